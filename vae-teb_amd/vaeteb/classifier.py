"""Config 4: the classification head trained jointly with SeqVaeTeb, on the HIP
kernels of libvaeteb.so (csrc/cls.hip + the shared linear / norm kernels).

Drop-in mirrors, same constructor arguments, forward / compute_loss contracts
and state_dict key names as the reference:
  FHRInception, FHRResidual, FHRInceptionTimeClassifier
                                  ref/model/inception_time.py:9-333
  SeqVaeTebClassifier             ref/model/vae_teb_model.py:1248-1526
Deviation: the reference's conv_long (kernel 40, padding 20)
returns L+1 positions and its concatenation raises for every L; the first L
are kept (the crop the golden fixtures were generated with).

Activations stay (B, L, C): the inception concatenation is four column slices
of one (B*L, 4f) buffer written in place by the branch convs, and the
reference's transposes around the convs and the attention vanish.
Dropout (nn.Dropout / Dropout1d / attention weights) uses a counter-hash mask
regenerated in the backward (seeds drawn from torch's CPU generator, so
torch.manual_seed makes runs repeatable).
"""
import ctypes
import math
import os

import torch
import torch.nn as nn

from . import _lib, ops
from ._lib import call, ptr
from .model import Activation, LayerNorm, Linear, SeqVaeTeb, _BatchNorm, _ConvWeight
from .ops import ACT, WS, _check, _ParamGrads, _st

_BN_WS = 4096 * 128 + 256


# the device seed offset of the classifier whose training forward is running (set for the
# duration of FHRInceptionTimeClassifier.forward): each dropout op keeps it with its host seed
_SEED_OFF = None


def _seed():
    """(host seed, device seed offset or None) of one dropout / attention-dropout op; the op
    keeps the pair for its backward (the same masks)."""
    return int(torch.randint(0, 2 ** 62, (1,)).item()), _SEED_OFF


# Dropout1d fused into the producing / consuming pass: the inception blocks' BatchNorm apply and
# backward (vt_batchnorm_{fwd,bwd}_dropout), the residual blocks' add + ReLU and its backward
# (vt_add_act_dropout_fwd, vt_act_dropout_bwd) — the same values as separate launches; 0: separate
BN_DROP_FUSE = int(os.environ.get("VAETEB_BN_DROP_FUSE", "1"))


def _sarg(seed):
    """The (seed, seed_offset pointer) call arguments of a _seed() pair (0 / NULL: no dropout)."""
    return (seed[0], ptr(seed[1])) if isinstance(seed, tuple) else (int(seed), None)


def _col(t, c0):
    """Device pointer of column c0 of a row-major (rows, C) buffer."""
    return t.data_ptr() + 4 * c0


def _zc(name, bf16):
    """The zero-pad conv entry point: exact fp32 (the parity path) or bf16 MFMA operands with fp32
    accumulation (vt_zconv16_*: the reference's 16-bit autocast, set_conv_precision("bf16"))."""
    assert name != "vt_zconv_bwd_weight_ws_floats"
    return name.replace("vt_zconv_", "vt_zconv16_") if bf16 else name


def _zcall(name, bf16, *args):
    """One zero-pad conv call (vt_zconv_fwd / _bwd_data / _bwd_weight arguments); bf16: the
    vt_zconv16_* kernel, whose forward / backward-data also take the workspace of the call's
    bf16 tap image (WS slot 6: the classifier's convolutions run in stream order)."""
    if bf16 and name in ("vt_zconv_fwd", "vt_zconv_bwd_data"):
        Cin, Cout, K = args[4], args[6], args[7]
        f = ctypes.c_int64()
        call("vt_zconv16_ws_floats", Cin, Cout, K, ctypes.byref(f))
        ws = WS.get(int(f.value), torch.device("cuda", torch.cuda.current_device()), 6)
        call(_zc(name, True), *args[:-1], ptr(ws), ws.numel(), args[-1])
    else:
        call(_zc(name, bf16), *args)


_TAPS_ELEMS = {}


def _tap_images(ws, flip, slot):
    """bf16 tap images of the block's weights ws = [(W, Cin, Cout, K), ...] in one launch
    (vt_zconv16_taps; flip: the backward-data images) -> one device pointer per weight, valid
    until the next use of WS slot `slot` (the block's convolutions run right after, in stream order)."""
    sizes = []
    for w, ci, co, k in ws:
        key = (co, ci, k) if flip else (ci, co, k)
        n = _TAPS_ELEMS.get(key)
        if n is None:
            e = ctypes.c_int64()
            call("vt_zconv16_taps_elems", *key, ctypes.byref(e))
            n = _TAPS_ELEMS[key] = (int(e.value) + 7) // 8 * 8   # 16-byte aligned images
        sizes.append(n)
    buf = WS.get((sum(sizes) + 1) // 2, ws[0][0].device, slot)
    base, ptrs = buf.data_ptr(), []
    for n in sizes:
        ptrs.append(base)
        base += 2 * n
    m = len(ws)
    W = (ctypes.c_int64 * m)(*[w.data_ptr() for w, _, _, _ in ws])
    Ci = (ctypes.c_int * m)(*[ci for _, ci, _, _ in ws])
    Co = (ctypes.c_int * m)(*[co for _, _, co, _ in ws])
    Ks = (ctypes.c_int * m)(*[k for _, _, _, k in ws])
    T = (ctypes.c_int64 * m)(*ptrs)
    call("vt_zconv16_taps", m, ctypes.addressof(W), ctypes.addressof(Ci), ctypes.addressof(Co), ctypes.addressof(Ks),
         int(flip), ctypes.addressof(T), _st())
    return ptrs


def _dw_ws(B, Cin, Cout, K, device):
    f = ctypes.c_int64()
    call("vt_zconv_bwd_weight_ws_floats", B, Cin, Cout, K, ctypes.byref(f))
    return WS.get(int(f.value), device, 4)


# ------------------------------------------------------------------ ops
class _InceptionF(torch.autograd.Function):
    """FHRInception.forward (ref/model/inception_time.py:89-117) in one op:
    bottleneck1 -> {conv 5, 15, 40} | maxpool3 -> bottleneck2 written as the
    column slices of the concatenation, train-mode BatchNorm + ReLU, Dropout1d."""

    @staticmethod
    def forward(ctx, x, wb1, ws, wm, wl, wb2, g, b, run_mean, run_var, momentum, eps, p, seed, bf16=False):
        _check(x, wb1, ws, wm, wl, wb2, g, b)
        x = x.contiguous()
        B, L, Cin = x.shape
        f = wb1.shape[0]
        C4 = 4 * f
        st = _st()
        x0 = torch.empty((B, L, f), device=x.device)
        cat = torch.empty((B, L, C4), device=x.device)
        mp = torch.empty_like(x)
        if bf16:   # the five tap images in one launch, then the convolutions read them
            T = _tap_images([(wb1, Cin, f, 1), (ws, f, f, 5), (wm, f, f, 15), (wl, f, f, 40), (wb2, Cin, f, 1)],
                            False, 7)
            call("vt_zconv16_fwd_t", ptr(x), Cin, B, L, Cin, T[0], f, 1, 0, ptr(x0), f, 0, st)
            for j, (K, P) in enumerate(((5, 2), (15, 7), (40, 20))):
                call("vt_zconv16_fwd_t", ptr(x0), f, B, L, f, T[1 + j], f, K, P, _col(cat, j * f), C4, 0, st)
            call("vt_maxpool3_fwd", ptr(x), B, L, Cin, ptr(mp), st)
            call("vt_zconv16_fwd_t", ptr(mp), Cin, B, L, Cin, T[4], f, 1, 0, _col(cat, 3 * f), C4, 0, st)
        else:
            call("vt_zconv_fwd", ptr(x), Cin, B, L, Cin, ptr(wb1), f, 1, 0, ptr(x0), f, 0, st)
            for j, (w, K, P) in enumerate(((ws, 5, 2), (wm, 15, 7), (wl, 40, 20))):
                call("vt_zconv_fwd", ptr(x0), f, B, L, f, ptr(w), f, K, P, _col(cat, j * f), C4, 0, st)
            call("vt_maxpool3_fwd", ptr(x), B, L, Cin, ptr(mp), st)
            call("vt_zconv_fwd", ptr(mp), Cin, B, L, Cin, ptr(wb2), f, 1, 0, _col(cat, 3 * f), C4, 0, st)
        y = torch.empty_like(cat)
        mean = torch.empty(C4, device=x.device)
        rstd = torch.empty(C4, device=x.device)
        bws = WS.get(_BN_WS, x.device, 5)
        if p > 0 and BN_DROP_FUSE:   # BN + ReLU + Dropout1d in the apply pass (the separate calls' values)
            call("vt_batchnorm_fwd_dropout", ptr(cat), B * L, C4, ptr(g), ptr(b), ACT["relu"], eps, momentum, ptr(y),
                 ptr(mean), ptr(rstd), ptr(run_mean), ptr(run_var), L, float(p), *_sarg(seed), ptr(bws), bws.numel(),
                 st)
        else:
            call("vt_batchnorm_fwd", ptr(cat), B * L, C4, ptr(g), ptr(b), ACT["relu"], eps, momentum, ptr(y),
                 ptr(mean), ptr(rstd), ptr(run_mean), ptr(run_var), ptr(bws), bws.numel(), st)
            if p > 0:
                call("vt_dropout_apply", ptr(y), y.numel(), C4, L, float(p), *_sarg(seed), ptr(y), st)
        ctx.save_for_backward(x, x0, mp, cat, mean, rstd)
        ctx.params = (wb1, ws, wm, wl, wb2, g, b)
        ctx.cfg = (p, seed, bf16)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, x0, mp, cat, mean, rstd = ctx.saved_tensors
        wb1, ws, wm, wl, wb2, g, b = ctx.params
        p, seed, bf16 = ctx.cfg
        B, L, Cin = x.shape
        f = wb1.shape[0]
        C4 = 4 * f
        st = _st()
        gy = gy.contiguous()
        if p > 0 and not BN_DROP_FUSE:
            gd = torch.empty_like(gy)
            call("vt_dropout_apply", ptr(gy), gy.numel(), C4, L, float(p), *_sarg(seed), ptr(gd), st)
            gy = gd
        gcat = torch.empty_like(cat)
        pbn = _ParamGrads([g, b], [True, True])
        bws = WS.get(_BN_WS, x.device, 5)
        # the Dropout1d mask applied as the BatchNorm backward reads gy (p = 0: plain backward)
        pf = float(p) if BN_DROP_FUSE else 0.0
        call("vt_batchnorm_bwd_dropout", ptr(gy), ptr(cat), B * L, C4, ptr(mean), ptr(rstd), ptr(g), ptr(b),
             ACT["relu"], L, pf, *_sarg(seed), ptr(gcat), ptr(pbn.out[0]), ptr(pbn.out[1]), pbn.acc, ptr(bws),
             bws.numel(), st)
        pw = _ParamGrads([wb1, ws, wm, wl, wb2], [True] * 5)
        gx0 = torch.empty_like(x0)
        # backward-data taps: one launch for the block's five flipped images (bf16)
        T = _tap_images([(wb1, Cin, f, 1), (ws, f, f, 5), (wm, f, f, 15), (wl, f, f, 40), (wb2, Cin, f, 1)],
                        True, 7) if bf16 else None
        bd = (lambda j, w: T[j]) if bf16 else (lambda j, w: ptr(w))
        zbd = "vt_zconv16_bwd_data_t" if bf16 else "vt_zconv_bwd_data"
        for j, (w, K, P) in enumerate(((ws, 5, 2), (wm, 15, 7), (wl, 40, 20))):
            call(zbd, _col(gcat, j * f), C4, B, L, f, bd(1 + j, w), f, K, P, ptr(gx0), f, int(j > 0), st)
            dws = _dw_ws(B, f, f, K, x.device)
            _zcall("vt_zconv_bwd_weight", bf16, _col(gcat, j * f), C4, ptr(x0), f, B, L, f, f, K, P,
                   ptr(pw.out[1 + j]), pw.acc, ptr(dws), dws.numel(), st)
        gmp = torch.empty_like(mp)
        call(zbd, _col(gcat, 3 * f), C4, B, L, Cin, bd(4, wb2), f, 1, 0, ptr(gmp), Cin, 0, st)
        dws = _dw_ws(B, Cin, f, 1, x.device)
        _zcall("vt_zconv_bwd_weight", bf16, _col(gcat, 3 * f), C4, ptr(mp), Cin, B, L, Cin, f, 1, 0, ptr(pw.out[4]),
               pw.acc, ptr(dws), dws.numel(), st)
        gx = None
        if ctx.needs_input_grad[0]:
            gx = torch.empty_like(x)
            call("vt_maxpool3_bwd", ptr(gmp), ptr(x), B, L, Cin, ptr(gx), 0, st)
            call(zbd, ptr(gx0), f, B, L, Cin, bd(0, wb1), f, 1, 0, ptr(gx), Cin, 1, st)
        _zcall("vt_zconv_bwd_weight", bf16, ptr(gx0), f, ptr(x), Cin, B, L, Cin, f, 1, 0, ptr(pw.out[0]), pw.acc,
               ptr(dws), dws.numel(), st)
        gws = pw.result()
        gg, gb = pbn.result()
        return (gx, *gws, gg, gb) + (None,) * 7


class _ResidualF(torch.autograd.Function):
    """FHRResidual.forward (ref/model/inception_time.py:152-170):
    relu(y + BN(bottleneck(x))) then Dropout1d."""

    @staticmethod
    def forward(ctx, x, y, w, g, b, run_mean, run_var, momentum, eps, p, seed, bf16=False):
        _check(x, y, w, g, b)
        x, y = x.contiguous(), y.contiguous()
        B, L, Cin = x.shape
        C4 = w.shape[0]
        st = _st()
        r = torch.empty((B, L, C4), device=x.device)
        _zcall("vt_zconv_fwd", bf16, ptr(x), Cin, B, L, Cin, ptr(w), C4, 1, 0, ptr(r), C4, 0, st)
        rb = torch.empty_like(r)
        mean = torch.empty(C4, device=x.device)
        rstd = torch.empty(C4, device=x.device)
        bws = WS.get(_BN_WS, x.device, 5)
        call("vt_batchnorm_fwd", ptr(r), B * L, C4, ptr(g), ptr(b), ACT["none"], eps, momentum, ptr(rb), ptr(mean),
             ptr(rstd), ptr(run_mean), ptr(run_var), ptr(bws), bws.numel(), st)
        s = torch.empty_like(r)
        out = s
        if p > 0 and BN_DROP_FUSE:   # s = relu(y + rb) saved, out = Dropout1d(s): one pass
            out = torch.empty_like(s)
            call("vt_add_act_dropout_fwd", ptr(y), ptr(rb), s.numel(), C4, ACT["relu"], L, float(p), *_sarg(seed),
                 ptr(s), ptr(out), st)
        else:
            call("vt_add_act_fwd", ptr(y), ptr(rb), s.numel(), ACT["relu"], ptr(s), st)
            if p > 0:
                out = torch.empty_like(s)
                call("vt_dropout_apply", ptr(s), s.numel(), C4, L, float(p), *_sarg(seed), ptr(out), st)
        ctx.save_for_backward(x, r, s, mean, rstd)
        ctx.params = (w, g, b)
        ctx.cfg = (p, seed, bf16)
        return out

    @staticmethod
    def backward(ctx, gout):
        x, r, s, mean, rstd = ctx.saved_tensors
        w, g, b = ctx.params
        p, seed, bf16 = ctx.cfg
        B, L, Cin = x.shape
        C4 = w.shape[0]
        st = _st()
        gout = gout.contiguous()
        gs = torch.empty_like(s)
        if p > 0 and BN_DROP_FUSE:   # Dropout1d(gout) relu'(s) in one pass
            call("vt_act_dropout_bwd", ptr(gout), ptr(s), s.numel(), C4, ACT["relu"], L, float(p), *_sarg(seed),
                 ptr(gs), st)
        else:
            src = gout
            if p > 0:
                call("vt_dropout_apply", ptr(gout), gout.numel(), C4, L, float(p), *_sarg(seed), ptr(gs), st)
                src = gs
            call("vt_act_bwd", ptr(src), ptr(s), s.numel(), ACT["relu"], ptr(gs), st)
        gr = torch.empty_like(r)
        pbn = _ParamGrads([g, b], [True, True])
        bws = WS.get(_BN_WS, x.device, 5)
        call("vt_batchnorm_bwd", ptr(gs), ptr(r), B * L, C4, ptr(mean), ptr(rstd), ptr(g), ptr(b), ACT["none"],
             ptr(gr), ptr(pbn.out[0]), ptr(pbn.out[1]), pbn.acc, ptr(bws), bws.numel(), st)
        pw = _ParamGrads([w], [True])
        dws = _dw_ws(B, Cin, C4, 1, x.device)
        _zcall("vt_zconv_bwd_weight", bf16, ptr(gr), C4, ptr(x), Cin, B, L, Cin, C4, 1, 0, ptr(pw.out[0]), pw.acc,
               ptr(dws), dws.numel(), st)
        gx = None
        if ctx.needs_input_grad[0]:
            gx = torch.empty_like(x)
            _zcall("vt_zconv_bwd_data", bf16, ptr(gr), C4, B, L, Cin, ptr(w), C4, 1, 0, ptr(gx), Cin, 0, st)
        gw, = pw.result()
        gg, gb = pbn.result()
        return gx, gs, gw, gg, gb, None, None, None, None, None, None, None


class _AttnCoreF(torch.autograd.Function):
    """softmax(Q K^T / sqrt(d)) (dropout) V over packed in-projections (B, S, 3E)."""

    @staticmethod
    def forward(ctx, qkv, H, p, seed):
        _check(qkv)
        qkv = qkv.contiguous()
        B, S, E3 = qkv.shape
        E = E3 // 3
        scale = 1.0 / math.sqrt(E // H)
        out = torch.empty((B, S, E), device=qkv.device)
        lse = torch.empty((B, H, S), device=qkv.device)
        call("vt_attn_fwd", ptr(qkv), B, S, H, scale, float(p), *_sarg(seed), ptr(out), ptr(lse), _st())
        ctx.save_for_backward(qkv, out, lse)
        ctx.cfg = (H, scale, p, seed)
        return out

    @staticmethod
    def backward(ctx, gout):
        qkv, out, lse = ctx.saved_tensors
        H, scale, p, seed = ctx.cfg
        B, S, _ = qkv.shape
        dqkv = torch.empty_like(qkv)
        call("vt_attn_bwd", ptr(qkv), ptr(out), ptr(gout.contiguous()), ptr(lse), B, S, H, scale, float(p), *_sarg(seed),
             ptr(dqkv), _st())
        return dqkv, None, None, None


class _AddF(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, b):
        _check(a, b)
        y = torch.empty_like(a)
        call("vt_add_act_fwd", ptr(a.contiguous()), ptr(b.contiguous()), y.numel(), 0, ptr(y), _st())
        return y

    @staticmethod
    def backward(ctx, gy):
        return gy, gy


class _ActF(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, act):
        _check(x)
        x = x.contiguous()
        y = torch.empty_like(x)
        call("vt_act_fwd", ptr(x), x.numel(), ACT[act], ptr(y), _st())
        ctx.save_for_backward(x)
        ctx.act = act
        return y

    @staticmethod
    def backward(ctx, gy):
        x, = ctx.saved_tensors
        gx = torch.empty_like(x)
        call("vt_act_bwd", ptr(gy.contiguous()), ptr(x), x.numel(), ACT[ctx.act], ptr(gx), _st())
        return gx, None


class _DropoutF(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, p, seed):
        _check(x)
        x = x.contiguous()
        y = torch.empty_like(x)
        call("vt_dropout_apply", ptr(x), x.numel(), x.shape[-1], 0, float(p), *_sarg(seed), ptr(y), _st())
        ctx.cfg = (p, seed)
        return y

    @staticmethod
    def backward(ctx, gy):
        p, seed = ctx.cfg
        gy = gy.contiguous()
        gx = torch.empty_like(gy)
        call("vt_dropout_apply", ptr(gy), gy.numel(), gy.shape[-1], 0, float(p), *_sarg(seed), ptr(gx), _st())
        return gx, None, None


class _TimeMeanF(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        _check(x)
        x = x.contiguous()
        B, L, C = x.shape
        y = torch.empty((B, C), device=x.device)
        call("vt_time_mean_fwd", ptr(x), B, L, C, ptr(y), _st())
        ctx.shape = (B, L, C)
        return y

    @staticmethod
    def backward(ctx, gy):
        B, L, C = ctx.shape
        gx = torch.empty((B, L, C), device=gy.device)
        call("vt_time_mean_bwd", ptr(gy.contiguous()), B, L, C, ptr(gx), 0, _st())
        return gx


class _CrossEntropyF(torch.autograd.Function):
    """nn.CrossEntropyLoss() (mean); also returns the softmax probabilities."""

    @staticmethod
    def forward(ctx, logits, labels):
        _check(logits)
        logits = logits.contiguous()
        labels = labels.to(device=logits.device, dtype=torch.int64).contiguous()
        B, C = logits.shape
        loss = torch.empty((), device=logits.device)
        probs = torch.empty_like(logits)
        call("vt_cross_entropy_fwd", ptr(logits), ptr(labels), B, C, ptr(loss), ptr(probs), _st())
        ctx.save_for_backward(probs, labels)
        ctx.mark_non_differentiable(probs)
        return loss, probs

    @staticmethod
    def backward(ctx, gloss, gprobs):
        probs, labels = ctx.saved_tensors
        B, C = probs.shape
        gl = torch.empty_like(probs)
        call("vt_cross_entropy_bwd", ptr(probs), ptr(labels), B, C, ptr(gloss.contiguous()), ptr(gl), _st())
        return gl, None


def cross_entropy(logits, labels):
    """(mean CE loss, softmax probabilities)."""
    return _CrossEntropyF.apply(logits, labels)


def _dropout(x, p, training):
    return _DropoutF.apply(x, p, _seed()) if (training and p > 0) else x


def _no_grad_check(*ts):
    if torch.is_grad_enabled() and any(t.requires_grad for t in ts):
        raise RuntimeError("eval-mode classifier blocks are inference-only (run under torch.no_grad())")


def _inception_eval(m, x):
    """FHRInception in eval mode: BatchNorm with the running statistics, no dropout."""
    _no_grad_check(x, m.bottleneck1.weight)
    x = x.contiguous()
    B, L, Cin = x.shape
    f = m.bottleneck1.weight.shape[0]
    C4 = 4 * f
    st = _st()
    x0 = torch.empty((B, L, f), device=x.device)
    bf16 = m.bf16
    _zcall("vt_zconv_fwd", bf16, ptr(x), Cin, B, L, Cin, ptr(m.bottleneck1.weight), f, 1, 0, ptr(x0), f, 0, st)
    cat = torch.empty((B, L, C4), device=x.device)
    for j, (w, K, P) in enumerate(((m.conv_short.weight, 5, 2), (m.conv_medium.weight, 15, 7),
                                   (m.conv_long.weight, 40, 20))):
        _zcall("vt_zconv_fwd", bf16, ptr(x0), f, B, L, f, ptr(w), f, K, P, _col(cat, j * f), C4, 0, st)
    mp = torch.empty_like(x)
    call("vt_maxpool3_fwd", ptr(x), B, L, Cin, ptr(mp), st)
    _zcall("vt_zconv_fwd", bf16, ptr(mp), Cin, B, L, Cin, ptr(m.bottleneck2.weight), f, 1, 0, _col(cat, 3 * f), C4,
           0, st)
    bn = m.batch_norm
    call("vt_batchnorm_eval", ptr(cat), B * L, C4, ptr(bn.running_mean), ptr(bn.running_var), bn.eps, ptr(bn.weight),
         ptr(bn.bias), ACT["relu"], ptr(cat), st)
    return cat


def _residual_eval(m, x, y):
    _no_grad_check(x, y, m.bottleneck.weight)
    x, y = x.contiguous(), y.contiguous()
    B, L, Cin = x.shape
    C4 = m.bottleneck.weight.shape[0]
    st = _st()
    r = torch.empty((B, L, C4), device=x.device)
    _zcall("vt_zconv_fwd", m.bf16, ptr(x), Cin, B, L, Cin, ptr(m.bottleneck.weight), C4, 1, 0, ptr(r), C4, 0, st)
    bn = m.batch_norm
    call("vt_batchnorm_eval", ptr(r), B * L, C4, ptr(bn.running_mean), ptr(bn.running_var), bn.eps, ptr(bn.weight),
         ptr(bn.bias), ACT["none"], ptr(r), st)
    call("vt_add_act_fwd", ptr(y), ptr(r), r.numel(), ACT["relu"], ptr(r), st)
    return r


# -------------------------------------------------------------- modules
class FHRInception(nn.Module):
    """ref/model/inception_time.py:9-117 (kaiming fan_out init, :80-87)."""

    def __init__(self, input_size, filters, dropout=0.1):
        super().__init__()
        self.bottleneck1 = _ConvWeight(input_size, filters, 1)
        self.conv_short = _ConvWeight(filters, filters, 5)
        self.conv_medium = _ConvWeight(filters, filters, 15)
        self.conv_long = _ConvWeight(filters, filters, 40)
        self.bottleneck2 = _ConvWeight(input_size, filters, 1)
        self.batch_norm = _BatchNorm(4 * filters, momentum=0.1)
        self.dropout = dropout
        self.bf16 = False   # bf16-MFMA convolutions (FHRInceptionTimeClassifier.set_conv_precision)
        for m in (self.bottleneck1, self.conv_short, self.conv_medium, self.conv_long, self.bottleneck2):
            nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")

    def forward(self, x):
        if not self.training:
            return _inception_eval(self, x)
        bn = self.batch_norm
        p = self.dropout
        y = _InceptionF.apply(x, self.bottleneck1.weight, self.conv_short.weight, self.conv_medium.weight,
                              self.conv_long.weight, self.bottleneck2.weight, bn.weight, bn.bias, bn.running_mean,
                              bn.running_var, bn.momentum, bn.eps, p, _seed() if p > 0 else 0, self.bf16)
        bn.num_batches_tracked.add_(1)
        return y


class FHRResidual(nn.Module):
    """ref/model/inception_time.py:119-170."""

    def __init__(self, input_size, filters, dropout=0.1):
        super().__init__()
        self.bottleneck = _ConvWeight(input_size, 4 * filters, 1)
        self.batch_norm = _BatchNorm(4 * filters, momentum=0.1)
        self.dropout = dropout
        self.bf16 = False
        nn.init.kaiming_normal_(self.bottleneck.weight, mode="fan_out", nonlinearity="relu")

    def forward(self, x, y):
        bn = self.batch_norm
        if not self.training:
            return _residual_eval(self, x, y)
        p = self.dropout
        out = _ResidualF.apply(x, y, self.bottleneck.weight, bn.weight, bn.bias, bn.running_mean, bn.running_var,
                               bn.momentum, bn.eps, p, _seed() if p > 0 else 0, self.bf16)
        bn.num_batches_tracked.add_(1)
        return out


class MultiheadAttention(nn.Module):
    """nn.MultiheadAttention(embed_dim, num_heads, dropout, batch_first=True)
    self-attention with its parameter names (in_proj_weight / in_proj_bias /
    out_proj); head dim 32."""

    def __init__(self, embed_dim, num_heads, dropout=0.0, batch_first=True):
        super().__init__()
        if not batch_first or embed_dim // num_heads != 32 or embed_dim % num_heads:
            raise ValueError("MultiheadAttention: batch_first with head dim 32 only")
        self.embed_dim, self.num_heads, self.dropout = embed_dim, num_heads, dropout
        self.in_proj_weight = nn.Parameter(torch.empty(3 * embed_dim, embed_dim))
        self.in_proj_bias = nn.Parameter(torch.zeros(3 * embed_dim))
        self.out_proj = Linear(embed_dim, embed_dim)
        nn.init.xavier_uniform_(self.in_proj_weight)
        nn.init.zeros_(self.out_proj.bias)

    def forward(self, query, key=None, value=None):
        """Self-attention only (the reference calls attention(y, y, y)); returns
        (attn_output, None) like need_weights=False."""
        if (key is not None and key is not query) or (value is not None and value is not query):
            raise NotImplementedError("MultiheadAttention: self-attention only")
        qkv = ops.linear(query, self.in_proj_weight, self.in_proj_bias)
        p = self.dropout if self.training else 0.0
        o = _AttnCoreF.apply(qkv, self.num_heads, p, _seed() if p > 0 else 0)
        return self.out_proj(o), None


class FHRInceptionTimeClassifier(nn.Module):
    """ref/model/inception_time.py:185-333: same constructor, forward
    x (B, S, latent) -> logits (B, num_classes), same state_dict keys."""

    def __init__(self, input_size=32, num_classes=2, filters=32, depth=6, dropout=0.2, use_attention=True):
        super().__init__()
        self.input_size, self.num_classes, self.filters = input_size, num_classes, filters
        self.depth, self.dropout, self.use_attention = depth, dropout, use_attention
        self.input_projection = nn.Sequential(LayerNorm(input_size), Linear(input_size, input_size),
                                              Activation("gelu"), Activation("dropout"))
        self.inception_blocks = nn.ModuleList()
        self.residual_blocks = nn.ModuleList()
        for d in range(depth):
            self.inception_blocks.append(FHRInception(input_size if d == 0 else 4 * filters, filters, dropout))
            if d % 3 == 2:
                self.residual_blocks.append(FHRResidual(input_size if d == 2 else 4 * filters, filters, dropout))
        if use_attention:
            self.attention = MultiheadAttention(4 * filters, 4, dropout=dropout, batch_first=True)
            self.attention_norm = LayerNorm(4 * filters)
        f = filters
        self.classifier = nn.Sequential(Linear(4 * f, 2 * f), LayerNorm(2 * f), Activation("gelu"),
                                        Activation("dropout"), Linear(2 * f, f), LayerNorm(f), Activation("gelu"),
                                        Activation("dropout"), Linear(f, num_classes))

    def set_conv_precision(self, precision):
        """"fp32": the inception / residual convolutions on the exact-fp32 kernels (parity mode);
        "bf16": on bf16 MFMA with fp32 accumulation (vt_zconv16_*), the reference's 16-bit
        autocast training precision (ref/model/graph_model.py:510) in bf16: forward,
        backward-data and weight gradient."""
        if precision not in ("fp32", "bf16"):
            raise ValueError(f"conv precision must be 'fp32' or 'bf16', got {precision!r}")
        for m in self.modules():
            if isinstance(m, (FHRInception, FHRResidual)):
                m.bf16 = precision == "bf16"
        return self

    def forward(self, x):
        global _SEED_OFF
        if self.training and self.dropout > 0 and x.is_cuda:
            # a device-side seed offset added to every host-drawn dropout seed.  Eager steps draw
            # fresh host seeds (torch's CPU generator: torch.manual_seed makes runs repeatable);
            # a captured step freezes them, so its forward advances the offset on the device
            # once (a kernel in the graph): every replay draws new masks, and its backward reads
            # the same offset as its forward (each op keeps this model's offset tensor, _seed())
            off = getattr(self, "_seed_off", None)
            if off is None or off.device != x.device:
                self._seed_off = off = torch.zeros(1, dtype=torch.int64, device=x.device)
            if torch.cuda.is_current_stream_capturing():
                call("vt_dropout_seed_advance", off.data_ptr(), _st())
            prev, _SEED_OFF = _SEED_OFF, off
            try:
                return self._forward(x)
            finally:
                _SEED_OFF = prev
        return self._forward(x)

    def _forward(self, x):
        tr = self.training
        ip = self.input_projection
        h = ip[0](x)
        h = _ActF.apply(ip[1](h), "gelu")
        x = _dropout(h, self.dropout * 0.5, tr)             # (B, S, latent): no transpose needed
        residual_inputs, ri = [x], 0
        y = x
        for d in range(self.depth):
            y = self.inception_blocks[d](x if d == 0 else y)
            if d % 3 == 2:
                y = self.residual_blocks[ri](residual_inputs[ri], y)
                residual_inputs.append(y)
                ri += 1
                x = y
        if self.use_attention:
            attn_out, _ = self.attention(y)
            y = self.attention_norm(_AddF.apply(y, attn_out))
        pooled = _TimeMeanF.apply(y)                        # AdaptiveAvgPool1d(1) over time
        c = self.classifier
        h = _dropout(c[1](c[0](pooled), "gelu"), self.dropout, tr)
        h = _dropout(c[5](c[4](h), "gelu"), self.dropout, tr)
        return c[8](h)


class SeqVaeTebClassifier(nn.Module):
    """ref/model/vae_teb_model.py:1248-1526.  freeze_vae=False is the multi-task
    configuration of BASELINE.json config 4 (ELBO with beta 1 + CE, end to end);
    freeze_vae=True (the reference default) runs the VAE in eval mode without
    gradients and trains the classifier only."""

    def __init__(self, input_channels=76, sequence_length=300, latent_dim_source=32, latent_dim_target=32,
                 latent_dim_z=32, decimation_factor=16, warmup_period=30, num_classes=2, classifier_filters=32,
                 classifier_depth=6, classifier_dropout=0.2, use_attention=True, freeze_vae=True,
                 pretrained_vae_path=None, **vae_kwargs):
        super().__init__()
        self.freeze_vae, self.num_classes, self.latent_dim_z = freeze_vae, num_classes, latent_dim_z
        self.vae_model = SeqVaeTeb(input_channels=input_channels, sequence_length=sequence_length,
                                   latent_dim_source=latent_dim_source, latent_dim_target=latent_dim_target,
                                   latent_dim_z=latent_dim_z, decimation_factor=decimation_factor,
                                   warmup_period=warmup_period, **vae_kwargs)
        if pretrained_vae_path is not None:
            self.load_pretrained_vae(pretrained_vae_path)
        if freeze_vae:
            self.freeze_vae_parameters()
        self.classifier = FHRInceptionTimeClassifier(input_size=latent_dim_z, num_classes=num_classes,
                                                     filters=classifier_filters, depth=classifier_depth,
                                                     dropout=classifier_dropout, use_attention=use_attention)
        # the VAE's conv precision (SeqVaeTeb(conv_precision=...)) applies to the classifier's convs too
        if vae_kwargs.get("conv_precision") == "bf16":
            self.classifier.set_conv_precision("bf16")

    def load_pretrained_vae(self, path):
        """ref :1322-1348 (weights-only load; keys model_state_dict / state_dict / bare)."""
        ck = torch.load(path, map_location="cpu", weights_only=True)
        sd = ck.get("model_state_dict", ck.get("state_dict", ck)) if isinstance(ck, dict) else ck
        return self.vae_model.load_state_dict(sd, strict=False)

    def freeze_vae_parameters(self):
        for p in self.vae_model.parameters():
            p.requires_grad = False

    def unfreeze_vae_parameters(self):
        for p in self.vae_model.parameters():
            p.requires_grad = True

    def extract_latent_features(self, y_st, y_ph, x_ph, return_all_outputs=False, eps=None):
        """ref :1350-1390: a frozen VAE runs in eval mode without gradients."""
        if self.freeze_vae:
            self.vae_model.eval()
        with torch.set_grad_enabled(torch.is_grad_enabled() and not self.freeze_vae):
            out = self.vae_model(y_st, y_ph, x_ph, eps=eps)
        return (out["z"], out) if return_all_outputs else out["z"]

    def predict(self, y_st, y_ph, x_ph, return_probabilities=True):
        """ref :1500-1526."""
        self.eval()
        with torch.no_grad():
            out = self.forward(y_st, y_ph, x_ph)
        return (out["predictions"], out["probabilities"]) if return_probabilities else out["predictions"]

    def forward(self, y_st, y_ph, x_ph, labels=None, return_latent=False, eps=None):
        z = self.extract_latent_features(y_st, y_ph, x_ph, eps=eps)
        logits = self.classifier(z)
        loss, probs = (None, None)
        if labels is not None:
            loss, probs = cross_entropy(logits, labels)
        else:
            probs = torch.softmax(logits, dim=-1)
        out = {"logits": logits, "probabilities": probs, "predictions": torch.argmax(logits, dim=-1),
               "classification_loss": loss}
        if return_latent:
            out["latent_z"] = z
        return out

    def compute_loss(self, y_st, y_ph, x_ph, labels, y_raw=None, compute_vae_loss=False, vae_loss_weight=0.1,
                     eps=None):
        """ref :1440-1498 — same keys; the VAE loss uses beta = 1."""
        if compute_vae_loss and y_raw is not None:
            z, fw = self.extract_latent_features(y_st, y_ph, x_ph, return_all_outputs=True, eps=eps)
            vae_total = self.vae_model.compute_loss(fw, y_st, y_ph, y_raw, compute_kld_loss=True,
                                                    beta=1.0)["total_loss"]
        else:
            z = self.extract_latent_features(y_st, y_ph, x_ph, eps=eps)
            vae_total = torch.zeros((), device=z.device)
        logits = self.classifier(z)
        ce, probs = cross_entropy(logits, labels)
        return {"classification_loss": ce, "vae_loss": vae_total, "total_loss": ce + vae_loss_weight * vae_total,
                "logits": logits, "probabilities": probs, "predictions": torch.argmax(logits, dim=-1)}
