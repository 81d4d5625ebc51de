"""Autograd wrappers of the HIP kernels (every compute op of the training step).

Each Function calls into libvaeteb.so through the C ABI (vaeteb._lib); the
tensors are only device buffers here.  Activations are (rows, C) row-major
with rows = B*S (or B*L for the conv stacks), the layout the kernels assume,
so no transposes are needed between the MLP, conv and LSTM stages (the
reference transposes to (B, C, L) for torch's conv1d at
ref/model/vae_teb_model.py:539,545,693,917).
"""
import ctypes
import os

import torch

from . import _lib
from ._lib import call, ptr

ACT = {"none": 0, "relu": 1, "gelu": 2, "tanh": 3}


# --------------------------------------------------------------- workspace
class _Workspace:
    """Grow-only scratch per (device, stream); ops are stream-ordered on the
    current stream, so consecutive ops on one stream may reuse it, and ops on
    concurrent streams (the two encoders) never share it."""

    def __init__(self):
        self.buf = {}

    def get(self, nfloats, device, slot=0):
        key = (device.index, slot, _lib.stream() if device.type == "cuda" else 0)
        b = self.buf.get(key)
        if b is None or b.numel() < nfloats:
            b = torch.empty(max(int(nfloats), 1 << 20), dtype=torch.float32, device=device)
            self.buf[key] = b
        return b


WS = _Workspace()
CAPTURE_TRACE = os.environ.get("VAETEB_CAPTURE_TRACE", "0") == "1"   # diagnostic: capture state dumps
WS_LINEAR = 1 << 25  # 128 MiB of split-K partials (a 4096x4097 head gradient fits unsplit)


def _st():
    return _lib.stream()


def _check(*ts):
    for t in ts:
        if t is not None and (t.dtype != torch.float32 or not t.is_cuda):
            raise TypeError(f"expected a CUDA float32 tensor, got {t.dtype} on {t.device}")


# ------------------------------------------------------- 16-bit operand format
# A module's 16-bit flag (Linear.mfma, ResidualMLP.bf16, ConvBlock.bf16): False (fp32 kernels),
# "bf16" (or True) or "fp16" — the operand type of the library's 16-bit MFMA kernels (csrc/h16.h).
# Every op that launches them selects the format first, in its forward and in its backward, so
# models of either format can share a process; fp16 is the reference's autocast width and is
# trained with the dynamic loss scale of vaeteb.train.Trainer (GradScaler).
def h16_flag(flag):
    """Normalise a 16-bit flag: False, "bf16" or "fp16"."""
    if not flag:
        return False
    return "fp16" if flag == "fp16" else "bf16"


def _h16(flag):
    if flag:
        _lib.set_h16(flag == "fp16")


def _shadow_dtype():
    return torch.float16 if _lib._H16[0] == 1 else torch.bfloat16


# ----------------------------------------------------------- gradient sink
# Parameters whose .grad is a persistent view of the trainer's flat gradient
# buffer (vaeteb.train.FlatState sets p._vt_sink) receive their gradient
# directly from the kernel, accumulated in place (the buffer is zeroed once
# per step), and the op returns None to autograd for them: no per-parameter
# AccumulateGrad add kernel (~540 launches per step).  GRAD_READY(p) is then
# called instead of the post-accumulate-grad hook (bucketed all-reduce).
GRAD_READY = None
SIDE_STREAMS = []   # extra streams the model runs work on (see SeqVaeTeb.concurrent_encoders)
GRAD_STREAM = None  # side stream for weight gradients off the data-gradient chain (set by SeqVaeTeb)
HEAD_GRAD_STREAM = None  # ... for the bf16-MFMA decoder-head weight gradients (set by SeqVaeTeb)
# first-writer gradient groups of the current Trainer step (vaeteb.train.FlatState.first_writer):
# id(weight) -> [weight, bias]; LinearF's weight-gradient call writes the group's first gradient
# with accumulate = 0 and removes it
FIRST_WRITER = {}
FIRST_WRITER_HIT = []   # group indices LinearF wrote this step (FlatState.finish_first_writer)

# decoder-head weight gradients (bf16 MFMA, in-place sinks) enqueued at the end of the backward
# when they have no side stream (VAETEB_HEAD_DW_DEFER=1)
HEAD_DW_DEFER = os.environ.get("VAETEB_HEAD_DW_DEFER", "0") == "1"
_DEFERRED = []


def _flush_deferred():
    """Run the work deferred to the end of this backward pass, in the order it was deferred
    (an autograd engine callback, queued by the first deferral of a pass)."""
    work = list(_DEFERRED)
    _DEFERRED.clear()
    for fn in work:
        fn()


def _defer(fn):
    if not _DEFERRED:
        torch.autograd.Variable._execution_engine.queue_callback(_flush_deferred)
    _DEFERRED.append(fn)


# diagnostic: join the head weight-gradient branch back right after its kernel (capture probe)
HEAD_GRAD_JOIN = os.environ.get("VAETEB_HEAD_GRAD_JOIN", "0") == "1"
LSTM_GRAD_STREAM = None  # ... for the LSTM weight gradients (set by SeqVaeTeb)
# LSTM input projections inside the recurrence kernels (vt_lstm_layer_{fwd,bwd}_x) for
# input sizes <= 64; 0: separate skinny GEMMs (the same results bit for bit)
LSTM_FUSED = int(os.environ.get("VAETEB_LSTM_FUSED", "1"))
# LSTM parameter gradients (in-place sinks) issued after the whole backward recurrence
# chain (on LSTM_GRAD_STREAM when set) instead of after each layer's recurrence
LSTM_GRAD_DEFER = int(os.environ.get("VAETEB_LSTM_GRAD_DEFER", "1"))
# 16-bit LSTM layers two at a time (vt_lstm16_pair_fwd / _bwd: the upper layer one chunk
# behind the lower in the same workgroup, bit-identical to the per-layer kernels)
LSTM_PAIR = int(os.environ.get("VAETEB_L16_PAIR", "1"))
_L16_PAIR_NS = 4 if os.environ.get("VAETEB_L16_PAIR_NS") == "4" else 2
# 4-layer 16-bit LSTMs as ONE launch each way (vt_lstm16_quad_fwd / _bwd: the two layer pairs
# concurrent, chained chunk by chunk through per-chunk flags; bit-identical to the pair launches)
LSTM_CHAIN_FWD = int(os.environ.get("VAETEB_L16_CHAIN_FWD", "1"))
LSTM_CHAIN_BWD = int(os.environ.get("VAETEB_L16_CHAIN_BWD", "1"))


def _l16_pair_fits(S):
    """The pair forward stages its lower layer's input in LDS: NS x ceil16(S) rows of 144 B
    within 120 KB (csrc/lstm16.hip fwd2_stage_bytes)."""
    return _L16_PAIR_NS * ((S + 15) // 16) * 16 * 72 * 2 <= 120 * 1024
# bf16 ResidualMLP backward split in two (vt_resmlp_bf16_bwd_data on the chain, the weight gradients
# from the saved dZ rows on the weight-gradient side stream); 0: the one-kernel backward
MLPB_SPLIT = int(os.environ.get("VAETEB_MLPB_SPLIT", "0"))
# bf16 conv backward-data written straight into dX where the fold is a crop; 0: gpad + fold
CONV_DIRECT_DX = int(os.environ.get("VAETEB_CONV_DIRECT_DX", "1"))
# conv-block backward as vt_batchnorm_bwd_x16 + vt_conv1d_bwd_dx16 (bf16 operand written once,
# upsample fold inside the conv); 0: the fused-staging kernels (vt_conv1d_bwd_*_bf16_bn)
CONV_BWD16 = int(os.environ.get("VAETEB_CONV_BWD16", "1"))


class _ParamGrads:
    """Gradient destinations of an op's parameters: all their .grad sinks
    (accumulate = 1) or, if any of them has none, fresh tensors (accumulate = 0)."""

    def __init__(self, params, needed):
        self.params, self.needed = params, needed
        sinks = [p.grad if (n and getattr(p, "_vt_sink", False) and p.grad is not None and p.grad.is_contiguous())
                 else None for p, n in zip(params, needed)]
        self.direct = all(sk is not None for sk, n in zip(sinks, needed) if n) and any(needed)
        if self.direct:
            self.out = sinks
        else:
            self.out = [torch.empty_like(p) if n else None for p, n in zip(params, needed)]
        self.acc = 1 if self.direct else 0

    def result(self):
        """What backward returns for the parameters (None when written in place)."""
        if not self.direct:
            return list(self.out)
        if GRAD_READY is not None:
            for p, n in zip(self.params, self.needed):
                if n:
                    GRAD_READY(p)
        return [None] * len(self.params)


# ------------------------------------------------------------------ Linear
def mfma_ok(K, N):
    """bf16 MFMA path available for a K -> N linear (vt_mfma_supported)."""
    return bool(_lib.lib().fns["vt_mfma_supported"](K, N))


_SHADOW = {}
# Shadows written ahead by prepare_shadows(): key -> event recorded after them on the
# prepass stream.  A forward that finds its weight here waits on the event instead of
# rewriting the shadow on its own (critical-path) stream; each entry serves one use.
_PREPARED = {}


# Shadows the trainer's optimizer step wrote together with the weights (Trainer._update:
# vt_adamw_step_dev_shadow / vt_conv1d_bf16_shadow_batch): key -> the weight's torch version
# counter at that time.  A forward finding its weight here at the same version uses the shadow
# as it is; any torch-side in-place change of the weight (load_state_dict, copy_) bumps the
# counter and the shadow is rewritten, and every other optimizer path clears the table.
_FRESH = {}


def mark_fresh(key, w):
    import weakref
    _FRESH[key] = (weakref.ref(w), w._version)


def _fresh(key, w):
    # the same tensor object (an address reused by a later model is not a match) at the same version
    e = _FRESH.get(key)
    return e is not None and e[0]() is w and e[1] == w._version


def _take_prepared(key):
    slot = _PREPARED.pop(key, None)
    if slot is None:
        return False
    _lib.wait_mark(slot)
    return True


def _weight_shadow(w, prepass=False):
    """16-bit images of an fp32 master weight W [N, K] in the current format (bf16 / fp16):
    (W16 [N, K], W16t [K, N]), rewritten from W on every forward unless the optimizer step wrote
    them with the weights (_fresh) or the prepass did (_take_prepared)."""
    N, K = w.shape
    key = (w.data_ptr(), N, K)
    sh = _SHADOW.get(key)
    dt = _shadow_dtype()
    if sh is None or sh[0].dtype != dt:
        sh = (torch.empty((N, K), dtype=dt, device=w.device),
              torch.empty((K, N), dtype=dt, device=w.device))
        _SHADOW[key] = sh
        _FRESH.pop(key, None)
    if prepass or not (_take_prepared(key) or _fresh(key, w)):
        call("vt_mfma_weight_shadow", ptr(w), N, K, ptr(sh[0]), ptr(sh[1]), _st())
    return sh


def prepare_shadows(head_weights, conv_weights, stream, extra=None):
    """Write the bf16 shadows of this forward's bf16 conv weights and MFMA head
    weights on `stream` ahead of the forward (they depend only on the weights,
    which change only in the optimizer step), off the activation chain; the ops
    then wait on an event instead of shadowing in line (the convs' event first:
    they are needed early, the 4096^2 heads late).  extra(): more weight-only work
    for the same stream (the BatchNorm step counters).  Same kernels, same bits."""
    _PREPARED.clear()
    _lib.wait_for(stream)
    with torch.cuda.stream(stream):
        for group, fn in ((conv_weights, _conv_shadow), (head_weights, _weight_shadow)):
            if not group:
                continue
            for w in group:
                fn(w, prepass=True)
            slot = _lib.mark(stream)
            for w in group:
                _PREPARED[(w.data_ptr(), *w.shape)] = slot
        if extra is not None:
            extra()


class LinearF(torch.autograd.Function):
    """nn.Linear; mfma=True routes the three GEMMs to the bf16 MFMA kernels
    (vt_mfma_linear_*, on bf16 shadows of the fp32 weight), else the fp32
    kernels (vt_linear_*)."""

    @staticmethod
    def forward(ctx, x, w, b, mfma=False):
        _check(x, w, b)
        K = x.shape[-1]
        N = w.shape[0]
        x2 = x.reshape(-1, K).contiguous()
        R = x2.shape[0]
        y = torch.empty((R, N), device=x.device)
        mfma = h16_flag(mfma) if mfma_ok(K, N) else False
        w16t = None
        if mfma:
            _h16(mfma)
            w16, w16t = _weight_shadow(w)
            ws = WS.get(WS_LINEAR, x.device, 1)
            call("vt_mfma_linear_fwd", ptr(x2), R, K, ptr(w16), N, ptr(b), ptr(y), ptr(ws), ws.numel(), _st())
        else:
            call("vt_linear_fwd", ptr(x2), R, K, ptr(w), N, ptr(b), ptr(y), _st())
        ctx.save_for_backward(x2, w16t)
        ctx.w, ctx.b = w, b
        ctx.shape = x.shape
        ctx.mfma = mfma
        return y.reshape(*x.shape[:-1], N)

    @staticmethod
    def backward(ctx, gy):
        x2, w16t = ctx.saved_tensors
        w, b = ctx.w, ctx.b
        _h16(ctx.mfma)
        N, K = w.shape
        R = x2.shape[0]
        gy2 = gy.reshape(R, N).contiguous()
        gx = None
        ws = WS.get(WS_LINEAR, w.device, 1)
        if ctx.needs_input_grad[0]:
            gx = torch.empty_like(x2)
            if ctx.mfma:
                call("vt_mfma_linear_bwd_data", ptr(gy2), R, N, ptr(w16t), K, ptr(gx), 0, ptr(ws), ws.numel(),
                     _st())
            else:
                call("vt_linear_bwd_data", ptr(gy2), R, N, ptr(w), K, ptr(gx), 0, _st())
            gx = gx.reshape(ctx.shape)
        want_b = b is not None and ctx.needs_input_grad[2]
        pg = _ParamGrads([w, b], [ctx.needs_input_grad[1], want_b])
        gw_t, gb_t = pg.out
        ent = FIRST_WRITER.pop(id(w), None)
        if ent is not None:
            grp, overwrite, gi = ent
            if pg.direct and gw_t is not None and (b is None or gb_t is not None) and len(grp) == (1 if b is None else 2):
                FIRST_WRITER_HIT.append(gi)
                if overwrite:
                    pg.acc = 0   # the first gradient of this step into an unzeroed range: overwrite
            else:
                FIRST_WRITER[id(w)] = ent   # not written here: handled after the backward
        if gw_t is not None:
            pre = "vt_mfma_" if ctx.mfma else "vt_"
            side = HEAD_GRAD_STREAM if (ctx.mfma and pg.direct and HEAD_GRAD_STREAM is not None) else None
            if side is None and ctx.mfma and pg.direct and HEAD_DW_DEFER and GRAD_READY is None:
                # no side stream for them (under capture the branch is dropped, model.py): the
                # heads' weight gradients are enqueued at the end of this backward instead of
                # between the decoder's data-gradient kernels, where the data chain waited for
                # them; same kernels and operands, same bits (in-place sinks; single process
                # only: with bucketed all-reduce hooks the heads' bucket must be ready early)
                cs = torch.cuda.current_stream()

                def run(gy2=gy2, x2=x2, pg=pg, cs=cs, R=R, N=N, K=K, pre=pre, fmt=ctx.mfma):
                    _h16(fmt)
                    with torch.cuda.stream(cs):
                        ws_d = WS.get(WS_LINEAR, gy2.device, 1)
                        call(pre + "linear_bwd_weight", ptr(gy2), R, N, ptr(x2), K, ptr(pg.out[0]), ptr(pg.out[1]),
                             pg.acc, ptr(ws_d), ws_d.numel(), _st())
                    pg.result()
                _defer(run)
                return gx, None, None, None
            if side is not None and side.cuda_stream != _lib.stream():
                # the decoder heads' 4096 x 4096 weight gradients are off the data-gradient
                # chain: a side stream idle during the decoder backward (in-place sinks)
                _lib.wait_for(side)
                with torch.cuda.stream(side):
                    ws_s = WS.get(WS_LINEAR, w.device, 1)
                    call(pre + "linear_bwd_weight", ptr(gy2), R, N, ptr(x2), K, ptr(gw_t), ptr(gb_t), pg.acc,
                         ptr(ws_s), ws_s.numel(), _st())
                gy2.record_stream(side)
                x2.record_stream(side)
                if CAPTURE_TRACE and torch.cuda.is_current_stream_capturing():   # diagnostic (capture_probe.py)
                    import sys
                    print(f"[capture] head branch enqueued on side stream:\n{_lib.capture_info(side)}\n"
                          f"[capture] the decoder's stream:\n{_lib.capture_info()}", file=sys.stderr, flush=True)
                if HEAD_GRAD_JOIN:   # diagnostic (tools/capture_probe.py model_head_join)
                    _lib.wait_for(_lib.stream(), side)
            else:
                call(pre + "linear_bwd_weight", ptr(gy2), R, N, ptr(x2), K, ptr(gw_t), ptr(gb_t), pg.acc, ptr(ws),
                     ws.numel(), _st())
        elif gb_t is not None:
            call("vt_colsum", ptr(gy2), R, N, ptr(gb_t), pg.acc, ptr(ws), ws.numel(), _st())
        gw, gb = pg.result()
        return gx, gw, gb, None


# ---------------------------------------------- fused Linear -> LN -> act
class LinearLNActF(torch.autograd.Function):
    """act(LayerNorm(x W^T + b)) — a ResidualMLP hidden layer
    (ref/model/vae_teb_model.py:336-403) in one pass over the rows
    (vt_linear_ln_fwd: the LN statistics are taken in the GEMM epilogue).
    Backward: vt_layernorm_bwd, then the linear's input / weight gradients."""

    @staticmethod
    def forward(ctx, x, w, b, g, beta, act, eps):
        _check(x, w, b, g, beta)
        K = x.shape[-1]
        N = w.shape[0]
        x2 = x.reshape(-1, K).contiguous()
        R = x2.shape[0]
        y = torch.empty((R, N), device=x.device)
        xhat = torch.empty_like(y)
        rstd = torch.empty(R, device=x.device)
        call("vt_linear_ln_fwd", ptr(x2), R, K, ptr(w), N, ptr(b), ptr(g), ptr(beta), ACT[act], eps, ptr(y),
             ptr(xhat), ptr(rstd), _st())
        ctx.save_for_backward(x2, xhat, rstd)
        ctx.params = (w, b, g, beta)
        ctx.act, ctx.shape = act, x.shape
        return y.reshape(*x.shape[:-1], N)

    @staticmethod
    def backward(ctx, gy):
        x2, xhat, rstd = ctx.saved_tensors
        w, b, g, beta = ctx.params
        N, K = w.shape
        R = x2.shape[0]
        gy2 = gy.reshape(R, N).contiguous()
        gh = torch.empty_like(xhat)
        nig = ctx.needs_input_grad
        pln = _ParamGrads([g, beta], [True, True])
        ws2 = WS.get(2 * N * max(1024, R if N > 512 else 0), x2.device, 2)
        call("vt_layernorm_bwd", ptr(gy2), ptr(xhat), ptr(rstd), R, N, ptr(g), ptr(beta), ACT[ctx.act], ptr(gh),
             ptr(pln.out[0]), ptr(pln.out[1]), pln.acc, ptr(ws2), ws2.numel(), _st())
        gx = None
        if nig[0]:
            gx = torch.empty_like(x2)
            call("vt_linear_bwd_data", ptr(gh), R, N, ptr(w), K, ptr(gx), 0, _st())
            gx = gx.reshape(ctx.shape)
        ws = WS.get(WS_LINEAR, x2.device, 1)
        pl = _ParamGrads([w, b], [nig[1], b is not None and nig[2]])
        gw_t, gb_t = pl.out
        if gw_t is not None:
            call("vt_linear_bwd_weight", ptr(gh), R, N, ptr(x2), K, ptr(gw_t), ptr(gb_t), pl.acc, ptr(ws), ws.numel(),
                 _st())
        elif gb_t is not None:
            call("vt_colsum", ptr(gh), R, N, ptr(gb_t), pl.acc, ptr(ws), ws.numel(), _st())
        gw, gb = pl.result()
        gg, gbeta = pln.result()
        return gx, gw, gb, gg, gbeta, None, None


def linear_ln_fused_ok(K, N):
    return N <= 256


# ------------------------------------------------------- whole ResidualMLP
class MlpSpec:
    """Static description of one ResidualMLP for vt_resmlp_* (ctypes arrays
    built once): widths, LayerNorm / activation per layer, skip kind, eps."""

    MAX_LAYERS, MAX_WIDTH = 34, 144   # VT_MLP_MAX_LAYERS / VT_MLP_MAX_WIDTH

    def __init__(self, dims, layer_ln, layer_act, skip, eps):
        import ctypes
        self.L = len(dims) - 1
        self.dims_l, self.skip, self.eps = list(dims), int(skip), float(eps)
        self.dims = (ctypes.c_int * len(dims))(*dims)
        self.ln = (ctypes.c_int * self.L)(*[int(v) for v in layer_ln])
        self.act = (ctypes.c_int * self.L)(*[ACT[a] if isinstance(a, str) else int(a) for a in layer_act])
        self.n_params = 4 * self.L + 4
        self._sizes = {}
        self.param_ptrs = None           # ctypes array of the parameter pointers (set by the owner)
        self._grad_key, self._grad_ptrs = None, None

    @classmethod
    def supported(cls, dims):
        return len(dims) - 1 <= cls.MAX_LAYERS and max(dims) <= cls.MAX_WIDTH

    def split_sizes(self, rows):
        """(dZ bf16 elements, bwd_data workspace floats, bwd_weight workspace floats, supported) of
        the split bf16 backward (vt_resmlp_bf16_bwd_data / _bwd_weight)."""
        s = self._sizes.get((rows, "split"))
        if s is None:
            import ctypes
            arr = (ctypes.c_int64 * 4)()
            call("vt_resmlp_bf16_split_sizes", self.L, self.dims, self.ln, self.act, self.skip, rows, arr)
            s = self._sizes[(rows, "split")] = tuple(arr)
        return s

    def sizes(self, rows, bf16=False):
        s = self._sizes.get((rows, bf16))
        if s is None:
            import ctypes
            arr = (ctypes.c_int64 * 3)()
            call("vt_resmlp_bf16_sizes" if bf16 else "vt_resmlp_sizes", self.L, self.dims, self.ln, self.act,
                 self.skip, rows, arr)
            s = self._sizes[(rows, bf16)] = tuple(arr)
        return s

    @staticmethod
    def pointers(ts):
        import ctypes
        return (ctypes.c_void_p * len(ts))(*[None if t is None else t.data_ptr() for t in ts])

    def plan_handle(self, rows, params):
        """The library's cached plan of this stack at `rows` rows (vt_resmlp_bf16_plan), for the
        batched image pass; keyed by the parameter addresses (a moved parameter is a new plan)."""
        pp = self.param_ptrs if self.param_ptrs is not None else self.pointers(params)
        key = (rows, tuple(pp))
        h = getattr(self, "_handles", {}).get(key)
        if h is None:
            import ctypes
            hv = ctypes.c_int64()
            call("vt_resmlp_bf16_plan", self.L, self.dims, self.ln, self.act, self.skip, self.eps, pp, rows,
                 ctypes.byref(hv), _st())
            self.__dict__.setdefault("_handles", {})[key] = h = hv.value
        return h

    def grad_pointers(self, ts):
        """Pointer array of the gradient destinations, reused while they stay put
        (the trainer's in-place gradient sinks)."""
        key = tuple(0 if t is None else t.data_ptr() for t in ts)
        if key != self._grad_key:
            import ctypes
            self._grad_key = key
            self._grad_ptrs = (ctypes.c_void_p * len(ts))(*[k or None for k in key])
        return self._grad_ptrs


# plans whose 16-bit weight images the model's batched pass (mlp_prep_batch) prepared for the coming
# forward: each such forward skips its own image pass once (vt_resmlp_bf16_fwd_prepped)
_MLP_PREPPED = set()
MLP_PREP_BATCH = int(os.environ.get("VAETEB_MLP_PREP_BATCH", "1"))


def mlp_prep_batch(stacks, rows):
    """One launch building the 16-bit weight images of every (spec, params) stack at `rows` rows
    (vt_resmlp_bf16_prep_batch) in the current format — the per-stack image passes of the step's
    16-bit ResidualMLP forwards (14 launches of ~7 us each on the forward chain) become one."""
    if not stacks:
        return
    import ctypes
    hs = [spec.plan_handle(rows, params) for spec, params in stacks]
    for i in range(0, len(hs), 32):
        chunk = hs[i:i + 32]
        call("vt_resmlp_bf16_prep_batch", len(chunk), (ctypes.c_int64 * len(chunk))(*chunk), _st())
    _MLP_PREPPED.update(hs)


class ResMLPF(torch.autograd.Function):
    """A whole ResidualMLP (ref/model/vae_teb_model.py:336-403): one forward
    launch (vt_resmlp_fwd) and the backward launches of vt_resmlp_bwd (chain,
    fixed-order sums).  bf16=True: the bf16-MFMA family (vt_resmlp_bf16_*: the
    Linear layers in 16 bit as under the reference's autocast, LayerNorm and
    every reduction fp32).  params in MlpSpec order:
    [g_in, b_in, (W, b, g, beta) per layer, W_skip, b_skip] (None if absent)."""

    @staticmethod
    def forward(ctx, x, spec, bf16, *params):
        _check(x, *params)
        d0, DL = spec.dims_l[0], spec.dims_l[-1]
        x2 = x.reshape(-1, d0).contiguous()
        R = x2.shape[0]
        n_xh, n_rs, _ = spec.sizes(R, bool(bf16))
        _h16(bf16)
        out = torch.empty((R, DL), device=x.device)
        xh = torch.empty(n_xh, device=x.device)
        rs = torch.empty(n_rs, device=x.device)
        pp = spec.param_ptrs if spec.param_ptrs is not None else spec.pointers(params)
        fn = "vt_resmlp_fwd"
        if bf16:
            fn = "vt_resmlp_bf16_fwd"
            if _MLP_PREPPED:
                h = spec.plan_handle(R, params)
                if h in _MLP_PREPPED:          # images prepared by this step's batched pass
                    _MLP_PREPPED.discard(h)
                    fn = "vt_resmlp_bf16_fwd_prepped"
        call(fn, spec.L, spec.dims, spec.ln, spec.act, spec.skip, spec.eps, pp, ptr(x2), R, ptr(out), ptr(xh),
             ptr(rs), _st())
        ctx.save_for_backward(xh, rs)
        ctx.spec, ctx.params, ctx.shape, ctx.R, ctx.bf16 = spec, params, x.shape, R, bf16
        return out.reshape(*x.shape[:-1], DL)

    @staticmethod
    def backward(ctx, gout):
        xh, rs = ctx.saved_tensors
        spec, params, R, bf16 = ctx.spec, ctx.params, ctx.R, ctx.bf16
        _h16(bf16)
        d0, DL = spec.dims_l[0], spec.dims_l[-1]
        g2 = gout.reshape(R, DL).contiguous()
        present = [i for i, p in enumerate(params) if p is not None]
        need = ctx.needs_input_grad[3:]
        pg = _ParamGrads([params[i] for i in present], [bool(need[i]) for i in present])
        grads = [None] * len(params)
        for i, gt in zip(present, pg.out):
            grads[i] = gt
        dx = torch.empty((R, d0), device=xh.device)
        pp = spec.param_ptrs if spec.param_ptrs is not None else spec.pointers(params)
        split = bf16 == "bf16" and MLPB_SPLIT and spec.split_sizes(R)[3]   # (no fp16 form of the split)
        if split:
            # the data-gradient chain here; the weight gradients from the saved dZ rows on the
            # weight-gradient side stream when they are written in place (off the critical chain)
            n_dz, n_wx, n_ww, _ = spec.split_sizes(R)
            dz16 = torch.empty(n_dz, dtype=torch.bfloat16, device=xh.device)
            wsx = WS.get(n_wx, xh.device, 5)
            gp = spec.grad_pointers(grads)
            call("vt_resmlp_bf16_bwd_data", spec.L, spec.dims, spec.ln, spec.act, spec.skip, spec.eps, pp, ptr(g2),
                 ptr(xh), ptr(rs), R, ptr(dx), gp, pg.acc, ptr(dz16), ptr(wsx), wsx.numel(), _st())
            side = GRAD_STREAM if (pg.direct and GRAD_STREAM is not None) else None
            if side is not None and side.cuda_stream != _lib.stream():
                _lib.wait_for(side)
                with torch.cuda.stream(side):
                    wsw = torch.empty(n_ww, device=xh.device)
                    call("vt_resmlp_bf16_bwd_weight", spec.L, spec.dims, spec.ln, spec.act, spec.skip, spec.eps, pp,
                         ptr(xh), ptr(dz16), R, gp, pg.acc, ptr(wsw), wsw.numel(), _st())
                dz16.record_stream(side)
                xh.record_stream(side)
            else:
                wsw = torch.empty(n_ww, device=xh.device)
                call("vt_resmlp_bf16_bwd_weight", spec.L, spec.dims, spec.ln, spec.act, spec.skip, spec.eps, pp,
                     ptr(xh), ptr(dz16), R, gp, pg.acc, ptr(wsw), wsw.numel(), _st())
        else:
            ws_floats = spec.sizes(R, bool(bf16))[2]
            ws = WS.get(ws_floats, xh.device, 5)
            call("vt_resmlp_bf16_bwd" if bf16 else "vt_resmlp_bwd", spec.L, spec.dims, spec.ln, spec.act, spec.skip,
                 spec.eps, pp, ptr(g2), ptr(xh), ptr(rs), R, ptr(dx), spec.grad_pointers(grads), pg.acc, ptr(ws),
                 ws.numel(), _st())
        res = pg.result()
        out = [None] * len(params)
        for i, gt in zip(present, res):
            out[i] = gt
        return (dx.reshape(ctx.shape), None, None, *out)


def resmlp(x, spec, params, bf16=False):
    return ResMLPF.apply(x, spec, h16_flag(bf16), *params)


# -------------------------------------------------------- LayerNorm + act
class LayerNormActF(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, g, b, act, eps):
        _check(x, g, b)
        C = x.shape[-1]
        x2 = x.reshape(-1, C).contiguous()
        R = x2.shape[0]
        y = torch.empty_like(x2)
        xhat = torch.empty_like(x2)
        rstd = torch.empty(R, device=x.device)
        call("vt_layernorm_fwd", ptr(x2), R, C, ptr(g), ptr(b), ACT[act], eps, ptr(y), ptr(xhat), ptr(rstd), _st())
        ctx.save_for_backward(xhat, rstd)
        ctx.params = (g, b)
        ctx.act, ctx.shape = act, x.shape
        return y.reshape(x.shape)

    @staticmethod
    def backward(ctx, gy):
        xhat, rstd = ctx.saved_tensors
        g, b = ctx.params
        R, C = xhat.shape
        gy2 = gy.reshape(R, C).contiguous()
        gx = torch.empty_like(xhat)
        pg = _ParamGrads([g, b], [True, True])
        need = 2 * C * max(1024, R if C > 512 else 0)
        ws = WS.get(need, xhat.device, 2)
        call("vt_layernorm_bwd", ptr(gy2), ptr(xhat), ptr(rstd), R, C, ptr(g), ptr(b), ACT[ctx.act], ptr(gx),
             ptr(pg.out[0]), ptr(pg.out[1]), pg.acc, ptr(ws), ws.numel(), _st())
        gg, gbeta = pg.result()
        return gx.reshape(ctx.shape), gg, gbeta, None, None


# ------------------------------------------------- Conv1d + BatchNorm + act
_CONV_WS = {}
_CONV_SHADOW = {}


def _conv_shadow(w, prepass=False):
    """16-bit shadows (the current format) of a conv weight W [Cout][Cin][K]
    (vt_conv1d_bf16_shadow): w16 [Cout][K][ceil32(Cin)] and the transposed / flipped w16t
    [Cin][K][ceil32(Cout)], rewritten from W on every forward (unless fresh / prepared)."""
    Cout, Cin, K = w.shape
    key = (w.data_ptr(), Cout, Cin, K)
    sh = _CONV_SHADOW.get(key)
    dt = _shadow_dtype()
    if sh is None or sh[0].dtype != dt:
        up32 = lambda n: (n + 31) // 32 * 32
        sh = (torch.empty(Cout * K * up32(Cin), dtype=dt, device=w.device),
              torch.empty(Cin * K * up32(Cout), dtype=dt, device=w.device))
        _CONV_SHADOW[key] = sh
        _FRESH.pop(key, None)
    if prepass or not (_take_prepared(key) or _fresh(key, w)):
        call("vt_conv1d_bf16_shadow", ptr(w), Cout, Cin, K, ptr(sh[0]), ptr(sh[1]), _st())
    return sh


def _conv_bn_ws(*shape):
    n = _CONV_WS.get(shape)
    if n is None:
        import ctypes
        f = ctypes.c_int64()
        call("vt_conv1d_bn_workspace_floats", *shape, ctypes.byref(f))
        n = _CONV_WS[shape] = max(int(f.value), 4096 * shape[3] + 2 * shape[3])
    return n


class ConvBNActF(torch.autograd.Function):
    """(B, L, Cin) -> (B, L_out, Cout): conv (implicit GEMM with fused
    padding/upsampling) -> train-mode BatchNorm (running stats updated) -> act.

    Conv-stack fold (bf16 only, round 5; ConvStack): xin = (mean, rstd, gamma, beta, act code)
    of the PREVIOUS block means x is that block's pre-BN conv output and its BatchNorm +
    activation are applied while this block stages its windows (forward and weight gradient:
    vt_conv1d_bn_fwd_bf16_in / vt_conv1d_bwd_weight_bf16_in); vout returns this block's pre-BN
    output in place of y (with its mean / rstd, non-differentiable) for the next block to stage
    the same way — the inner blocks' y is never written or read.  The gradient autograd passes
    back for that output is dL/dy (the next block's backward-data conv output), as for y."""

    @staticmethod
    def forward(ctx, x, w, g, b, run_mean, run_var, mode, up, act, momentum, eps, bf16=False, xin=None, vout=False):
        _check(x, w, g, b)
        if (xin is not None or vout) and bf16 != "bf16":
            raise ValueError("the conv-stack BatchNorm fold needs the bf16 conv kernels (no fp32 / fp16 form)")
        _h16(bf16)
        B, L, Cin = x.shape
        Cout, _, K = w.shape
        x = x.contiguous()
        Lo = _lib.lib().fns["vt_conv1d_out_len"](L, K, mode, up)
        conv = torch.empty((B, Lo, Cout), device=x.device)
        y = None if vout else torch.empty_like(conv)
        mean = torch.empty(Cout, device=x.device)
        rstd = torch.empty(Cout, device=x.device)
        ws = WS.get(_conv_bn_ws(B, L, Cin, Cout, K, mode, up), x.device, 2)
        w16t = None
        if bf16:
            w16, w16t = _conv_shadow(w)
            tail = (B, L, Cin, ptr(w16), Cout, K, mode, up, ptr(g), ptr(b), ACT[act], eps, momentum, ptr(conv),
                    None if vout else ptr(y), ptr(mean), ptr(rstd), ptr(run_mean), ptr(run_var), ptr(ws), ws.numel(),
                    _st())
            if xin is not None:
                call("vt_conv1d_bn_fwd_bf16_in", ptr(x), *(ptr(t) for t in xin[:4]), xin[4], *tail)
            else:
                call("vt_conv1d_bn_fwd_bf16", ptr(x), *tail)
        else:
            call("vt_conv1d_bn_fwd", ptr(x), B, L, Cin, ptr(w), Cout, K, mode, up, ptr(g), ptr(b), ACT[act], eps,
                 momentum, ptr(conv), ptr(y), ptr(mean), ptr(rstd), ptr(run_mean), ptr(run_var), ptr(ws), ws.numel(),
                 _st())
        ctx.save_for_backward(x, conv, mean, rstd, w16t, *(xin[:4] if xin is not None else ()))
        ctx.params = (w, g, b)
        ctx.cfg = (mode, up, act, bf16)
        ctx.in_act = None if xin is None else xin[4]
        if vout:
            ctx.mark_non_differentiable(mean, rstd)
            ctx.set_materialize_grads(False)   # no zero-filled gradients for mean / rstd
            return conv, mean, rstd
        return y

    @staticmethod
    def backward(ctx, gy, *_):
        x, conv, mean, rstd, w16t, *xin = ctx.saved_tensors
        if gy is None:   # vout with its output unused (set_materialize_grads(False))
            gy = torch.zeros_like(conv)
        w, g, b = ctx.params
        mode, up, act, bf16 = ctx.cfg
        _h16(bf16)
        # the input is the previous block's pre-BN output: its BatchNorm + act in the weight
        # gradient's staging (the backward-data output below is dL/d(that block's y), as always)
        inb = (*(ptr(t) for t in xin), ctx.in_act) if xin else None
        B, L, Cin = x.shape
        Cout, _, K = w.shape
        Lo = conv.shape[1]
        gy = gy.contiguous()
        pbn = _ParamGrads([g, b], [True, True])
        ws = WS.get(4096 * Cout + 2 * Cout, x.device, 2)
        M = B * Lo
        fused = bf16 and ctx.needs_input_grad[0]
        pad = K - 1 if mode == 0 else (K - 1) // 2
        # two-launch backward (vt_batchnorm_bwd_x16 + vt_conv1d_bwd_dx16): every geometry of the
        # model's blocks (causal; reflect with L_up > pad, x2 upsample folded in the conv)
        # (and within the two kernels' limits: K <= 11, B <= 65535 workgroup rows, the BN-gradient
        # row image of Cout <= 1024 channels in LDS; other shapes keep the fused-staging kernels)
        bwd16 = fused and CONV_BWD16 and K <= 11 and B <= 65535 and Cout <= 1024 and \
            (mode == 1 and L * (2 if up else 1) > pad or mode == 0 and not up)
        if bwd16:
            bnp = torch.empty(6 * Cout, device=x.device)
            call("vt_batchnorm_bwd_coef", ptr(gy), ptr(conv), M, Cout, ptr(mean), ptr(rstd), ptr(g), ptr(b),
                 ACT[act], ptr(pbn.out[0]), ptr(pbn.out[1]), pbn.acc, ptr(bnp), ptr(ws), ws.numel(), _st())
            c32 = (Cout + 31) // 32 * 32
            dxbn = torch.empty(M * c32, dtype=_shadow_dtype(), device=x.device)
            call("vt_batchnorm_bwd_x16", ptr(gy), ptr(conv), ptr(bnp), ACT[act], M, Cout, ptr(dxbn), _st())
            srcs = (dxbn,)
            dw_args = lambda wsx: (ptr(dxbn), c32, ptr(x), B, L, Cin, Cout, K, mode, up, ptr(pw.out[0]), pw.acc,
                                   ptr(wsx), wsx.numel(), _st())
            fn = "vt_conv1d_bwd_weight_bf16_dy16s"
            if inb:
                dw_args = lambda wsx: (None, ptr(dxbn), c32, ptr(x), *inb, B, L, Cin, Cout, K, mode, up,
                                       ptr(pw.out[0]), pw.acc, ptr(wsx), wsx.numel(), _st())
                fn = "vt_conv1d_bwd_weight_bf16_in"
        elif fused:
            # fused BatchNorm backward: only the column sums here; the bf16 backward-data
            # conv forms the BN input gradient while staging its operand from (gy, conv,
            # bnp) and leaves it in bf16 (dxbn) for the weight gradient
            bnp = torch.empty(6 * Cout, device=x.device)
            call("vt_batchnorm_bwd_coef", ptr(gy), ptr(conv), M, Cout, ptr(mean), ptr(rstd), ptr(g), ptr(b),
                 ACT[act], ptr(pbn.out[0]), ptr(pbn.out[1]), pbn.acc, ptr(bnp), ptr(ws), ws.numel(), _st())
            dxbn = torch.empty(M * ((Cout + 7) // 8 * 8), dtype=torch.bfloat16, device=x.device)
            srcs = (dxbn,)
            dw_args = lambda wsx: (ptr(dxbn), ptr(x), B, L, Cin, Cout, K, mode, up, ptr(pw.out[0]), pw.acc,
                                   ptr(wsx), wsx.numel(), _st())
            fn = "vt_conv1d_bwd_weight_bf16_dy16"
            if inb:
                dw_args = lambda wsx: (None, ptr(dxbn), (Cout + 7) // 8 * 8, ptr(x), *inb, B, L, Cin, Cout, K, mode,
                                       up, ptr(pw.out[0]), pw.acc, ptr(wsx), wsx.numel(), _st())
                fn = "vt_conv1d_bwd_weight_bf16_in"
        else:
            gconv = torch.empty_like(conv)
            call("vt_batchnorm_bwd", ptr(gy), ptr(conv), M, Cout, ptr(mean), ptr(rstd), ptr(g), ptr(b), ACT[act],
                 ptr(gconv), ptr(pbn.out[0]), ptr(pbn.out[1]), pbn.acc, ptr(ws), ws.numel(), _st())
            srcs = (gconv,)
            dw_args = lambda wsx: (ptr(gconv), ptr(x), B, L, Cin, Cout, K, mode, up, ptr(pw.out[0]), pw.acc,
                                   ptr(wsx), wsx.numel(), _st())
            fn = "vt_conv1d_bwd_weight_bf16" if bf16 else "vt_conv1d_direct_bwd_weight"
            if inb:   # a folded input is the previous block's output: it always needs its gradient
                raise RuntimeError("conv-stack fold: the block input's gradient is required")
        gx = None
        if ctx.needs_input_grad[0]:
            gx = torch.empty_like(x)
            if bwd16:
                edge = WS.get(max(B * 2 * pad * Cin, 1), x.device, 3)
                call("vt_conv1d_bwd_dx16", ptr(dxbn), B, L, Cin, ptr(w16t), Cout, K, mode, up, ptr(gx), ptr(edge),
                     _st())
            elif fused and CONV_DIRECT_DX and not up and (mode == 0 or L > pad):
                # the fold is a crop: the conv writes gx itself (reflect: + the mirrored edge rows)
                edge = WS.get(max(B * 2 * pad * Cin, 1), x.device, 3)
                call("vt_conv1d_bwd_dx_bf16_bn", ptr(gy), ptr(conv), ptr(bnp), ACT[act], M, B, L, Cin, ptr(w16t),
                     Cout, K, mode, up, ptr(gx), ptr(edge), ptr(dxbn), _st())
            else:
                gpad = WS.get(B * (Lo + K - 1) * Cin, x.device, 3)
                if fused:
                    call("vt_conv1d_bwd_gpad_bf16_bn", ptr(gy), ptr(conv), ptr(bnp), ACT[act], M, B, L, Cin,
                         ptr(w16t), Cout, K, mode, up, ptr(gpad), ptr(dxbn), _st())
                else:
                    call("vt_conv1d_direct_bwd_gpad", ptr(gconv), B, L, Cin, ptr(w), Cout, K, mode, up, ptr(gpad),
                         _st())
                call("vt_conv1d_fold", ptr(gpad), B, L, Cin, Cout, K, mode, up, ptr(gx), 0, _st())
        pw = _ParamGrads([w], [ctx.needs_input_grad[1]])
        if pw.out[0] is not None:
            side = GRAD_STREAM if (pw.direct and GRAD_STREAM is not None) else None
            if side is not None and side.cuda_stream != _lib.stream():
                # the weight gradient is off the data-gradient chain: compute it on a
                # side stream (written in place into the flat gradient buffer, joined
                # at the end of the backward / before a bucket's all-reduce)
                _lib.wait_for(side)
                with torch.cuda.stream(side):
                    ws1 = WS.get(WS_LINEAR, x.device, 1)
                    call(fn, *dw_args(ws1))
                for t in (*srcs, x, *xin):   # xin: the folded input's BatchNorm, read by the staging
                    t.record_stream(side)
            else:
                ws1 = WS.get(WS_LINEAR, x.device, 1)
                call(fn, *dw_args(ws1))
        gw, = pw.result()
        gg, gb = pbn.result()
        return gx, gw, gg, gb, None, None, None, None, None, None, None, None, None, None


class SyncConvBNActF(torch.autograd.Function):
    """ConvBNActF with cross-rank BatchNorm statistics (torch.nn.SyncBatchNorm semantics,
    Lightning sync_batchnorm=True: ref/model/graph_model.py:517): the per-channel sums
    are all-reduced over `group` twice in the forward (sum, then the centred sum of
    squares: two-pass, as the single-rank path) and once in the backward (sum dz, sum
    dz xhat, for dx); dgamma / dbeta are this rank's own sums (the data-parallel
    gradient all-reduce averages them, as DDP does for SyncBatchNorm's grad_weight)."""

    @staticmethod
    def forward(ctx, x, w, g, b, run_mean, run_var, mode, up, act, momentum, eps, bf16, group):
        import torch.distributed as dist
        if x.is_cuda and torch.cuda.is_current_stream_capturing():
            # the BatchNorm statistics are all-reduced inside the op: a collective cannot be
            # captured into a hipGraph (Trainer.capture / the native executor)
            raise RuntimeError("SyncBatchNorm conv blocks cannot be captured into a hipGraph "
                               "(cross-rank statistics need a collective inside the step); train them eagerly")
        _check(x, w, g, b)
        B, L, Cin = x.shape
        Cout, _, K = w.shape
        x = x.contiguous()
        Lo = _lib.lib().fns["vt_conv1d_out_len"](L, K, mode, up)
        conv = torch.empty((B, Lo, Cout), device=x.device)
        if bf16:
            _h16(bf16)
            w16, w16t = _conv_shadow(w)
            call("vt_conv1d_fwd_bf16", ptr(x), B, L, Cin, ptr(w16), Cout, K, mode, up, ptr(conv), _st())
        else:
            w16t = None
            call("vt_conv1d_direct_fwd", ptr(x), B, L, Cin, ptr(w), Cout, K, mode, up, ptr(conv), _st())
        M = B * Lo
        mean = torch.empty(Cout, device=x.device)
        rstd = torch.empty(Cout, device=x.device)
        sums = torch.empty(2 * Cout + 1, dtype=torch.float64, device=x.device)
        ws = WS.get(4096 * Cout * 2 + 2 * Cout, x.device, 2)
        for which, outs in ((0, (ptr(mean), None, None, None)), (1, (ptr(mean), ptr(rstd), ptr(run_mean),
                                                                     ptr(run_var)))):
            call("vt_syncbn_sums", ptr(conv), None, M, Cout, which, ptr(mean), None, None, None, 0, ptr(sums),
                 ptr(ws), ws.numel(), _st())
            dist.all_reduce(sums, op=dist.ReduceOp.SUM, group=group)   # counts add up too (sums[2C])
            call("vt_syncbn_stats", ptr(sums), Cout, which, eps, momentum, *outs, None, None, 0, _st())
        y = torch.empty_like(conv)
        call("vt_batchnorm_apply", ptr(conv), M, Cout, ptr(mean), ptr(rstd), ptr(g), ptr(b), ACT[act], ptr(y), _st())
        ctx.save_for_backward(x, conv, mean, rstd, w16t)
        ctx.params = (w, g, b)
        ctx.cfg = (mode, up, act, bf16, group)
        return y

    @staticmethod
    def backward(ctx, gy):
        import torch.distributed as dist
        x, conv, mean, rstd, w16t = ctx.saved_tensors
        w, g, b = ctx.params
        mode, up, act, bf16, group = ctx.cfg
        _h16(bf16)
        B, L, Cin = x.shape
        Cout, _, K = w.shape
        Lo = conv.shape[1]
        M = B * Lo
        gy = gy.contiguous()
        pbn = _ParamGrads([g, b], [True, True])
        sums = torch.empty(2 * Cout + 1, dtype=torch.float64, device=x.device)
        ws = WS.get(4096 * Cout * 2 + 2 * Cout, x.device, 2)
        call("vt_syncbn_sums", ptr(conv), ptr(gy), M, Cout, 2, ptr(mean), ptr(rstd), ptr(g), ptr(b), ACT[act],
             ptr(sums), ptr(ws), ws.numel(), _st())
        call("vt_syncbn_stats", ptr(sums), Cout, 2, 0.0, 0.0, None, None, None, None, ptr(pbn.out[0]),
             ptr(pbn.out[1]), pbn.acc, _st())
        dist.all_reduce(sums, op=dist.ReduceOp.SUM, group=group)
        gconv = torch.empty_like(conv)
        call("vt_syncbn_bwd_dx", ptr(gy), ptr(conv), M, Cout, ptr(mean), ptr(rstd), ptr(g), ptr(b), ACT[act],
             ptr(sums), ptr(gconv), ptr(ws), _st())
        gx = None
        if ctx.needs_input_grad[0]:
            gx = torch.empty_like(x)
            gpad = WS.get(B * (Lo + K - 1) * Cin, x.device, 3)
            if bf16:
                call("vt_conv1d_bwd_gpad_bf16", ptr(gconv), B, L, Cin, ptr(w16t), Cout, K, mode, up, ptr(gpad), _st())
            else:
                call("vt_conv1d_direct_bwd_gpad", ptr(gconv), B, L, Cin, ptr(w), Cout, K, mode, up, ptr(gpad), _st())
            call("vt_conv1d_fold", ptr(gpad), B, L, Cin, Cout, K, mode, up, ptr(gx), 0, _st())
        pw = _ParamGrads([w], [ctx.needs_input_grad[1]])
        if pw.out[0] is not None:
            ws1 = WS.get(WS_LINEAR, x.device, 1)
            fn = "vt_conv1d_bwd_weight_bf16" if bf16 else "vt_conv1d_direct_bwd_weight"
            call(fn, ptr(gconv), ptr(x), B, L, Cin, Cout, K, mode, up, ptr(pw.out[0]), pw.acc, ptr(ws1), ws1.numel(),
                 _st())
        gw, = pw.result()
        gg, gb = pbn.result()
        return gx, gw, gg, gb, None, None, None, None, None, None, None, None, None, None, None


def sync_conv_bn_act(x, w, g, b, run_mean, run_var, mode, up=False, act="relu", momentum=0.9, eps=1e-5, bf16=False,
                     group=None):
    return SyncConvBNActF.apply(x, w, g, b, run_mean, run_var, int(mode), int(up), act, momentum, eps,
                                h16_flag(bf16), group)


def conv_bn_eval(x, w, g, b, run_mean, run_var, mode, up=False, act="relu", eps=1e-5, bf16=False):
    """Eval-mode ConvBlock: conv -> BatchNorm with the running statistics -> act
    (validation / frozen-VAE / predict path; not differentiable)."""
    _check(x, w, g, b)
    if torch.is_grad_enabled() and (x.requires_grad or w.requires_grad):
        raise RuntimeError("eval-mode conv blocks are inference-only (run under torch.no_grad())")
    B, L, Cin = x.shape
    Cout, _, K = w.shape
    x = x.contiguous()
    Lo = _lib.lib().fns["vt_conv1d_out_len"](L, K, mode, up)
    conv = torch.empty((B, Lo, Cout), device=x.device)
    if bf16:
        _h16(h16_flag(bf16))
        w16, _ = _conv_shadow(w)
        call("vt_conv1d_fwd_bf16", ptr(x), B, L, Cin, ptr(w16), Cout, K, mode, up, ptr(conv), _st())
    else:
        call("vt_conv1d_direct_fwd", ptr(x), B, L, Cin, ptr(w), Cout, K, mode, up, ptr(conv), _st())
    call("vt_batchnorm_eval", ptr(conv), B * Lo, Cout, ptr(run_mean), ptr(run_var), eps, ptr(g), ptr(b), ACT[act],
         ptr(conv), _st())
    return conv


# ---------------------------------------------------------------------- LSTM
class LSTMF(torch.autograd.Function):
    """Multi-layer unidirectional LSTM, batch_first, zero initial state.
    params: flat list [w_ih_l0, w_hh_l0, b_ih_l0, b_hh_l0, w_ih_l1, ...]."""

    @staticmethod
    def forward(ctx, x, half, *params):
        _check(x, *params)
        B, S, _ = x.shape
        nl = len(params) // 4
        H = params[1].shape[1]
        saved = []
        pairs = []   # lower layers of the layer pairs run by vt_lstm16_pair_fwd
        inp = x.contiguous()
        l = 0
        while l < nl:
            w_ih, w_hh, b_ih, b_hh = params[4 * l: 4 * l + 4]
            In = inp.shape[-1]
            h = torch.empty((B, S, H), device=x.device)
            c = torch.empty_like(h)
            gates = torch.empty((B, S, 4 * H), device=x.device)
            h16 = half and In <= 64 and In % 4 == 0
            if h16 and LSTM_PAIR and LSTM_CHAIN_FWD and l == 0 and nl == 4 and H == 64 and _l16_pair_fits(S):
                # all four layers in one launch: pair (2, 3) consumes layer 1's h chunk by chunk
                hs = [h] + [torch.empty_like(h) for _ in range(3)]
                cs = [c] + [torch.empty_like(h) for _ in range(3)]
                gs = [gates] + [torch.empty_like(gates) for _ in range(3)]
                pv = (ctypes.c_void_p * 16)(*[ptr(t) for t in params])
                ov = (ctypes.c_void_p * 12)(*[ptr(t) for i in range(4) for t in (hs[i], cs[i], gs[i])])
                call("vt_lstm16_quad_fwd", ptr(inp), In, ctypes.addressof(pv), B, S, H, ctypes.addressof(ov), _st())
                saved += [inp, hs[0], cs[0], gs[0], hs[0], hs[1], cs[1], gs[1],
                          hs[1], hs[2], cs[2], gs[2], hs[2], hs[3], cs[3], gs[3]]
                pairs += [0, 2]
                inp = hs[3]
                l = 4
                continue
            if h16 and LSTM_PAIR and l + 1 < nl and H <= 64 and _l16_pair_fits(S):
                # layers l and l + 1 in one launch (the upper one chunk behind the lower)
                w_ih1, w_hh1, b_ih1, b_hh1 = params[4 * l + 4: 4 * l + 8]
                h1, c1 = torch.empty_like(h), torch.empty_like(h)
                gates1 = torch.empty_like(gates)
                call("vt_lstm16_pair_fwd", ptr(inp), In, ptr(w_ih), ptr(b_ih), ptr(w_hh), ptr(b_hh), ptr(w_ih1),
                     ptr(b_ih1), ptr(w_hh1), ptr(b_hh1), B, S, H, ptr(h), ptr(c), ptr(gates), ptr(h1), ptr(c1),
                     ptr(gates1), _st())
                saved += [inp, h, c, gates, h, h1, c1, gates1]
                pairs.append(l)
                inp = h1
                l += 2
                continue
            if h16:
                # 16-bit MFMA recurrence over sample tiles (f16 operands, fp32 state); no h_{t-1}
                # output: the weight gradient reads it from h (vt_lstm16_layer_bwd_weight)
                call("vt_lstm16_layer_fwd", ptr(inp), In, ptr(w_ih), ptr(b_ih), ptr(w_hh), ptr(b_hh), B, S, H, ptr(h),
                     None, ptr(c), ptr(gates), _st())
                saved += [inp, h, c, gates]
                inp = h
                l += 1
                continue
            hp = torch.empty_like(h)
            if LSTM_FUSED and In <= 64:
                # input projection inside the recurrence kernel (bitwise the unfused result)
                call("vt_lstm_layer_fwd_x", ptr(inp), In, ptr(w_ih), ptr(b_ih), ptr(w_hh), ptr(b_hh), B, S, H, ptr(h),
                     ptr(hp), ptr(c), ptr(gates), _st())
            else:
                # gin = X W_ih^T + b_ih, overwritten in place by the post-activation gates
                call("vt_linear_fwd", ptr(inp), B * S, In, ptr(w_ih), 4 * H, ptr(b_ih), ptr(gates), _st())
                call("vt_lstm_layer_fwd", ptr(gates), ptr(w_hh), ptr(b_hh), B, S, H, ptr(h), ptr(hp), ptr(c),
                     ptr(gates), _st())
            saved += [inp, hp, c, gates]
            inp = h
            l += 1
        ctx.save_for_backward(*saved)
        ctx.params = params
        ctx.nl = nl
        ctx.half = bool(half)
        ctx.pairs = pairs
        return inp

    @staticmethod
    def backward(ctx, gy):
        saved, params = ctx.saved_tensors, ctx.params
        nl = ctx.nl
        gy = gy.contiguous()
        B, S, H = gy.shape
        grads = [None] * len(params)
        dh = gy
        ws = WS.get(WS_LINEAR, gy.device, 1)
        gx = None
        deferred = []

        def wgrad(l, dg, half):
            """every parameter gradient of layer l from its dgates (in place / deferred / on the
            weight-gradient side stream, as configured)"""
            inp, hp = saved[4 * l], saved[4 * l + 1]
            w_ih, w_hh, b_ih, b_hh = params[4 * l: 4 * l + 4]
            In = inp.shape[-1]
            wfn = "vt_lstm16_layer_bwd_weight" if half else "vt_lstm_layer_bwd_weight"
            if (LSTM_FUSED or half) and In + H + 1 <= 144:
                # every parameter gradient of the layer in one pass over dg
                pg = _ParamGrads([w_ih, w_hh, b_ih, b_hh], [True] * 4)
                if pg.direct and LSTM_GRAD_DEFER:
                    # in-place sinks: issued after the last layer's recurrence (below), so
                    # the layer-to-layer dh chain is not interrupted by them
                    deferred.append((dg, inp, In, hp, pg, wfn))
                    return
                side = LSTM_GRAD_STREAM if (pg.direct and LSTM_GRAD_STREAM is not None) else None
                if side is not None and side.cuda_stream != _lib.stream():
                    # off the layer-to-layer chain (in-place sinks; same kernels, same bits)
                    _lib.wait_for(side)
                    with torch.cuda.stream(side):
                        ws_s = WS.get(WS_LINEAR, gy.device, 1)
                        call(wfn, ptr(dg), ptr(inp), In, ptr(hp), B, S, H,
                             *[ptr(t) for t in pg.out], pg.acc, ptr(ws_s), ws_s.numel(), _st())
                    for t in (dg, inp, hp):
                        t.record_stream(side)
                else:
                    call(wfn, ptr(dg), ptr(inp), In, ptr(hp), B, S, H,
                         *[ptr(t) for t in pg.out], pg.acc, ptr(ws), ws.numel(), _st())
                grads[4 * l: 4 * l + 4] = pg.result()
                return
            pw = _ParamGrads([w_ih, w_hh], [True, True])
            # b_ih and b_hh receive the same gradient (the sum of dg over rows), written
            # by one column sum per bias straight into its gradient sink (no device copy:
            # a memcpy node would not survive the native step executor, csrc/stepgraph.cpp)
            pb = _ParamGrads([b_ih, b_hh], [True, True])
            side = LSTM_GRAD_STREAM if (pw.direct and LSTM_GRAD_STREAM is not None) else None
            if side is not None and side.cuda_stream != _lib.stream():
                # weight gradients (in-place sinks) off the recurrence chain on a side
                # stream; the returned bias gradient stays here (same kernels and
                # summation orders as the serial branch below: bitwise equal)
                _lib.wait_for(side)
                with torch.cuda.stream(side):
                    ws_s = WS.get(WS_LINEAR, gy.device, 1)
                    call("vt_linear_bwd_weight", ptr(dg), B * S, 4 * H, ptr(inp), In, ptr(pw.out[0]), None, pw.acc,
                         ptr(ws_s), ws_s.numel(), _st())
                    call("vt_linear_bwd_weight", ptr(dg), B * S, 4 * H, ptr(hp), H, ptr(pw.out[1]), None, pw.acc,
                         ptr(ws_s), ws_s.numel(), _st())
                for t in (dg, inp, hp):
                    t.record_stream(side)
            else:
                call("vt_linear_bwd_weight", ptr(dg), B * S, 4 * H, ptr(inp), In, ptr(pw.out[0]), None, pw.acc,
                     ptr(ws), ws.numel(), _st())
                call("vt_linear_bwd_weight", ptr(dg), B * S, 4 * H, ptr(hp), H, ptr(pw.out[1]), None, pw.acc,
                     ptr(ws), ws.numel(), _st())
            for gb in pb.out:
                call("vt_colsum", ptr(dg), B * S, 4 * H, ptr(gb), pb.acc, ptr(ws), ws.numel(), _st())
            gw_ih, gw_hh = pw.result()
            grads[4 * l: 4 * l + 4] = [gw_ih, gw_hh, *pb.result()]

        l = nl - 1
        if LSTM_CHAIN_BWD and ctx.pairs == [0, 2] and nl == 4:
            # the four layers' backward in one launch: layer 2's dX (dmid, the gradient at layer
            # 1's outputs) handed to layers 1, 0 chunk by chunk (vt_lstm16_quad_bwd)
            In0 = saved[0].shape[-1]
            dgs = [torch.empty((B, S, 4 * H), device=gy.device) for _ in range(4)]
            dmid = torch.empty((B, S, H), device=gy.device)
            need_dx = ctx.needs_input_grad[0]
            gin = torch.empty((B, S, In0), device=gy.device) if need_dx else None
            wv = (ctypes.c_void_p * 8)(*[ptr(params[4 * k + i]) for k in range(4) for i in (0, 1)])
            gv = (ctypes.c_void_p * 8)(*[ptr(saved[4 * k + i]) for k in range(4) for i in (3, 2)])
            dv = (ctypes.c_void_p * 4)(*[ptr(t) for t in dgs])
            call("vt_lstm16_quad_bwd", ptr(dh), ctypes.addressof(wv), ctypes.addressof(gv), In0, B, S, H,
                 ctypes.addressof(dv), ptr(dmid), ptr(gin) if need_dx else None, _st())
            for k in (3, 2, 1, 0):
                wgrad(k, dgs[k], True)
            if need_dx:
                dh = gx = gin
            l = -1
        while l >= 0:
            if l - 1 in ctx.pairs:
                # layers l (upper) and l - 1 (lower) in one launch: the upper layer's dX goes
                # to the lower layer through LDS (vt_lstm16_pair_bwd)
                lo = l - 1
                inpL, _, cL, gatesL = saved[4 * lo: 4 * lo + 4]
                _, _, cU, gatesU = saved[4 * l: 4 * l + 4]
                InL = inpL.shape[-1]
                dgU = torch.empty((B, S, 4 * H), device=gy.device)
                dgL = torch.empty_like(dgU)
                need_dx = lo > 0 or ctx.needs_input_grad[0]
                gin = torch.empty((B, S, InL), device=gy.device) if need_dx else None
                call("vt_lstm16_pair_bwd", ptr(dh), ptr(gatesU), ptr(cU), ptr(params[4 * l + 1]), ptr(params[4 * l]),
                     ptr(gatesL), ptr(cL), ptr(params[4 * lo + 1]), ptr(params[4 * lo]), InL, B, S, H, ptr(dgU),
                     ptr(dgL), ptr(gin) if need_dx else None, _st())
                wgrad(l, dgU, True)
                wgrad(lo, dgL, True)
                if need_dx:
                    dh = gx = gin
                l -= 2
                continue
            inp, hp, c, gates = saved[4 * l: 4 * l + 4]
            w_ih, w_hh = params[4 * l], params[4 * l + 1]
            In = inp.shape[-1]
            half = ctx.half and In <= 64 and In % 4 == 0   # hp is then h (read shifted by one step)
            dg = torch.empty((B, S, 4 * H), device=gy.device)
            need_dx = l > 0 or ctx.needs_input_grad[0]
            fused = LSTM_FUSED and In <= 64
            gin = torch.empty((B, S, In), device=gy.device) if need_dx else None
            if half:
                # bf16-MFMA recurrence, dX = dG W_ih inside; dG in fp32 for the weight gradients
                call("vt_lstm16_layer_bwd", ptr(dh), ptr(gates), ptr(c), ptr(w_hh), ptr(w_ih), In, B, S, H, ptr(dg),
                     ptr(gin) if need_dx else None, _st())
            elif fused:
                # dX = dG W_ih inside the recurrence kernel (bitwise the unfused result)
                call("vt_lstm_layer_bwd_x", ptr(dh), ptr(gates), ptr(c), ptr(w_hh), ptr(w_ih), In, B, S, H, ptr(dg),
                     ptr(gin) if need_dx else None, _st())
            else:
                call("vt_lstm_layer_bwd", ptr(dh), ptr(gates), ptr(c), ptr(w_hh), B, S, H, ptr(dg), _st())
                if need_dx:
                    call("vt_linear_bwd_data", ptr(dg), B * S, 4 * H, ptr(w_ih), In, ptr(gin), 0, _st())
            wgrad(l, dg, half)
            if need_dx:
                dh = gin
                gx = gin
            l -= 1
        if deferred:
            # the layers' parameter gradients after the whole recurrence chain, on the
            # weight-gradient side stream when there is one (joined before the bucket
            # all-reduce / the end of the backward), else in line; same kernels and
            # summation orders as in line per layer: the same bits
            side = LSTM_GRAD_STREAM
            on_side = side is not None and side.cuda_stream != _lib.stream()
            if on_side:
                _lib.wait_for(side)
            with torch.cuda.stream(side if on_side else torch.cuda.current_stream()):
                ws_d = WS.get(WS_LINEAR, gy.device, 1)
                for dg, inp, In, hp, pg, wfn in deferred:
                    call(wfn, ptr(dg), ptr(inp), In, ptr(hp), B, S, H,
                         *[ptr(t) for t in pg.out], pg.acc, ptr(ws_d), ws_d.numel(), _st())
            for dg, inp, In, hp, pg, wfn in deferred:
                if on_side:
                    for t in (dg, inp, hp):
                        t.record_stream(side)
                pg.result()
        return (gx, None, *grads)


# ---------------------------------------------------------------------- ELBO
class LatentF(torch.autograd.Function):
    """(mu_c, lv_q, mu_y, lv_p, eps) -> (z, mu_post, kl): fused reparameterisation
    + KL (vt_elbo_latent_*)."""

    @staticmethod
    def forward(ctx, mu_c, lv_q, mu_y, lv_p, eps):
        _check(mu_c, lv_q, mu_y, lv_p, eps)
        ins = [t.contiguous() for t in (mu_c, lv_q, mu_y, lv_p, eps)]
        D = mu_c.shape[-1]
        rows = mu_c.numel() // D
        z, mp = torch.empty_like(ins[0]), torch.empty_like(ins[0])
        kl = torch.empty((), device=mu_c.device)
        ws = WS.get(_lib.lib().fns["vt_elbo_workspace_floats"](), mu_c.device, 4)
        call("vt_elbo_latent_fwd", *[ptr(t) for t in ins], rows, D, ptr(z), ptr(mp), ptr(kl), ptr(ws), _st())
        ctx.save_for_backward(*ins)
        ctx.dims = (rows, D)
        return z, mp, kl

    @staticmethod
    def backward(ctx, gz, gmp, gkl):
        ins = ctx.saved_tensors
        rows, D = ctx.dims
        outs = [torch.empty_like(ins[0]) for _ in range(4)]
        gz = gz.contiguous() if gz is not None else None
        gmp = gmp.contiguous() if gmp is not None else None
        gkl = gkl.reshape(1).contiguous() if gkl is not None else None
        call("vt_elbo_latent_bwd", *[ptr(t) for t in ins], rows, D, ptr(gz), ptr(gmp), ptr(gkl), *[ptr(t) for t in outs],
             _st())
        return outs[0], outs[1], outs[2], outs[3], None


class OutputLossF(torch.autograd.Function):
    """(mu_pr, lv_pr, y_raw, lin, y_st, y_ph) -> (nll, mse) with gradients
    computed in the forward (vt_elbo_output_fwd) and scaled in the backward."""

    @staticmethod
    def forward(ctx, mu, lv, y, lin, y_st, y_ph):
        _check(mu, lv, y)
        mu, lv, y = mu.contiguous(), lv.contiguous(), y.contiguous()
        use_mse = lin is not None and lin.shape[-1] == 87 and y_st.shape[-1] == 43 and y_ph.shape[-1] == 44
        out = torch.zeros(2, device=mu.device)
        g_mu, g_lv = torch.empty_like(mu), torch.empty_like(lv)
        ws = WS.get(_lib.lib().fns["vt_elbo_workspace_floats"](), mu.device, 4)
        if use_mse:
            lin, y_st, y_ph = lin.contiguous(), y_st.contiguous(), y_ph.contiguous()
            g_lin = torch.empty_like(lin)
            rows = lin.numel() // 87
            call("vt_elbo_output_fwd", ptr(mu), ptr(lv), ptr(y), mu.numel(), ptr(lin), ptr(y_st), ptr(y_ph), rows, 43,
                 44, ptr(g_mu), ptr(g_lv), ptr(g_lin), out.data_ptr(), out.data_ptr() + 4, ptr(ws), _st())
        else:
            g_lin = torch.zeros_like(lin) if lin is not None else None
            call("vt_elbo_output_fwd", ptr(mu), ptr(lv), ptr(y), mu.numel(), None, None, None, 0, 0, 0, ptr(g_mu),
                 ptr(g_lv), None, out.data_ptr(), out.data_ptr() + 4, ptr(ws), _st())
        ctx.save_for_backward(g_mu, g_lv, g_lin if g_lin is not None else torch.empty(0, device=mu.device))
        ctx.has_lin = lin is not None
        return out[0], out[1]

    @staticmethod
    def backward(ctx, gnll, gmse):
        g_mu, g_lv, g_lin = ctx.saved_tensors
        # scale the unit-upstream gradients by the incoming device scalars (no host sync)
        for t, s in ((g_mu, gnll), (g_lv, gnll), (g_lin, gmse)):
            if t.numel() and s is not None:
                call("vt_scale_by_device_scalar", ptr(t), t.numel(), ptr(s.reshape(1).contiguous()), _st())
        return g_mu, g_lv, None, (g_lin if ctx.has_lin else None), None, None


# ------------------------------------------------------------- functional API
class CatLastF(torch.autograd.Function):
    """torch.cat(xs, dim=-1) of fp32 device tensors (the encoders' concatenations,
    ref/model/vae_teb_model.py: cross_modal_fusion(cat([a, b])) and the conditional encoder's
    mlp(cat([h_x, h_y]))) by vt_copy_cols, and its backward: each input's gradient as its own
    contiguous tensor, one column-range copy each — the consumers' backward kernels need contiguous
    rows, and ATen's copy of a strided column slice ran at ~0.1 TB/s (46 us for one half on the
    critical chain).  Pure copies: the same values as torch.cat and its autograd split."""

    @staticmethod
    def forward(ctx, *xs):
        xs = [x.contiguous() for x in xs]
        widths = [int(x.shape[-1]) for x in xs]
        W, lead = sum(widths), tuple(xs[0].shape[:-1])
        R = xs[0].numel() // widths[0]
        out = torch.empty(*lead, W, device=xs[0].device, dtype=torch.float32)
        c0 = 0
        for x, w in zip(xs, widths):
            call("vt_copy_cols", ptr(x), R, w, 0, w, ptr(out), W, c0, _st())
            c0 += w
        ctx.widths, ctx.lead, ctx.R = widths, lead, R
        return out

    @staticmethod
    def backward(ctx, g):
        g = g.contiguous()
        W = sum(ctx.widths)
        outs, c0 = [], 0
        for w, need in zip(ctx.widths, ctx.needs_input_grad):
            d = None
            if need:
                d = torch.empty(*ctx.lead, w, device=g.device, dtype=torch.float32)
                call("vt_copy_cols", ptr(g), ctx.R, W, c0, w, ptr(d), w, 0, _st())
            outs.append(d)
            c0 += w
        return tuple(outs)


class ClampF(torch.autograd.Function):
    """torch.clamp(x, lo, hi) with its backward in one pass (vt_clamp_bwd: (lo <= x <= hi) ? g : 0,
    autograd's where((x >= lo) & (x <= hi), g, 0) — four ATen launches on the critical chain); the
    forward is ATen's clamp (NaN propagating as the reference's)."""

    @staticmethod
    def forward(ctx, x, lo, hi):
        ctx.save_for_backward(x)
        ctx.lo, ctx.hi = float(lo), float(hi)
        return torch.clamp(x, lo, hi)

    @staticmethod
    def backward(ctx, g):
        (x,) = ctx.saved_tensors
        g = g.contiguous()
        gx = torch.empty_like(x)
        call("vt_clamp_bwd", ptr(g), ptr(x), x.numel(), ctx.lo, ctx.hi, ptr(gx), _st())
        return gx, None, None


def clamp(x, lo, hi):
    """The encoders' logvar clamp: ClampF on a contiguous fp32 device tensor, torch.clamp otherwise."""
    if x.is_cuda and x.dtype == torch.float32 and x.is_contiguous() and x.numel() > 0 and x.requires_grad:
        return ClampF.apply(x, lo, hi)
    return torch.clamp(x, lo, hi)


def cat_last(xs):
    """The last-axis concatenation of the encoders: CatLastF for fp32 device tensors of equal leading
    shape, torch.cat otherwise."""
    if len(xs) > 1 and all(x.is_cuda and x.dtype == torch.float32 and x.shape[:-1] == xs[0].shape[:-1]
                           and x.numel() > 0 for x in xs):
        return CatLastF.apply(*xs)
    return torch.cat(xs, dim=-1)


def linear(x, w, b=None, mfma=False):
    return LinearF.apply(x, w, b, mfma)


def linear_ln_act(x, w, b, g, beta, act="none", eps=1e-5):
    return LinearLNActF.apply(x, w, b, g, beta, act, eps)


def layer_norm_act(x, g, b, act="none", eps=1e-5):
    return LayerNormActF.apply(x, g, b, act, eps)


def conv_bn_act(x, w, g, b, run_mean, run_var, mode, up=False, act="relu", momentum=0.9, eps=1e-5, bf16=False,
                xin=None, vout=False):
    """xin / vout: the conv-stack BatchNorm fold (ConvBNActF); vout returns (pre-BN output, its
    BatchNorm as the next block's xin)."""
    out = ConvBNActF.apply(x, w, g, b, run_mean, run_var, int(mode), int(up), act, momentum, eps, h16_flag(bf16), xin,
                           bool(vout))
    if not vout:
        return out
    conv, mean, rstd = out
    return conv, (mean, rstd, g, b, ACT[act])


def lstm(x, params, half=False):
    """half: the 16-bit MFMA recurrences (vt_lstm16_layer_*: f16 forward / bf16 backward
    operands, fp32 accumulation and cell state), the reference's 16-bit autocast width."""
    return LSTMF.apply(x, bool(half), *params)


def latent(mu_c, lv_q, mu_y, lv_p, eps):
    return LatentF.apply(mu_c, lv_q, mu_y, lv_p, eps)


def output_losses(mu, lv, y, lin=None, y_st=None, y_ph=None):
    return OutputLossF.apply(mu, lv, y, lin, y_st, y_ph)
