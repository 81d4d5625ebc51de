"""16-bit MFMA LSTM recurrences (vt_lstm16_layer_fwd / _bwd, csrc/lstm16.hip) on MI355X.

The kernels compute a definite 16-bit model of nn.LSTM (ref/model/vae_teb_model.py:
474-480, :647-653 under the reference's 16-mixed autocast, graph_model.py:510,
:709-711): forward operands x, h_{t-1} and the pre-scaled W_ih, W_hh (gate rows times
-log2 e, or -2 log2 e for g, in fp32) rounded to f16, sigmoid = 1 / (1 + 2^p) and
tanh = 2 sigmoid(2x) - 1 in the forward, backward operands
dg and W_hh / W_ih rounded to bf16, the parameter gradients from bf16-rounded dg, x and
h_{t-1} (bf16 MFMA, skdw16.hip), everything else (accumulation, biases, cell state,
activations, outputs, dgates) fp32.  The oracle here is that model
restated in fp64 on the CPU (`_emu`), with torch's fp64 nn.LSTM as the exact model.

Tolerance: two correct implementations of the same 16-bit model differ by
rounding-boundary flips (an h or dg within fp32 rounding of an f16 / bf16 boundary rounds
the other way, and the recurrence carries the difference), so the bound is the distance
between the model computed in fp64 and the SAME model computed in fp32 (`_emu(dt=fp32)`):
rel-L2(ours, emu64) <= 3 x rel-L2(emu32, emu64) + 2e-5 on outputs, dx and every
parameter gradient (+ 2 % of the gradient's own bf16 operand-rounding effect: its x / h
operands are the recurrence's fp32 outputs, whose ~1e-6 differences between two correct
implementations flip ~1e-4 of their bf16 roundings by one ulp — a rounding the kernel
did not apply would cost 100 % of that effect) — and that bound must stay inside the 16-bit model's own distance to
the exact LSTM (asserted for 1-2 layers; through 4 layers x 48 steps the flips make the
floor ~1/2 of that distance, and the 4-layer case bounds gross errors only).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ops():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from vaeteb import ops as o
    return o


def rel(a, b):
    a = torch.as_tensor(a).detach().double().cpu()
    b = torch.as_tensor(b).detach().double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def _emu(x, params, gy, dt=torch.float64):
    """Restatement of the 16-bit model the kernels compute (layer by layer, forward
    then a hand-written backward) in arithmetic dtype dt; returns y, dx and the
    parameter grads (float64 tensors)."""
    B, S, _ = x.shape
    nl = len(params) // 4
    H = params[1].shape[1]
    h16 = lambda t: t.to(torch.float16).to(dt)
    b16 = lambda t: t.to(torch.float32).to(torch.bfloat16).to(dt)
    # the forward's weights / biases pre-scaled in fp32 before the f16 rounding (gate rows
    # i, f, o by -log2 e, g by -2 log2 e): the MFMA yields p with sigmoid = 1 / (1 + 2^p)
    nl2e = torch.tensor(-1.44269504088896341, dtype=torch.float32)
    sc = torch.cat([torch.full((H,), float(nl2e)), torch.full((H,), float(nl2e)),
                    torch.full((H,), float(2 * nl2e)), torch.full((H,), float(nl2e))])
    saved, inp = [], x.to(dt)
    for l in range(nl):
        w_ih, w_hh, b_ih, b_hh = params[4 * l: 4 * l + 4]
        wx = h16(w_ih.float() * sc[:, None])
        wh = h16(w_hh.float() * sc[:, None])
        bias = ((b_ih.float() + b_hh.float()) * sc).to(dt)
        G = h16(inp) @ wx.T + bias
        h = torch.zeros(B, H, dtype=dt)
        c = torch.zeros(B, H, dtype=dt)
        hs, hps, cs, gs = [], [], [], []
        for t in range(S):
            p = G[:, t] + h16(h) @ wh.T
            i, f, g, o = (1 / (1 + torch.pow(2.0, p))).split(H, dim=1)
            g = 2 * g - 1
            hps.append(h)
            c = f * c + i * g
            # the kernel's tanh(c) = 2 / (1 + 2^(-2 log2(e) c)) - 1 (absolute, not relative,
            # accuracy near 0: the fp32 restatement carries the same cancellation)
            h = o * (2 / (1 + torch.pow(2.0, float(2 * nl2e) * c)) - 1)
            hs.append(h), cs.append(c), gs.append(torch.cat([i, f, g, o], 1))
        saved.append((inp, torch.stack(hps, 1), torch.stack(cs, 1), torch.stack(gs, 1)))
        inp = torch.stack(hs, 1)
    y = inp
    grads = [None] * len(params)
    qround = [0.0] * len(params)
    dh_out = gy.to(dt)
    for l in reversed(range(nl)):
        xin, hp, cs, gs = saved[l]
        w_ih, w_hh = params[4 * l].to(dt), params[4 * l + 1].to(dt)
        dg = torch.zeros(B, S, 4 * H, dtype=dt)
        dhr = torch.zeros(B, H, dtype=dt)
        dc = torch.zeros(B, H, dtype=dt)
        for t in reversed(range(S)):
            i, f, g, o = gs[:, t].split(H, dim=1)
            c = cs[:, t]
            cp = cs[:, t - 1] if t > 0 else torch.zeros_like(c)
            dh = dh_out[:, t] + dhr
            tc = torch.tanh(c)
            dc = dc + dh * o * (1 - tc * tc)
            d = torch.cat([dc * g * i * (1 - i), dc * cp * f * (1 - f), dc * i * (1 - g * g), dh * tc * o * (1 - o)], 1)
            dc = dc * f
            dg[:, t] = d
            dhr = b16(d) @ b16(w_hh)
        dx = b16(dg) @ b16(w_ih)
        grads[4 * l] = torch.einsum("bsg,bsi->gi", b16(dg), b16(xin))
        grads[4 * l + 1] = torch.einsum("bsg,bsi->gi", b16(dg), b16(hp))
        grads[4 * l + 2] = b16(dg).sum((0, 1))
        grads[4 * l + 3] = b16(dg).sum((0, 1))
        # the same gradients on the unrounded operands: the size of the bf16 operand rounding
        qround[4 * l] = rel(grads[4 * l], torch.einsum("bsg,bsi->gi", dg, xin))
        qround[4 * l + 1] = rel(grads[4 * l + 1], torch.einsum("bsg,bsi->gi", dg, hp))
        qround[4 * l + 2] = qround[4 * l + 3] = rel(grads[4 * l + 2], dg.sum((0, 1)))
        dh_out = dx
    _emu.qround = qround
    return y.double(), dh_out.double(), [g.double() for g in grads]


def _exact(x, params, gy, In):
    ref = torch.nn.LSTM(In, 64, len(params) // 4, batch_first=True).double()
    with torch.no_grad():
        for p, q in zip(ref.parameters(), params):
            p.copy_(q)
    xr = x.double().clone().requires_grad_()
    yr, _ = ref(xr)
    (yr * gy.double()).sum().backward()
    return yr.detach(), xr.grad, [p.grad for p in ref.parameters()]


@pytest.mark.parametrize("In,B,S,nl", [(20, 8, 48, 4), (32, 5, 33, 2), (64, 3, 16, 1), (8, 4, 5, 2), (64, 6, 40, 2)])
def test_lstm16_vs_16bit_model(ops, In, B, S, nl):
    """Ragged batch (B % 4 != 0: the last 4-sample tile masked), S not a multiple of the
    16-step chunk, In = 8 / 20 / 32 / 64 (one or two input k-steps, 1-4 dX column tiles)."""
    torch.manual_seed(7 + In + S)
    ref = torch.nn.LSTM(In, 64, nl, batch_first=True)
    params = [p.detach().clone() for p in ref.parameters()]
    x = torch.randn(B, S, In)
    gy = torch.randn(B, S, 64)
    ye, dxe, ge = _emu(x, params, gy)
    q = [0.0, 0.0] + list(_emu.qround)
    y3, dx3, g3 = _emu(x, params, gy, torch.float32)
    yx, dxx, gx = _exact(x, params, gy, In)
    pd = [p.cuda().requires_grad_() for p in params]
    xd = x.cuda().requires_grad_()
    y = ops.lstm(xd, pd, half=True)
    (y * gy.cuda()).sum().backward()
    torch.cuda.synchronize()
    names = ["y", "dx"] + [f"{n}_l{l}" for l in range(nl) for n in ("w_ih", "w_hh", "b_ih", "b_hh")]
    for n, ours, e, e32, ex, qr in zip(names, [y, xd.grad] + [p.grad for p in pd], [ye, dxe] + ge, [y3, dx3] + g3,
                                      [yx, dxx] + gx, q):
        d, floor, model = rel(ours, e), rel(e32, e), rel(e, ex)
        assert d <= 3 * floor + 2e-5 + 0.02 * qr, (n, d, floor, model, qr)
        if nl <= 2:   # shallow: the bound separates the 16-bit model from the exact one (4 layers
            # x 48 steps of bf16 flips make the model's own fp32/fp64 floor ~1/3 of its distance)
            assert 3 * floor + 2e-5 + 0.02 * qr < model, (n, floor, model, qr)


def test_lstm16_no_dx_and_outputs(ops):
    """Layer entry points directly: h / h_{t-1} / c / gates of the forward are the fp32
    outputs the backward and the weight gradients consume; dx = null and dgates = null
    are accepted (first layer without an input gradient)."""
    from vaeteb import _lib
    torch.manual_seed(3)
    B, S, In, H = 4, 20, 32, 64
    ref = torch.nn.LSTM(In, H, 1, batch_first=True)
    w_ih, w_hh, b_ih, b_hh = [p.detach().cuda().contiguous() for p in ref.parameters()]
    x = torch.randn(B, S, In, device="cuda")
    h, hp, c = (torch.empty(B, S, H, device="cuda") for _ in range(3))
    gates = torch.empty(B, S, 4 * H, device="cuda")
    P = lambda t: t.data_ptr()
    st = torch.cuda.current_stream().cuda_stream
    _lib.call("vt_lstm16_layer_fwd", P(x), In, P(w_ih), P(b_ih), P(w_hh), P(b_hh), B, S, H, P(h), P(hp), P(c),
              P(gates), st)
    torch.cuda.synchronize()
    assert torch.equal(hp[:, 1:], h[:, :-1]) and torch.count_nonzero(hp[:, 0]) == 0
    i, f, g, o = gates.view(B, S, H, 4).unbind(-1)   # [B, S, H, 4] (i, f, g~, o) per unit
    cp = torch.cat([torch.zeros_like(c[:, :1]), c[:, :-1]], 1)
    assert rel(c, f * cp + i * g) < 1e-6
    assert rel(h, o * torch.tanh(c)) < 1e-6
    assert bool((i > 0).all() and (i < 1).all() and (g.abs() <= 1).all())
    dh = torch.randn(B, S, H, device="cuda")
    dg = torch.empty(B, S, 4 * H, device="cuda")
    _lib.call("vt_lstm16_layer_bwd", P(dh), P(gates), P(c), P(w_hh), P(w_ih), In, B, S, H, P(dg), None, st)
    dg2 = torch.empty_like(dg)
    dx = torch.empty(B, S, In, device="cuda")
    _lib.call("vt_lstm16_layer_bwd", P(dh), P(gates), P(c), P(w_hh), P(w_ih), In, B, S, H, P(dg2), P(dx), st)
    _lib.call("vt_lstm16_layer_bwd", P(dh), P(gates), P(c), P(w_hh), P(w_ih), In, B, S, H, None, P(dx), st)
    torch.cuda.synchronize()
    assert torch.equal(dg, dg2)
    with pytest.raises(ValueError):
        _lib.call("vt_lstm16_layer_fwd", P(x), 30, P(w_ih), P(b_ih), P(w_hh), P(b_hh), B, S, H, P(h), P(hp), P(c),
                  P(gates), st)


@pytest.mark.parametrize("In,B,S", [(20, 3, 37), (64, 4, 16), (32, 5, 256), (64, 8, 300), (20, 2, 1)])
def test_lstm16_weight_grad_bf16(ops, In, B, S):
    """vt_lstm16_layer_bwd_weight (bf16 MFMA, h_{t-1} read from h, zero at t = 0) == the
    parameter gradients of bf16-rounded dg, x, h_{t-1} summed in fp64 (rel-L2 <= 1e-5: fp32
    accumulation order only); the exact-fp32 entry point on the same operands stays within
    bf16 rounding of it."""
    from vaeteb import _lib
    torch.manual_seed(In + S)
    H = 64
    dg = torch.randn(B, S, 4 * H, device="cuda")
    x = torch.randn(B, S, In, device="cuda")
    h = torch.randn(B, S, H, device="cuda")
    hp = torch.cat([torch.zeros_like(h[:, :1]), h[:, :-1]], 1).contiguous()
    ws = torch.empty(32 << 20, device="cuda")
    P = lambda t: t.data_ptr()
    st = torch.cuda.current_stream().cuda_stream
    outs = []
    for fn, hh in (("vt_lstm_layer_bwd_weight", hp), ("vt_lstm16_layer_bwd_weight", h)):
        o = [torch.full((4 * H, In), float("nan"), device="cuda"), torch.full((4 * H, H), float("nan"), device="cuda"),
             torch.empty(4 * H, device="cuda"), torch.empty(4 * H, device="cuda")]
        _lib.call(fn, P(dg), P(x), In, P(hh), B, S, H, *[P(t) for t in o], 0, P(ws), ws.numel(), st)
        outs.append(o)
    torch.cuda.synchronize()
    b16 = lambda t: t.cpu().bfloat16().double()
    g16 = b16(dg)
    ref = [torch.einsum("bsg,bsi->gi", g16, b16(x)), torch.einsum("bsg,bsi->gi", g16, b16(hp)), g16.sum((0, 1)),
           g16.sum((0, 1))]
    for ours, fp32, r in zip(outs[1], outs[0], ref):
        assert rel(ours, r) <= 1e-5, (rel(ours, r), rel(fp32, r))
        assert rel(fp32, r) <= 2e-2   # the exact gradient, within bf16 operand rounding


@pytest.mark.parametrize("In,B,S", [(20, 3, 37), (64, 4, 16)])
def test_lstm16_weight_grad_reads_h_shifted(ops, In, B, S):
    """With the bf16 kernel off (VAETEB_L16_DW16=0, checked in a fresh process):
    vt_lstm16_layer_bwd_weight (h_{t-1} read from h, zero at t = 0) == vt_lstm_layer_bwd_weight
    on an explicit h_{t-1} tensor, bit for bit (same kernel and summation order)."""
    import os
    import subprocess
    import sys
    code = f"""
import torch, sys
sys.path.insert(0, {repr(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "vae-teb_amd"))})
from vaeteb import _lib
torch.manual_seed({In} + {S})
B, S, In, H = {B}, {S}, {In}, 64
dg = torch.randn(B, S, 4 * H, device="cuda")
x = torch.randn(B, S, In, device="cuda")
h = torch.randn(B, S, H, device="cuda")
hp = torch.cat([torch.zeros_like(h[:, :1]), h[:, :-1]], 1).contiguous()
ws = torch.empty(32 << 20, device="cuda")
P = lambda t: t.data_ptr()
st = torch.cuda.current_stream().cuda_stream
outs = []
for fn, hh in (("vt_lstm_layer_bwd_weight", hp), ("vt_lstm16_layer_bwd_weight", h)):
    o = [torch.empty(4 * H, In, device="cuda"), torch.empty(4 * H, H, device="cuda"),
         torch.empty(4 * H, device="cuda"), torch.empty(4 * H, device="cuda")]
    _lib.call(fn, P(dg), P(x), In, P(hh), B, S, H, *[P(t) for t in o], 0, P(ws), ws.numel(), st)
    outs.append(o)
torch.cuda.synchronize()
assert all(torch.equal(a, b) for a, b in zip(*outs))
print("ok")
"""
    env = dict(os.environ, VAETEB_L16_DW16="0")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "ok" in r.stdout, r.stderr[-2000:]



@pytest.mark.parametrize("In,B,S,nl", [(20, 256, 256, 4), (32, 256, 256, 4), (32, 5, 37, 2), (64, 3, 16, 3),
                                       (20, 2, 1, 2), (32, 7, 300, 4), (8, 4, 33, 2), (20, 3, 17, 2)])
def test_lstm16_pair_bitwise_per_layer(ops, monkeypatch, In, B, S, nl):
    """vt_lstm16_pair_fwd / _bwd (two layers per workgroup, the upper one chunk behind) ==
    the per-layer kernels bit for bit: outputs, dx and every parameter gradient, at the bench
    geometry (B = 256, S = 256, the encoders' input sizes 20 / 32, 4 layers = 2 pairs), a
    ragged batch, S = 1, S not a multiple of the chunk, S = 300, and an odd layer count (a
    pair + one single layer)."""
    torch.manual_seed(11 + In + S + nl)
    ref = torch.nn.LSTM(In, 64, nl, batch_first=True)
    params = [p.detach().cuda() for p in ref.parameters()]
    x = torch.randn(B, S, In, device="cuda")
    gy = torch.randn(B, S, 64, device="cuda")
    outs, names = [], []
    real_call = ops.call
    monkeypatch.setattr(ops, "LSTM_CHAIN_FWD", 0)   # the pair launches themselves (chained: the test below)
    monkeypatch.setattr(ops, "LSTM_CHAIN_BWD", 0)
    for pair in (0, 1):
        monkeypatch.setattr(ops, "LSTM_PAIR", pair)
        called = []
        monkeypatch.setattr(ops, "call", lambda name, *a: (called.append(name), real_call(name, *a))[1])
        pd = [p.clone().requires_grad_() for p in params]
        xd = x.clone().requires_grad_()
        y = ops.lstm(xd, pd, half=True)
        y.backward(gy)
        torch.cuda.synchronize()
        outs.append([y.detach(), xd.grad] + [p.grad for p in pd])
        names.append(called)
    assert "vt_lstm16_pair_fwd" not in names[0] and "vt_lstm16_pair_bwd" not in names[0]
    assert names[1].count("vt_lstm16_pair_fwd") == nl // 2 and names[1].count("vt_lstm16_pair_bwd") == nl // 2
    for k, (a, b) in enumerate(zip(*outs)):
        assert torch.equal(a, b), (k, (a != b).sum().item(), (a - b).abs().max().item())


@pytest.mark.parametrize("In,B,S", [(20, 256, 256), (32, 256, 256), (20, 256, 300), (32, 64, 17), (20, 6, 40)])
def test_lstm16_quad_chained_bitwise_pairs(ops, monkeypatch, In, B, S):
    """vt_lstm16_quad_fwd / _bwd (round 6: the encoder's four layers in one launch each way, pair
    (2, 3) consuming layer 1's h — and in the backward layers (1, 0) consuming layer 2's dX — chunk
    by chunk through per-chunk flags) == the two pair launches bit for bit: output, dx and every
    parameter gradient; at the bench geometry (B = 256: 128 workgroups per pair, chained), S = 300,
    S not a multiple of the chunk, and B = 6 (3 workgroups per pair: not a multiple of 8, so the
    library runs the pairs one after the other).  Repeated twice in the process (the flags are left
    zero for the next launch), and no bounded wait timed out."""
    import ctypes
    from vaeteb import _lib
    torch.manual_seed(5 + In + S + B)
    ref = torch.nn.LSTM(In, 64, 4, batch_first=True)
    params = [p.detach().cuda() for p in ref.parameters()]
    x = torch.randn(B, S, In, device="cuda")
    gy = torch.randn(B, S, 64, device="cuda")
    cnt = ctypes.c_int()
    _lib.call("vt_lstm16_chain_errors", ctypes.byref(cnt), 1)
    outs, names = [], []
    real_call = ops.call
    for chain in (0, 1, 1):
        monkeypatch.setattr(ops, "LSTM_CHAIN_FWD", chain)
        monkeypatch.setattr(ops, "LSTM_CHAIN_BWD", chain)
        called = []
        monkeypatch.setattr(ops, "call", lambda name, *a: (called.append(name), real_call(name, *a))[1])
        pd = [p.clone().requires_grad_() for p in params]
        xd = x.clone().requires_grad_()
        y = ops.lstm(xd, pd, half=True)
        y.backward(gy)
        torch.cuda.synchronize()
        outs.append([y.detach(), xd.grad] + [p.grad for p in pd])
        names.append(called)
    assert names[0].count("vt_lstm16_pair_fwd") == 2 and "vt_lstm16_quad_fwd" not in names[0]
    assert names[1].count("vt_lstm16_quad_fwd") == 1 and names[1].count("vt_lstm16_quad_bwd") == 1
    _lib.call("vt_lstm16_chain_errors", ctypes.byref(cnt), 1)
    assert cnt.value == 0, cnt.value
    for run in (1, 2):
        for k, (a, b) in enumerate(zip(outs[0], outs[run])):
            assert torch.equal(a, b), (run, k, (a != b).sum().item(), (a - b).abs().max().item())
