"""HIP model ops and the full SeqVaeTeb step vs torch references (MI355X).

Op tests compare each HIP kernel with the plain-PyTorch fp64 CPU version of
the same op (tolerance rel-L2 <= 1e-5 unless stated).  The model tests load the
deterministic weights (tests/golden_util.py) and compare forward outputs, the
loss parts and every gradient with the REFERENCE's own values in
tests/golden/model_s*.npz (fp32 CPU reference vs fp32 HIP: different
summation orders through a 4-layer LSTM and 17 train-mode BatchNorms, so
per-tensor rel-L2 <= 2e-4 for gradients and 1e-5 for the losses).
"""
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ops():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from vaeteb import ops as o
    return o


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def _leaf(t, dev="cuda"):
    return t.detach().to(dev, torch.float32).requires_grad_(True)


@pytest.mark.parametrize("R,K,N", [(1000, 130, 103), (65, 32, 32), (300, 64, 256), (17, 4096, 4096)])
def test_linear(ops, R, K, N):
    torch.manual_seed(R)
    x, w, b = torch.randn(R, K, dtype=torch.float64), torch.randn(N, K, dtype=torch.float64) / K ** 0.5, \
        torch.randn(N, dtype=torch.float64)
    gy = torch.randn(R, N, dtype=torch.float64)
    xr, wr, br = x.clone().requires_grad_(), w.clone().requires_grad_(), b.clone().requires_grad_()
    (F.linear(xr, wr, br) * gy).sum().backward()
    xd, wd, bd = _leaf(x), _leaf(w), _leaf(b)
    y = ops.linear(xd, wd, bd)
    (y * gy.float().cuda()).sum().backward()
    assert rel(y, F.linear(x, w, b)) < 1e-5
    assert rel(xd.grad, xr.grad) < 1e-5 and rel(wd.grad, wr.grad) < 1e-5 and rel(bd.grad, br.grad) < 1e-5


@pytest.mark.parametrize("R,K,N", [(70000, 20, 256), (4099, 256, 64), (1000, 145, 200), (33, 3, 5)])
def test_linear_skinny_shapes(ops, R, K, N):
    """The skinny fp32-MFMA path (N <= 256): LSTM projections (256 gates),
    their input gradient (256 -> 64), ragged sizes and partial row tiles."""
    test_linear(ops, R, K, N)


@pytest.mark.parametrize("R,K,N", [(1000, 130, 103), (4100, 64, 64), (77, 32, 20), (300, 87, 256)])
@pytest.mark.parametrize("act", ["none", "relu", "gelu"])
def test_linear_ln_act(ops, R, K, N, act):
    """Fused Linear -> LayerNorm -> act (vt_linear_ln_fwd) vs torch fp64."""
    torch.manual_seed(R + N)
    x, w, b = torch.randn(R, K, dtype=torch.float64), torch.randn(N, K, dtype=torch.float64) / K ** 0.5, \
        torch.randn(N, dtype=torch.float64)
    g, be = 1 + 0.1 * torch.randn(N, dtype=torch.float64), 0.1 * torch.randn(N, dtype=torch.float64)
    gy = torch.randn(R, N, dtype=torch.float64)
    leaves = [t.clone().requires_grad_() for t in (x, w, b, g, be)]
    fn = {"none": lambda t: t, "relu": F.relu, "gelu": F.gelu}[act]
    yr = fn(F.layer_norm(F.linear(*leaves[:3]), (N,), leaves[3], leaves[4], 1e-5))
    (yr * gy).sum().backward()
    dl = [_leaf(t) for t in (x, w, b, g, be)]
    y = ops.linear_ln_act(*dl, act)
    (y * gy.float().cuda()).sum().backward()
    assert rel(y, yr) < 1e-5
    for a, e, n in zip([t.grad for t in dl], [t.grad for t in leaves], "xwbgB"):
        assert rel(a, e) < 2e-5, n


@pytest.mark.parametrize("C", [16, 44, 130, 4096])
@pytest.mark.parametrize("act", ["none", "relu", "gelu"])
def test_layernorm_act(ops, C, act):
    torch.manual_seed(C)
    R = 512 if C < 4096 else 8
    x = torch.randn(R, C, dtype=torch.float64) * 3 + 1
    g, b = 1 + 0.1 * torch.randn(C, dtype=torch.float64), 0.1 * torch.randn(C, dtype=torch.float64)
    gy = torch.randn(R, C, dtype=torch.float64)
    xr, gr, br = x.clone().requires_grad_(), g.clone().requires_grad_(), b.clone().requires_grad_()
    fn = {"none": lambda t: t, "relu": F.relu, "gelu": F.gelu}[act]
    yr = fn(F.layer_norm(xr, (C,), gr, br, 1e-5))
    (yr * gy).sum().backward()
    xd, gd, bd = _leaf(x), _leaf(g), _leaf(b)
    y = ops.layer_norm_act(xd, gd, bd, act)
    (y * gy.float().cuda()).sum().backward()
    assert rel(y, yr) < 1e-5
    for a, e in ((xd.grad, xr.grad), (gd.grad, gr.grad), (bd.grad, br.grad)):
        assert rel(a, e) < 2e-5


def _ref_conv_block(x_blc, w, g, b, rm, rv, causal, up, tanh):
    """Plain-torch version of the reference block on (B, L, C) input."""
    x = x_blc.transpose(1, 2)
    K = w.shape[-1]
    if causal:
        x = F.pad(x, (K - 1, 0))
    else:
        if up:
            x = F.interpolate(x, scale_factor=2, mode="linear", align_corners=False)
        p = (K - 1) // 2
        if p > 0:
            if x.shape[-1] <= p:
                x = F.pad(x, (p, p), mode="replicate")
            else:
                x = torch.cat([x[..., 1:p + 1].flip(-1), x, x[..., -p - 1:-1].flip(-1)], -1)
    y = F.batch_norm(F.conv1d(x, w), rm, rv, g, b, True, 0.9, 1e-5)
    y = torch.tanh(y) if tanh else F.relu(y)
    return y.transpose(1, 2)


@pytest.mark.parametrize("B,L,Cin,Cout,K,causal,up,tanh", [
    (8, 64, 16, 16, 7, True, False, False),
    (4, 40, 32, 32, 3, True, False, False),
    (4, 16, 87, 77, 11, False, False, False),
    (4, 32, 77, 66, 9, False, True, False),
    (3, 4, 87, 77, 11, False, False, False),     # L <= pad: replicate fallback
    (2, 3, 8, 6, 5, False, True, False),         # upsample then replicate
    (4, 256, 11, 1, 3, False, False, False),
    (8, 256, 16, 2, 3, False, False, True),
    (2, 1024, 33, 22, 3, False, True, False),    # decoder L6 geometry (x2 upsample to 2048)
    (3, 300, 1, 16, 3, True, False, False),      # Cin = 1 (tiny encoder)
    (2, 512, 55, 44, 5, False, False, False),
])
def test_conv_bn_act(ops, B, L, Cin, Cout, K, causal, up, tanh):
    torch.manual_seed(B * 1000 + L)
    x = torch.randn(B, L, Cin, dtype=torch.float64)
    w = torch.randn(Cout, Cin, K, dtype=torch.float64) / (Cin * K) ** 0.5
    g, b = 1 + 0.1 * torch.randn(Cout, dtype=torch.float64), 0.1 * torch.randn(Cout, dtype=torch.float64)
    rm, rv = torch.randn(Cout, dtype=torch.float64) * 0.1, torch.rand(Cout, dtype=torch.float64) + 0.5
    xr, wr, gr, br = [t.clone().requires_grad_() for t in (x, w, g, b)]
    rmr, rvr = rm.clone(), rv.clone()
    yr = _ref_conv_block(xr, wr, gr, br, rmr, rvr, causal, up, tanh)
    gy = torch.randn_like(yr)
    (yr * gy).sum().backward()
    xd, wd, gd, bd = [_leaf(t) for t in (x, w, g, b)]
    rmd, rvd = rm.float().cuda(), rv.float().cuda()
    y = ops.conv_bn_act(xd, wd, gd, bd, rmd, rvd, mode=0 if causal else 1, up=up, act="tanh" if tanh else "relu")
    (y * gy.float().cuda()).sum().backward()
    assert y.shape == yr.shape
    assert rel(y, yr) < 1e-5
    assert rel(rmd, rmr) < 1e-6 and rel(rvd, rvr) < 1e-6
    for a, e, n in ((xd.grad, xr.grad, "x"), (wd.grad, wr.grad, "w"), (gd.grad, gr.grad, "g"), (bd.grad, br.grad, "b")):
        assert rel(a, e) < 5e-5, n


@pytest.mark.parametrize("In,B,S", [(20, 4, 33), (32, 3, 16)])
def test_lstm(ops, In, B, S):
    torch.manual_seed(In)
    ref = torch.nn.LSTM(In, 64, 4, batch_first=True).double()
    x = torch.randn(B, S, In, dtype=torch.float64)
    gy = torch.randn(B, S, 64, dtype=torch.float64)
    xr = x.clone().requires_grad_()
    yr, _ = ref(xr)
    (yr * gy).sum().backward()
    params = [_leaf(p) for p in ref.parameters()]   # order: w_ih, w_hh, b_ih, b_hh per layer
    xd = _leaf(x)
    y = ops.lstm(xd, params)
    (y * gy.float().cuda()).sum().backward()
    assert rel(y, yr) < 1e-5
    assert rel(xd.grad, xr.grad) < 2e-5
    for p, pr in zip(params, ref.parameters()):
        assert rel(p.grad, pr.grad) < 2e-5


@pytest.mark.parametrize("In,B,S", [(20, 3, 33), (32, 2, 16), (64, 2, 47), (64, 3, 256), (7, 2, 5), (48, 2, 18)])
def test_lstm_fused_projection_bitwise(ops, In, B, S, monkeypatch):
    """vt_lstm_layer_{fwd,bwd}_x (input projections inside the recurrence) give
    the bits of the separate skinny GEMM + recurrence path: the same MFMA chains.
    vt_lstm_layer_bwd_weight gives the weight gradients of the two separate
    vt_linear_bwd_weight calls bit for bit."""
    torch.manual_seed(100 + In)
    ref = torch.nn.LSTM(In, 64, 4, batch_first=True)
    x = torch.randn(B, S, In)
    gy = torch.randn(B, S, 64).cuda()
    outs = []
    for fused in (0, 1):
        monkeypatch.setattr(ops, "LSTM_FUSED", fused)
        params = [_leaf(p) for p in ref.parameters()]
        xd = _leaf(x)
        y = ops.lstm(xd, params)
        (y * gy).sum().backward()
        outs.append([y.detach(), xd.grad] + [p.grad for p in params])
    # y, dx and the weight gradients: the same MFMA chains (bitwise); the bias
    # gradients come from vt_lstm_layer_bwd_weight's ones-column instead of a
    # column-sum kernel (another fixed summation order)
    for i, (a, e) in enumerate(zip(*outs)):
        if i >= 2 and (i - 2) % 4 >= 2:
            assert rel(a, e) < 1e-6, i
        else:
            assert torch.equal(a, e), i


def _load_model(S):
    from golden_util import det_fill_
    from vaeteb.model import SeqVaeTeb
    return det_fill_(SeqVaeTeb(sequence_length=S)).cuda()


@pytest.mark.parametrize("name", ["model_s16_b4", "model_s4_b3"])
def test_model_step_vs_reference_golden(golden, name):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    g = golden(name)
    S = int(g["S"])
    m = _load_model(S)
    m.train()
    T = lambda k: torch.from_numpy(g[k]).cuda()
    fw = m(T("y_st"), T("y_ph"), T("x_ph"), eps=T("eps"))
    L = m.compute_loss(fw, T("y_st"), T("y_ph"), T("y_raw"), compute_kld_loss=True, beta=float(g["beta"]))
    for k in ("mse_loss", "nll_loss", "kld_loss", "total_loss"):
        exp = float(g["loss_" + k])
        assert abs(L[k].item() - exp) <= 1e-5 * abs(exp) + 1e-7, (k, L[k].item(), exp)
    for k in ("z", "mu_pr", "logvar_pr", "mu_post", "logvar_post", "mu_prior", "logvar_prior", "linear_output"):
        # fp32 vs fp32 in different summation orders through the LSTMs, 17
        # BatchNorms and the heads: a few 1e-5 on the deepest outputs
        assert rel(fw[k], torch.from_numpy(g["fw_" + k])) < 5e-5, k
    L["total_loss"].backward()
    names = list(g["param_names"])
    params = dict(m.named_parameters())
    worst = max((rel(params[k].grad, torch.from_numpy(g[f"grad_{i}"])), k) for i, k in enumerate(names))
    assert worst[0] < 2e-4, worst
    sd = m.state_dict()
    for i, k in enumerate(list(g["bn_names"])):
        assert rel(sd[k], torch.from_numpy(g[f"bn_{i}"])) < 1e-5, k


@pytest.mark.parametrize("concurrent", [False, True])
def test_measure_transfer_entropy_vs_reference_golden(golden, concurrent):
    """SeqVaeTeb.measure_transfer_entropy (ref/model/vae_teb_model.py:1194-1226): after
    one train-mode forward (running statistics updated), eval-mode BatchNorm, no
    gradients; elementwise KL (B, S, 32) and its mean vs the reference, model left in
    eval mode."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    g, t = golden("model_s16_b4"), golden("te_s16_b4")
    m = _load_model(16)
    m.concurrent_encoders = concurrent
    m.train()
    T = lambda k: torch.from_numpy(g[k]).cuda()
    with torch.no_grad():
        m(T("y_st"), T("y_ph"), T("x_ph"), eps=T("eps"))
    sd = m.state_dict()
    for i, k in enumerate(list(t["bn_names"])):
        if not k.startswith("decoder."):   # the decoder's statistics depend on the reference's random eps
            assert rel(sd[k], torch.from_numpy(t[f"bn_{i}"])) < 1e-5, k
    te = m.measure_transfer_entropy(T("y_st"), T("y_ph"), T("x_ph"))
    assert not m.training and te.shape == (4, 16, 32) and not te.requires_grad
    assert rel(te, torch.from_numpy(t["te"])) < 5e-5
    te_mean = m.measure_transfer_entropy(T("y_st"), T("y_ph"), T("x_ph"), reduce_mean=True)
    assert abs(te_mean.item() - float(t["te_mean"])) <= 5e-5 * abs(float(t["te_mean"]))


def test_tiny_c1_vs_reference_golden(golden):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from golden_util import det_fill_
    from vaeteb.model import TinyVaeTeb
    g = golden("tiny_c1")
    m = det_fill_(TinyVaeTeb()).cuda().train()
    r = m(torch.from_numpy(g["x"]).cuda(), torch.from_numpy(g["eps"]).cuda())
    assert abs(r["total"].item() - float(g["total"])) <= 1e-5 * abs(float(g["total"]))
    r["total"].backward()
    for i, (k, p) in enumerate(m.named_parameters()):
        assert rel(p.grad, torch.from_numpy(g[f"grad_{i}"])) < 1e-4, k


def test_concurrent_encoders_bitwise_identical(golden):
    """The two encoders on two HIP streams (SeqVaeTeb(concurrent_encoders=True))
    give bit-identical losses, gradients and updated parameters to the serial
    run: every reduction has a fixed order, so stream interleaving must not
    change a single bit — and a missing cross-stream sync would."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from golden_util import det_fill_
    from vaeteb.model import SeqVaeTeb
    from vaeteb.train import Trainer
    g = golden("model_s16_b4")
    T = lambda k: torch.from_numpy(g[k]).cuda()
    res = []
    for conc in (False, True):
        m = det_fill_(SeqVaeTeb(sequence_length=16, concurrent_encoders=conc)).cuda()
        tr = Trainer(m, lr=1e-3)
        batch = {"fhr_st": T("y_st"), "fhr_ph": T("y_ph"), "fhr_up_ph": T("x_ph"), "fhr": T("y_raw")}
        for _ in range(2):
            L = tr.step(batch, eps=T("eps"))
        torch.cuda.synchronize()
        res.append((L["total_loss"].item(), tr.state.g.clone(), tr.state.p.clone()))
    assert res[0][0] == res[1][0]
    assert torch.equal(res[0][1], res[1][1]) and torch.equal(res[0][2], res[1][2])


def test_concurrent_frontend_and_encoders_bitwise_identical():
    """Raw windows -> front-end (cross pairs on the source encoder's stream) ->
    model step: bit-identical to the all-serial run."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from vaeteb import synthetic
    from vaeteb.frontend import FrontEnd, FrontEndPlan, load_stats
    from vaeteb.model import SeqVaeTeb
    from vaeteb.train import Trainer
    plan = FrontEndPlan(11, 4, 16, 4096, device="cuda")
    fe = FrontEnd(plan, load_stats(11, 4, 16, 4096))
    x = torch.from_numpy(synthetic.batch(5, 4, 4096)).cuda()
    res = []
    for conc in (False, True):
        torch.manual_seed(0)
        m = SeqVaeTeb(sequence_length=plan.S, scattering_channels=fe.C_st, phase_channels=fe.C_ph,
                      cross_phase_channels=fe.C_x, concurrent_encoders=conc).cuda()
        tr = Trainer(m, lr=1e-3, frontend=fe)
        eps = torch.randn(4, plan.S, 32, generator=torch.Generator().manual_seed(1)).cuda()
        L = tr.step({"x": x}, eps=eps)
        torch.cuda.synchronize()
        res.append((L["total_loss"].item(), tr.state.g.clone()))
    assert res[0][0] == res[1][0]
    assert torch.equal(res[0][1], res[1][1])


@pytest.mark.parametrize("concurrent", [False, True])
def test_graph_replay_bitwise_identical_to_eager(golden, concurrent):
    """Trainer.capture/replay (the whole step as one hipGraph) == eager steps,
    bit for bit, over several steps (device-side AdamW step counter, static
    inputs refreshed per replay, side streams joined inside the graph)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from golden_util import det_fill_
    from vaeteb.model import SeqVaeTeb
    from vaeteb.train import Trainer
    g = golden("model_s16_b4")
    T = lambda k: torch.from_numpy(g[k]).cuda()
    b0 = {"fhr_st": T("y_st"), "fhr_ph": T("y_ph"), "fhr_up_ph": T("x_ph"), "fhr": T("y_raw")}
    b1 = {k: v.flip(0).contiguous() for k, v in b0.items()}
    eps = T("eps")
    res = []
    for graph in (False, True):
        m = det_fill_(SeqVaeTeb(sequence_length=16, concurrent_encoders=concurrent)).cuda()
        tr = Trainer(m, lr=1e-3)
        if graph:
            tr.capture(b0, eps=eps, warmup=2)
            outs = [tr.replay(b, eps=eps)["total_loss"].item() for b in (b1, b0, b1)]
        else:
            for _ in range(2):
                tr.step(b0, eps=eps)
            outs = [tr.step(b, eps=eps)["total_loss"].item() for b in (b1, b0, b1)]
        torch.cuda.synchronize()
        res.append((outs, tr.state.p.clone(), tr.state.m.clone()))
    assert res[0][0] == res[1][0]
    assert torch.equal(res[0][1], res[1][1]) and torch.equal(res[0][2], res[1][2])


def test_graph_capture_bf16_paths_after_eager_steps(golden):
    """Capture after eager steps (a loss kept from them must not tie the
    parameters' AccumulateGrad nodes to another stream) with the bf16-MFMA
    decoder heads and bf16 conv blocks, concurrent encoders: replay == eager
    bit for bit (advisor round 1: this configuration crashed in
    hipStreamEndCapture)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from golden_util import det_fill_
    from vaeteb import ops
    from vaeteb.model import SeqVaeTeb
    from vaeteb.train import Trainer
    g = golden("model_s16_b4")
    T = lambda k: torch.from_numpy(g[k]).cuda()
    b0 = {"fhr_st": T("y_st"), "fhr_ph": T("y_ph"), "fhr_up_ph": T("x_ph"), "fhr": T("y_raw")}
    b1 = {k: v.flip(0).contiguous() for k, v in b0.items()}
    eps = T("eps")
    assert ops.mfma_ok(256, 256)   # R = 16 S = 256: the heads take the bf16 MFMA path
    res = []
    for graph in (False, True):
        m = det_fill_(SeqVaeTeb(sequence_length=16, concurrent_encoders=True, head_precision="bf16",
                                conv_precision="bf16")).cuda()
        tr = Trainer(m, lr=1e-3)
        kept = tr.step(b0, eps=eps)          # an eager step whose losses stay referenced
        if graph:
            tr.capture(b0, eps=eps, warmup=1)
            outs = [tr.replay(b, eps=eps)["total_loss"].item() for b in (b1, b0, b1)]
        else:
            tr.step(b0, eps=eps)
            outs = [tr.step(b, eps=eps)["total_loss"].item() for b in (b1, b0, b1)]
        torch.cuda.synchronize()
        assert kept["total_loss"].grad_fn is None
        res.append((outs, tr.state.p.clone()))
    assert res[0][0] == res[1][0]
    assert torch.equal(res[0][1], res[1][1])


@pytest.mark.parametrize("n_streams", [1, 2, 4])
def test_native_executor_bitwise_identical_to_eager(golden, n_streams):
    """The library's multi-stream executor over the captured step
    (Trainer.capture(native=True), csrc/stepgraph.cpp) == eager steps bit for bit:
    the same kernels and arguments, the capture's cross-stream dependencies kept
    as event waits whatever the stream count (concurrent encoders, bf16 heads /
    convs / MLPs: every side stream of the step)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from golden_util import det_fill_
    from vaeteb.model import SeqVaeTeb
    from vaeteb.train import Trainer
    g = golden("model_s16_b4")
    T = lambda k: torch.from_numpy(g[k]).cuda()
    b0 = {"fhr_st": T("y_st"), "fhr_ph": T("y_ph"), "fhr_up_ph": T("x_ph"), "fhr": T("y_raw")}
    b1 = {k: v.flip(0).contiguous() for k, v in b0.items()}
    eps0 = T("eps")
    eps1 = eps0.flip(0).contiguous()
    res = []
    for native in (False, True):
        m = det_fill_(SeqVaeTeb(sequence_length=16, concurrent_encoders=True, head_precision="bf16",
                                conv_precision="bf16", mlp_precision="bf16")).cuda()
        tr = Trainer(m, lr=1e-3)
        if native:
            cap = tr.capture(b0, eps=eps0, warmup=2, native=True, n_streams=n_streams)
            n_kernel, n_memcpy, n_memset, n_waits = cap.info()
            assert n_kernel > 100 and (n_streams > 1 or n_waits == 0)
            outs = [tr.replay(b, eps=e)["total_loss"].item() for b, e in ((b1, eps1), (b0, eps0), (b1, eps1))]
        else:
            for _ in range(2):
                tr.step(b0, eps=eps0)
            outs = [tr.step(b, eps=e)["total_loss"].item() for b, e in ((b1, eps1), (b0, eps0), (b1, eps1))]
        torch.cuda.synchronize()
        res.append((outs, tr.state.p.clone(), tr.state.m.clone(), tr.state.v.clone()))
    assert res[0][0] == res[1][0]
    for a, b in zip(res[0][1:], res[1][1:]):
        assert torch.equal(a, b)


def test_first_writer_group_reached_through_autograd():
    """Advisor r04 (low): once a first-writer group (a >= 2^20-element linear weight + bias)
    is confirmed, zero_grad leaves its range unzeroed for LinearF to overwrite.  A later step
    whose gradient for that weight arrives through autograd (AccumulateGrad, here F.linear)
    must see a zeroed range (not last step's values) and keep its gradient (not be zeroed
    after the backward)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from vaeteb import ops
    from vaeteb.train import FlatState
    torch.manual_seed(0)
    lin = torch.nn.Linear(1024, 1024).cuda()
    st = FlatState(lin)
    assert len(st.first_writer) == 1
    x = torch.randn(64, 1024, device="cuda")
    for i in range(3):                                # LinearF steps: the group gets confirmed
        st.zero_grad(first_writer=True)
        ops.LinearF.apply(x * (i + 1), lin.weight, lin.bias, False).square().sum().backward()
        st.finish_first_writer()
    assert st._fw_ok == {0}
    st.zero_grad(first_writer=True)                   # group left unzeroed (holds step 3's gradient)
    torch.nn.functional.linear(x, lin.weight, lin.bias).square().sum().backward()
    st.finish_first_writer()
    torch.cuda.synchronize()
    ref = torch.nn.Linear(1024, 1024).cuda()
    ref.load_state_dict(lin.state_dict())
    torch.nn.functional.linear(x, ref.weight, ref.bias).square().sum().backward()
    torch.testing.assert_close(lin.weight.grad, ref.weight.grad, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(lin.bias.grad, ref.bias.grad, rtol=1e-5, atol=1e-5)
    assert st._fw_ok == set() and 0 in st._fw_bad     # demoted: zeroed with the rest from now on


def test_native_replay_after_load_state_dict(golden):
    """Advisor r04 (medium): the captured forward trusts the bf16 head / conv shadows the
    optimizer pass wrote.  After a load_state_dict between replays the replay must compute with
    the LOADED weights (CapturedStep re-checks the weights' version counters and rewrites the
    shadows), exactly as an eager step from the same loaded state does — bit for bit."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from golden_util import det_fill_
    from vaeteb.model import SeqVaeTeb
    from vaeteb.train import Trainer
    g = golden("model_s16_b4")
    T = lambda k: torch.from_numpy(g[k]).cuda()
    b0 = {"fhr_st": T("y_st"), "fhr_ph": T("y_ph"), "fhr_up_ph": T("x_ph"), "fhr": T("y_raw")}
    b1 = {k: v.flip(0).contiguous() for k, v in b0.items()}
    eps0 = T("eps")
    torch.manual_seed(7)
    src = SeqVaeTeb(sequence_length=16)   # another model's weights (default init, not det_fill_)
    loaded = {k: v.cuda() for k, v in src.state_dict().items()}
    res = []
    for native in (False, True):
        m = det_fill_(SeqVaeTeb(sequence_length=16, concurrent_encoders=True, head_precision="bf16",
                                conv_precision="bf16", mlp_precision="bf16")).cuda()
        tr = Trainer(m, lr=1e-3)
        if native:
            tr.capture(b0, eps=eps0, warmup=2, native=True)
            outs = [tr.replay(b1, eps=eps0)["total_loss"].item()]
        else:
            for _ in range(2):
                tr.step(b0, eps=eps0)
            outs = [tr.step(b1, eps=eps0)["total_loss"].item()]
        torch.cuda.synchronize()
        m.load_state_dict(loaded)
        step = tr.replay if native else tr.step
        outs += [step(b, eps=eps0)["total_loss"].item() for b in (b0, b1)]
        torch.cuda.synchronize()
        res.append((outs, tr.state.p.clone()))
    assert res[0][0] == res[1][0], (res[0][0], res[1][0])
    assert torch.equal(res[0][1], res[1][1])


@pytest.mark.parametrize("B", [4, 256])
def test_native_executor_with_frontend_bitwise_identical_to_eager(B):
    """The step captured from RAW windows (the front-end inside the graph, its cross pairs
    on the source encoder's stream) replayed by the executor == eager steps from the same
    windows, bit for bit (losses, parameters, Adam moments), at the benchmarked front-end
    (J=11 Q=4 T=16, N=4096) and bench precision; B = 256 is the bench's own batch (the
    128-workgroup LSTM grids, the > 64-slab split sums and the XCD-remapped front-end at
    their bench sizes)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from golden_util import det_fill_
    from vaeteb import synthetic
    from vaeteb.frontend import FrontEnd, FrontEndPlan, load_stats
    from vaeteb.model import SeqVaeTeb
    from vaeteb.train import Trainer
    fe = FrontEnd(FrontEndPlan(11, 4, 16, 4096, device="cuda"), load_stats())
    xs = [torch.from_numpy(synthetic.batch(1000 * i, B, 4096)).cuda() for i in range(2)]
    S = fe.plan.S
    epss = [torch.randn(B, S, 32, generator=torch.Generator().manual_seed(i)).cuda() for i in range(2)]
    res = []
    for native in (False, True):
        m = det_fill_(SeqVaeTeb(sequence_length=S, scattering_channels=fe.C_st, phase_channels=fe.C_ph,
                                cross_phase_channels=fe.C_x, concurrent_encoders=True, head_precision="bf16",
                                conv_precision="bf16", mlp_precision="bf16", lstm_precision="16-mixed")).cuda()
        tr = Trainer(m, lr=1e-3, frontend=fe)
        if native:
            cap = tr.capture({"x": xs[0]}, eps=epss[0], warmup=2, native=True)
            outs = [cap.replay({"x": xs[i % 2]}, eps=epss[i % 2])["total_loss"].item() for i in (1, 0, 1)]
        else:
            for _ in range(2):
                tr.step({"x": xs[0]}, eps=epss[0])
            outs = [tr.step({"x": xs[i % 2]}, eps=epss[i % 2])["total_loss"].item() for i in (1, 0, 1)]
        torch.cuda.synchronize()
        res.append((outs, tr.state.p.clone(), tr.state.m.clone(), tr.state.v.clone()))
    assert res[0][0] == res[1][0]
    for a, b in zip(res[0][1:], res[1][1:]):
        assert torch.equal(a, b)


def test_native_executor_requires_eps(golden):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from golden_util import det_fill_
    from vaeteb.model import SeqVaeTeb
    from vaeteb.train import Trainer
    g = golden("model_s16_b4")
    T = lambda k: torch.from_numpy(g[k]).cuda()
    b0 = {"fhr_st": T("y_st"), "fhr_ph": T("y_ph"), "fhr_up_ph": T("x_ph"), "fhr": T("y_raw")}
    tr = Trainer(det_fill_(SeqVaeTeb(sequence_length=16)).cuda(), lr=1e-3)
    with pytest.raises(ValueError):
        tr.capture(b0, native=True)


@pytest.mark.parametrize("defer", [0, 1])
def test_prepass_and_deferred_lstm_grads_bitwise(golden, monkeypatch, defer):
    """bf16 heads / convs with the weight-only prepass (shadows + BatchNorm counters
    ahead of the forward on a side stream) and the LSTM parameter gradients deferred
    to a side stream: bit-identical losses, gradients and parameters to the serial
    in-line run, and every BatchNorm counted exactly once per step."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from golden_util import det_fill_
    from vaeteb import model as MD, ops
    from vaeteb.model import ConvBlock, SeqVaeTeb
    from vaeteb.train import Trainer
    monkeypatch.setattr(ops, "LSTM_GRAD_DEFER", defer)
    g = golden("model_s16_b4")
    T = lambda k: torch.from_numpy(g[k]).cuda()
    res = []
    for conc, prepass in ((False, 0), (True, 1), (True, 0)):
        monkeypatch.setattr(MD, "PREPASS", prepass)
        m = det_fill_(SeqVaeTeb(sequence_length=16, concurrent_encoders=conc, head_precision="bf16",
                                conv_precision="bf16")).cuda()
        tr = Trainer(m, lr=1e-3)
        batch = {"fhr_st": T("y_st"), "fhr_ph": T("y_ph"), "fhr_up_ph": T("x_ph"), "fhr": T("y_raw")}
        for i in range(3):
            if i == 1:
                m.prepass()   # ahead of the forward, as Trainer.loss does before the front-end
            L = tr.step(batch, eps=T("eps"))
        torch.cuda.synchronize()
        counts = {int(mm.bn_layer.num_batches_tracked) for mm in m.modules() if isinstance(mm, ConvBlock)}
        assert counts == {3}, counts
        assert set(m.state_dict().keys()) == set(det_fill_(SeqVaeTeb(sequence_length=16)).state_dict().keys())
        res.append((L["total_loss"].item(), tr.state.g.clone(), tr.state.p.clone()))
    for r in res[1:]:
        assert res[0][0] == r[0]
        assert torch.equal(res[0][1], r[1]) and torch.equal(res[0][2], r[2])


_HANDOFF_SCRIPT = r"""
import sys, numpy as np, torch
sys.path[:0] = [{pkg!r}]
from vaeteb import ops
d = np.load({inp!r})
x = torch.from_numpy(d["x"]).cuda()
params = [torch.from_numpy(d[f"p{{i}}"]).cuda() for i in range(4)]
ops.LSTM_FUSED = 1
y = ops.lstm(x, params)
torch.cuda.synchronize()
np.save({out!r}, y.cpu().numpy())
"""


@pytest.mark.parametrize("In,B,S", [(64, 4, 64), (20, 3, 48), (32, 2, 80)])
def test_lstm_fused_chunk_handoff_bitwise_fresh_process(ops, tmp_path, In, B, S):
    """The fused forward kernel (k_lstm_fwd_x) issues the NEXT chunk's input projection
    behind each step's barrier and hands it to the lanes at the chunk boundary; round 2
    found an operand read hoisted ahead of that barrier, which made the first steps of
    a process intermittently wrong.  Pinned here: S a multiple of the 16-step chunk with
    several chunks, the layer's outputs bitwise equal to the plain path (separate
    projection GEMM + recurrence) on 8 back-to-back launches in this process AND on the
    first launch of a fresh process."""
    import subprocess
    import sys
    import numpy as np
    torch.manual_seed(In * 10 + S)
    ref = torch.nn.LSTM(In, 64, 1, batch_first=True)
    x = torch.randn(B, S, In)
    params = [p.detach().clone() for p in ref.parameters()]
    ops.LSTM_FUSED = 0
    try:
        with torch.no_grad():
            y0 = ops.lstm(x.cuda(), [p.cuda() for p in params])
        ops.LSTM_FUSED = 1
        with torch.no_grad():
            for _ in range(8):
                y1 = ops.lstm(x.cuda(), [p.cuda() for p in params])
                assert torch.equal(y0, y1), (y0 != y1).nonzero()[:4]
    finally:
        ops.LSTM_FUSED = 1
    inp, out = str(tmp_path / "in.npz"), str(tmp_path / "out.npy")
    np.savez(inp, x=x.numpy(), **{f"p{i}": p.numpy() for i, p in enumerate(params)})
    pkg = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "vae-teb_amd")
    code = _HANDOFF_SCRIPT.format(pkg=pkg, inp=inp, out=out)
    subprocess.run([sys.executable, "-c", code], check=True, timeout=120)
    assert np.array_equal(np.load(out), y0.cpu().numpy())


@pytest.mark.parametrize("native", [False, True])
def test_head_weight_grads_deferred_bitwise(golden, monkeypatch, native):
    """VAETEB_HEAD_DW_DEFER: the bf16-MFMA heads' weight gradients enqueued at the end of the
    backward (an autograd-engine callback) instead of between the decoder's data-gradient
    kernels == in line, bit for bit (eager steps, and the captured step on the native
    executor, where the heads have no side stream)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from golden_util import det_fill_
    from vaeteb import ops
    from vaeteb.model import SeqVaeTeb
    from vaeteb.train import Trainer
    g = golden("model_s16_b4")
    T = lambda k: torch.from_numpy(g[k]).cuda()
    b0 = {"fhr_st": T("y_st"), "fhr_ph": T("y_ph"), "fhr_up_ph": T("x_ph"), "fhr": T("y_raw")}
    b1 = {k: v.flip(0).contiguous() for k, v in b0.items()}
    eps0 = T("eps")
    eps1 = eps0.flip(0).contiguous()
    res = []
    for defer in (False, True):
        monkeypatch.setattr(ops, "HEAD_DW_DEFER", defer)
        m = det_fill_(SeqVaeTeb(sequence_length=16, concurrent_encoders=True, head_precision="bf16",
                                conv_precision="bf16", mlp_precision="bf16")).cuda()
        tr = Trainer(m, lr=1e-3)
        if native:
            tr.capture(b0, eps=eps0, warmup=2, native=True)
            outs = [tr.replay(b, eps=e)["total_loss"].item() for b, e in ((b1, eps1), (b0, eps0))]
        else:
            outs = [tr.step(b, eps=e)["total_loss"].item() for b, e in ((b0, eps0), (b1, eps1), (b0, eps0))]
        torch.cuda.synchronize()
        assert not ops._DEFERRED
        res.append((outs, tr.state.p.clone(), tr.state.g.clone()))
    assert res[0][0] == res[1][0]
    for a, b in zip(res[0][1:], res[1][1:]):
        assert torch.equal(a, b)


@pytest.mark.parametrize("native", [False, True])
def test_first_writer_head_gradients_bitwise(monkeypatch, native):
    """FlatState.first_writer (Trainer steps): the four R x R decoder-head weights (+ biases) are
    not zeroed by zero_grad and their weight-gradient kernel overwrites instead of accumulating
    == zeroing everything, bit for bit: losses, parameters, moments and the last step's
    gradients (S = 256: R = 4096, the bench's heads; eager steps and the native replay)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from golden_util import det_fill_, traj_inputs
    from vaeteb import ops, train
    from vaeteb.model import SeqVaeTeb
    from vaeteb.train import Trainer
    res = []
    for fw in (False, True):
        monkeypatch.setattr(train, "FIRST_WRITER", fw)
        m = det_fill_(SeqVaeTeb(sequence_length=256, concurrent_encoders=True, head_precision="bf16",
                                conv_precision="bf16", mlp_precision="bf16", lstm_precision="16-mixed")).cuda()
        tr = Trainer(m, lr=1e-3)
        assert len(tr.state.first_writer) == 4
        batches = []
        for t in range(3):
            y_st, y_ph, x_ph, y_raw, eps = [torch.from_numpy(a).cuda() for a in traj_inputs(256, 2, t)]
            batches.append(({"fhr_st": y_st, "fhr_ph": y_ph, "fhr_up_ph": x_ph, "fhr": y_raw}, eps))
        if native:
            tr.capture(batches[0][0], eps=batches[0][1], warmup=1, native=True)
            outs = [tr.replay(b, eps=e)["total_loss"].item() for b, e in batches[1:]]
        else:
            outs = [tr.step(b, eps=e)["total_loss"].item() for b, e in batches]
        torch.cuda.synchronize()
        assert not ops.FIRST_WRITER
        res.append((outs, tr.state.p.clone(), tr.state.m.clone(), tr.state.v.clone(), tr.state.g.clone()))
    assert res[0][0] == res[1][0]
    for a, b in zip(res[0][1:], res[1][1:]):
        assert torch.equal(a, b)
