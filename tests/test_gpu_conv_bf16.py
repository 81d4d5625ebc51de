"""bf16-MFMA conv kernels (csrc/conv_bf16.hip) — the 16-bit-autocast precision
of the reference's training (ref/model/graph_model.py:510, :709-711).

Per geometry of SeqVaeTeb's conv blocks (causal encoder blocks, reflect /
replicate decoder blocks with and without the x2 upsample):
  * exact: small-integer activations and weights are exact in bf16 and their
    sums exact in fp32, so forward and backward-data must equal the exact-fp32
    kernels (conv.hip, themselves checked against torch in test_gpu_model.py)
    bit for bit — this pins fragment maps, tap order / flip, padding, upsample;
  * bf16 model: random operands vs the fp32 kernels run on the bf16-ROUNDED
    operands: rel-L2 <= 1e-5 (accumulation order only);
  * vs fp32: rel-L2 <= 1e-2 (bf16 has an 8-bit mantissa: ~3e-3 expected);
  * model: a full SeqVaeTeb step with bf16 convs stays within 1e-2 of fp32.
The exact / rounded-model / weight-gradient cases also run with the fp16 operand format
(round 6, csrc/h16.h: the same kernels instantiated for _Float16, the model rounding to fp16).
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

GEOS = [  # B, L, Cin, Cout, K, mode, up
    (4, 64, 16, 16, 5, 0, 0), (3, 70, 32, 32, 7, 0, 0), (2, 40, 87, 77, 11, 1, 0), (2, 48, 77, 66, 9, 1, 1),
    (2, 100, 33, 22, 3, 1, 1), (2, 300, 11, 1, 3, 1, 0), (3, 3, 20, 13, 9, 1, 0), (2, 64, 44, 33, 5, 1, 1),
]


@pytest.fixture(scope="module")
def L():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from vaeteb import _lib
    return _lib


def _rel(a, b):
    return ((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30)).item()


FMTS = ["bf16", "fp16"]
DT = {"bf16": torch.bfloat16, "fp16": torch.float16}


def _fmt(L, fmt):
    L.set_h16(fmt == "fp16")
    return lambda t: t.to(DT[fmt]).float()


def _shadow(L, w):
    Cout, Cin, K = w.shape
    up = lambda n: (n + 31) // 32 * 32
    dt = torch.float16 if L.h16() == "fp16" else torch.bfloat16
    w16 = torch.empty(Cout * K * up(Cin), dtype=dt, device="cuda")
    w16t = torch.empty(Cin * K * up(Cout), dtype=dt, device="cuda")
    L.call("vt_conv1d_bf16_shadow", L.ptr(w), Cout, Cin, K, L.ptr(w16), L.ptr(w16t), L.stream())
    return w16, w16t


def _run(L, x, w, mode, up, dy):
    B, Lin, Cin = x.shape
    Cout, _, K = w.shape
    Lo = L.lib().fns["vt_conv1d_out_len"](Lin, K, mode, up)
    y32, y16 = (torch.empty(B, Lo, Cout, device="cuda") for _ in range(2))
    L.call("vt_conv1d_direct_fwd", L.ptr(x), B, Lin, Cin, L.ptr(w), Cout, K, mode, up, L.ptr(y32), L.stream())
    w16, w16t = _shadow(L, w)
    L.call("vt_conv1d_fwd_bf16", L.ptr(x), B, Lin, Cin, L.ptr(w16), Cout, K, mode, up, L.ptr(y16), L.stream())
    g32, g16 = (torch.empty(B, Lo + K - 1, Cin, device="cuda") for _ in range(2))
    L.call("vt_conv1d_direct_bwd_gpad", L.ptr(dy), B, Lin, Cin, L.ptr(w), Cout, K, mode, up, L.ptr(g32), L.stream())
    L.call("vt_conv1d_bwd_gpad_bf16", L.ptr(dy), B, Lin, Cin, L.ptr(w16t), Cout, K, mode, up, L.ptr(g16),
           L.stream())
    return y32, y16, g32, g16


def _ints(shape, seed, lo=-3, hi=4):
    g = torch.Generator().manual_seed(seed)
    return torch.randint(lo, hi, shape, generator=g).float().cuda()


@pytest.mark.parametrize("fmt", FMTS)
@pytest.mark.parametrize("geo", GEOS)
def test_conv_bf16_exact_integer(L, geo, fmt):
    _fmt(L, fmt)
    B, Lin, Cin, Cout, K, mode, up = geo
    Lo = L.lib().fns["vt_conv1d_out_len"](Lin, K, mode, up)
    # even integers keep the x2 upsample's 1/4, 3/4 weights exact in bf16
    x = _ints((B, Lin, Cin), 1) * 4
    w = _ints((Cout, Cin, K), 2)
    dy = _ints((B, Lo, Cout), 3)
    y32, y16, g32, g16 = _run(L, x, w, mode, up, dy)
    assert torch.equal(y16, y32)
    assert torch.equal(g16, g32)


@pytest.mark.parametrize("fmt", FMTS)
@pytest.mark.parametrize("geo", GEOS)
def test_conv_bf16_random(L, geo, fmt):
    rb = _fmt(L, fmt)
    B, Lin, Cin, Cout, K, mode, up = geo
    Lo = L.lib().fns["vt_conv1d_out_len"](Lin, K, mode, up)
    torch.manual_seed(sum(geo))
    x = torch.randn(B, Lin, Cin, device="cuda")
    w = torch.randn(Cout, Cin, K, device="cuda") / (Cin * K) ** 0.5
    dy = torch.randn(B, Lo, Cout, device="cuda")
    y32, y16, g32, g16 = _run(L, x, w, mode, up, dy)
    assert _rel(y16, y32) < 1e-2 and _rel(g16, g32) < 1e-2
    # the bf16 model: fp32 kernels on bf16-rounded operands (the forward rounds
    # the upsampled / padded window values, so round x before a non-upsampling conv only)
    if not up:
        y32b, _, _, _ = _run(L, rb(x), rb(w), mode, up, rb(dy))
        assert _rel(y16, y32b) < 1e-5
    _, _, g32b, _ = _run(L, x, rb(w), mode, up, rb(dy))
    assert _rel(g16, g32b) < 1e-5


def _dw(L, fn, dy, x, mode, up, Cout, K):
    B, Lin, Cin = x.shape
    dw = torch.empty(Cout, Cin, K, device="cuda")
    ws = torch.empty(1 << 24, device="cuda")
    L.call(fn, L.ptr(dy), L.ptr(x), B, Lin, Cin, Cout, K, mode, up, L.ptr(dw), 0, L.ptr(ws), ws.numel(), L.stream())
    return dw


@pytest.mark.parametrize("fmt", FMTS)
@pytest.mark.parametrize("geo", GEOS)
def test_conv_bf16_weight_grad(L, geo, fmt):
    """dW on bf16 MFMA (transposed LDS reads): exact on small integers, bf16
    model 1e-5, vs fp32 1e-2."""
    rb = _fmt(L, fmt)
    B, Lin, Cin, Cout, K, mode, up = geo
    Lo = L.lib().fns["vt_conv1d_out_len"](Lin, K, mode, up)
    x, dy = _ints((B, Lin, Cin), 4) * 4, _ints((B, Lo, Cout), 5)
    assert torch.equal(_dw(L, "vt_conv1d_bwd_weight_bf16", dy, x, mode, up, Cout, K),
                       _dw(L, "vt_conv1d_direct_bwd_weight", dy, x, mode, up, Cout, K))
    torch.manual_seed(sum(geo) + 1)
    x, dy = torch.randn(B, Lin, Cin, device="cuda"), torch.randn(B, Lo, Cout, device="cuda")
    d16 = _dw(L, "vt_conv1d_bwd_weight_bf16", dy, x, mode, up, Cout, K)
    assert _rel(d16, _dw(L, "vt_conv1d_direct_bwd_weight", dy, x, mode, up, Cout, K)) < 1e-2
    if not up:
        assert _rel(d16, _dw(L, "vt_conv1d_direct_bwd_weight", rb(dy), rb(x), mode, up, Cout, K)) < 1e-5


def test_model_bf16_convs_close_to_fp32(golden):
    """Full SeqVaeTeb training step (S = 16, reference golden weights/inputs):
    bf16 convs vs the exact-fp32 step.  The ELBO parts agree within 1e-2.
    Gradients: this small-batch model is rounding-sensitive (deep LayerNorm /
    ReLU chains, BatchNorm over B*L = 64 rows: fp32 summation-order changes
    alone move encoder gradients by 2e-4, test_gpu_model.py), so the bf16
    gradients are held to the scale of the model's own sensitivity: their
    deviation from the fp32 step (aggregate rel-L2 over the decoder conv stack
    and heads, and over all parameters) must not exceed 3x that of an fp32 step
    whose inputs carry a 4e-3 relative perturbation (bf16's rounding step)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from golden_util import det_fill_
    from vaeteb.model import SeqVaeTeb
    g = golden("model_s16_b4")
    batch = {k: torch.from_numpy(g[k]).cuda() for k in ("y_st", "y_ph", "x_ph", "y_raw")}
    eps = torch.from_numpy(g["eps"]).cuda()
    gen = torch.Generator(device="cuda").manual_seed(7)
    pert = {k: v * (1 + 4e-3 * torch.randn(v.shape, device="cuda", generator=gen)) if k != "y_raw" else v
            for k, v in batch.items()}
    res = {}
    for name, prec, b in (("fp32", "fp32", batch), ("bf16", "bf16", batch), ("pert", "fp32", pert)):
        m = det_fill_(SeqVaeTeb(sequence_length=16)).cuda()
        m.set_conv_precision(prec)
        out = m(b["y_st"], b["y_ph"], b["x_ph"], eps=eps)
        loss = m.compute_loss(out, b["y_st"], b["y_ph"], b["y_raw"], beta=float(g["beta"]))
        loss["total_loss"].backward()
        res[name] = (loss, {n: p.grad.detach().double().clone() for n, p in m.named_parameters()})
    for k in ("total_loss", "nll_loss", "mse_loss", "kld_loss"):
        a, b = res["bf16"][0][k].item(), res["fp32"][0][k].item()
        assert abs(a - b) <= 1e-2 * abs(b), (k, a, b)

    def dev(name, prefix):
        ref = res["fp32"][1]
        num = sum((res[name][1][n] - v).norm() ** 2 for n, v in ref.items() if n.startswith(prefix))
        den = sum(v.norm() ** 2 for n, v in ref.items() if n.startswith(prefix))
        return (num / den).sqrt().item()
    for prefix in (("decoder.conv.", "decoder.output_"), ""):
        assert dev("bf16", prefix) <= 3 * dev("pert", prefix) + 1e-3, (prefix, dev("bf16", prefix),
                                                                         dev("pert", prefix))


@pytest.mark.parametrize("geo", GEOS)
@pytest.mark.parametrize("act", [1, 3])
def test_fused_batchnorm_backward_bitwise(L, geo, act):
    """vt_batchnorm_bwd_coef + vt_conv1d_bwd_gpad_bf16_bn (the BN input gradient formed
    while the backward-data conv stages its operand, also left in bf16) +
    vt_conv1d_bwd_weight_bf16_dy16 == vt_batchnorm_bwd's materialised dx fed to the
    unfused bf16 kernels, bit for bit; dgamma / dbeta equal."""
    B, Lin, Cin, Cout, K, mode, up = geo
    Lo = L.lib().fns["vt_conv1d_out_len"](Lin, K, mode, up)
    M = B * Lo
    torch.manual_seed(sum(geo) + act)
    x = torch.randn(B, Lin, Cin, device="cuda")
    w = torch.randn(Cout, Cin, K, device="cuda") / (Cin * K) ** 0.5
    conv = torch.randn(B, Lo, Cout, device="cuda") * 2 + 0.3
    gy = torch.randn(B, Lo, Cout, device="cuda")
    mean = conv.reshape(-1, Cout).mean(0)
    rstd = 1 / (conv.reshape(-1, Cout).var(0, unbiased=False) + 1e-5).sqrt()
    gam = 1 + 0.1 * torch.randn(Cout, device="cuda")
    bet = 0.1 * torch.randn(Cout, device="cuda")
    _, w16t = _shadow(L, w)
    ws = torch.empty(4096 * Cout + 2 * Cout, device="cuda")
    wsw = torch.empty(8 << 20, device="cuda")
    # unfused reference
    dx = torch.empty_like(conv)
    dg0, db0 = torch.empty(Cout, device="cuda"), torch.empty(Cout, device="cuda")
    L.call("vt_batchnorm_bwd", L.ptr(gy), L.ptr(conv), M, Cout, L.ptr(mean), L.ptr(rstd), L.ptr(gam), L.ptr(bet), act,
           L.ptr(dx), L.ptr(dg0), L.ptr(db0), 0, L.ptr(ws), ws.numel(), L.stream())
    gp0 = torch.empty(B, Lo + K - 1, Cin, device="cuda")
    L.call("vt_conv1d_bwd_gpad_bf16", L.ptr(dx), B, Lin, Cin, L.ptr(w16t), Cout, K, mode, up, L.ptr(gp0), L.stream())
    dw0 = torch.empty(Cout, Cin, K, device="cuda")
    L.call("vt_conv1d_bwd_weight_bf16", L.ptr(dx), L.ptr(x), B, Lin, Cin, Cout, K, mode, up, L.ptr(dw0), 0,
           L.ptr(wsw), wsw.numel(), L.stream())
    # fused
    bnp = torch.empty(6 * Cout, device="cuda")
    dg1, db1 = torch.empty(Cout, device="cuda"), torch.empty(Cout, device="cuda")
    L.call("vt_batchnorm_bwd_coef", L.ptr(gy), L.ptr(conv), M, Cout, L.ptr(mean), L.ptr(rstd), L.ptr(gam),
           L.ptr(bet), act, L.ptr(dg1), L.ptr(db1), 0, L.ptr(bnp), L.ptr(ws), ws.numel(), L.stream())
    gp1 = torch.empty_like(gp0)
    cp = (Cout + 7) // 8 * 8
    dxbn = torch.full((M, cp), float("nan"), dtype=torch.bfloat16, device="cuda")
    L.call("vt_conv1d_bwd_gpad_bf16_bn", L.ptr(gy), L.ptr(conv), L.ptr(bnp), act, M, B, Lin, Cin, L.ptr(w16t), Cout,
           K, mode, up, L.ptr(gp1), L.ptr(dxbn), L.stream())
    dw1 = torch.empty_like(dw0)
    L.call("vt_conv1d_bwd_weight_bf16_dy16", L.ptr(dxbn), L.ptr(x), B, Lin, Cin, Cout, K, mode, up, L.ptr(dw1), 0,
           L.ptr(wsw), wsw.numel(), L.stream())
    torch.cuda.synchronize()
    # the bf16 side output is dx rounded to bf16, zero in the channel padding, every row written
    assert torch.equal(dxbn[:, :Cout].float(), dx.reshape(M, Cout).bfloat16().float())
    assert (dxbn[:, Cout:] == 0).all()
    assert torch.equal(dg0, dg1) and torch.equal(db0, db1)
    assert torch.equal(gp0, gp1), ((gp0 != gp1).sum().item(), gp0.numel(), (gp0 - gp1).abs().max().item(),
                                   gp0.abs().max().item(), (dw0 != dw1).sum().item())
    assert torch.equal(dw0, dw1)


@pytest.mark.parametrize("geo", [(2, 40, 20, 17, 5, 0, 0), (3, 33, 33, 22, 3, 1, 0), (2, 256, 87, 77, 11, 1, 0),
                                 (2, 6, 9, 7, 11, 1, 0), (2, 3, 5, 6, 5, 1, 0), (2, 1024, 55, 44, 5, 1, 0),
                                 (1, 7, 16, 16, 7, 0, 0)])
def test_backward_data_direct_dx_bitwise(L, geo):
    """vt_conv1d_bwd_dx_bf16_bn (dX written by the conv, reflect edges added back)
    == vt_conv1d_bwd_gpad_bf16_bn + vt_conv1d_fold, bit for bit; dxbn equal."""
    B, Lin, Cin, Cout, K, mode, up = geo
    pad = K - 1 if mode == 0 else (K - 1) // 2
    if mode == 1 and Lin <= pad:
        with pytest.raises(ValueError):
            L.call("vt_conv1d_bwd_dx_bf16_bn", None, None, None, 1, 1, B, Lin, Cin, None, Cout, K, mode, up, None,
                   None, None, L.stream())
        return
    Lo = L.lib().fns["vt_conv1d_out_len"](Lin, K, mode, up)
    M = B * Lo
    torch.manual_seed(sum(geo))
    w = torch.randn(Cout, Cin, K, device="cuda") / (Cin * K) ** 0.5
    conv = torch.randn(B, Lo, Cout, device="cuda") * 2 + 0.3
    gy = torch.randn(B, Lo, Cout, device="cuda")
    bnp = torch.cat([conv.reshape(-1, Cout).mean(0), 1 / (conv.reshape(-1, Cout).var(0) + 1e-5).sqrt(),
                     1 + 0.1 * torch.randn(Cout, device="cuda"), 0.1 * torch.randn(Cout, device="cuda"),
                     torch.randn(Cout, device="cuda"), torch.randn(Cout, device="cuda")]).contiguous()
    _, w16t = _shadow(L, w)
    cp = (Cout + 7) // 8 * 8
    gp = torch.empty(B, Lo + K - 1, Cin, device="cuda")
    d0 = torch.full((M, cp), float("nan"), dtype=torch.bfloat16, device="cuda")
    L.call("vt_conv1d_bwd_gpad_bf16_bn", L.ptr(gy), L.ptr(conv), L.ptr(bnp), 1, M, B, Lin, Cin, L.ptr(w16t), Cout,
           K, mode, up, L.ptr(gp), L.ptr(d0), L.stream())
    dx0 = torch.empty(B, Lin, Cin, device="cuda")
    L.call("vt_conv1d_fold", L.ptr(gp), B, Lin, Cin, Cout, K, mode, up, L.ptr(dx0), 0, L.stream())
    dx1 = torch.full((B, Lin, Cin), float("nan"), device="cuda")
    edge = torch.full((max(B * 2 * pad * Cin, 1),), float("nan"), device="cuda")
    d1 = torch.full((M, cp), float("nan"), dtype=torch.bfloat16, device="cuda")
    L.call("vt_conv1d_bwd_dx_bf16_bn", L.ptr(gy), L.ptr(conv), L.ptr(bnp), 1, M, B, Lin, Cin, L.ptr(w16t), Cout, K,
           mode, up, L.ptr(dx1), L.ptr(edge), L.ptr(d1), L.stream())
    torch.cuda.synchronize()
    assert torch.equal(dx0, dx1), ((dx0 != dx1).sum().item(), dx0.numel())
    assert torch.equal(d0, d1)


@pytest.mark.parametrize("geo", GEOS)
def test_window_staging_channel_lanes_bitwise(L, geo):
    """vt_conv_bf16_set_staging: the channel-lane window staging (default) and the
    octet staging give the same bits — forward, backward-data with the fused
    BatchNorm backward, and its bf16 side output."""
    B, Lin, Cin, Cout, K, mode, up = geo
    Lo = L.lib().fns["vt_conv1d_out_len"](Lin, K, mode, up)
    M = B * Lo
    torch.manual_seed(7 * sum(geo))
    x = torch.randn(B, Lin, Cin, device="cuda")
    w = torch.randn(Cout, Cin, K, device="cuda") / (Cin * K) ** 0.5
    conv = torch.randn(B, Lo, Cout, device="cuda") * 2 + 0.3
    gy = torch.randn(B, Lo, Cout, device="cuda")
    bnp = torch.cat([conv.reshape(-1, Cout).mean(0), 1 / (conv.reshape(-1, Cout).var(0) + 1e-5).sqrt(),
                     1 + 0.1 * torch.randn(Cout, device="cuda"), 0.1 * torch.randn(Cout, device="cuda"),
                     torch.randn(Cout, device="cuda"), torch.randn(Cout, device="cuda")]).contiguous()
    w16, w16t = _shadow(L, w)
    cp = (Cout + 7) // 8 * 8
    outs = []
    try:
        for cl in (0, 2):
            L.call("vt_conv_bf16_set_staging", cl)
            y = torch.full((B, Lo, Cout), float("nan"), device="cuda")
            L.call("vt_conv1d_fwd_bf16", L.ptr(x), B, Lin, Cin, L.ptr(w16), Cout, K, mode, up, L.ptr(y), L.stream())
            gp = torch.full((B, Lo + K - 1, Cin), float("nan"), device="cuda")
            d = torch.full((M, cp), float("nan"), dtype=torch.bfloat16, device="cuda")
            L.call("vt_conv1d_bwd_gpad_bf16_bn", L.ptr(gy), L.ptr(conv), L.ptr(bnp), 3, M, B, Lin, Cin, L.ptr(w16t),
                   Cout, K, mode, up, L.ptr(gp), L.ptr(d), L.stream())
            torch.cuda.synchronize()
            outs.append((y, gp, d))
    finally:
        L.call("vt_conv_bf16_set_staging", 1)
    for a, b in zip(*outs):
        assert torch.equal(a, b), ((a != b).sum().item(), a.numel())
