"""Two-launch conv-block backward (csrc/conv_bwd16.hip): vt_batchnorm_bwd_x16 (the
BatchNorm input gradient written once in bf16, rows of ceil32(C)) + vt_conv1d_bwd_dx16
(backward-data on that operand, the x2-upsample fold applied inside the conv) +
vt_conv1d_bwd_weight_bf16_dy16s must equal the fused-staging path it replaces —
vt_batchnorm_bwd_coef + vt_conv1d_bwd_gpad_bf16_bn + vt_conv1d_fold +
vt_conv1d_bwd_weight_bf16_dy16 — bit for bit (same element function, same MFMA
accumulation order, the fold's arithmetic in the fold's order).  That path is itself
pinned to the unfused kernels (test_gpu_conv_bf16.py) and, through them, to torch
(ref/model/vae_teb_model.py:128-253).
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

GEOS = [  # B, L_in, Cin, Cout, K, mode, up — the model's blocks and ragged / edge tilings
    (4, 64, 16, 16, 5, 0, 0), (3, 70, 32, 32, 7, 0, 0), (2, 256, 32, 32, 3, 0, 0),
    (2, 256, 87, 77, 11, 1, 0), (3, 256, 77, 66, 9, 1, 1), (2, 512, 66, 55, 7, 1, 1), (2, 1024, 55, 44, 5, 1, 0),
    (2, 1024, 44, 33, 5, 1, 1), (2, 2048, 33, 22, 3, 1, 1), (2, 4096, 22, 11, 3, 1, 0), (2, 4096, 11, 1, 3, 1, 0),
    (2, 62, 77, 66, 9, 1, 1), (2, 61, 77, 66, 9, 1, 1), (3, 30, 77, 66, 9, 1, 1), (2, 3, 20, 13, 9, 1, 1),
    (2, 37, 44, 33, 5, 1, 1), (2, 100, 33, 22, 3, 1, 1), (2, 6, 9, 7, 11, 1, 0), (1, 7, 16, 16, 7, 0, 0),
    (2, 40, 120, 100, 3, 1, 1),
]


@pytest.fixture(scope="module")
def L():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from vaeteb import _lib
    return _lib


def _shadow(L, w):
    Cout, Cin, K = w.shape
    up = lambda n: (n + 31) // 32 * 32
    w16 = torch.empty(Cout * K * up(Cin), dtype=torch.bfloat16, device="cuda")
    w16t = torch.empty(Cin * K * up(Cout), dtype=torch.bfloat16, device="cuda")
    L.call("vt_conv1d_bf16_shadow", L.ptr(w), Cout, Cin, K, L.ptr(w16), L.ptr(w16t), L.stream())
    return w16, w16t


@pytest.mark.parametrize("geo", GEOS)
@pytest.mark.parametrize("act", [1, 3])
def test_bwd16_bitwise_vs_fused_staging(L, geo, act):
    B, Lin, Cin, Cout, K, mode, up = geo
    Lo = L.lib().fns["vt_conv1d_out_len"](Lin, K, mode, up)
    M = B * Lo
    pad = K - 1 if mode == 0 else (K - 1) // 2
    torch.manual_seed(sum(geo) + 11 * act)
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
    bnp = torch.empty(6 * Cout, device="cuda")
    dg, db = torch.empty(Cout, device="cuda"), torch.empty(Cout, device="cuda")
    L.call("vt_batchnorm_bwd_coef", L.ptr(gy), L.ptr(conv), M, Cout, L.ptr(mean), L.ptr(rstd), L.ptr(gam),
           L.ptr(bet), act, L.ptr(dg), L.ptr(db), 0, L.ptr(bnp), L.ptr(ws), ws.numel(), L.stream())
    # fused staging (reference path)
    cp = (Cout + 7) // 8 * 8
    d0 = torch.full((M, cp), float("nan"), dtype=torch.bfloat16, device="cuda")
    gp = torch.empty(B, Lo + K - 1, Cin, device="cuda")
    L.call("vt_conv1d_bwd_gpad_bf16_bn", L.ptr(gy), L.ptr(conv), L.ptr(bnp), act, M, B, Lin, Cin, L.ptr(w16t), Cout,
           K, mode, up, L.ptr(gp), L.ptr(d0), L.stream())
    dx0 = torch.empty(B, Lin, Cin, device="cuda")
    L.call("vt_conv1d_fold", L.ptr(gp), B, Lin, Cin, Cout, K, mode, up, L.ptr(dx0), 0, L.stream())
    dw0 = torch.empty(Cout, Cin, K, device="cuda")
    L.call("vt_conv1d_bwd_weight_bf16_dy16", L.ptr(d0), L.ptr(x), B, Lin, Cin, Cout, K, mode, up, L.ptr(dw0), 0,
           L.ptr(wsw), wsw.numel(), L.stream())
    # two-launch path
    c32 = (Cout + 31) // 32 * 32
    d1 = torch.full((M, c32), float("nan"), dtype=torch.bfloat16, device="cuda")
    L.call("vt_batchnorm_bwd_x16", L.ptr(gy), L.ptr(conv), L.ptr(bnp), act, M, Cout, L.ptr(d1), L.stream())
    dw1 = torch.empty_like(dw0)
    L.call("vt_conv1d_bwd_weight_bf16_dy16s", L.ptr(d1), c32, L.ptr(x), B, Lin, Cin, Cout, K, mode, up, L.ptr(dw1), 0,
           L.ptr(wsw), wsw.numel(), L.stream())
    torch.cuda.synchronize()
    assert torch.equal(d1[:, :Cout], d0[:, :Cout])
    assert (d1[:, Cout:] == 0).all()
    assert torch.equal(dw0, dw1)
    supported = (mode == 1 and Lin * (2 if up else 1) > pad) or (mode == 0 and not up)
    dx1 = torch.full((B, Lin, Cin), float("nan"), device="cuda")
    edge = torch.full((max(B * 2 * pad * Cin, 1),), float("nan"), device="cuda")
    if not supported:
        with pytest.raises(ValueError):
            L.call("vt_conv1d_bwd_dx16", L.ptr(d1), B, Lin, Cin, L.ptr(w16t), Cout, K, mode, up, L.ptr(dx1),
                   L.ptr(edge), L.stream())
        return
    L.call("vt_conv1d_bwd_dx16", L.ptr(d1), B, Lin, Cin, L.ptr(w16t), Cout, K, mode, up, L.ptr(dx1), L.ptr(edge),
           L.stream())
    torch.cuda.synchronize()
    assert torch.equal(dx0, dx1), ((dx0 != dx1).sum().item(), dx0.numel(), (dx0 - dx1).abs().max().item())


def test_bwd16_block_matches_fused_in_autograd(L):
    """ConvBlock backward through ops.ConvBNActF with the two-launch path (default) and with
    VAETEB_CONV_BWD16=0 (fused staging): identical input and parameter gradients."""
    from vaeteb import ops
    from vaeteb.model import ConvBlock
    torch.manual_seed(3)
    for (a, b, k, causal, u, L_) in [(77, 66, 9, False, True, 256), (87, 77, 11, False, False, 256),
                                     (16, 16, 5, True, False, 256)]:
        blk = ConvBlock(a, b, k, causal=causal, up=u).cuda()
        blk.bf16 = True
        x = torch.randn(4, L_, a, device="cuda", requires_grad=True)
        gy = torch.randn(4, L_ * (2 if u else 1), b, device="cuda")
        res = []
        for flag in (1, 0):
            ops.CONV_BWD16 = flag
            try:
                x.grad = None
                for p in blk.parameters():
                    p.grad = None
                blk(x).backward(gy)
                torch.cuda.synchronize()
                res.append([x.grad.clone()] + [p.grad.clone() for p in blk.parameters()])
            finally:
                ops.CONV_BWD16 = 1
        for t0, t1 in zip(*res):
            assert torch.equal(t0, t1)


FWD_GEOS = GEOS + [(2, 5, 33, 22, 3, 1, 1), (2, 2, 20, 13, 9, 1, 0), (3, 1, 8, 8, 3, 1, 0), (2, 9, 16, 16, 11, 0, 0),
                   (2, 300, 1, 16, 3, 0, 0), (2, 40, 130, 100, 5, 1, 1), (2, 257, 87, 77, 1, 1, 0)]


@pytest.mark.parametrize("geo", FWD_GEOS)
def test_flat_staged_forward_bitwise(L, geo):
    """vt_conv_bf16_set_kernels: the flat-staged forward (conv_fwd16.hip, default) and
    k_conv_bf16 give the same conv output, BatchNorm statistics and running statistics,
    bit for bit (same tiles, accumulation order and interpolation arithmetic)."""
    B, Lin, Cin, Cout, K, mode, up = geo
    Lo = L.lib().fns["vt_conv1d_out_len"](Lin, K, mode, up)
    torch.manual_seed(5 * sum(geo))
    x = torch.randn(B, Lin, Cin, device="cuda")
    w = torch.randn(Cout, Cin, K, device="cuda") / (Cin * K) ** 0.5
    w16, _ = _shadow(L, w)
    gam = 1 + 0.1 * torch.randn(Cout, device="cuda")
    bet = 0.1 * torch.randn(Cout, device="cuda")
    ws = torch.empty(1 << 22, device="cuda")
    outs = []
    try:
        for flags in (0, 7):
            L.call("vt_conv_bf16_set_kernels", flags)
            conv = torch.full((B, Lo, Cout), float("nan"), device="cuda")
            y = torch.full_like(conv, float("nan"))
            mean, rstd = torch.empty(Cout, device="cuda"), torch.empty(Cout, device="cuda")
            rm, rv = torch.zeros(Cout, device="cuda"), torch.ones(Cout, device="cuda")
            L.call("vt_conv1d_bn_fwd_bf16", L.ptr(x), B, Lin, Cin, L.ptr(w16), Cout, K, mode, up, L.ptr(gam),
                   L.ptr(bet), 1, 1e-5, 0.9, L.ptr(conv), L.ptr(y), L.ptr(mean), L.ptr(rstd), L.ptr(rm), L.ptr(rv),
                   L.ptr(ws), ws.numel(), L.stream())
            y2 = torch.full_like(conv, float("nan"))
            L.call("vt_conv1d_fwd_bf16", L.ptr(x), B, Lin, Cin, L.ptr(w16), Cout, K, mode, up, L.ptr(y2), L.stream())
            torch.cuda.synchronize()
            outs.append((conv, y, mean, rstd, rm, rv, y2))
    finally:
        L.call("vt_conv_bf16_set_kernels", 11)
    for a, b in zip(*outs):
        assert torch.equal(a, b), ((a != b).sum().item(), a.numel())


@pytest.mark.parametrize("geo", [g for g in FWD_GEOS if g[2] <= 128 and g[3] <= 128] +
                         [(8, 2048, 33, 22, 3, 1, 1), (8, 4096, 22, 11, 3, 1, 0), (8, 4096, 11, 1, 3, 1, 0),
                          (16, 256, 16, 16, 7, 0, 0), (16, 256, 32, 32, 3, 0, 0), (4, 1000, 20, 30, 5, 1, 1)])
def test_flat_staged_weight_grad_bitwise(L, geo):
    """vt_conv_bf16_set_kernels bit 1: the flat-staged, prefetching weight gradient
    (k_cdw16, default) and k_conv_dw_bf16 on the same bf16 dY rows give the same dW bit for
    bit (same splits, chunks, pairs and MFMA order; the window's values by up_lerp)."""
    B, Lin, Cin, Cout, K, mode, up = geo
    Lo = L.lib().fns["vt_conv1d_out_len"](Lin, K, mode, up)
    M = B * Lo
    torch.manual_seed(9 * sum(geo))
    x = torch.randn(B, Lin, Cin, device="cuda")
    c32 = (Cout + 31) // 32 * 32
    d16 = torch.zeros(M, c32, dtype=torch.bfloat16, device="cuda")
    d16[:, :Cout] = torch.randn(M, Cout, device="cuda").bfloat16()
    wsw = torch.empty(8 << 20, device="cuda")
    outs = []
    try:
        for flags in (0, 7, 11, 15):
            L.call("vt_conv_bf16_set_kernels", flags)
            dw = torch.full((Cout, Cin, K), float("nan"), device="cuda")
            L.call("vt_conv1d_bwd_weight_bf16_dy16s", L.ptr(d16), c32, L.ptr(x), B, Lin, Cin, Cout, K, mode, up,
                   L.ptr(dw), 0, L.ptr(wsw), wsw.numel(), L.stream())
            torch.cuda.synchronize()
            outs.append(dw)
    finally:
        L.call("vt_conv_bf16_set_kernels", 11)
    for o in outs[1:]:
        assert torch.equal(outs[0], o), ((outs[0] != o).sum().item(), o.numel())
