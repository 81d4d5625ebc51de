"""bf16 MFMA GEMMs of the decoder heads (vt_mfma_linear_*, csrc/mfma.hip).

Three checks per entry point:
  * exact: small-integer operands are exact in bf16 and their products/sums
    exact in fp32, so the kernel must match an fp64 matmul bit for bit — this
    pins the MFMA operand/accumulator lane maps, the transposed B staging, the
    zero padding and the split-K slab reduction;
  * bf16 model: random operands vs an fp64 matmul of the bf16-ROUNDED operands
    (what the kernel computes up to fp32 accumulation order), rel. 1e-5;
  * vs the fp32 op: rel. error of the bf16 product vs the fp32 one < 1e-2
    (bf16 has an 8-bit mantissa: expected ~3e-3).
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def L():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from vaeteb import _lib
    return _lib


def _ws(L, R, K, N):
    import ctypes
    n = ctypes.c_int64(0)
    rc = L.lib().fns["vt_mfma_workspace_floats"](R, K, N, ctypes.addressof(n))
    assert rc == 0
    return torch.empty(n.value + 64, device="cuda")


def _ints(*shape, lo=-3, hi=4, seed=0):
    g = torch.Generator().manual_seed(seed)
    return torch.randint(lo, hi, shape, generator=g).float().cuda()


def _rel(a, b):
    return ((a.double() - b.double()).norm() / b.double().norm()).item()


def _shadow(L, w):
    N, K = w.shape
    w16 = torch.empty(N, K, dtype=torch.bfloat16, device="cuda")
    w16t = torch.empty(K, N, dtype=torch.bfloat16, device="cuda")
    L.call("vt_mfma_weight_shadow", L.ptr(w), N, K, L.ptr(w16), L.ptr(w16t), L.stream())
    return w16, w16t


def _fwd(L, x, w, b):
    R, K = x.shape
    N = w.shape[0]
    y = torch.empty(R, N, device="cuda")
    ws = _ws(L, R, K, N)
    w16, _ = _shadow(L, w)
    L.call("vt_mfma_linear_fwd", L.ptr(x), R, K, L.ptr(w16), N, L.ptr(b), L.ptr(y), L.ptr(ws), ws.numel(),
           L.stream())
    return y


def _bwd_data(L, gy, w, acc=None):
    R, N = gy.shape
    K = w.shape[1]
    gx = acc.clone() if acc is not None else torch.empty(R, K, device="cuda")
    ws = _ws(L, R, K, N)
    _, w16t = _shadow(L, w)
    L.call("vt_mfma_linear_bwd_data", L.ptr(gy), R, N, L.ptr(w16t), K, L.ptr(gx), int(acc is not None), L.ptr(ws),
           ws.numel(), L.stream())
    return gx


def _bwd_weight(L, gy, x, with_bias=True, acc=None):
    R, N = gy.shape
    K = x.shape[1]
    gw = acc.clone() if acc is not None else torch.empty(N, K, device="cuda")
    gb = torch.empty(N, device="cuda") if with_bias else None
    ws = _ws(L, R, K, N)
    L.call("vt_mfma_linear_bwd_weight", L.ptr(gy), R, N, L.ptr(x), K, L.ptr(gw), L.ptr(gb), int(acc is not None),
           L.ptr(ws), ws.numel(), L.stream())
    return gw, gb


# (R, K, N): the S=16 head (256), a ragged batch, the S=256 head at batch 256
# (4096: split-K 4), and the S=300 reference head (4800: split-K 3); the weight
# gradient takes the direct kernel (k_mfma_dw) when N and K are multiples of 128
# (ragged 37 / 300 rows: masked chunk rows) and the split-K path otherwise
SHAPES = [(64, 256, 256), (7, 128, 192), (256, 4096, 4096), (256, 4800, 4800), (300, 640, 320), (37, 128, 256),
          (300, 384, 640)]


@pytest.mark.parametrize("R,K,N", SHAPES)
def test_mfma_exact_integer(L, R, K, N):
    x, w, b = _ints(R, K, seed=1), _ints(N, K, seed=2), _ints(N, seed=3)
    gy = _ints(R, N, seed=4)
    y = _fwd(L, x, w, b)
    assert torch.equal(y, (x.double() @ w.double().T + b.double()).float())
    gx = _bwd_data(L, gy, w)
    assert torch.equal(gx, (gy.double() @ w.double()).float())
    gw, gb = _bwd_weight(L, gy, x)
    assert torch.equal(gw, (gy.double().T @ x.double()).float())
    assert torch.equal(gb, gy.double().sum(0).float())


@pytest.mark.parametrize("R,K,N", [(32, 128, 64), (100, 256, 128)])
def test_mfma_accumulate(L, R, K, N):
    x, w, gy = _ints(R, K, seed=5), _ints(N, K, seed=6), _ints(R, N, seed=7)
    a0, w0 = _ints(R, K, seed=8), _ints(N, K, seed=9)
    gx = _bwd_data(L, gy, w, acc=a0)
    assert torch.equal(gx, (a0.double() + gy.double() @ w.double()).float())
    gw, _ = _bwd_weight(L, gy, x, with_bias=False, acc=w0)
    assert torch.equal(gw, (w0.double() + gy.double().T @ x.double()).float())


@pytest.mark.parametrize("R,K,N", SHAPES[2:4])
def test_mfma_random_vs_bf16_model_and_fp32(L, R, K, N):
    torch.manual_seed(0)
    x = torch.randn(R, K, device="cuda")
    w = torch.randn(N, K, device="cuda") / K ** 0.5
    b = torch.randn(N, device="cuda")
    gy = torch.randn(R, N, device="cuda")
    bf = lambda t: t.bfloat16().double()
    y = _fwd(L, x, w, b)
    assert _rel(y, bf(x) @ bf(w).T + b.double()) < 1e-5
    assert _rel(y, x.double() @ w.double().T + b.double()) < 1e-2
    gx = _bwd_data(L, gy, w)
    assert _rel(gx, bf(gy) @ bf(w)) < 1e-5
    assert _rel(gx, gy.double() @ w.double()) < 1e-2
    gw, gb = _bwd_weight(L, gy, x)
    assert _rel(gw, bf(gy).T @ bf(x)) < 1e-5
    assert _rel(gw, gy.double().T @ x.double()) < 1e-2
    assert _rel(gb, gy.double().sum(0)) < 1e-6


def test_mfma_shadow_is_bf16_and_transpose(L):
    w = torch.randn(192, 320, device="cuda")
    w16, w16t = _shadow(L, w)
    assert torch.equal(w16, w.bfloat16()) and torch.equal(w16t, w.bfloat16().T.contiguous())


def test_mfma_rejects_unsupported_shapes(L):
    assert L.lib().fns["vt_mfma_supported"](4800, 4800) == 1
    assert L.lib().fns["vt_mfma_supported"](100, 64) == 0
    x, w = torch.zeros(4, 100, device="cuda"), torch.zeros(64, 100, device="cuda")
    with pytest.raises(ValueError, match="multiples of 64"):
        _shadow(L, w)
    y = torch.empty(4, 64, device="cuda")
    ws = torch.empty(1 << 20, device="cuda")
    with pytest.raises(ValueError, match="multiples of 64"):
        L.call("vt_mfma_linear_fwd", L.ptr(x), 4, 100, L.ptr(y), 64, None, L.ptr(y), L.ptr(ws), ws.numel(),
               L.stream())


def test_model_bf16_heads_close_to_fp32(golden):
    """SeqVaeTeb(S=16) with the heads on bf16 MFMA vs the all-fp32 model on the
    reference golden batch: same loss to 1e-2 relative, gradients aligned."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from golden_util import det_fill_
    from vaeteb.model import SeqVaeTeb
    g = golden("model_s16_b4")
    out = {}
    for prec in ("fp32", "bf16"):
        m = det_fill_(SeqVaeTeb(sequence_length=16, head_precision=prec)).cuda()
        assert all(bool(l.mfma) == (prec == "bf16") for l in m.decoder.output_mu.modules() if hasattr(l, "mfma"))
        ins = [torch.from_numpy(g[k]).cuda() for k in ("y_st", "y_ph", "x_ph", "eps", "y_raw")]
        fo = m(*ins[:3], eps=ins[3])
        loss = m.compute_loss(fo, ins[0], ins[1], ins[4], beta=float(g["beta"]))["total_loss"]
        loss.backward()
        out[prec] = (loss.item(), torch.cat([p.grad.reshape(-1) for p in m.parameters()]))
    (l32, g32), (l16, g16) = out["fp32"], out["bf16"]
    assert abs(l16 - l32) <= 1e-2 * abs(l32)
    cos = torch.nn.functional.cosine_similarity(g16, g32, dim=0).item()
    assert cos > 0.999, cos
