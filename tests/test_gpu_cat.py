"""vt_copy_cols / ops.cat_last (csrc/cols.hip): the encoders' last-axis concatenation and its
backward split, against torch.cat and its autograd bit for bit (pure copies), on the 16-B path
(widths multiples of 4) and the element path (ragged widths)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("widths", [(16, 16), (32, 32), (5, 3, 8), (130, 2)])
def test_cat_last_matches_torch_cat(widths):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from vaeteb import ops
    g = torch.Generator(device="cuda").manual_seed(sum(widths))
    xs = [torch.randn(4, 37, w, device="cuda", generator=g, requires_grad=True) for w in widths]
    ref = [x.detach().clone().requires_grad_(True) for x in xs]
    out = ops.cat_last(xs)
    exp = torch.cat(ref, dim=-1)
    assert isinstance(out.grad_fn, ops.CatLastF._backward_cls) and torch.equal(out, exp)
    gy = torch.randn(exp.shape, device="cuda", generator=g)
    out.backward(gy)
    exp.backward(gy)
    torch.cuda.synchronize()
    for x, r in zip(xs, ref):
        assert x.grad.is_contiguous() and torch.equal(x.grad, r.grad)


def test_cat_last_one_input_without_grad():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from vaeteb import ops
    a = torch.randn(2, 8, 16, device="cuda", requires_grad=True)
    b = torch.randn(2, 8, 16, device="cuda")
    ops.cat_last([a, b]).sum().backward()
    assert torch.equal(a.grad, torch.ones_like(a)) and b.grad is None


def test_clamp_backward_one_pass_matches_autograd():
    """ops.clamp (ClampF: ATen's clamp forward, vt_clamp_bwd backward) == torch.clamp and its autograd
    bit for bit, including inputs exactly at the bounds (gradient kept), beyond them (zeroed) and
    NaN (forward NaN, gradient zeroed, as where((x >= lo) & (x <= hi), g, 0))."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from vaeteb import ops
    g = torch.Generator(device="cuda").manual_seed(11)
    x0 = torch.randn(3, 50, 32, device="cuda", generator=g) * 12
    x0.view(-1)[:4] = torch.tensor([10.0, -10.0, float("nan"), 10.000001], device="cuda")
    x, r = x0.clone().requires_grad_(True), x0.clone().requires_grad_(True)
    y, e = ops.clamp(x, -10, 10), torch.clamp(r, -10, 10)
    assert isinstance(y.grad_fn, ops.ClampF._backward_cls)
    assert torch.equal(torch.nan_to_num(y, nan=7.0), torch.nan_to_num(e, nan=7.0))
    gy = torch.randn(y.shape, device="cuda", generator=g)
    y.backward(gy)
    e.backward(gy)
    torch.cuda.synchronize()
    assert torch.equal(x.grad, r.grad)
