"""Conv-stack BatchNorm fold (round 5, model.ConvStack / ops.ConvBNActF xin / vout): an inner
block hands the next its pre-BN conv output and BatchNorm, and the next block applies
act(BN(.)) while staging its windows (vt_conv1d_bn_fwd_bf16_in, vt_conv1d_bwd_weight_bf16_in)
instead of reading a materialised y.  The staged bf16 operand is the value the BatchNorm-apply
pass would have written (one element function, bnbwd.h bn_fwd_val), so the folded stack must
equal the unfolded one BIT FOR BIT: outputs, input gradient, every parameter gradient and the
running statistics — for the model's stacks (decoder: reflect padding, x2 upsampling, K 11..3;
encoders: causal K 3/5/7) and ragged lengths.  The unfolded stack is itself pinned to torch /
the reference through test_gpu_conv_bf16.py, test_gpu_conv_bwd16.py and the model goldens
(ref/model/vae_teb_model.py:128-253).
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


STACKS = {
    # name: (blocks (cin, cout, k, causal, up, tanh), B, L)
    "decoder": ([(87, 77, 11, False, False, False), (77, 66, 9, False, True, False), (66, 55, 7, False, True, False),
                 (55, 44, 5, False, False, False), (44, 33, 5, False, True, False), (33, 22, 3, False, True, False),
                 (22, 11, 3, False, False, False), (11, 1, 3, False, False, False)], 3, 20),
    "decoder_ragged": ([(87, 77, 11, False, False, False), (77, 66, 9, False, True, False),
                        (66, 55, 7, False, True, False)], 2, 7),
    "source_enc": ([(32, 32, 3, True, False, False), (32, 32, 5, True, False, False),
                    (32, 32, 7, True, False, False)], 4, 256),
    "target_enc": ([(16, 16, 3, True, False, False), (16, 16, 5, True, False, False),
                    (16, 16, 7, True, False, False)], 3, 130),
    "tanh_tail": ([(8, 16, 3, False, False, False), (16, 2, 3, False, False, True)], 2, 64),
}


def _stack(spec, seed):
    from vaeteb.model import ConvBlock, ConvStack
    torch.manual_seed(seed)
    st = ConvStack(*[ConvBlock(a, b, k, causal=c, up=u, tanh=t) for a, b, k, c, u, t in spec]).cuda()
    with torch.no_grad():
        for blk in st:
            blk.bf16 = True
            blk.bn_layer.weight.uniform_(0.5, 1.5)
            blk.bn_layer.bias.uniform_(-0.3, 0.3)
    return st


def _run(st, x, gy):
    x = x.clone().requires_grad_(True)
    y = st(x)
    y.backward(gy)
    torch.cuda.synchronize()
    out = {"y": y.detach().clone(), "dx": x.grad.clone()}
    for n, p in st.named_parameters():
        out["grad." + n] = p.grad.clone()
    for n, b in st.named_buffers():
        out["buf." + n] = b.clone()
    return out


@pytest.mark.parametrize("name", list(STACKS))
def test_conv_stack_fold_bitwise(name):
    _need_gpu()
    from vaeteb import model
    spec, B, L = STACKS[name]
    Lo = L
    for a, b, k, c, u, t in spec:
        Lo *= 2 if u else 1
    x = torch.randn(B, L, spec[0][0], device="cuda")
    gy = torch.randn(B, Lo, spec[-1][1], device="cuda")
    res = []
    saved = model.CONV_FOLD
    for fold in (0, 1):
        model.CONV_FOLD = fold
        try:
            res.append(_run(_stack(spec, 11), x, gy))
        finally:
            model.CONV_FOLD = saved
    ref, got = res
    assert ref.keys() == got.keys()
    bad = [k for k in ref if not torch.equal(ref[k], got[k])]
    assert not bad, [(k, (ref[k] - got[k]).abs().max().item()) for k in bad]
    assert torch.isfinite(got["dx"]).all()


def test_conv_stack_fold_eval_and_fp32_unfolded():
    """Evaluation mode and the exact-fp32 conv kernels keep the per-block path (no fold)."""
    _need_gpu()
    spec, B, L = STACKS["target_enc"]
    st = _stack(spec, 5)
    x = torch.randn(B, L, 16, device="cuda")
    st.eval()
    with torch.no_grad():
        y0 = st(x)
        y1 = torch.nn.Sequential.forward(st, x)
    assert torch.equal(y0, y1)
    st.train()
    for blk in st:
        blk.bf16 = False
    y2 = st(x)
    y3 = torch.nn.Sequential.forward(st, x)
    assert torch.allclose(y2, y3, rtol=0, atol=0)
