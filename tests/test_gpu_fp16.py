"""The fp16 operand format (round 6; csrc/h16.h) and its dynamic loss scale (MI355X).

The reference trains under Lightning precision="16-mixed" / torch.amp.autocast('cuda') with
torch.amp.GradScaler('cuda') (ref/model/graph_model.py:510, 670, 709-726): Linear / conv / LSTM
operands in fp16, fp32 accumulation, the backward on loss * scale, an overflowing step skipped.
Here the decoder heads, conv blocks and ResidualMLP linears run their 16-bit MFMA kernels with
_Float16 operands (head / conv / mlp precision "fp16") and vaeteb.train.Trainer keeps the scale
on the device (vt_grad_norm_clip_scaled, vt_adamw_step_dev*_skip).  Tests:
  * the format is per op: bf16 results are bit-identical before and after fp16 launches;
  * each fp16 kernel family against the exact fp32 kernels is ~8x closer than its bf16 form
    (fp16 keeps 11 significant bits, bf16 8) — forward and every gradient;
  * GradScaler semantics: growth after growth_interval clean steps, an overflowing step (inf
    gradient) skipped — no parameter, moment or step-counter change — and the scale halved;
  * the fp16 step at the bench geometry (S = 256) inside the reference's OWN fp16 spread
    (tests/golden/model_s256_b2_amp.npz emu_fp16_*: the reference step under an emulation of
    CUDA fp16 autocast + GradScaler), which is ~8x tighter than the bf16 spread the bf16 step is
    held to;
  * the 20-step lr = 1e-5 trajectory in fp16 (tests/golden/traj_s256_b2_lr1e-5.npz: the
    emulated-fp16 members) — test_gpu_parity_s256.py::test_s256_trajectory_low_lr_binds_every_step[fp16].
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def rel(a, b):
    a = torch.as_tensor(a).detach().double().cpu()
    b = torch.as_tensor(b).detach().double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def test_format_is_per_op_bf16_bits_unchanged():
    """A bf16 head GEMM gives the same bits before and after fp16 launches of the same op (the
    library format is selected by each op), and the fp16 result differs (another operand type)."""
    _need_gpu()
    from vaeteb import _lib, ops
    torch.manual_seed(0)
    x = torch.randn(256, 4096, device="cuda")
    w = torch.randn(1024, 4096, device="cuda") * 0.02
    b = torch.randn(1024, device="cuda")
    y1 = ops.linear(x, w, b, "bf16")
    y2 = ops.linear(x, w, b, "fp16")
    assert _lib.h16() == "fp16"
    y3 = ops.linear(x, w, b, True)   # True == bf16
    assert _lib.h16() == "bf16"
    torch.cuda.synchronize()
    assert torch.equal(y1, y3)
    assert not torch.equal(y1, y2)
    # the fp16 GEMM IS the fp16-rounded product (RNE operand conversion, fp32 accumulation)
    assert rel(y2, x.half().double() @ w.half().double().t() + b.double()) < 1e-5
    ref = x.double() @ w.double().t() + b.double()
    e16 = rel(y2, ref)
    eb = rel(y1, ref)
    # the head GEMM rounds only its operands: fp16 ~2^-11, bf16 ~2^-8 relative per operand
    assert e16 < 2e-3 and e16 < eb / 4, (e16, eb)


def _fam_errors(precision, build, attr, S=64, B=4, seed=0):
    """rel-L2 of the forward output and of every parameter gradient of one module at `precision`
    against the same module on the exact fp32 kernels (same weights and inputs)."""
    from golden_util import det_fill_
    torch.manual_seed(seed)
    m32 = det_fill_(build()).cuda()
    m16 = det_fill_(build()).cuda()
    for m, p in ((m32, "fp32"), (m16, precision)):
        for mod in m.modules():
            if hasattr(mod, attr) and not isinstance(mod, torch.nn.Sequential):
                setattr(mod, attr, False if p == "fp32" else p)
    x = torch.randn(B, S, m32.in_dim, device="cuda")
    outs, grads = [], []
    for m in (m32, m16):
        m.train()
        xi = x.clone().requires_grad_(True)
        y = m(xi)
        g = torch.cos(torch.arange(y.numel(), device="cuda", dtype=torch.float32)).view_as(y)
        y.backward(g)
        torch.cuda.synchronize()
        outs.append(y.detach())
        grads.append([xi.grad.detach()] + [p.grad.detach().clone() for p in m.parameters()])
    fw = rel(outs[1], outs[0])
    gr = np.array([rel(a, b) for a, b in zip(grads[1], grads[0]) if b.norm() > 0])
    return fw, float(np.median(gr)), float(np.max(gr)), gr


class _Mlp(torch.nn.Module):
    def __init__(self):
        super().__init__()
        from vaeteb.model import ResidualMLP
        self.in_dim = 44
        self.mlp = ResidualMLP(44, (64, 64, 64, 32))

    def forward(self, x):
        return self.mlp(x)


class _Conv(torch.nn.Module):
    def __init__(self):
        super().__init__()
        from vaeteb.model import ConvBlock, ConvStack
        self.in_dim = 44
        self.conv = ConvStack(ConvBlock(44, 33, 5, causal=False, up=True), ConvBlock(33, 22, 3, causal=False, up=True),
                              ConvBlock(22, 16, 7, causal=True))

    def forward(self, x):
        return self.conv(x)


class _Head(torch.nn.Module):
    def __init__(self):
        super().__init__()
        from vaeteb.model import ResidualMLP
        self.in_dim = 1024
        self.head = ResidualMLP(1024, (1024, 1024), final_activation=False, use_skip_connection=False)

    def forward(self, x):
        return self.head(x.reshape(-1, 1024)).reshape(x.shape)


@pytest.mark.parametrize("fam", ["mlp", "conv", "head"])
def test_fp16_family_closer_to_fp32_than_bf16(fam):
    """Per kernel family (ResidualMLP stack, conv stack with x2 upsample / reflect / causal
    blocks, decoder-head GEMMs): the fp16 forward output and gradients against the exact fp32
    kernels, next to the bf16 ones.  fp16 keeps 3 more significant bits than bf16: the forward
    error must be >= 4x smaller (measured ~8x) and under 2e-3; the gradients carry the same
    rounding amplified by cancelling reductions (BatchNorm / LayerNorm parameter gradients), so
    their median error must be >= 2x smaller (measured 2.3-5.9x) and most gradients closer."""
    _need_gpu()
    build = {"mlp": _Mlp, "conv": _Conv, "head": _Head}[fam]
    attr = "mfma" if fam == "head" else "bf16"
    S = 4 if fam == "head" else 64
    eb = _fam_errors("bf16", build, attr, S=S)
    eh = _fam_errors("fp16", build, attr, S=S)
    closer = float(np.mean(eh[3] < eb[3]))
    print(f"{fam}: bf16 fw {eb[0]:.2e} grad median {eb[1]:.2e} max {eb[2]:.2e}; "
          f"fp16 fw {eh[0]:.2e} grad median {eh[1]:.2e} max {eh[2]:.2e}; fp16 closer on {closer:.2f} of the gradients")
    print("  per gradient (fp16, bf16):", [(round(a, 5), round(b, 5)) for a, b in zip(eh[3], eb[3])])
    assert eh[0] < 2e-3 and eh[0] * 4 < eb[0], (eh[:3], eb[:3])
    assert eh[1] * 2 < eb[1], (eh[:3], eb[:3])
    assert closer >= 0.75, closer


def _small_batch(S=16, B=2, seed=0):
    rng = np.random.default_rng(seed)
    b = {k: torch.from_numpy(rng.standard_normal(s).astype(np.float32)).cuda() for k, s in
         (("fhr_st", (B, S, 43)), ("fhr_ph", (B, S, 44)), ("fhr_up_ph", (B, S, 130)), ("fhr", (B, 16 * S)))}
    eps = torch.from_numpy(rng.standard_normal((B, S, 32)).astype(np.float32)).cuda()
    return b, eps


def _fp16_model(S=16):
    from golden_util import det_fill_
    from vaeteb.model import SeqVaeTeb
    m = det_fill_(SeqVaeTeb(sequence_length=S, head_precision="fp16", conv_precision="fp16", mlp_precision="fp16",
                            lstm_precision="16-mixed")).cuda()
    assert m.loss_scaling and m.h16_format == "fp16"
    return m


def test_loss_scale_growth_and_overflow_skip():
    """GradScaler semantics on the device (torch.amp.GradScaler defaults 2.0 / 0.5, interval here 2):
    clean steps grow the scale every 2 steps; a step whose scaled gradients overflow (init scale
    3e38: loss * scale is inf) is skipped — parameters, Adam moments and the AdamW step counter
    unchanged — with the scale halved and grad_norm reported as inf; training then resumes."""
    _need_gpu()
    from vaeteb.train import Trainer
    m = _fp16_model()
    tr = Trainer(m, lr=1e-3, init_scale=1024.0, growth_interval=2)
    assert tr.loss_scale
    for t in range(3):
        b, eps = _small_batch(seed=t)
        L = tr.step(b, eps=eps)
        assert np.isfinite(float(L["grad_norm"]))
    st = tr.scaler_state()
    assert st["scale"] == 2048.0 and st["growth_tracker"] == 1 and not st["found_inf"] and st["skipped_steps"] == 0, st
    # an overflowing step: the scale so large that the scaled backward seeds are inf in fp32
    tr.scaler[0] = 3.0e38
    p0, m0, v0 = tr.state.p.clone(), tr.state.m.clone(), tr.state.v.clone()
    step0 = int(tr.step_dev.item())
    b, eps = _small_batch(seed=9)
    L = tr.step(b, eps=eps)
    torch.cuda.synchronize()
    st = tr.scaler_state()
    assert st["found_inf"] and st["skipped_steps"] == 1 and st["growth_tracker"] == 0, st
    assert st["scale"] == pytest.approx(1.5e38, rel=1e-6), st
    assert not np.isfinite(float(L["grad_norm"]))
    assert torch.equal(tr.state.p, p0) and torch.equal(tr.state.m, m0) and torch.equal(tr.state.v, v0)
    assert int(tr.step_dev.item()) == step0
    # back to a sane scale: the next steps update again
    tr.scaler[0] = 512.0
    b, eps = _small_batch(seed=10)
    L = tr.step(b, eps=eps)
    torch.cuda.synchronize()
    assert np.isfinite(float(L["grad_norm"])) and not tr.scaler_state()["found_inf"]
    assert int(tr.step_dev.item()) == step0 + 1 and not torch.equal(tr.state.p, p0)


def test_fp16_scaled_step_equals_unscaled_gradient_math():
    """The scale cancels: one fp16 step with loss scale 2^10 and one with 2^14 (both exact powers
    of two, no overflow) give gradients that differ only by fp16 rounding of the scaled
    backward operands — the pre-clip norms agree to 1e-3 and the updated parameters to 1e-3
    rel-L2 (the same AdamW step on nearly the same gradient)."""
    _need_gpu()
    from vaeteb.train import Trainer
    out = []
    for sc in (2.0 ** 10, 2.0 ** 14):
        m = _fp16_model()
        tr = Trainer(m, lr=1e-3, init_scale=sc)
        b, eps = _small_batch(seed=3)
        L = tr.step(b, eps=eps)
        torch.cuda.synchronize()
        out.append((float(L["grad_norm"]), tr.state.p.clone()))
    assert abs(out[0][0] - out[1][0]) <= 1e-3 * out[1][0], (out[0][0], out[1][0])
    assert rel(out[0][1], out[1][1]) < 1e-3


def test_s256_fp16_step_within_reference_fp16_spread(golden):
    """The all-fp16 step (heads, convs, MLP linears fp16 operands; 16-mixed LSTM) at the bench
    geometry S = 256, B = 2 vs the reference's fp32 golden step, bounded by the reference's OWN fp16
    autocast spread (emu_fp16 of model_s256_b2_amp.npz): every forward output within 2x the
    reference's fp16 rel-L2, every loss within 3x the reference's fp16 ensemble deviation (+1e-6
    relative; below), gradient median / max within 2x the reference's fp16 median / max.  (One backward, unscaled here: the
    Trainer's loss scale is exercised by the trajectory test.)  The reference's fp16 spread is
    ~8x tighter than its bf16 spread, which the bf16 step is held to
    (test_gpu_parity_s256.py::test_s256_bf16_step_within_reference_autocast_spread)."""
    _need_gpu()
    from test_gpu_parity_s256 import FW_KEYS, LOSSES, _forward_backward, _grad_rels, _model
    g = golden("model_s256_b2")
    ga = golden("model_s256_b2_amp")
    m = _model(256, head_precision="fp16", conv_precision="fp16", mlp_precision="fp16", lstm_precision="16-mixed",
               concurrent_encoders=True)
    fw, L = _forward_backward(m, g)
    report = {}
    for k in FW_KEYS:
        r = rel(fw[k], g["fw_" + k])
        spread = float(ga[f"emu_fp16_fwrel_{k}"])
        report[k] = (round(r, 6), round(spread, 6))
        assert r <= 2 * spread, (k, r, spread)
    # losses: the reference's fp16 ENSEMBLE (emu_fp16 + three runs from one-ulp perturbed weights,
    # tests/golden/model_s256_b2_fp16ens.npz, tools/gen_golden.py amp_fp16_ens) at 3x.  Measured: the
    # reference's members shift the KL loss by +6.6e-5 .. +8.5e-5 relative, ours by +1.9e-4; the shift
    # is deterministic (weight / bias rounding), per stack additive (tools/fp16_diag2.py: the
    # conditional encoder's fc_mu +2.6e-4, the target encoder's pre_output -1.4e-4), and the two
    # implementations round different things — the reference's autocast rounds every Linear's bias
    # and output to fp16 (fc_mu's output IS the posterior mean), ours keeps both in fp32 — so their
    # deterministic parts differ by more than the members' one-ulp scatter
    ge = golden("model_s256_b2_fp16ens")
    members = ["emu_fp16"] + [f"emu_fp16_p{int(s_)}" for s_ in ge["seeds"]]
    src = lambda m_, k: float((ga if m_ == "emu_fp16" else ge)[f"{m_}_loss_{k}"])
    for k in LOSSES:
        exp = float(g["loss_" + k])
        dev = max(abs(src(m_, k) - exp) for m_ in members)
        got = L[k].item()
        report[k] = (abs(got - exp) / abs(exp), dev / abs(exp))
        assert abs(got - exp) <= 3 * dev + 1e-6 * abs(exp), (k, got, exp, dev)
    ours = {k: r for r, k in _grad_rels(m, g) if not k.endswith("(l2)")}
    names = list(ga["param_names"])
    ref = np.asarray(ga["emu_fp16_grad_rel"], np.float64)
    o = np.array([ours[k] for k in names])
    print("fp16 vs fp32 (ours, ref fp16 spread):", report)
    print(f"grad rel: ours median {np.median(o):.3e} max {o.max():.3e}; ref fp16 median {np.median(ref):.3e} "
          f"max {ref.max():.3e}")
    assert np.median(o) <= 2 * np.median(ref), (np.median(o), np.median(ref))
    assert o.max() <= 2 * ref.max(), (o.max(), ref.max())
