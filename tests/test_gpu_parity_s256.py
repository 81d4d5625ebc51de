"""The benchmarked geometry pinned end to end (MI355X).

`bench.py` trains SeqVaeTeb at S = 256 / R = 4096 with every GEMM-shaped op on bf16
MFMA.  These tests pin that configuration to the reference and the oracle:

  (a) the exact-fp32 HIP step at S = 256, B = 2 vs the REFERENCE's own fp32 step
      (tests/golden/model_s256_b2.npz, tools/gen_golden.py): losses 1e-5 relative,
      forward outputs 5e-5, BatchNorm running statistics 1e-5, post-AdamW parameter
      norms 1e-5; every gradient (the head weights by their first 16 rows and their
      norms) within 3x the reference's OWN fp32 error + 2e-5 rel-L2: the fixture
      stores each gradient's distance between the reference's fp32 and fp64 steps
      (median 1.8e-4, up to 5.9e-3 for the conditional encoder's logvar head at
      S = 256: 256 LSTM steps and 17 train-mode BatchNorms amplify rounding), so a
      second fp32 implementation cannot be held to a fixed 2e-4 there.
  (b) the all-bf16 HIP step (decoder heads + conv blocks + ResidualMLP linears, the
      bench default; with and without the 16-bit LSTM recurrences) at the same inputs, bounded by the reference's OWN spread at
      16-bit precision (tests/golden/model_s256_b2_amp.npz: the reference step under
      torch.autocast('cpu', bfloat16) and under an emulation of CUDA autocast in
      bf16, each compared with the reference fp32 step).  Tolerance:
        - each forward output: rel-L2 to fp32 <= 2x the larger bf16 spread;
        - each loss: |ours - fp32| <= 2x the larger bf16 deviation + 1e-6 relative;
        - gradients: median over parameters of rel-L2 to fp32 <= 2x the reference's
          median, max over parameters <= 2x the reference's max.
      The reference's fp16 spread (its literal precision, CUDA autocast fp16 +
      GradScaler, emulated) is ~8x smaller; bf16 is the documented deviation.
  (c) the literal BASELINE config 2 (Scattering1D J=6 Q=1 T=16 front-end, encoder
      widths 8 / 13 / 7) end to end: raw windows -> HIP front-end -> HIP fp32 step vs
      the oracle (oracle/frontend_ref.py + oracle/model_ref.py, fp64) on the same
      windows; features within 2x the reference engine's own fp32 error, the model
      step on the GPU's features vs the fp64 oracle: per gradient within 10x the oracle's
      own fp32 error (+2e-5), and the median over parameters of that error ratio <= 2
      (the conditional encoder's logvar-head gradients are chaotic in fp32: one of them
      measured 8x, the median ~1), and the end-to-end losses within 2x the loss spread
      the reference's own fp32 front-end error causes.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

BF16_MODES = ("cpu_bf16", "emu_bf16")
FW_KEYS = ("z", "linear_output", "mu_pr", "logvar_pr", "mu_prior", "logvar_prior", "mu_post", "logvar_post")
LOSSES = ("mse_loss", "nll_loss", "kld_loss", "total_loss")


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def rel(a, b):
    a = torch.as_tensor(a).detach().double().cpu()
    b = torch.as_tensor(b).detach().double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def _model(S, **kw):
    from golden_util import det_fill_
    from vaeteb.model import SeqVaeTeb
    return det_fill_(SeqVaeTeb(sequence_length=S, **kw)).cuda()


def _forward_backward(m, g):
    T = lambda k: torch.from_numpy(g[k]).cuda()
    m.train()
    fw = m(T("y_st"), T("y_ph"), T("x_ph"), eps=T("eps"))
    L = m.compute_loss(fw, T("y_st"), T("y_ph"), T("y_raw"), compute_kld_loss=True, beta=float(g["beta"]))
    L["total_loss"].backward()
    torch.cuda.synchronize()
    return fw, L


def _grad_rels(m, g, scaled=False):
    """rel-L2 of every parameter gradient vs the golden: full tensors, the R x R head
    weights by their first 16 rows (+ their fp64 norms, for the rows not stored).
    scaled: divided by the tolerance 2e-5 + 3 x the reference's own fp32 error."""
    params = dict(m.named_parameters())
    out = []
    for i, k in enumerate(list(g["param_names"])):
        gr = params[k].grad
        tol = (2e-5 + 3 * float(g["grad_rel64"][i])) if scaled else 1.0
        if f"grad_{i}" in g.files:
            out.append((rel(gr, g[f"grad_{i}"]) / tol, k))
        else:
            out.append((rel(gr[:16], g[f"gradrows_{i}"]) / tol, k))
        l2 = float(g["grad_l2"][i])
        out.append((abs(gr.double().norm().item() - l2) / max(l2, 1e-30) / tol, k + " (l2)"))
    return out


@pytest.mark.parametrize("name", ["model_s256_b2", "model_s300_b2"])
def test_fp32_step_vs_reference_golden_training_geometry(golden, name):
    """S = 256 (the bench's 4096-point windows) and S = 300 / R = 4800 (the reference's own
    production geometry: 5760-point windows trimmed to 300 steps, its unmodified 4800 x 4800
    heads)."""
    _need_gpu()
    g = golden(name)
    S = int(g["S"])
    m = _model(S)
    fw, L = _forward_backward(m, g)
    for k in LOSSES:
        exp = float(g["loss_" + k])
        assert abs(L[k].item() - exp) <= 1e-5 * abs(exp) + 1e-7, (k, L[k].item(), exp)
    for k in FW_KEYS:
        assert g["fw_" + k].shape == tuple(fw[k].shape), k    # every step (crosses the LSTM chunk hand-offs)
        assert rel(fw[k], g["fw_" + k]) < 5e-5, k
    worst = max(_grad_rels(m, g, scaled=True))
    assert worst[0] <= 1.0, worst       # in units of the tolerance
    sd = m.state_dict()
    for i, k in enumerate(list(g["bn_names"])):
        assert rel(sd[k], g[f"bn_{i}"]) < 1e-5, k

    # one full Trainer step (clip 1.0 + AdamW as ref/model/graph_model.py:654-660,724)
    from vaeteb.train import Trainer
    m2 = _model(S)
    p0 = {k: v.detach().double().cpu() for k, v in m2.state_dict().items()}
    tr = Trainer(m2, lr=1e-3)
    T = lambda k: torch.from_numpy(g[k]).cuda()
    Ls = tr.step({"fhr_st": T("y_st"), "fhr_ph": T("y_ph"), "fhr_up_ph": T("x_ph"), "fhr": T("y_raw")}, eps=T("eps"))
    assert abs(Ls["total_loss"].item() - float(g["loss_total_loss"])) <= 1e-5 * abs(float(g["loss_total_loss"]))
    # global norm vs the reference's, within 1e-4 + 3 x the reference's own fp32 spread of it
    # (each parameter's fp32-vs-fp64 gradient error weighted by its share of the squared norm:
    # 2.4e-4 at S = 256, 3.3e-3 at S = 300, where the decoder convs' gradients carry 3.8e-3)
    l2 = np.asarray(g["grad_l2"], np.float64)
    spread = float((l2 ** 2 * np.asarray(g["grad_rel64"], np.float64)).sum() / (l2 ** 2).sum())
    gn = float(g["grad_norm_total"])
    assert abs(Ls["grad_norm"].item() - gn) <= (1e-4 + 3 * spread) * gn, (Ls["grad_norm"].item(), gn, spread)
    # post-AdamW parameter norms: 1e-5 relative, plus what sign-ambiguous updates can move
    # the norm.  A first AdamW step moves each element by lr g / (|g| + eps) ~ lr sign(g), so
    # an element whose reference gradient lies within 3x the reference's own fp32 noise of
    # zero (noise per element: rel64 ||g|| / sqrt(n)) can legitimately step the other way,
    # a change of <= 2 lr that moves the norm by <= 2 lr (|p0_j| + 2 lr) / ||p||, summed over
    # those elements (S = 300: the input LayerNorm's bias has 3).  Counted from the full
    # reference gradients; the head weights (16 rows stored) keep the strict bound.
    sd2 = m2.state_dict()
    for i, k in enumerate(list(g["param_names"])):
        a = sd2[k].double().norm().item()
        amb = 0.0
        if f"grad_{i}" in g.files:
            gr = np.abs(np.asarray(g[f"grad_{i}"], np.float64)).reshape(-1)
            noise = float(g["grad_rel64"][i]) * float(g["grad_l2"][i]) / np.sqrt(gr.size)
            pj = p0[k].reshape(-1).abs().numpy()[gr <= 3 * noise]
            amb = float((2 * tr.lr * (pj + 2 * tr.lr)).sum()) / max(float(g["after_l2"][i]), 1e-30)
        tol = 1e-5 * float(g["after_l2"][i]) + 1e-7 + amb
        assert abs(a - float(g["after_l2"][i])) <= tol, (k, a, float(g["after_l2"][i]), amb)


@pytest.mark.parametrize("lstm", ["fp32", "16-mixed"])
def test_s256_bf16_step_within_reference_autocast_spread(golden, lstm):
    """lstm "16-mixed": the encoders' LSTMs on the 16-bit MFMA recurrences as well (the
    reference's autocast runs its LSTM in 16 bits; the Emu16 spread rounds the LSTM operands
    and stores h / c in 16 bits)."""
    _need_gpu()
    g = golden("model_s256_b2")
    ga = golden("model_s256_b2_amp")
    m = _model(256, head_precision="bf16", conv_precision="bf16", mlp_precision="bf16", lstm_precision=lstm,
               concurrent_encoders=True)
    fw, L = _forward_backward(m, g)
    report = {}
    for k in FW_KEYS:
        r = rel(fw[k], g["fw_" + k])
        spread = max(float(ga[f"{mode}_fwrel_{k}"]) for mode in BF16_MODES)
        report[k] = (r, spread, float(ga[f"emu_fp16_fwrel_{k}"]))
        assert r <= 2 * spread, (k, r, spread)
    for k in LOSSES:
        exp = float(g["loss_" + k])
        dev = max(abs(float(ga[f"{mode}_loss_{k}"]) - exp) for mode in BF16_MODES)
        got = L[k].item()
        report[k] = (abs(got - exp) / abs(exp), dev / abs(exp))
        assert abs(got - exp) <= 2 * dev + 1e-6 * abs(exp), (k, got, exp, dev)
    ours = {}
    for r, k in _grad_rels(m, g):
        if not k.endswith("(l2)"):
            ours[k] = r
    names = list(ga["param_names"])
    ref = np.max([ga[f"{mode}_grad_rel"] for mode in BF16_MODES], axis=0)
    o = np.array([ours[k] for k in names])
    print("bf16 vs fp32 (ours, ref bf16 spread, ref fp16 spread):", report)
    print(f"grad rel: ours median {np.median(o):.3e} max {o.max():.3e}; ref bf16 median {np.median(ref):.3e} "
          f"max {ref.max():.3e}; ref fp16 median {np.median(ga['emu_fp16_grad_rel']):.3e}")
    assert np.median(o) <= 2 * np.median(ref), (np.median(o), np.median(ref))
    assert o.max() <= 2 * ref.max(), (o.max(), ref.max())
    # the binding part: every parameter whose gradient the reference's own 16-bit step keeps
    # within 0.5 rel-L2 of fp32 (the decoder heads — 97 % of the gradient's squared norm —
    # the decoder MLPs, ~1/4 of the parameters) is held to 2x that spread, a bound below the
    # 1.0 a zero or unrelated gradient scores; the others are chaotic in the reference itself
    # (their 16-bit gradients sit 0.5-2.5 rel-L2 from fp32) and keep the aggregate bounds
    tight = [(o[i] / (2 * ref[i]), names[i]) for i in range(len(names)) if ref[i] < 0.5]
    print(f"{len(tight)} parameters with a binding bound; worst (ours / 2 x ref spread): {max(tight)}")
    assert len(tight) >= 100 and max(tight)[0] <= 1.0, max(tight)
    # the whole gradient vector (squared-norm weighted): the reference's bf16 spread is 0.47
    l2 = np.asarray(g["grad_l2"], np.float64)
    w = l2 ** 2 / (l2 ** 2).sum()
    assert float((w * o).sum()) <= 2 * float((w * ref).sum()), (float((w * o).sum()), float((w * ref).sum()))


def _traj_run(precision, lr=1e-3):
    """20 Trainer steps (clip 1.0 + AdamW, ref/model/graph_model.py:700-726) at S = 256,
    B = 2 on the trajectory fixture's batches and noise; per-step losses and pre-clip
    gradient norms, and the last step's mu_pr."""
    from golden_util import traj_inputs
    from vaeteb.train import Trainer
    kw = dict(head_precision=precision, conv_precision=precision, mlp_precision=precision,
              lstm_precision="16-mixed" if precision != "fp32" else "fp32", concurrent_encoders=True)
    m = _model(256, **kw)
    tr = Trainer(m, lr=lr)
    rec = {k: [] for k in (*LOSSES, "grad_norm")}
    last = None
    for t in range(20):
        y_st, y_ph, x_ph, y_raw, eps = [torch.from_numpy(a).cuda() for a in traj_inputs(256, 2, t)]
        batch = {"fhr_st": y_st, "fhr_ph": y_ph, "fhr_up_ph": x_ph, "fhr": y_raw}
        if t == 19:   # the last step's forward outputs: the model's forward before this step's update
            with torch.no_grad():
                m.train()
                last = m(y_st, y_ph, x_ph, eps=eps)["mu_pr"].double().cpu()
        L = tr.step(batch, eps=eps)
        for k in rec:
            rec[k].append(float(L[k]))
        if tr.loss_scale and tr.scaler_state()["found_inf"]:
            rec["grad_norm"][-1] = 0.0   # a skipped step: the reference's record (tools/gen_golden.py Emu16)
    return {k: np.array(v) for k, v in rec.items()}, last


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_s256_training_trajectory_vs_reference(golden, precision):
    """the ELBO over 20 training steps (a new batch per step, as the
    reference's loop) vs the reference's own trajectory (tests/golden/traj_s256_b2.npz).
    This model is chaotic under AdamW: the first update moves every head weight by ~lr,
    with a sign that rounding noise decides wherever a gradient is near 0, so the
    reference's fp32 trajectory leaves its own fp64 trajectory by 1e-3 at step 2 and by
    tens of percent (NLL) later, and so do fp32 runs of it from one-ulp perturbed initial
    weights.  The bound at step t is therefore an envelope: env(t) = the running maximum
    over steps s <= t of the reference ensemble's deviation from its base fp32 run —
      fp32 (exact kernels): the fp64 run and seven one-ulp perturbed fp32 runs;
          |ours - ref fp32| <= 1e-4 |ref| + 3 env(t)  (step 0: the fp64 distance only);
      bf16 (the bench precision: bf16 heads / convs / MLP linears, 16-mixed LSTM): those
          and the emulated-bf16-autocast runs (base + five perturbed);
          |ours - ref fp32| <= 1e-4 |ref| + 2 env(t);
    for each of the four losses at every step, the pre-clip gradient norm while the ensemble
    agrees within 50 % (the first steps), and the last step's mu_pr within 2x the ensemble's
    largest deviation at that step."""
    _need_gpu()
    d = golden("traj_s256_b2")
    ours, mu_pr = _traj_run(precision)
    r32 = lambda k: np.asarray(d[f"fp32_{k}"], np.float64)
    # every member the fixture holds (round 4: fp64, fp32_p1-p7; bf16 adds emu_bf16 and
    # emu_bf16_p1-p5)
    names = [k[: -len("_total_loss")] for k in d.files if k.endswith("_total_loss")]
    members = ["fp64"] + sorted(m for m in names if m.startswith("fp32_p"))
    if precision == "bf16":
        members += sorted(m for m in names if m.startswith("emu_bf16"))
    factor = 3.0 if precision == "fp32" else 2.0
    for k in (*LOSSES, "grad_norm"):
        ref = r32(k)
        devs = {m: np.abs(np.asarray(d[f"{m}_{k}"], np.float64) - ref) for m in members}
        dev = np.max(list(devs.values()), axis=0)
        # step 0 (the first forward / backward, at exactly the reference's weights): the fp32
        # test is held to the fp64 distance only (the one-ulp perturbed fp32 members start from
        # other weights); from step 1 on, one update's sign noise is in every member
        dev[0] = max(v[0] for m, v in devs.items() if not m.startswith("fp32_p"))
        env = np.maximum.accumulate(dev)
        err = np.abs(ours[k] - ref)
        bound = 1e-4 * np.abs(ref) + factor * env + 1e-7
        # the pre-clip gradient norm is held only while the reference ensemble itself agrees
        # within 50 % (steps 0-3 or so): later the NLL head's exp(-logvar) makes it swing by
        # 10-40x between members, and a bound of that size pins nothing
        held = np.ones_like(err, dtype=bool) if k != "grad_norm" else env < 0.5 * np.abs(ref)
        print(f"{precision} {k}: ours-ref {np.round(err / np.abs(ref), 5).tolist()}\n"
              f"   bound/|ref| {np.round(bound / np.abs(ref), 5).tolist()}  (held at {int(held.sum())} steps)")
        assert held[0] and (err <= bound)[held].all(), (k, int(np.argmax((err - bound) * held)), ours[k].tolist(),
                                                        ref.tolist())
    ref_mu = np.asarray(d["fp32_mu_pr"], np.float64)
    dev = max(rel(np.asarray(d[f"{m}_mu_pr"]), ref_mu) for m in members)
    got = rel(mu_pr, ref_mu)
    print(f"{precision} last-step mu_pr rel-L2 {got:.4f} (reference ensemble spread {dev:.4f})")
    assert got <= 2 * dev + 1e-4, (got, dev)

@pytest.mark.parametrize("precision", ["fp32", "bf16", "fp16"])
def test_s256_trajectory_low_lr_binds_every_step(golden, precision):
    """the 20-step trajectory at lr = 1e-5 (tests/golden/
    traj_s256_b2_lr1e-5.npz, tools/gen_golden.py traj_lowlr), where the reference does not
    amplify rounding into O(1) swings: its fp32 run stays within ~2e-4 of its fp64 run over all
    20 steps.  So the bound binds at EVERY step, for every loss AND the pre-clip gradient norm
    (no held mask): env(t) = running max over the reference ensemble of |member - fp32 base|
    (fp64 + the one-ulp perturbed fp32 members; for the bench precision also the emulated bf16
    autocast runs), exact fp32: |ours - ref| <= 1e-5 |ref| + 3 env(t); bf16 (bf16 heads / convs
    / MLP linears, 16-mixed LSTM): |ours - ref| <= 1e-5 |ref| + 2 env(t); fp16 (round 6: fp16
    heads / convs / MLP linears with the trainer's dynamic loss scale, 16-mixed LSTM) the same
    with the emulated fp16-autocast + GradScaler members in the envelope instead of the bf16 ones
    (a skipped step's gradient norm recorded as 0, as the reference's emulation does), at 3 env(t)."""
    _need_gpu()
    d = golden("traj_s256_b2_lr1e-5")
    assert float(d["lr"]) == 1e-5
    ours, mu_pr = _traj_run(precision, lr=1e-5)
    r32 = lambda k: np.asarray(d[f"fp32_{k}"], np.float64)
    names = [k[: -len("_total_loss")] for k in d.files if k.endswith("_total_loss")]
    members = ["fp64"] + sorted(m for m in names if m.startswith("fp32_p"))
    if precision in ("bf16", "fp16"):
        members += sorted(m for m in names if m.startswith("emu_" + precision))
    # fp16: 3x (as test_gpu_fp16.py::test_s256_fp16_step_within_reference_fp16_spread): the reference's
    # autocast rounds Linear biases / outputs to fp16 and ours keeps them fp32, so the deterministic
    # rounding shifts of the two fp16 implementations differ (step 0 KL: ours 2.1x the members')
    factor = 2.0 if precision == "bf16" else 3.0
    for k in (*LOSSES, "grad_norm"):
        ref = r32(k)
        env = np.maximum.accumulate(np.max([np.abs(np.asarray(d[f"{m}_{k}"], np.float64) - ref) for m in members],
                                           axis=0))
        err = np.abs(ours[k] - ref)
        bound = 1e-5 * np.abs(ref) + factor * env + 1e-7
        print(f"{precision} lr 1e-5 {k}: ours-ref / |ref| {np.round(err / np.abs(ref), 6).tolist()}\n"
              f"   bound / |ref| {np.round(bound / np.abs(ref), 6).tolist()}")
        assert (err <= bound).all(), (k, int(np.argmax(err - bound)), ours[k].tolist(), ref.tolist())
    # the bound binds: it stays far below the quantities themselves
    assert (1e-5 * np.abs(r32("total_loss")) + factor * np.maximum.accumulate(
        np.max([np.abs(np.asarray(d[f"{m}_total_loss"], np.float64) - r32("total_loss")) for m in members], axis=0))
        < 0.02 * np.abs(r32("total_loss"))).all()
    ref_mu = np.asarray(d["fp32_mu_pr"], np.float64)
    dev = max(rel(np.asarray(d[f"{m}_mu_pr"]), ref_mu) for m in members)
    got = rel(mu_pr, ref_mu)
    print(f"{precision} lr 1e-5 last-step mu_pr rel-L2 {got:.5f} (reference ensemble spread {dev:.5f})")
    assert got <= 2 * dev + 1e-5, (got, dev)


def _oracle_features(fe, x, st, dtype, engine):
    """Oracle front-end (the reference's two calls, create_hdf5_dataset.py:418-441)
    + normalisation, model layout (B, S, C)."""
    from oracle import frontend_ref as F
    old = F.FFT_ENGINE
    F.FFT_ENGINE = engine
    try:
        ofe = F.PhaseFrontEnd(fe.plan.J, fe.plan.Q, fe.plan.T, fe.plan.N, dtype=dtype)
        pm, cm = ofe.masks()
        rp = ofe.forward(x, compute_phase=True, pair_subset=pm)
        rc = ofe.forward(x, compute_phase=False, compute_cross_phase=True, pair_subset=cm)
    finally:
        F.FFT_ENGINE = old
    tt = lambda a: np.ascontiguousarray(np.asarray(a, np.float64).transpose(0, 2, 1))
    return {"fhr_st": tt(F.normalize(rp["scattering"], "fhr_st", st["fhr_st_mean"], st["fhr_st_variance"])),
            "fhr_ph": tt(F.normalize(rp["phase_corr"], "fhr_ph", st["fhr_ph_mean"], st["fhr_ph_variance"])),
            "fhr_up_ph": tt(F.normalize(rc["cross_phase_corr"], "fhr_up_ph", st["fhr_up_ph_mean"],
                                        st["fhr_up_ph_variance"])),
            "fhr": np.asarray(F.normalize(x[:, 0], "fhr", st["fhr_mean"], st["fhr_variance"]), np.float64)}


def _oracle_step(feats, eps, widths, dtype=torch.float64, S=256):
    from golden_util import det_fill_
    from oracle import model_ref as M
    ref = det_fill_(M.SeqVaeTebRef(S, *widths)).to(dtype)
    T = lambda a: torch.from_numpy(np.asarray(a)).to(dtype)
    fw, L, grads, gn = M.train_step(ref, {"y_st": T(feats["fhr_st"]), "y_ph": T(feats["fhr_ph"]),
                                          "x_ph": T(feats["fhr_up_ph"]), "y_raw": T(feats["fhr"])},
                                    T(eps), 1e-5)
    return fw, L, grads, ref.state_dict()


def _relu_kinks(feats, eps, widths, factor=10.0, S=256):
    """ReLU inputs of the oracle's training forward on these features that sit within `factor` x
    the fp32-vs-fp64 distance of the kink: |x64| <= factor |x32 - x64| (x32 != x64).  At such a unit
    the derivative's 0 / 1 is decided by fp32 rounding — the fp32 oracle and any other fp32 step
    (ours) may take different sides — and one flipped unit moves its layer's weight gradient by
    ~1 / (B S) of its norm.  Returns (count, smallest |x64| / |x32 - x64|)."""
    import torch.nn.functional as Fn
    from golden_util import det_fill_
    from oracle import model_ref as M
    rec = {}
    orig = Fn.relu
    for dt in (torch.float64, torch.float32):
        rec[dt] = []

        def relu(x, inplace=False, _r=rec[dt]):
            _r.append(x.detach().double().clone())
            return orig(x, inplace=inplace)
        ref = det_fill_(M.SeqVaeTebRef(S, *widths)).to(dt)
        ref.train()
        T = lambda a: torch.from_numpy(np.asarray(a)).to(dt)
        Fn.relu = relu
        try:
            with torch.no_grad():
                ref(T(feats["fhr_st"]), T(feats["fhr_ph"]), T(feats["fhr_up_ph"]), T(eps))
        finally:
            Fn.relu = orig
    n, worst = 0, float("inf")
    for a, b in zip(rec[torch.float64], rec[torch.float32]):
        d = (b - a).abs()
        m = d > 0
        if not m.any():
            continue
        ratio = a.abs()[m] / d[m]
        n += int((ratio <= factor).sum())
        worst = min(worst, ratio.min().item())
    return n, worst


def test_j6_config2_step_end_to_end_vs_oracle():
    """BASELINE config 2's literal variant: raw windows -> FrontEnd(J=6, Q=1, T=16) ->
    SeqVaeTeb(widths 8 / 13 / 7) train step, vs the oracle on the same windows."""
    _need_gpu()
    from vaeteb import synthetic
    from vaeteb.frontend import FrontEnd, FrontEndPlan, load_stats
    from vaeteb.train import Trainer
    torch.set_num_threads(min(16, torch.get_num_threads()))
    st = load_stats(6, 1, 16, 4096)
    fe = FrontEnd(FrontEndPlan(6, 1, 16, 4096, device="cuda"), st)
    widths = (fe.C_st, fe.C_ph, fe.C_x)
    assert widths == (8, 13, 7) and fe.plan.S == 256
    B = 2
    # window seed 4244: the fp64 oracle's gradients are a smooth function of the features
    # there (checked below).  Seeds 4242/4243/4245 put a sample near a kink of the model
    # (a ReLU / clamp boundary): a 1e-6 relative perturbation of the features moves the
    # oracle's own gradients by ~1e-3, so ANY fp32 front-end, the reference's included,
    # lands on either side of it and no gradient bound of the fp32 error's size holds there
    x = synthetic.batch(4244, B, 4096)
    eps = np.random.default_rng(6).standard_normal((B, 256, 32)).astype(np.float32)
    feats = {k: v.detach().cpu().double().numpy() for k, v in fe(torch.from_numpy(x).cuda()).items()}

    # features vs the fp64 oracle, within 2x the reference engine's own fp32 error
    f64 = _oracle_features(fe, x, st, np.float64, "numpy")
    f32 = _oracle_features(fe, x, st, np.float32, "torch")
    for k in ("fhr_st", "fhr_ph", "fhr_up_ph", "fhr"):
        assert feats[k].shape == f64[k].shape, k
        assert rel(feats[k], f64[k]) <= 2 * rel(f32[k], f64[k]) + 1e-6, (k, rel(feats[k], f64[k]),
                                                                          rel(f32[k], f64[k]))

    # the HIP fp32 step on the GPU's features vs the fp64 oracle step on the same features
    m = _model(256, scattering_channels=widths[0], phase_channels=widths[1], cross_phase_channels=widths[2])
    tr = Trainer(m, lr=1e-3, frontend=fe)
    L = tr.step({"x": torch.from_numpy(x).cuda()}, eps=torch.from_numpy(eps).cuda())
    torch.cuda.synchronize()
    fw_o, L_o, g_o, sd_o = _oracle_step(feats, eps, widths)
    # the oracle's own fp32 reproducibility: the plain fp32 step and ENS steps from one-ulp perturbed
    # initial weights (golden_util.perturb_ulp_, as the bench-batch test).  Round 6 finding
    # (tools/j6_step_diag.py): at this window one ReLU unit of the target encoder's mu_layer sits
    # within fp32 rounding of its kink — the fp32 steps that flip it (our step on the half-image pair
    # kernel's features; the oracle's member 3; our own one-ulp members) move mu_layer's weight
    # gradients by up to 1.1e-2 while the fp64 step moves by 3e-6 for the same feature change, and
    # our flipped step equals that oracle member gradient for gradient.  So each gradient is held to
    # the ensemble's largest distance, as at B = 256, not to the one plain fp32 run.
    from golden_util import det_fill_, perturb_ulp_
    from oracle import model_ref as M

    def member(seed):
        ref = det_fill_(M.SeqVaeTebRef(256, *widths))
        if seed:
            perturb_ulp_(ref, seed)
        Tf = lambda a: torch.from_numpy(np.asarray(a)).float()
        _, _, g, _ = M.train_step(ref, {"y_st": Tf(feats["fhr_st"]), "y_ph": Tf(feats["fhr_ph"]),
                                        "x_ph": Tf(feats["fhr_up_ph"]), "y_raw": Tf(feats["fhr"])}, Tf(eps), 1e-5)
        return g, ref.state_dict()
    ENS = 4
    members = [member(s) for s in range(ENS + 1)]          # seed 0: the plain fp32 oracle step
    g_o32, sd_o32 = members[0]
    # precondition: the oracle is well-conditioned at these features (a 1e-6 relative
    # perturbation, below fp32 rounding, moves its fp64 gradients by far less than the bounds)
    prng = np.random.default_rng(4244)
    _, _, g_p, sd_p = _oracle_step({k: v * (1 + 1e-6 * prng.standard_normal(v.shape)) for k, v in feats.items()},
                                   eps, widths)
    sens = np.median([rel(g_p[k], gr) for k, gr in g_o.items() if gr.norm() > 0])
    assert sens <= 5e-5, f"oracle ill-conditioned at this window (perturbed median rel {sens:.2e})"
    assert L["mse_loss"].item() == 0.0       # 8 + 13 != 87: the reference's MSE branch is off
    for k in ("nll_loss", "kld_loss", "total_loss"):
        exp = L_o[k].item()
        assert abs(L[k].item() - exp) <= 1e-5 * abs(exp) + 1e-7, (k, L[k].item(), exp)
    params = dict(m.named_parameters())
    env = {k: max(rel(g[k], gr) for g, _ in members) for k, gr in g_o.items() if gr.norm() > 0}
    worst, ratios = [], []
    for k, gr in g_o.items():
        if gr.norm() == 0:      # decoder.linear: no MSE term, no gradient
            worst.append((params[k].grad.abs().max().item() * 1e30, k, 0.0, 0.0, 0.0))
            continue
        e_ours = rel(params[k].grad, gr)
        ratios.append(e_ours / max(env[k], 1e-12))
        # + the gradient's own conditioning at these features: how far the fp64 oracle's gradient
        # moves for the 1e-6 feature perturbation above (a fp32 front-end's rounding is that size)
        e_pert = rel(g_p[k], gr)
        worst.append((e_ours / (2e-5 + 10 * env[k] + 2 * e_pert), k, e_ours, env[k], e_pert))
    # fixed bounds from the errors measured here (round 4: median 6.8e-6, p90 1.0e-5) over the
    # gradients every ensemble member gets within 1e-4 of fp64 (a clean fp32 gradient lands ~1e-5
    # away; a member that flips the kink unit moves the gradients upstream of it by 1e-4 .. 1e-2):
    # the per-parameter bound above is relative to the ensemble, which is large for the chaotic
    # ones, so these aggregates are what a regression of the HIP gradients would fail
    errs = np.array([rel(params[k].grad, g_o[k]) for k in env if env[k] < 1e-4])
    print(f"J6 grads vs fp64 oracle: median ours/ensemble error ratio {np.median(ratios):.2f}, "
          f"worst {max(worst)}; ours rel-L2 over {len(errs)} well-conditioned gradients: median "
          f"{np.median(errs):.3e} p90 {np.percentile(errs, 90):.3e} max {errs.max():.3e}")
    assert len(errs) >= 100 and np.median(errs) <= 2e-5 and np.percentile(errs, 90) <= 5e-5, errs
    assert np.median(ratios) <= 2.0, np.median(ratios)
    worst = max(worst)
    assert worst[0] <= 1.0, worst
    # after clip + AdamW: within 10x the ensemble's largest fp32-vs-fp64 distance (+1e-6), as the
    # gradients (AdamW carries a gradient's error into the step: the conditional encoder's
    # logvar-head LayerNorm weight measured 4.8x), + twice the parameter's own conditioning (the
    # 1e-6 feature perturbation of the fp64 step: a bias whose gradient entries sit near AdamW's eps
    # moves by ~lr).  With the MSE term off, decoder.linear's biases feed only BatchNorm-normalised
    # channels: their exact gradient is 0 and an fp32 step gives rounding noise, which AdamW scales
    # to lr-sized steps — the reference's fp32 step does the same, so only that bound is
    # meaningful there
    sd = m.state_dict()
    worst = max((rel(sd[k], v) / (1e-6 + 10 * max(rel(sm[k], v) for _, sm in members) + 2 * rel(sd_p[k], v)), k,
                 rel(sd[k], v), rel(sd_o32[k], v), rel(sd_p[k], v)) for k, v in sd_o.items()
                if v.dtype == torch.float64 and v.norm() > 0)
    print(f"J6 parameters after clip + AdamW: worst {worst}")
    assert worst[0] <= 1.0, worst

    # end to end: the oracle step on its own fp64 features; the spread the reference's own
    # fp32 front-end error causes in the losses sets the bound
    _, L64, _, _ = _oracle_step(f64, eps, widths)
    _, L32, _, _ = _oracle_step(f32, eps, widths)
    for k in ("nll_loss", "kld_loss", "total_loss"):
        a, e, r32 = L[k].item(), L64[k].item(), L32[k].item()
        assert abs(a - e) <= 2 * abs(r32 - e) + 1e-5 * abs(e), (k, a, e, r32)


def test_production_geometry_end_to_end_vs_oracle():
    """The reference's production data path on the MI355X: raw 5760-point windows ->
    FrontEnd(J=11 Q=4 T=16, N=5760, trim 30 steps: ref/hdf5_dataset/hdf5_dataset.py:359-364)
    -> SeqVaeTeb(sequence_length=300, R = 4800) fp32 train step, vs the oracle front-end
    (fp64, trimmed the same way) and the oracle step (fp64) on the GPU's features, with the
    tolerances of the J=6 test.  Normalisation statistics: the frozen N=4096 per-channel
    statistics (the same transform for every position, so valid for any window length)."""
    _need_gpu()
    from vaeteb import synthetic
    from vaeteb.frontend import FrontEnd, FrontEndPlan, load_stats
    from vaeteb.train import Trainer
    torch.set_num_threads(min(16, torch.get_num_threads()))
    st = load_stats(11, 4, 16, 4096)
    fe = FrontEnd(FrontEndPlan(11, 4, 16, 5760, device="cuda"), st, trim=30)
    assert fe.plan.S == 360 and fe.S_out == 300 and fe.N_out == 4800
    widths = (fe.C_st, fe.C_ph, fe.C_x)
    B = 2
    x = synthetic.batch(5760, B, 5760)
    eps = np.random.default_rng(7).standard_normal((B, 300, 32)).astype(np.float32)
    feats = {k: v.detach().cpu().double().numpy() for k, v in fe(torch.from_numpy(x).cuda()).items()}
    f64 = _oracle_features(fe, x, st, np.float64, "numpy")
    f32 = _oracle_features(fe, x, st, np.float32, "torch")
    for d in (f64, f32):
        for k in ("fhr_st", "fhr_ph", "fhr_up_ph"):
            d[k] = d[k][:, 30:330]
        d["fhr"] = d["fhr"][:, 480:5280]
    for k in ("fhr_st", "fhr_ph", "fhr_up_ph", "fhr"):
        assert feats[k].shape == f64[k].shape, k
        assert rel(feats[k], f64[k]) <= 2 * rel(f32[k], f64[k]) + 1e-6, (k, rel(feats[k], f64[k]),
                                                                          rel(f32[k], f64[k]))
    m = _model(300, scattering_channels=widths[0], phase_channels=widths[1], cross_phase_channels=widths[2])
    tr = Trainer(m, lr=1e-3, frontend=fe)
    L = tr.step({"x": torch.from_numpy(x).cuda()}, eps=torch.from_numpy(eps).cuda())
    torch.cuda.synchronize()
    _, L_o, g_o, _ = _oracle_step(feats, eps, widths, S=300)
    _, _, g_o32, _ = _oracle_step(feats, eps, widths, torch.float32, S=300)
    for k in ("mse_loss", "nll_loss", "kld_loss", "total_loss"):
        exp = L_o[k].item()
        assert abs(L[k].item() - exp) <= 1e-5 * abs(exp) + 1e-7, (k, L[k].item(), exp)
    params = dict(m.named_parameters())
    worst, ratios = [], []
    for k, gr in g_o.items():
        e_ours, e_ref = rel(params[k].grad, gr), rel(g_o32[k], gr)
        ratios.append(e_ours / max(e_ref, 1e-12))
        worst.append((e_ours / (2e-5 + 10 * e_ref), k))
    # fixed bounds from the errors measured here (round 4: median 6.4e-6, p90 1.1e-5, max 2.7e-4
    # over every gradient; the oracle's own fp32 step is 8e-3 off in median at S = 300, so the
    # ratio bound above does not bind — these do)
    errs = np.array([rel(params[k].grad, gr) for k, gr in g_o.items()])
    e32 = np.array([rel(g_o32[k], gr) for k, gr in g_o.items()])
    print(f"S=300 grads vs fp64 oracle: median ours/oracle-fp32 error ratio {np.median(ratios):.2f}, "
          f"worst {max(worst)}; ours rel-L2 median {np.median(errs):.3e} p90 {np.percentile(errs, 90):.3e} "
          f"max {errs.max():.3e}; oracle fp32 median {np.median(e32):.3e} max {e32.max():.3e}")
    assert np.median(errs) <= 2e-5 and np.percentile(errs, 90) <= 5e-5 and errs.max() <= 2e-3, errs
    assert np.median(ratios) <= 2.0, np.median(ratios)
    assert max(worst)[0] <= 1.0, max(worst)


def test_bench_batch_fp32_step_vs_fp64_oracle():
    """the bench's own batch.  One exact-fp32 c2 step at B = 256 —
    raw windows -> FrontEnd(J=11 Q=4 T=16) -> SeqVaeTeb(S = 256) — against the fp64 oracle step
    (oracle/model_ref.py, run on this box's host) on the same features: the 17 train-mode
    BatchNorms then reduce over 65,536 (encoders) to 1,048,576 (last decoder block) rows with the
    kernels' split partials, the MLPs / LSTMs run their full 256-sample grids, the heads their
    256-row GEMMs.

    At this batch an fp32 step is not a fixed distance from fp64: the oracle's own fp32 step run
    from initial weights perturbed by one ulp lands anywhere in a spread as wide as the distance
    itself (CPU measurement, tools/b256_ensemble.py: pre-clip norm gap +2.0e-5 for the plain fp32
    run, -2.3e-5 .. -1.3e-4 for four one-ulp members; whole-gradient rel-L2 3.2e-4 .. 6.4e-4;
    median per-gradient 5.5e-4 .. 1.1e-3).  So the bound is that ENSEMBLE, computed here: the
    plain fp32 oracle step and ENS one-ulp perturbed fp32 oracle steps (golden_util.perturb_ulp_),
    each compared with the fp64 step, and the HIP step held to 1.5x the ensemble's largest
    distance for the pre-clip norm, the whole gradient and the median / p90 of the per-gradient
    rel-L2, every single gradient within 10x its largest member distance + 2e-5.  Losses within
    1e-5; the pre-clip norm equal to the fp64 norm of the gradients it reduced; the four head
    gradients' norms as before.  The front-end rows at B = 256 are those of B = 4 runs bit for bit
    (test_gpu_frontend.py), and a B = 4 slice of them is held to the fp64 oracle front-end here.
    (Round 6 finding: the LSTM cell on the libm expf / tanhf / IEEE divide instead of the hardware
    v_exp / v_rcp forms moved this step's norm gap from +3.6e-5 to -1.7e-4 — the same scatter as
    the oracle's members, not a bias of the approximations)"""
    _need_gpu()
    import time
    from golden_util import det_fill_, perturb_ulp_
    from oracle import model_ref as M
    from vaeteb import synthetic
    from vaeteb.frontend import FrontEnd, FrontEndPlan, load_stats
    from vaeteb.train import Trainer
    torch.set_num_threads(min(16, torch.get_num_threads()))
    st = load_stats(11, 4, 16, 4096)
    fe = FrontEnd(FrontEndPlan(11, 4, 16, 4096, device="cuda"), st)
    widths = (fe.C_st, fe.C_ph, fe.C_x)
    B, S = 256, fe.plan.S
    assert S == 256
    x = synthetic.batch(777, B, 4096)
    eps = np.random.default_rng(8).standard_normal((B, S, 32)).astype(np.float32)
    feats = {k: v.detach().cpu().double().numpy() for k, v in fe(torch.from_numpy(x).cuda()).items()}
    rows = [0, 1, 254, 255]
    f64 = _oracle_features(fe, x[rows], st, np.float64, "numpy")
    f32 = _oracle_features(fe, x[rows], st, np.float32, "torch")
    for k in ("fhr_st", "fhr_ph", "fhr_up_ph", "fhr"):
        assert rel(feats[k][rows], f64[k]) <= 2 * rel(f32[k], f64[k]) + 1e-6, k
    m = _model(S, scattering_channels=widths[0], phase_channels=widths[1], cross_phase_channels=widths[2])
    tr = Trainer(m, lr=1e-3, frontend=fe)
    L = tr.step({"x": torch.from_numpy(x).cuda()}, eps=torch.from_numpy(eps).cuda())
    torch.cuda.synchronize()
    gn = float(L["grad_norm"])

    def member(seed):   # the oracle's fp32 step from one-ulp perturbed initial weights
        ref = perturb_ulp_(det_fill_(M.SeqVaeTebRef(S, *widths)), seed)
        T = lambda a: torch.from_numpy(np.asarray(a)).float()
        _, _, g, _ = M.train_step(ref, {"y_st": T(feats["fhr_st"]), "y_ph": T(feats["fhr_ph"]),
                                        "x_ph": T(feats["fhr_up_ph"]), "y_raw": T(feats["fhr"])}, T(eps), 1e-5)
        return g
    ENS = 4
    t0 = time.time()
    _, L_o, g_o, _ = _oracle_step(feats, eps, widths)
    t1 = time.time()
    _, _, g_o32, _ = _oracle_step(feats, eps, widths, torch.float32)
    members = [g_o32] + [member(s) for s in range(1, ENS + 1)]
    print(f"oracle steps at B={B}: fp64 {t1 - t0:.1f} s, {ENS + 1} fp32 {time.time() - t1:.1f} s")
    for k in LOSSES:
        exp = L_o[k].item()
        assert abs(L[k].item() - exp) <= 1e-5 * abs(exp) + 1e-7, (k, L[k].item(), exp)
    norm = lambda gs: torch.sqrt(sum((g.double() ** 2).sum() for g in gs)).item()
    gn_o = norm(g_o.values())
    params = dict(m.named_parameters())
    heads = {k for k, p in params.items() if p.numel() >= 1 << 20}
    assert len(heads) == 4, heads
    flat = lambda gs: torch.cat([g.detach().double().cpu().reshape(-1) for g in gs])
    go = flat(g_o[k] for k in g_o)
    names = [k for k in g_o if k not in heads and g_o[k].norm() > 0]

    def dist(g):   # (norm gap, whole-gradient rel-L2, per-gradient rel-L2 of the non-head gradients)
        return (abs(norm(g[k] for k in g_o) - gn_o) / gn_o, (flat(g[k] for k in g_o) - go).norm().item() / go.norm().item(),
                np.array([rel(g[k], g_o[k]) for k in names]))
    ours = dist({k: params[k].grad for k in g_o})
    ens = [dist(g) for g in members]
    # the well-conditioned gradients: those the plain fp32 oracle step gets within 1e-3 of fp64
    good = ens[0][2] < 1e-3
    assert good.sum() >= 300, good.sum()
    gn_d = norm(p.grad for p in params.values())
    print(f"grad norm: ours {gn:.7f} (fp64 norm of our gradients {gn_d:.7f}), oracle fp64 {gn_o:.7f}")
    for tag, (ng, ev, per) in [("ours", ours)] + [(f"fp32 member {i}", e) for i, e in enumerate(ens)]:
        print(f"  {tag}: norm gap {ng:.3e}, whole-gradient rel-L2 {ev:.3e}, over {good.sum()} well-conditioned "
              f"non-head gradients median {np.median(per[good]):.3e} p90 {np.percentile(per[good], 90):.3e} "
              f"max {per[good].max():.3e}")
    hn = {}
    for k in sorted(heads):
        hn[k] = (params[k].grad.double().norm().item(), g_o[k].double().norm().item(), g_o32[k].double().norm().item())
        print(f"{k}: |grad| ours {hn[k][0]:.7f}, oracle fp64 {hn[k][1]:.7f}, fp32 {hn[k][2]:.7f}; rel-L2 ours "
              f"{rel(params[k].grad, g_o[k]):.3e}, oracle fp32 {rel(g_o32[k], g_o[k]):.3e}")
    env = np.max(np.stack([e[2] for e in ens]), 0)     # per gradient: the ensemble's largest distance
    table = sorted(zip(ours[2], env, names), reverse=True)
    for e, e32, k in table[:10]:
        print(f"  worst: {k}: ours {e:.3e}, fp32 ensemble max {e32:.3e}")
    env_ng, env_ev = max(e[0] for e in ens), max(e[1] for e in ens)
    env_med = max(np.median(e[2][good]) for e in ens)
    env_p90 = max(np.percentile(e[2][good], 90) for e in ens)
    assert abs(gn - gn_d) <= 1e-6 * gn_d, (gn, gn_d)
    assert ours[0] <= 1.5 * env_ng + 1e-6, (ours[0], env_ng)
    assert ours[1] <= 1.5 * env_ev, (ours[1], env_ev)
    assert np.median(ours[2][good]) <= 1.5 * env_med, (np.median(ours[2][good]), env_med)
    assert np.percentile(ours[2][good], 90) <= 1.5 * env_p90, (np.percentile(ours[2][good], 90), env_p90)
    for k, (a, e, e32_) in hn.items():
        assert abs(a - e) <= max(1e-5 * e, 2 * abs(e32_ - e)), (k, a, e, e32_)
    worst = max((e / (2e-5 + 10 * e32), k) for e, e32, k in table)
    assert worst[0] <= 1.0, worst
