"""HIP front-end vs the oracle and the reference's golden outputs (MI355X).

Tolerances (DESIGN.md "Parity tolerances"):
  * FFT rows: relative L2 <= 2e-6 vs numpy fp64.
  * analytic signals / scattering: relative L2 per row vs the fp64 oracle,
    bounded (max and median over rows) by 2x the error of the oracle run in
    fp32 with torch.fft — the reference's own FFT engine and precision
    (oracle.frontend_ref.FFT_ENGINE = "torch") — plus a 1e-6 floor.
  * phase-harmonic pairs: errors normalised by the cancellation-free scale
    ||lowpass(|a_i||a_j|)||; the max and median over channels must stay
    within 2x the reference's (or the fp32 oracle's) own fp32-vs-fp64 error
    (+1e-5 / +1e-6 floors) — see tests/test_oracle.py for why per-channel
    agreement between fp32 implementations is not attainable.
"""
import numpy as np
import pytest
import torch

from oracle import frontend_ref as F

pytestmark = pytest.mark.gpu


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda")


def rel_rows(a, b):
    return np.sqrt((np.abs(a - b) ** 2).sum(-1) / np.maximum((np.abs(b) ** 2).sum(-1), 1e-30))


def torch_engine(fn, *a, **k):
    """Run an oracle call with the reference's FFT engine (torch.fft, CPU fp32)."""
    old = F.FFT_ENGINE
    F.FFT_ENGINE = "torch"
    try:
        return fn(*a, **k)
    finally:
        F.FFT_ENGINE = old


def assert_ref_precision(err, ref_err, floor_max=1e-6, floor_med=1e-7, what=""):
    assert err.max() <= 2 * ref_err.max() + floor_max, (what, err.max(), ref_err.max())
    assert np.median(err) <= 2 * np.median(ref_err) + floor_med, (what, np.median(err), np.median(ref_err))


@pytest.fixture(scope="module")
def lib():
    from vaeteb import _lib
    return _lib


@pytest.mark.parametrize("n", [4, 8, 16, 32, 64, 128, 256, 512, 1024, 2048, 4096, 8192])
@pytest.mark.parametrize("inverse", [0, 1])
def test_fft_rows(lib, n, inverse):
    dev = _dev()
    from vaeteb.filter_bank import twiddles
    rng = np.random.default_rng(n)
    x = (rng.standard_normal((5, n)) + 1j * rng.standard_normal((5, n))).astype(np.complex64)
    xt = torch.from_numpy(x).to(dev)
    out = torch.empty_like(xt)
    # a length-n FFT read from the 8192 table with stride (tests the strided twiddle path)
    tw = torch.from_numpy(twiddles(8192)).to(dev)
    lib.call("vt_fft", xt.data_ptr(), out.data_ptr(), 5, n, inverse, tw.data_ptr(), 8192 // n, lib.stream())
    ref = np.fft.ifft(x.astype(np.complex128)) if inverse else np.fft.fft(x.astype(np.complex128))
    assert rel_rows(out.cpu().numpy(), ref).max() < 2e-6


@pytest.fixture(scope="module")
def fe11():
    dev = _dev()
    from vaeteb.frontend import FrontEnd, FrontEndPlan, load_stats
    return FrontEnd(FrontEndPlan(11, 4, 16, 4096, device=dev), load_stats(11, 4, 16, 4096))


@pytest.fixture(scope="module")
def fe6():
    dev = _dev()
    from vaeteb.frontend import FrontEnd, FrontEndPlan, load_stats
    return FrontEnd(FrontEndPlan(6, 1, 16, 4096, device=dev), load_stats(6, 1, 16, 4096))


def _golden_x(golden, J, Q):
    return golden(f"frontend_j{J}q{Q}t16_n4096")


@pytest.mark.parametrize("cfg", ["fe11", "fe6"])
def test_scattering_vs_oracle(request, cfg):
    fe = request.getfixturevalue(cfg)
    p = fe.plan
    from vaeteb import synthetic
    x = synthetic.batch(500, 4, 4096)
    r = fe.raw(torch.from_numpy(x).cuda())
    S = r["fhr_st"].cpu().numpy()
    S64 = F.scattering1d(x[:, 0], p.J, p.Q, p.T, 1, dtype=np.float64)
    S32 = torch_engine(F.scattering1d, x[:, 0], p.J, p.Q, p.T, 1)
    assert S.shape == S64.shape
    assert_ref_precision(rel_rows(S, S64), rel_rows(S32, S64), what="scattering")


@pytest.fixture(scope="module")
def fe11_5760():
    dev = _dev()
    from vaeteb.frontend import FrontEnd, FrontEndPlan, load_stats
    return FrontEnd(FrontEndPlan(11, 4, 16, 5760, device=dev), load_stats(11, 4, 16, 4096))


@pytest.mark.parametrize("J,Q,N", [(11, 4, 4096), (6, 1, 4096), (11, 4, 5760)])
def test_frontend_vs_reference_golden(golden, request, J, Q, N):
    """Feed the reference's fixture windows; compare against the reference's own outputs.
    N = 5760 is the reference's own dataset window (create_hdf5_dataset.py:360: 360 steps)."""
    fe = request.getfixturevalue({(11, 4096): "fe11", (6, 4096): "fe6", (11, 5760): "fe11_5760"}[(J, N)])
    g = golden(f"frontend_j{J}q{Q}t16_n{N}")
    x = g["x"]
    r = fe.raw(torch.from_numpy(x).cuda())
    assert_ref_precision(rel_rows(r["fhr_st"].cpu().numpy(), g["fhr_st64"]), rel_rows(g["fhr_st"], g["fhr_st64"]),
                         what="fhr_st")
    pairs = r["pairs"].cpu().numpy()
    nph = fe.C_ph
    fe64 = F.PhaseFrontEnd(J, Q, 16, N, dtype=np.float64)
    a64 = fe64.analytic(x[:, [0, 1]])
    pm, cm = g["phase_mask"], g["cross_mask"]
    for key, out, sel, ai, aj in (("fhr_ph", pairs[:, :nph], pm, a64[:, 0], a64[:, 0]),
                                  ("fhr_up_ph", pairs[:, nph:], cm, a64[:, 0], a64[:, 1])):
        ii, jj = fe64.i_idx[sel], fe64.j_idx[sel]
        scale = np.sqrt((fe64._lowpass(np.abs(ai[:, ii]) * np.abs(aj[:, jj]) + 0j, fe.plan.S) ** 2).sum(-1))
        err = np.sqrt(((out - g[key + "64"]) ** 2).sum(-1)) / scale
        ref_err = np.sqrt(((g[key] - g[key + "64"]) ** 2).sum(-1)) / scale
        assert err.max() <= 2 * ref_err.max() + 1e-5, (key, err.max(), ref_err.max())
        assert np.median(err) <= 2 * np.median(ref_err) + 1e-6, (key, np.median(err), np.median(ref_err))


def test_analytic_signals(fe11):
    """The analytic slots in their complex form (vt_fe_set_analytic_polar(0)) vs the oracle;
    the default polar form {arg / 2 pi, |a|} is the same signal to fp32 rounding."""
    p, t = fe11.plan, fe11.tab
    from vaeteb import _lib, synthetic
    fns = _lib.lib().fns
    x = synthetic.batch(700, 2, 4096)
    prev = fns["vt_fe_set_analytic_polar"](1)
    try:
        fe11.raw(torch.from_numpy(x).cuda())
        pol = fe11._bufs["analytic"].double().cpu().numpy().copy()
        fns["vt_fe_set_analytic_polar"](0)
        fe11.raw(torch.from_numpy(x).cuda())
        an = torch.view_as_complex(fe11._bufs["analytic"]).cpu().numpy()
    finally:
        fns["vt_fe_set_analytic_polar"](prev)
    from_polar = pol[..., 1] * np.exp(2j * np.pi * pol[..., 0])
    used = sorted({int(s) for s in t["items"].cpu().numpy()[:, 2] if s >= 0})
    assert rel_rows(from_polar[:, used].reshape(-1, p.N), an[:, used].reshape(-1, p.N)).max() < 1e-6
    a64 = F.PhaseFrontEnd(11, 4, 16, 4096, dtype=np.float64).analytic(x[:, [0, 1]])
    a32 = torch_engine(F.PhaseFrontEnd(11, 4, 16, 4096).analytic, x[:, [0, 1]])
    items = t["items"].cpu().numpy()
    errs, ref_errs = [], []
    for chan, filt, slot, _, _ in items:
        if slot < 0:
            continue
        errs.append(rel_rows(an[:, slot], a64[:, chan, filt]))
        ref_errs.append(rel_rows(a32[:, chan, filt], a64[:, chan, filt]))
    assert_ref_precision(np.array(errs), np.array(ref_errs), what="analytic")


@pytest.mark.parametrize("B,polar", [(3, 0), (4, 0), (8, 0), (4, 1), (8, 1)])
def test_pairs_random_inputs_vs_oracle(fe11, B, polar):
    """Bigger random batch: HIP fp32 vs oracle fp64, distribution-bounded by the
    oracle's own fp32 error on the same inputs.  B = 4 / 8: every launch's item count
    (B x 44, B x 130, B x 174) is a multiple of 8, so the XCD-aware item order the bench
    runs (xcd_item, csrc/frontend.hip) is active; B = 3 keeps the identity order."""
    from vaeteb import _lib, synthetic
    x = synthetic.batch(900, B, 4096)
    prev = _lib.lib().fns["vt_fe_set_analytic_polar"](polar)   # polar = 1: the default polar slots
    try:
        r = fe11.raw(torch.from_numpy(x).cuda())
        pairs = r["pairs"].cpu().numpy()
    finally:
        _lib.lib().fns["vt_fe_set_analytic_polar"](prev)
    p = fe11.plan
    o32 = F.PhaseFrontEnd(11, 4, 16, 4096)
    o64 = F.PhaseFrontEnd(11, 4, 16, 4096, dtype=np.float64)
    a64 = o64.analytic(x[:, [0, 1]])
    nph = fe11.C_ph
    for key, sel, cross in (("ph", p.phase_mask, False), ("x", p.cross_mask, True)):
        r32 = torch_engine(o32.forward, x, compute_phase=not cross, compute_cross_phase=cross, pair_subset=sel)
        r64 = o64.forward(x, compute_phase=not cross, compute_cross_phase=cross, pair_subset=sel)
        k = "cross_phase_corr" if cross else "phase_corr"
        out = pairs[:, nph:] if cross else pairs[:, :nph]
        ii, jj = o64.i_idx[sel], o64.j_idx[sel]
        aj = a64[:, 1] if cross else a64[:, 0]
        scale = np.sqrt((o64._lowpass(np.abs(a64[:, 0][:, ii]) * np.abs(aj[:, jj]) + 0j, 256) ** 2).sum(-1))
        err = np.sqrt(((out - r64[k]) ** 2).sum(-1)) / scale
        ref_err = np.sqrt(((r32[k] - r64[k]) ** 2).sum(-1)) / scale
        assert err.max() <= 2 * ref_err.max() + 1e-5, (key, err.max(), ref_err.max())
        assert np.median(err) <= 2 * np.median(ref_err) + 1e-6, (key, np.median(err), np.median(ref_err))


def test_normalised_outputs(fe11):
    """Full fused path (raw -> log/asinh -> z-score -> (B,S,C)) vs oracle."""
    from vaeteb import synthetic
    from vaeteb.frontend import load_stats
    st = load_stats(11, 4, 16, 4096)
    x = synthetic.batch(1200, 2, 4096)
    out = fe11(torch.from_numpy(x).cuda())
    raw = fe11.raw(torch.from_numpy(x).cuda())
    S = raw["fhr_st"].cpu().numpy()
    pr = raw["pairs"].cpu().numpy()
    nph = fe11.C_ph
    exp = {"fhr_st": F.normalize(S, "fhr_st", st["fhr_st_mean"], st["fhr_st_variance"]),
           "fhr_ph": F.normalize(pr[:, :nph], "fhr_ph", st["fhr_ph_mean"], st["fhr_ph_variance"]),
           "fhr_up_ph": F.normalize(pr[:, nph:], "fhr_up_ph", st["fhr_up_ph_mean"], st["fhr_up_ph_variance"])}
    for k, e in exp.items():
        got = out[k].cpu().numpy().transpose(0, 2, 1)
        assert np.allclose(got, e, rtol=1e-5, atol=1e-5), k
    fhr = F.normalize(x[:, 0], "fhr", st["fhr_mean"], st["fhr_variance"])
    assert np.allclose(out["fhr"].cpu().numpy(), fhr, rtol=1e-6, atol=1e-6)


def test_wrong_shape_raises(fe11):
    with pytest.raises(ValueError):
        fe11.raw(torch.zeros(2, 1, 4096, device="cuda"))


def test_pairs_direct_columns_match_staged(fe11):
    """vt_fe_set_pairs_direct(1) (padded product columns formed in registers from
    HBM) against the default LDS-staged product: same per-sample arithmetic and
    FFT; the compiler contracts the product differently in the two paths, so they
    agree to fp32 rounding (1e-5 of the batch's largest coefficient), not bitwise."""
    from vaeteb import _lib, synthetic
    fns = _lib.lib().fns
    x = torch.from_numpy(synthetic.batch(901, 4, 4096)).cuda()
    prev = fns["vt_fe_set_pairs_direct"](0)
    try:
        staged = fe11.raw(x)["pairs"].clone()
        fns["vt_fe_set_pairs_direct"](1)
        direct = fe11.raw(x)["pairs"].clone()
    finally:
        fns["vt_fe_set_pairs_direct"](prev)
    torch.cuda.synchronize()
    diff = (staged - direct).abs().max().item()
    assert diff <= 1e-5 * staged.abs().max().item(), diff


def test_pairs_polar_slots_match_complex(fe11):
    """The pair features from polar analytic slots (the default, vt_fe_set_analytic_polar(1):
    |a_i| |a_j| and one fused angle per element) against the complex slots with the per-pair
    accelerated product: the same quantity in fp32, to 1e-5 of the batch's largest
    coefficient (and against the fp64 oracle: test_pairs_random_inputs_vs_oracle[polar])."""
    from vaeteb import _lib, synthetic
    fns = _lib.lib().fns
    x = torch.from_numpy(synthetic.batch(902, 4, 4096)).cuda()
    prev = fns["vt_fe_set_analytic_polar"](1)
    try:
        polar = fe11.raw(x)["pairs"].clone()
        fns["vt_fe_set_analytic_polar"](0)
        cplx = fe11.raw(x)["pairs"].clone()
    finally:
        fns["vt_fe_set_analytic_polar"](prev)
    torch.cuda.synchronize()
    diff = (polar - cplx).abs().max().item()
    assert diff <= 1e-5 * cplx.abs().max().item(), diff


def test_frontend_bench_batch_rows_equal_small_batch(fe11):
    """The front-end at the bench's batch (B = 256) vs a B = 4 run of its first four
    windows, bit for bit (every output is per sample; the XCD-aware item order is active
    in both, at different item counts, so this pins the remapped indexing at bench size)."""
    from vaeteb import synthetic
    x = torch.from_numpy(synthetic.batch(70_000, 256, 4096)).cuda()
    big = {k: v.clone() for k, v in fe11(x).items()}
    small = fe11(x[:4].contiguous())
    torch.cuda.synchronize()
    for k, v in small.items():
        assert big[k].shape[0] == 256, k
        assert torch.equal(big[k][:4], v), (k, (big[k][:4] - v).abs().max().item())
    raw_big = {k: v.clone() for k, v in fe11.raw(x).items()}
    raw_small = fe11.raw(x[252:].contiguous())     # the LAST four rows: the far end of the remap
    torch.cuda.synchronize()
    for k, v in raw_small.items():
        assert torch.equal(raw_big[k][252:], v), k


@pytest.mark.parametrize("B", [8, 64])
def test_pairs_persistent_kernel_bitwise(fe11, B):
    """k_fe_pairs8k_p (persistent workgroups, the one-wave inverse of item i overlapped with
    item i+1's product on the other seven waves) == the one-item-per-workgroup kernel, bit for
    bit; default grid and a small grid (many items per workgroup)."""
    from vaeteb import _lib, synthetic
    fns = _lib.lib().fns
    x = torch.from_numpy(synthetic.batch(5150, B, 4096)).cuda()
    prev = fns["vt_fe_set_pairs_persist"](0)
    prev_half = fns["vt_fe_set_pairs_half"](0)     # the full-image kernel the persistent form mirrors
    try:
        ref = fe11.raw(x)["pairs"].clone()
        fns["vt_fe_set_pairs_persist"](-1)
        got = fe11.raw(x)["pairs"].clone()
        fns["vt_fe_set_pairs_persist"](64)
        got_small = fe11.raw(x)["pairs"].clone()
    finally:
        fns["vt_fe_set_pairs_persist"](prev)
        fns["vt_fe_set_pairs_half"](prev_half)
    torch.cuda.synchronize()
    assert torch.equal(got, ref) and torch.equal(got_small, ref)


@pytest.mark.parametrize("B", [4, 8])
def test_pairs_full_image_kernel_vs_oracle(fe11, B):
    """The full-image pair kernel (k_fe_pairs8k, vt_fe_set_pairs_half(0), the default of rounds
    2-5) held to the fp64 oracle as the default half-image kernel is in
    test_pairs_random_inputs_vs_oracle; the two forms agree to fp32 rounding (other DFT-16
    factorisation and summation order: 1e-5 of the batch's largest coefficient, not bitwise)."""
    from vaeteb import _lib, synthetic
    fns = _lib.lib().fns
    x = synthetic.batch(903, B, 4096)
    xt = torch.from_numpy(x).cuda()
    half = fe11.raw(xt)["pairs"].clone()
    prev = fns["vt_fe_set_pairs_half"](0)
    try:
        full = fe11.raw(xt)["pairs"].clone()
    finally:
        fns["vt_fe_set_pairs_half"](prev)
    torch.cuda.synchronize()
    diff = (half - full).abs().max().item()
    assert diff <= 1e-5 * full.abs().max().item(), diff
    p = fe11.plan
    o64 = F.PhaseFrontEnd(11, 4, 16, 4096, dtype=np.float64)
    o32 = F.PhaseFrontEnd(11, 4, 16, 4096)
    a64 = o64.analytic(x[:, [0, 1]])
    nph = fe11.C_ph
    out_all = full.cpu().numpy()
    for sel, cross in ((p.phase_mask, False), (p.cross_mask, True)):
        r32 = torch_engine(o32.forward, x, compute_phase=not cross, compute_cross_phase=cross, pair_subset=sel)
        r64 = o64.forward(x, compute_phase=not cross, compute_cross_phase=cross, pair_subset=sel)
        k = "cross_phase_corr" if cross else "phase_corr"
        out = out_all[:, nph:] if cross else out_all[:, :nph]
        ii, jj = o64.i_idx[sel], o64.j_idx[sel]
        aj = a64[:, 1] if cross else a64[:, 0]
        scale = np.sqrt((o64._lowpass(np.abs(a64[:, 0][:, ii]) * np.abs(aj[:, jj]) + 0j, 256) ** 2).sum(-1))
        err = np.sqrt(((out - r64[k]) ** 2).sum(-1)) / scale
        ref_err = np.sqrt(((r32[k] - r64[k]) ** 2).sum(-1)) / scale
        assert err.max() <= 2 * ref_err.max() + 1e-5, (k, err.max(), ref_err.max())
        assert np.median(err) <= 2 * np.median(ref_err) + 1e-6, (k, np.median(err), np.median(ref_err))
