"""Reference-API mirrors on the GPU: kymatio backend plugin `torch_hip`,
Scattering1D frontend (fused and generic paths) and KymatioPhaseScattering1D,
against kymatio's own known answers / backend tests and the reference's
golden outputs (tolerances as in test_gpu_frontend.py)."""
import numpy as np
import pytest
import torch

from oracle import frontend_ref as F

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def bk():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from vaeteb.scattering import TorchHipBackend1D
    return TorchHipBackend1D


def rel(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return np.sqrt((np.abs(a - b) ** 2).sum() / max((np.abs(b) ** 2).sum(), 1e-30))


# ------------------------------------------------------------ backend plugin
def test_backend_name_and_checks(bk):
    assert bk.name.startswith("torch")
    with pytest.raises(TypeError, match="should be complex"):
        bk.subsample_fourier(torch.randn(4, device="cuda"), 1)
    with pytest.raises(RuntimeError, match="contiguous"):
        bk.modulus(torch.randn(4, 6, 2, device="cuda").transpose(0, 1))
    with pytest.raises(ValueError, match="Indefinite padding"):
        bk.pad(torch.randn(2, 8, device="cuda"), 8, 1)


def test_pad_unpad(bk):
    # ref/kymatio/tests/scattering1d/test_torch_backend_1d.py:31-87, :177-197 semantics
    x = torch.randn(3, 5, 16, device="cuda")
    p = bk.pad(x, 7, 5)
    exp = np.pad(x.cpu().numpy(), ((0, 0), (0, 0), (7, 5)), mode="reflect")
    assert p.shape == (3, 5, 28, 1) and np.allclose(p[..., 0].cpu().numpy(), exp)
    assert torch.equal(bk.unpad(p, 7, 23), x)


@pytest.mark.parametrize("j", range(0, 8))
def test_subsample_fourier_is_time_subsampling(bk, j):
    # ref/kymatio/tests/scattering1d/test_torch_backend_1d.py:141-172
    rng = np.random.RandomState(42)
    x = rng.randn(2, 4, 2 ** 10) + 1j * rng.randn(2, 4, 2 ** 10)
    xf = np.fft.fft(x, axis=-1)
    xf_t = torch.from_numpy(np.stack([xf.real, xf.imag], -1).astype(np.float32)).cuda()
    sub = bk.subsample_fourier(xf_t, 2 ** j).cpu().numpy()
    xs = np.fft.ifft(sub[..., 0] + 1j * sub[..., 1], axis=-1)
    assert np.allclose(x[:, :, ::2 ** j], xs, atol=1e-5)


def test_fft_family_and_modulus_grad(bk):
    torch.manual_seed(0)
    x = torch.randn(3, 256, 2, device="cuda")
    xc = x[..., 0].double().cpu() + 1j * x[..., 1].double().cpu()
    f = bk.fft(x)
    assert rel(f[..., 0].cpu() + 1j * f[..., 1].cpu(), np.fft.fft(xc.numpy())) < 2e-6
    i = bk.ifft(x)
    assert rel(i[..., 0].cpu() + 1j * i[..., 1].cpu(), np.fft.ifft(xc.numpy())) < 2e-6
    r = torch.randn(3, 256, 1, device="cuda")
    rf = bk.rfft(r)
    assert rel(rf[..., 0].cpu() + 1j * rf[..., 1].cpu(), np.fft.fft(r[..., 0].double().cpu().numpy())) < 2e-6
    assert rel(bk.irfft(rf).cpu(), r.cpu()) < 2e-6
    # modulus + ModulusStable gradient (zero subgradient at 0)
    z = torch.randn(2, 64, 2, device="cuda")
    z[0, 0] = 0
    z.requires_grad_(True)
    m = bk.modulus(z)
    assert m.shape == (2, 64, 1)
    m.sum().backward()
    zz = z.detach()
    exp = zz / zz.norm(dim=-1, keepdim=True)
    exp[0, 0] = 0
    assert torch.allclose(z.grad, exp, atol=1e-6)


@pytest.mark.parametrize("n,rows", [(16384, 3), (32768, 2), (1 << 17, 1)])
def test_fft_four_step_long(bk, n, rows):
    """n > 8192 (config 5: n_pad = 32768) runs the four-step vt_fft_large
    (256-point column FFTs + twiddles, then n/256-point row FFTs): rel-L2 vs
    numpy fp64 <= 3e-6 (fp32, two passes of log2 n radix-4 stages)."""
    torch.manual_seed(n)
    x = torch.randn(rows, n, 2, device="cuda")
    xc = x[..., 0].double().cpu().numpy() + 1j * x[..., 1].double().cpu().numpy()
    f = bk.fft(x)
    assert rel(f[..., 0].cpu() + 1j * f[..., 1].cpu(), np.fft.fft(xc)) < 3e-6
    i = bk.ifft(x)
    assert rel(i[..., 0].cpu() + 1j * i[..., 1].cpu(), np.fft.ifft(xc)) < 3e-6
    assert rel(bk.ifft(f).cpu(), x.cpu()) < 3e-6


def test_cdgmm_real_and_complex(bk):
    A = torch.randn(2, 3, 16, 2, device="cuda")
    Br = torch.randn(16, 1, device="cuda")
    Bc = torch.randn(16, 2, device="cuda")
    Ac = A[..., 0] + 1j * A[..., 1]
    out = bk.cdgmm(A, Br)
    assert torch.allclose(out[..., 0] + 1j * out[..., 1], Ac * Br[..., 0], atol=1e-6)
    out = bk.cdgmm(A, Bc)
    assert torch.allclose(out[..., 0] + 1j * out[..., 1], Ac * (Bc[..., 0] + 1j * Bc[..., 1]), atol=1e-6)
    with pytest.raises(RuntimeError, match="not compatible"):
        bk.cdgmm(A, torch.randn(8, 2, device="cuda"))


# ------------------------------------------------------------ Scattering1D
def test_kymatio_known_answer_generic_path(golden):
    """kymatio's shipped test_data_1d.npz (J=6, Q=16, N=512, T=2^J, order 2) through
    the generic core over the HIP backend plugin."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from vaeteb.scattering import Scattering1D
    d = golden("kymatio_test_data_1d")
    x = torch.from_numpy(d["x"]).cuda()
    sc = Scattering1D(int(d["J"]), x.shape[-1], int(d["Q"]))
    for cascade in (True, False):
        sc.cascade = cascade
        S, _ = sc(x)
        assert S.shape == d["Sx"].shape
        assert np.allclose(S.cpu().numpy(), d["Sx"], rtol=1e-4, atol=1e-6)   # fp32 FFT engine differs from torch's


@pytest.mark.parametrize("name,fused", [("j11q4t16_n4096_o1", True), ("j6q1t16_n4096_o1", True),
                                        ("j6q1t16_n4096_o2", False), ("j8q12t256_n16384_o2", False)])
def test_scattering1d_vs_reference_golden(golden, name, fused):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import re
    from vaeteb.scattering import Scattering1D
    g = golden("scattering_" + name)
    J, Q, T, N, o = map(int, re.findall(r"\d+", name))
    sc = Scattering1D(J=J, shape=N, Q=Q, max_order=o, T=T)
    assert sc._fused_ok() == fused
    # non-fused configurations: the level-grouped cascade and the per-filter generic core
    for cascade in ((True,) if fused else (True, False)):
        sc.cascade = cascade
        S, S2 = sc(torch.from_numpy(g["x"]).cuda())
        assert S is S2 and S.shape == g["S"].shape
        got, exp64, ref32 = S.cpu().numpy(), g["S64"], g["S"]
        e = np.sqrt(((got - exp64) ** 2).sum(-1) / (exp64 ** 2).sum(-1))
        r = np.sqrt(((ref32 - exp64) ** 2).sum(-1) / (exp64 ** 2).sum(-1))
        assert e.max() <= 2 * r.max() + 1e-6, (cascade, e.max(), r.max())


# ------------------------------------------------ KymatioPhaseScattering1D
@pytest.fixture(scope="module")
def kps():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from vaeteb.frontend import KymatioPhaseScattering1D
    return KymatioPhaseScattering1D(J=11, Q=4, T=16, shape=4096, device=torch.device("cuda"), max_order=1)


def test_phase_module_all_903_pairs_vs_reference(golden, kps):
    g = golden("frontend_j11q4t16_n4096")
    x = torch.from_numpy(g["x"]).cuda()
    sel = kps.get_optimal_coefficients_for_fhr(11, 4, 16)
    assert (sel["recommendations"]["use_phase_mask"].cpu().numpy() == g["phase_mask"]).all()
    assert (sel["recommendations"]["use_cross_mask"].cpu().numpy() == g["cross_mask"]).all()
    rp = kps(x, compute_phase=True, compute_cross_phase=False, scattering_channel=0, phase_channels=[0])
    full = rp["phase_corr"].cpu().numpy()
    assert full.shape == g["phase_full"].shape and rp["autoc_idx"].numel() == 42
    # all-pair output against the fp64 oracle, scale-normalised, bounded by the
    # reference's fp32 outputs' own error distribution
    o64 = F.PhaseFrontEnd(11, 4, 16, 4096, dtype=np.float64)
    r64 = o64.forward(g["x"], compute_phase=True)["phase_corr"]
    a64 = o64.analytic(g["x"][:, 0])
    scale = np.sqrt((o64._lowpass(np.abs(a64[:, o64.i_idx]) * np.abs(a64[:, o64.j_idx]) + 0j, 256) ** 2).sum(-1))
    err = np.sqrt(((full - r64) ** 2).sum(-1)) / scale
    ref = np.sqrt(((g["phase_full"] - r64) ** 2).sum(-1)) / scale
    assert err.max() <= 2 * ref.max() + 1e-5 and np.median(err) <= 2 * np.median(ref) + 1e-6
    assert np.allclose(rp["scattering"].cpu().numpy(), g["fhr_st"], rtol=1e-3, atol=1e-4)


@pytest.mark.parametrize("border", ["reflect", "constant", "circular"])
@pytest.mark.parametrize("same_pairs,low_pass", [(False, True), (True, True), (True, False)])
def test_phase_module_cross_options(border, same_pairs, low_pass):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from vaeteb import synthetic
    from vaeteb.frontend import KymatioPhaseScattering1D
    m = KymatioPhaseScattering1D(J=6, Q=1, T=16, shape=4096, device=torch.device("cuda"), max_order=1,
                                 border_mode=border)
    x = synthetic.batch(77, 2, 4096)
    r = m(torch.from_numpy(x).cuda(), compute_phase=False, compute_cross_phase=True,
          cross_phase_same_pairs_only=same_pairs, cross_phase_low_pass=low_pass)["cross_phase_corr"].cpu().numpy()
    o = F.PhaseFrontEnd(6, 1, 16, 4096, dtype=np.float64)
    o.border_mode = border
    a = o.analytic(x[:, [0, 1]])
    sel = o.autoc_idx if same_pairs else np.arange(len(o.i_idx))
    ii, jj, pw = o.i_idx[sel], o.j_idx[sel], o.powers[sel]
    c = o._accelerate(a[:, 0][:, ii], pw[None, :, None]) * np.conj(a[:, 1][:, jj])
    exp = o._lowpass(c, 256) if low_pass else c.real
    assert r.shape == exp.shape
    scale = np.sqrt((np.abs(c) ** 2).sum(-1)) if not low_pass else \
        np.sqrt((o._lowpass(np.abs(c) + 0j, 256) ** 2).sum(-1))
    err = np.sqrt(((r - exp) ** 2).sum(-1)) / scale
    assert np.median(err) < 1e-5 and err.max() < 1e-3


def test_phase_module_input_validation(kps):
    with pytest.raises(ValueError):
        kps(torch.zeros(2, 3, 4, 4096, device="cuda"))
    with pytest.raises(ValueError):
        kps(torch.zeros(2, 4096, device="cuda"), compute_cross_phase=True)
    with pytest.raises(ValueError):
        kps(torch.zeros(2, 2, 4096, device="cuda"), scattering_channel=2)
