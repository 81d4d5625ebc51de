"""ORACLE — TEST INFRASTRUCTURE ONLY.  Never imported by the product path.

Plain-numpy CPU restatement of the reference front-end, used by tests/,
``__graft_entry__.smoke()`` and ``bench.py``'s cpu_baseline leg as the checker.
Pinned by tests/golden/*.npz, which were produced by running the reference
itself in the build container (tools/gen_golden.py) plus kymatio's own
known-answer file test_data_1d.npz.

Follows, structure for structure (FFT-domain periodisation, reflect padding,
crop-then-512-point-iFFT for the phase path):
  filter bank     ref/kymatio/kymatio/scattering1d/filter_bank.py:6-762
  padding/unpad   ref/kymatio/kymatio/scattering1d/utils.py:5-133
  Scattering1D    ref/kymatio/kymatio/scattering1d/core/scattering1d.py:197-399
                  (+ backend ops ref/kymatio/kymatio/scattering1d/backend/torch_backend.py:17-174)
  phase front-end ref/hdf5_dataset/kymatio_phase_scattering.py:60-760
  normalisation   ref/hdf5_dataset/hdf5_dataset.py:18-137

``dtype`` selects float32 (the reference's precision: complex64 filters,
``kymatio_phase_scattering.py:124-125``) or float64 (tolerance derivation).
"""
import math

import numpy as np


# ----------------------------------------------------------------- filter bank
def _adaptive_P(sigma, eps=1e-7):                       # filter_bank.py:6-48
    return int(math.ceil(math.sqrt(-2 * sigma ** 2 * math.log(eps)) + 1))


def _periodize(h, nper):                                # filter_bank.py:51-71 (mean!)
    return h.reshape(nper, h.shape[0] // nper).mean(axis=0)


def _l1_factor(hf):                                     # filter_bank.py:139-165
    return 1.0 / np.abs(np.fft.ifft(hf)).sum()


def morlet(N, xi, sigma, P_max=5, eps=1e-7):            # filter_bank.py:74-136
    P = min(_adaptive_P(sigma, eps), P_max)
    f = np.arange((1 - P) * N, P * N, dtype=float) / float(N)
    flow = np.fft.fftfreq(N) if P == 1 else f
    gab = _periodize(np.exp(-(f - xi) ** 2 / (2 * sigma ** 2)), 2 * P - 1)
    low = _periodize(np.exp(-(flow ** 2) / (2 * sigma ** 2)), 2 * P - 1)
    m = gab - (gab[0] / low[0]) * low
    return m * _l1_factor(m)


def gauss(N, sigma, P_max=5, eps=1e-7):                 # filter_bank.py:168-216
    P = min(_adaptive_P(sigma, eps), P_max)
    flow = np.fft.fftfreq(N) if P == 1 else np.arange((1 - P) * N, P * N, dtype=float) / float(N)
    g = _periodize(np.exp(-flow ** 2 / (2 * sigma ** 2)), 2 * P - 1)
    return g * _l1_factor(g)


def _sigma_psi(xi, Q, r=math.sqrt(0.5)):                 # filter_bank.py:219-251
    f = 1.0 / 2 ** (1.0 / Q)
    return xi * (1 - f) / (1 + f) / math.sqrt(2 * math.log(1.0 / r))


def _max_sub(xi, sigma, alpha=5.0):                      # filter_bank.py:306-337
    return int(math.floor(-math.log2(min(xi + alpha * sigma, 0.5))) - 1)


def _bank_params(sigma_min, Q, r=math.sqrt(0.5), alpha=5.0):   # filter_bank.py:412-487
    xi_max = max(1.0 / (1.0 + 2 ** (3.0 / Q)), 0.35)
    s_max = _sigma_psi(xi_max, Q, r)
    xs, ss, js = [], [], []
    if s_max <= sigma_min:
        last = s_max
    else:
        xi, s, j = xi_max, s_max, 0
        f = 1.0 / 2 ** (1.0 / Q)
        while s > sigma_min:
            xs.append(xi); ss.append(s); js.append(j)
            xi, s = xi * f, s * f
            j = _max_sub(xi, s, alpha)
        last = xs[-1]
    for q in range(1, Q):
        nx = (Q - q) / float(Q) * last
        xs.append(nx); ss.append(sigma_min); js.append(_max_sub(nx, sigma_min, alpha))
    return xs, ss, js


def filter_bank(J_support, J, Q, T, sigma0=0.1):         # filter_bank.py:490-762
    smin = sigma0 / 2 ** J
    x1, s1, j1 = _bank_params(smin, Q)
    x2, s2, j2 = _bank_params(smin, 1)
    N = 2 ** J_support
    psi2 = []
    for xi, s, j in zip(x2, s2, j2):
        sub = [a for a in j1 if j > a]
        lv = [morlet(N, xi, s)]
        lv += [_periodize(lv[0], 2 ** l) for l in range(1, (max(sub) if sub else 0) + 1)]
        psi2.append(dict(levels=lv, xi=xi, sigma=s, j=j))
    psi1 = [dict(levels=[morlet(N, xi, s)], xi=xi, sigma=s, j=j) for xi, s, j in zip(x1, s1, j1)]
    phi0 = gauss(N, sigma0 / T)
    phi = dict(levels=[phi0] + [_periodize(phi0, 2 ** l) for l in range(1, max(max(j1), max(j2)) + 1)],
               xi=0, sigma=sigma0 / T, j=0)
    # compute_temporal_support (filter_bank.py:254-303) on phi level 0
    h = np.abs(np.fft.ifft(phi0))[: N // 2]
    resid = np.cumsum(h[::-1])[::-1]
    ok = np.where(resid <= 1e-3)[0]
    t_max = int(ok.min() + 1) if ok.size else N // 2
    return phi, psi1, psi2, t_max


def padding_plan(N, J, Q, T):
    """J_pad, pad_left/right and border indices (base_frontend.py:27-77,
    utils.py:5-133)."""
    _, _, _, t_max = filter_bank(int(np.ceil(np.log2(N))), J, Q, T)
    min_pad = 3 * t_max
    J_pad = min(int(np.ceil(np.log2(N + 2 * min_pad))), int(np.floor(np.log2(3 * N - 2))))
    add = 2 ** J_pad - N
    pl, pr = add // 2, add - add // 2
    i0, i1 = {0: pl}, {0: pl + N}
    for j in range(1, J + 1):
        i0[j] = i0[j - 1] // 2 + i0[j - 1] % 2
        i1[j] = i1[j - 1] // 2 + i1[j - 1] % 2
    return J_pad, pl, pr, i0, i1


# ------------------------------------------------------------------ Scattering1D
def _sub(xf, k):                                          # torch_backend.py:18-48
    return xf.reshape(xf.shape[:-1] + (k, xf.shape[-1] // k)).mean(axis=-2)


# FFT engine: numpy (pocketfft) by default.  FFT_ENGINE = "torch" runs the
# transforms through torch.fft on the CPU — the engine the reference itself
# uses (torch_backend.py:7-9, kymatio_phase_scattering.py:223,236,252) — which
# the tests use to measure the reference's own fp32 rounding level.
FFT_ENGINE = "numpy"


def _fft(x, axis=-1):
    if FFT_ENGINE == "torch":
        import torch
        return torch.fft.fft(torch.from_numpy(np.ascontiguousarray(x)), dim=axis).numpy()
    return np.fft.fft(x, axis=axis)


def _ifft(x, axis=-1):
    if FFT_ENGINE == "torch":
        import torch
        return torch.fft.ifft(torch.from_numpy(np.ascontiguousarray(x)), dim=axis).numpy()
    return np.fft.ifft(x, axis=axis)


def scattering1d(x, J, Q, T, max_order=1, dtype=np.float32):
    """Averaged, vectorised Scattering1D (oversampling=0), returns (B, C, S)."""
    x = np.asarray(x)
    N = x.shape[-1]
    J_pad, pl, pr, i0, i1 = padding_plan(N, J, Q, T)
    phi, psi1, psi2, _ = filter_bank(J_pad, J, Q, T)
    rd, cd = np.dtype(dtype), (np.complex64 if dtype == np.float32 else np.complex128)
    cast = lambda a: np.asarray(a, rd)
    x = x.astype(rd).reshape(-1, N)
    U0 = np.pad(x, ((0, 0), (pl, pr)), mode="reflect")    # torch reflect == numpy reflect
    U0h = _fft(U0.astype(cd), axis=-1).astype(cd)
    lt = int(math.floor(math.log2(T)))
    out = [_ifft(_sub(U0h * cast(phi["levels"][0]), 2 ** lt)).real[:, i0[lt]:i1[lt]]]
    s2 = []
    for p1 in psi1:
        k1 = max(min(p1["j"], lt), 0)
        U1c = _ifft(_sub(U0h * cast(p1["levels"][0]), 2 ** k1)).astype(cd)
        U1 = np.abs(U1c).astype(rd)
        U1h = _fft(U1.astype(cd)).astype(cd)
        kJ = max(lt - k1, 0)
        out.append(_ifft(_sub(U1h * cast(phi["levels"][k1]), 2 ** kJ)).real[:, i0[kJ + k1]:i1[kJ + k1]])
        if max_order == 2:
            for p2 in psi2:
                if p2["j"] > p1["j"]:
                    k2 = max(min(p2["j"] - k1, lt - k1), 0)
                    U2 = np.abs(_ifft(_sub(U1h * cast(p2["levels"][k1]), 2 ** k2)).astype(cd)).astype(rd)
                    U2h = _fft(U2.astype(cd)).astype(cd)
                    k2J = max(lt - k2 - k1, 0)
                    s2.append(_ifft(_sub(U2h * cast(phi["levels"][k1 + k2]), 2 ** k2J)).real
                              [:, i0[k1 + k2 + k2J]:i1[k1 + k2 + k2J]])
    return np.stack(out + s2, axis=1).astype(rd)


# ------------------------------------------------------------- phase front-end
class PhaseFrontEnd:
    """Restatement of KymatioPhaseScattering1D (kymatio_phase_scattering.py:11)."""

    def __init__(self, J, Q, T, N, max_order=1, dtype=np.float32):
        self.J, self.Q, self.T, self.N, self.max_order = J, Q, T, N, max_order
        self.dtype = np.dtype(dtype)
        self.cdtype = np.complex64 if self.dtype == np.float32 else np.complex128
        self.J_pad, self.pl, self.pr, self.i0, self.i1 = padding_plan(N, J, Q, T)   # :100-113
        phi, psi1, _, _ = filter_bank(self.J_pad, J, Q, T)                            # :115-132
        self.psi1 = np.stack([p["levels"][0] for p in psi1]).astype(np.complex64).astype(self.cdtype)
        self.phi = phi["levels"][0].astype(np.complex64).astype(self.cdtype)
        self.xi = np.array([p["xi"] for p in psi1], np.float32)
        ii, jj, pw = [], [], []                                                        # :134-160
        for i in range(len(self.xi)):
            for j in range(len(self.xi)):
                if self.xi[j] >= self.xi[i]:
                    ii.append(i); jj.append(j)
                    pw.append(np.float32(self.xi[j] / self.xi[i]) if self.xi[i] > 1e-8 else np.float32(1.0))
        self.i_idx, self.j_idx = np.array(ii), np.array(jj)
        self.powers = np.array(pw, np.float32)
        self.autoc_idx = np.array([k for k in range(len(ii)) if ii[k] == jj[k]])

    # masks: get_optimal_coefficients_for_fhr (:635-760)
    def masks(self):
        xi, pw, ii, jj = self.xi, self.powers, self.i_idx, self.j_idx
        mn = 0.006 if self.J >= 11 else 0.003
        f = xi >= mn
        auto = np.zeros(len(ii), bool); auto[self.autoc_idx] = True
        phase = f[ii] & f[jj] & auto
        for r in (2, 3):
            phase |= f[ii] & f[jj] & (np.abs(pw - r) < 0.1) & (pw <= 8)
        cross = (xi < 0.02)[ii] & ((xi >= 0.04) & (xi <= 0.5))[jj] & (pw >= 1) & (pw <= 32)
        return phase, cross

    border_mode = "reflect"                                                          # :162-172

    def _reflect(self, x):                                                           # :174-205
        if self.border_mode == "constant":
            return np.pad(x, [(0, 0)] * (x.ndim - 1) + [(self.pl, self.pr)], mode="constant")
        if self.border_mode == "circular":
            return np.pad(x, [(0, 0)] * (x.ndim - 1) + [(self.pl, self.pr)], mode="wrap")
        left, right = self.pl, self.pr
        while left > 0:
            c = min(left, x.shape[-1] - 1)
            x = np.concatenate([x[..., 1:c + 1][..., ::-1], x], axis=-1); left -= c
        while right > 0:
            c = min(right, x.shape[-1] - 1)
            x = np.concatenate([x, x[..., -c - 1:-1][..., ::-1]], axis=-1); right -= c
        return x

    def analytic(self, x):                                                           # :220-231
        xf = _fft(self._reflect(x.astype(self.dtype)).astype(self.cdtype), axis=-1).astype(self.cdtype)
        a = _ifft(xf[..., None, :] * self.psi1, axis=-1).astype(self.cdtype)
        return a[..., self.i0[0]:self.i1[0]]

    def _accelerate(self, a, p):                                                     # :211-218
        mag = np.abs(a).astype(self.dtype)
        ph = (np.arctan2(a.imag, a.real).astype(self.dtype) * p).astype(self.dtype)
        return (mag * (np.cos(ph) + 1j * np.sin(ph)).astype(self.cdtype)).astype(self.cdtype)

    def _lowpass(self, c, target):                                                   # :233-273
        dec = max(1, min(c.shape[-1], c.shape[-1] // target)) if (target > 0 and c.shape[-1] > target) else 1
        cf = _fft(self._reflect(c), axis=-1).astype(self.cdtype) * self.phi
        if dec > 1:
            cf = cf[..., :max(cf.shape[-1] // dec, 1)]
            sm = _ifft(cf, axis=-1).astype(self.cdtype)
            s0 = self.pl // dec
            sm = sm[..., s0:min(s0 + self.N // dec, sm.shape[-1])]
        else:
            sm = _ifft(cf, axis=-1)[..., self.i0[0]:self.i1[0]]
        return sm.real.astype(self.dtype)

    def pairs(self, a_i, a_j, powers, target):
        out = []
        for k in range(0, a_i.shape[1], 64):            # chunk to bound memory
            c = self._accelerate(a_i[:, k:k + 64], powers[None, k:k + 64, None]) * np.conj(a_j[:, k:k + 64])
            out.append(self._lowpass(c.astype(self.cdtype), target))
        return np.concatenate(out, axis=1)

    def forward(self, x, compute_phase=True, compute_cross_phase=False, pair_subset=None):
        """x: (B, 2, N) [ch0 = fhr, ch1 = up].  Mirrors forward (:394-473) for the
        two calls of create_hdf5_dataset.py:421-432.  ``pair_subset`` (bool mask over
        the 903 pairs) restricts the computation (the result equals masking the
        full output, since pairs are independent)."""
        S = scattering1d(x[:, 0], self.J, self.Q, self.T, self.max_order, self.dtype)
        res = {"scattering": S}
        sel = np.ones(len(self.i_idx), bool) if pair_subset is None else pair_subset
        ii, jj, pw = self.i_idx[sel], self.j_idx[sel], self.powers[sel]
        if compute_cross_phase:
            a = self.analytic(x[:, [0, 1]])
            res["cross_phase_corr"] = self.pairs(a[:, 0][:, ii], a[:, 1][:, jj], pw, S.shape[-1])
        elif compute_phase:
            a = self.analytic(x[:, 0])
            res["phase_corr"] = self.pairs(a[:, ii], a[:, jj], pw, S.shape[-1])
        return res


# ------------------------------------------------------------- normalisation
def normalize(data, field, mean, var, log_eps=1e-6):
    """normalize_tensor_data (hdf5_dataset.py:18-137) with the dataset's channel
    config (hdf5_dataset.py:385-393): fhr/up z-score; fhr_st log on ch>=1;
    fhr_ph / fhr_up_ph asinh; then per-channel (x-mu)/(sigma+1e-8).  data (B,C,S)."""
    d = np.asarray(data, np.float32)
    if field in ("fhr", "up"):
        return ((d - np.float32(mean)) / (np.float32(np.sqrt(var)) + np.float32(1e-8))).astype(np.float32)
    t = d.copy()
    if field == "fhr_st":
        t[:, 1:] = np.log(np.maximum(t[:, 1:], 0) + np.float32(log_eps))
    else:
        t = np.arcsinh(t)
    m = np.asarray(mean, np.float32)[None, :, None]
    s = np.sqrt(np.asarray(var, np.float32)).astype(np.float32)[None, :, None]
    return ((t - m) / (s + np.float32(1e-8))).astype(np.float32)


def stats(field, data, log_eps=1e-6):
    """Per-channel mean/variance after the transform, float64 accumulation
    (calculate_dataset_stats.py:134-273).  data (W, C, S) or (W, N)."""
    d = np.asarray(data, np.float64)
    if field in ("fhr", "up"):
        m = d.mean()
        return m, max(0.0, (d ** 2).mean() - m ** 2)
    if field == "fhr_st":
        d = d.copy(); d[:, 1:] = np.log(np.maximum(d[:, 1:], 0) + log_eps)
    else:
        d = np.arcsinh(d)
    m = d.mean(axis=(0, 2))
    v = np.maximum((d ** 2).mean(axis=(0, 2)) - m ** 2, 0)
    return m.astype(np.float32), v.astype(np.float32)
