"""Host-side (init-time) Morlet/Gauss filter bank and padding plan.

Mirrors kymatio's filter construction, which the
reference runs once per transform on the host in numpy/scipy:
  ref/kymatio/kymatio/scattering1d/filter_bank.py:6-762
  ref/kymatio/kymatio/scattering1d/utils.py:5-133 (padding, border indices)
  ref/kymatio/kymatio/scattering1d/frontend/base_frontend.py:27-85 (build)
Everything is float64 here; the device tables are rounded to float32 once.
"""
import math
from dataclasses import dataclass, field

import numpy as np

R_PSI = math.sqrt(0.5)
SIGMA0 = 0.1
ALPHA = 5.0
P_MAX = 5
EPS = 1e-7
CRITERION = 1e-3


def _periods(sigma):
    return min(int(math.ceil(math.sqrt(-2 * sigma * sigma * math.log(EPS)) + 1)), P_MAX)


def _fold(h, k):
    """Periodise a Fourier filter by averaging k chunks (filter_bank.py:51-71)."""
    return h.reshape(k, -1).mean(axis=0)


def _l1_normalise(hf):
    return hf / np.abs(np.fft.ifft(hf)).sum()


def morlet_fourier(n, xi, sigma):
    P = _periods(sigma)
    grid = np.arange((1 - P) * n, P * n, dtype=np.float64) / n
    low_grid = grid if P > 1 else np.fft.fftfreq(n)
    gabor = _fold(np.exp(-((grid - xi) ** 2) / (2 * sigma * sigma)), 2 * P - 1)
    low = _fold(np.exp(-(low_grid ** 2) / (2 * sigma * sigma)), 2 * P - 1)
    return _l1_normalise(gabor - (gabor[0] / low[0]) * low)


def gauss_fourier(n, sigma):
    P = _periods(sigma)
    grid = np.arange((1 - P) * n, P * n, dtype=np.float64) / n if P > 1 else np.fft.fftfreq(n)
    return _l1_normalise(_fold(np.exp(-(grid ** 2) / (2 * sigma * sigma)), 2 * P - 1))


def _max_subsampling(xi, sigma):
    return int(math.floor(-math.log2(min(xi + ALPHA * sigma, 0.5)))) - 1


def wavelet_params(sigma_min, Q):
    """(xi, sigma, j) lists of a Morlet family (filter_bank.py:412-487)."""
    xi = max(1.0 / (1.0 + 2.0 ** (3.0 / Q)), 0.35)
    f = 1.0 / 2.0 ** (1.0 / Q)
    sigma = xi * (1 - f) / (1 + f) / math.sqrt(2 * math.log(1.0 / R_PSI))
    out = []
    if sigma <= sigma_min:
        last = sigma
    else:
        j = 0
        while sigma > sigma_min:
            out.append((xi, sigma, j))
            xi, sigma = xi * f, sigma * f
            j = _max_subsampling(xi, sigma)
        last = out[-1][0]
    for q in range(1, Q):
        nx = (Q - q) / float(Q) * last
        out.append((nx, sigma_min, _max_subsampling(nx, sigma_min)))
    return out


@dataclass
class Bank:
    psi1: np.ndarray          # (F1, n) real Fourier filters, level 0
    xi1: np.ndarray
    j1: np.ndarray
    psi2_levels: list         # per second-order filter: list of levels
    xi2: np.ndarray
    j2: np.ndarray
    phi_levels: list          # phi periodised 2^k, k = 0..max
    sigma_low: float
    t_max_phi: int


def build_bank(J_support, J, Q, T):
    """scattering_filter_factory (filter_bank.py:561-762)."""
    smin = SIGMA0 / 2 ** J
    p1 = wavelet_params(smin, Q)
    p2 = wavelet_params(smin, 1)
    n = 2 ** J_support
    j1s = [p[2] for p in p1]
    psi2 = []
    for xi, s, j in p2:
        below = [a for a in j1s if j > a]
        base = morlet_fourier(n, xi, s)
        psi2.append([base] + [_fold(base, 2 ** l) for l in range(1, (max(below) if below else 0) + 1)])
    psi1 = np.stack([morlet_fourier(n, xi, s) for xi, s, _ in p1])
    phi0 = gauss_fourier(n, SIGMA0 / T)
    nmax = max(max(j1s), max(p[2] for p in p2))
    phi = [phi0] + [_fold(phi0, 2 ** l) for l in range(1, nmax + 1)]
    # temporal support of phi (filter_bank.py:254-303)
    h = np.abs(np.fft.ifft(phi0))[: n // 2]
    tail = np.cumsum(h[::-1])[::-1]
    ok = np.nonzero(tail <= CRITERION)[0]
    t_max = int(ok[0] + 1) if ok.size else n // 2
    return Bank(psi1=psi1, xi1=np.array([p[0] for p in p1]), j1=np.array(j1s, dtype=np.int64), psi2_levels=psi2,
                xi2=np.array([p[0] for p in p2]), j2=np.array([p[2] for p in p2], dtype=np.int64), phi_levels=phi,
                sigma_low=SIGMA0 / T, t_max_phi=t_max)


@dataclass
class Padding:
    J_pad: int
    pad_left: int
    pad_right: int
    ind_start: dict = field(default_factory=dict)
    ind_end: dict = field(default_factory=dict)

    @property
    def n_pad(self):
        return 2 ** self.J_pad


def padding(N, J, Q, T):
    """J_pad, pads and border indices (base_frontend.py:57-77, utils.py:5-133)."""
    t_max = build_bank(int(math.ceil(math.log2(N))), J, Q, T).t_max_phi
    J_pad = min(int(math.ceil(math.log2(N + 2 * 3 * t_max))), int(math.floor(math.log2(3 * N - 2))))
    extra = 2 ** J_pad - N
    pl = extra // 2
    pr = extra - pl
    if max(pl, pr) >= N:
        raise ValueError("Too large padding value, will lead to NaN errors")
    i0, i1 = {0: pl}, {0: pl + N}
    for j in range(1, J + 1):
        i0[j] = (i0[j - 1] + 1) // 2
        i1[j] = (i1[j - 1] + 1) // 2
    return Padding(J_pad, pl, pr, i0, i1)


def lowpass_taps(phi0, tail_tol=1e-9):
    """h0 = ifft(phi_0) (real, even) truncated at the smallest radius whose l1
    tail sum_{|d|>radius} |h0(d)| is below `tail_tol` of sum |h0|.  Used to
    evaluate kymatio's periodise-and-iFFT low-pass as a short correlation
    (DESIGN.md §3).  Returns (h0[0..radius], radius)."""
    h = np.fft.ifft(phi0)
    assert np.abs(h.imag).max() <= 1e-12 * np.abs(h.real).max(), "phi_0 must be real"
    h = h.real
    n = len(h)
    assert np.allclose(h[1:n // 2], h[n - 1:n // 2:-1], rtol=0, atol=1e-15 * np.abs(h).max()), "phi_0 must be even"
    a = np.abs(h[: n // 2 + 1])
    total = np.abs(h).sum()
    # tail(r) = 2 * sum_{d=r+1}^{n/2-1} a[d] + a[n/2]
    inner = np.concatenate([np.cumsum(a[1:n // 2][::-1])[::-1], [0.0]])   # inner[r] = sum_{d=r+1}^{n/2-1}
    tail = 2 * inner + a[n // 2]
    radius = int(np.nonzero(tail <= tail_tol * total)[0][0]) if (tail <= tail_tol * total).any() else n // 2 - 1
    return h[: radius + 1].copy(), radius


def twiddles(n):
    k = np.arange(n, dtype=np.float64)
    w = np.exp(-2j * np.pi * k / n)
    return np.stack([w.real, w.imag], axis=-1).astype(np.float32)
