"""kymatio-compatible Scattering1D on MI355X and the `torch_hip` backend plugin.

Two entry points mirror the reference's plugin API:

* `TorchHipBackend1D` — a kymatio backend (name 'torch_hip', accepted by
  kymatio's frontend check `backend.name.startswith('torch')`,
  ref/kymatio/kymatio/frontend/base_frontend.py:16-34) whose classmethods
  (pad, unpad, rfft, irfft, fft, ifft, cdgmm, modulus, subsample_fourier,
  concatenate, ...) keep the trailing-dim-2 complex convention, the checks and
  the error messages of ref/kymatio/kymatio/scattering1d/backend/torch_backend.py:17-174
  and ref/kymatio/kymatio/backend/torch_backend.py:99-219, with the compute
  in HIP kernels.  It can be handed to the reference's own kymatio
  `Scattering1D(..., backend=TorchHipBackend1D)`.
* `Scattering1D` — the frontend (ref/kymatio/kymatio/scattering1d/frontend/torch_frontend.py:10-255):
  same constructor and `[S, S]` return.  The averaged first-order,
  oversampling-0 case (the one the VAE-TEB front-end uses) runs the fused
  kernels of vaeteb.frontend; everything else runs the generic scattering
  core below over the HIP backend plugin.
"""
import math

import numpy as np
import torch
import torch.nn as nn

from . import _lib
from .filter_bank import build_bank, padding, twiddles


# ------------------------------------------------------------------ backend
_TW = {}


def _tw(n, device):
    key = (n, str(device))
    if key not in _TW:
        _TW[key] = torch.from_numpy(twiddles(n)).to(device)
    return _TW[key]


class _ModulusStable(torch.autograd.Function):
    """ModulusStable (ref/kymatio/kymatio/backend/torch_backend.py:5-96) on HIP."""

    @staticmethod
    def forward(ctx, x):
        out = torch.empty(x.shape[:-1], dtype=x.dtype, device=x.device)
        _lib.call("vt_modulus", _lib.ptr(x), _lib.ptr(out), out.numel(), _lib.stream())
        ctx.save_for_backward(x, out)
        return out

    @staticmethod
    def backward(ctx, g):
        x, out = ctx.saved_tensors
        gi = torch.empty_like(x)
        _lib.call("vt_modulus_bwd", _lib.ptr(x), _lib.ptr(out), _lib.ptr(g.contiguous()), _lib.ptr(gi), out.numel(),
                  _lib.stream())
        return gi


class TorchHipBackend1D:
    name = "torch_hip"

    # --- checks (same messages as the reference backend)
    @classmethod
    def input_checks(cls, x):
        if x is None:
            raise TypeError("The input should be not empty.")
        cls.contiguous_check(x)

    @staticmethod
    def contiguous_check(x):
        if not x.is_contiguous():
            raise RuntimeError("Tensors must be contiguous.")

    @staticmethod
    def _is_complex(x):
        return x.shape[-1] == 2

    @staticmethod
    def _is_real(x):
        return x.shape[-1] == 1

    @classmethod
    def complex_check(cls, x):
        if not cls._is_complex(x):
            raise TypeError("The input should be complex (i.e. last dimension is 2).")

    @classmethod
    def real_check(cls, x):
        if not cls._is_real(x):
            raise TypeError("The input should be real.")

    @classmethod
    def complex_contiguous_check(cls, x):
        cls.complex_check(x)
        cls.contiguous_check(x)

    @staticmethod
    def _device_check(x):
        if not x.is_cuda:
            raise TypeError("Input must be on GPU.")

    # --- ops
    @classmethod
    def modulus(cls, x):
        cls.complex_contiguous_check(x)
        return _ModulusStable.apply(x)[..., None]

    @staticmethod
    def concatenate(arrays, dim=2):
        return torch.stack(arrays, dim=dim)

    @staticmethod
    def reshape(x, shape):
        return x.reshape(shape)

    @classmethod
    def cdgmm(cls, A, B):
        if not cls._is_real(B):
            cls.complex_contiguous_check(B)
        else:
            cls.contiguous_check(B)
        cls.complex_contiguous_check(A)
        if A.shape[-len(B.shape):-1] != B.shape[:-1]:
            raise RuntimeError("The filters are not compatible for multiplication.")
        if A.dtype is not B.dtype:
            raise TypeError("Input and filter must be of the same dtype.")
        if B.is_cuda and (not A.is_cuda or A.device.index != B.device.index):
            raise TypeError("Input and filter must be on the same GPU." if A.is_cuda else "Input must be on GPU.")
        if not B.is_cuda and A.is_cuda:
            raise TypeError("Input must be on CPU.")
        cls._device_check(A)
        n = B.numel() // B.shape[-1]
        C = torch.empty_like(A)
        _lib.call("vt_cdgmm", _lib.ptr(A), _lib.ptr(B), int(cls._is_real(B)), _lib.ptr(C), A.numel() // (2 * n), n,
                  _lib.stream())
        return C

    @classmethod
    def subsample_fourier(cls, x, k):
        cls.complex_check(x)
        cls._device_check(x)
        x = x.contiguous()
        N = x.shape[-2]
        out = torch.empty(x.shape[:-2] + (N // k, 2), dtype=x.dtype, device=x.device)
        _lib.call("vt_subsample_fourier", _lib.ptr(x), _lib.ptr(out), x.numel() // (2 * N), N, k, _lib.stream())
        return out

    @staticmethod
    def pad(x, pad_left, pad_right):
        if (pad_left >= x.shape[-1]) or (pad_right >= x.shape[-1]):
            raise ValueError("Indefinite padding size (larger than tensor).")
        x = x.contiguous()
        N = x.shape[-1]
        out = torch.empty(x.shape[:-1] + (N + pad_left + pad_right,), dtype=x.dtype, device=x.device)
        _lib.call("vt_pad_reflect", _lib.ptr(x), _lib.ptr(out), x.numel() // N, N, pad_left, pad_right, _lib.stream())
        return out[..., None]

    @staticmethod
    def unpad(x, i0, i1):
        x = x.reshape(x.shape[:-1])
        return x[..., i0:i1]

    @classmethod
    def _fft(cls, x, inverse):
        cls._device_check(x)
        n = x.shape[-2]
        if n > _MAX_FFT:
            raise ValueError(f"torch_hip backend: FFT length {n} exceeds {_MAX_FFT}")
        out = torch.empty_like(x)
        rows = x.numel() // (2 * n)
        if n <= _lib_max_fft():
            _lib.call("vt_fft", _lib.ptr(x), _lib.ptr(out), rows, n, int(inverse), _lib.ptr(_tw(n, x.device)), 1,
                      _lib.stream())
        else:   # four-step through HBM (config 5: n_pad = 32768)
            ws = torch.empty_like(x)
            _lib.call("vt_fft_large", _lib.ptr(x), _lib.ptr(out), _lib.ptr(ws), rows, n, int(inverse),
                      _lib.ptr(_tw(n, x.device)), _lib.stream())
        return out

    @classmethod
    def rfft(cls, x):
        cls.contiguous_check(x)
        cls.real_check(x)
        x_r = torch.zeros(x.shape[:-1] + (2,), dtype=x.dtype, device=x.device)
        x_r[..., 0] = x[..., 0]
        return cls._fft(x_r, False)

    @classmethod
    def irfft(cls, x):
        cls.contiguous_check(x)
        cls.complex_check(x)
        return cls._fft(x, True)[..., :1].contiguous()

    @classmethod
    def ifft(cls, x):
        cls.contiguous_check(x)
        cls.complex_check(x)
        return cls._fft(x, True)

    @classmethod
    def fft(cls, x):
        cls.contiguous_check(x)
        cls.complex_check(x)
        return cls._fft(x, False)

    @staticmethod
    def multiply(x, y):
        return torch.multiply(x, y)

    @classmethod
    def to_polar(cls, x):
        cls.complex_check(x)
        mag = cls.modulus(x)
        phase = torch.atan2(x[..., 1:2], x[..., 0:1])
        return mag, phase

    @classmethod
    def to_cartesian(cls, mag, phase):
        return torch.cat((torch.cos(phase) * mag, torch.sin(phase) * mag), -1)


def _lib_max_fft():
    return 8192     # VT_FFT_MAX_LDS: one workgroup's LDS; longer -> vt_fft_large


_MAX_FFT = 1 << 21


backend = TorchHipBackend1D


# ------------------------------------------------------------- generic core
def scattering1d_core(x, bk, J, T, psi1, psi2, phi, pad_left, pad_right, ind_start, ind_end, oversampling=0,
                      max_order=2, average=True, vectorize=True, out_type="array"):
    """The scattering cascade of ref/kymatio/kymatio/scattering1d/core/scattering1d.py:197-399
    written against a backend object (here the HIP plugin)."""
    U0h = bk.rfft(bk.pad(x, pad_left=pad_left, pad_right=pad_right))
    lt = int(math.floor(math.log2(T)))
    k0 = max(lt - oversampling, 0)
    s0 = bk.unpad(bk.irfft(bk.subsample_fourier(bk.cdgmm(U0h, phi["levels"][0]), 2 ** k0)), ind_start[k0],
                  ind_end[k0]) if average else x
    out = [{"coef": s0, "j": (), "n": ()}]
    out2 = []
    for n1, p1 in enumerate(psi1):
        j1 = p1["j"]
        k1 = max(min(j1 - oversampling, lt - oversampling), 0)
        U1c = bk.ifft(bk.subsample_fourier(bk.cdgmm(U0h, p1["levels"][0]), 2 ** k1))
        U1m = bk.modulus(U1c)
        U1h = bk.rfft(U1m) if (average or max_order > 1) else None
        if average:
            k1J = max(lt - k1 - oversampling, 0)
            s1 = bk.unpad(bk.irfft(bk.subsample_fourier(bk.cdgmm(U1h, phi["levels"][k1]), 2 ** k1J)),
                          ind_start[k1J + k1], ind_end[k1J + k1])
        else:
            s1 = bk.unpad(U1m, ind_start[k1], ind_end[k1])
        out.append({"coef": s1, "j": (j1,), "n": (n1,)})
        if max_order == 2:
            for n2, p2 in enumerate(psi2):
                j2 = p2["j"]
                if j2 <= j1:
                    continue
                k2 = max(min(j2 - k1 - oversampling, lt - k1 - oversampling), 0)
                U2m = bk.modulus(bk.ifft(bk.subsample_fourier(bk.cdgmm(U1h, p2["levels"][k1]), 2 ** k2)))
                if average:
                    k2J = max(lt - k2 - k1 - oversampling, 0)
                    s2 = bk.unpad(bk.irfft(bk.subsample_fourier(bk.cdgmm(bk.rfft(U2m), phi["levels"][k1 + k2]),
                                                                2 ** k2J)),
                                  ind_start[k1 + k2 + k2J], ind_end[k1 + k2 + k2J])
                else:
                    s2 = bk.unpad(U2m, ind_start[k1 + k2], ind_end[k1 + k2])
                out2.append({"coef": s2, "j": (j1, j2), "n": (n1, n2)})
    out += out2
    if out_type == "array" and vectorize:
        return bk.concatenate([o["coef"] for o in out])
    if out_type == "array":
        return {o["n"]: o["coef"] for o in out}
    for o in out:
        o.pop("n")
    return out


# ------------------------------------------------------------- batched cascade
class _Cascade:
    """The cascade of scattering1d_core (orders 1-2, average=True, array output)
    regrouped by subsampling level: every (sample, filter) row of a level is one
    launch of vt_scat_filter_sub (cdgmm + subsample), vt_scat_mod_spec (ifft ->
    modulus -> rfft in LDS) and vt_scat_lowpass (phi, subsample, irfft, unpad ->
    its output channel).  Same arithmetic and channel order as the reference
    loop (ref/kymatio/kymatio/scattering1d/core/scattering1d.py:197-399); ~3
    launches per level instead of ~6 per filter and per filter pair."""

    def __init__(self, sc, device):
        b, J, os_ = sc._bank, sc.J, sc.oversampling
        n = 2 ** sc.J_pad
        lt = int(math.floor(math.log2(sc.T)))
        self.n, self.dev = n, device
        pool, offs = [], {}

        def off(key, arr):
            if key not in offs:
                offs[key] = sum(len(a) for a in pool)
                pool.append(np.asarray(arr, np.float32).reshape(-1))
            return offs[key]

        i32 = lambda v: torch.tensor(v, dtype=torch.int32, device=device)
        i64 = lambda v: torch.tensor(v, dtype=torch.int64, device=device)
        ind0, ind1 = sc.ind_start, sc.ind_end
        k0 = max(lt - os_, 0)
        self.S = ind1[k0] - ind0[k0]
        self.s0 = (off(("phi", 0), b.phi_levels[0]), 2 ** k0, ind0[k0], ind1[k0], i32([0]))
        n_psi1 = len(b.xi1)
        groups = {}
        for n1 in range(n_psi1):
            k1 = max(min(int(b.j1[n1]) - os_, lt - os_), 0)
            groups.setdefault(k1, []).append(n1)
        order2 = []   # channel numbering of the reference loop: S0, S1 (n1), then S2 (n1, n2) in loop order
        if sc.max_order == 2:
            for n1 in range(n_psi1):
                for n2 in range(len(b.xi2)):
                    if int(b.j2[n2]) > int(b.j1[n1]):
                        order2.append((n1, n2))
        ch2 = {pr: 1 + n_psi1 + i for i, pr in enumerate(order2)}
        self.C = 1 + n_psi1 + len(order2)
        self.levels = []
        for k1, members in sorted(groups.items()):
            L = n // 2 ** k1
            k1J = max(lt - k1 - os_, 0)
            lvl = {"L": L, "k": 2 ** k1, "P": len(members), "a_idx": i32([0] * len(members)),
                   "f_off": i64([off(("psi1", m), b.psi1[m]) for m in members]),
                   "s1": (off(("phi", k1), b.phi_levels[k1]), 2 ** k1J, ind0[k1J + k1], ind1[k1J + k1],
                          i32([1 + m for m in members])), "sub": []}
            pos = {m: i for i, m in enumerate(members)}
            sub = {}
            for (n1, n2) in order2:
                if n1 not in pos:
                    continue
                k2 = max(min(int(b.j2[n2]) - k1 - os_, lt - k1 - os_), 0)
                sub.setdefault(k2, []).append((n1, n2))
            for k2, prs in sorted(sub.items()):
                k2J = max(lt - k2 - k1 - os_, 0)
                lvl["sub"].append({
                    "L": L // 2 ** k2, "k": 2 ** k2, "P": len(prs), "a_idx": i32([pos[a] for a, _ in prs]),
                    "f_off": i64([off(("psi2", c, k1), b.psi2_levels[c][k1]) for _, c in prs]),
                    "s2": (off(("phi", k1 + k2), b.phi_levels[k1 + k2]), 2 ** k2J, ind0[k1 + k2 + k2J],
                           ind1[k1 + k2 + k2J], i32([ch2[pr] for pr in prs]))})
            self.levels.append(lvl)
        self.pool = torch.from_numpy(np.concatenate(pool)).to(device)
        self.pad = (sc.pad_left, sc.pad_right)

    def _spectrum(self, A, B, a_rows, n_in, g):
        """U^ = rfft(|ifft(subsample(A[a_idx] . psi, k))|) for every (b, p) row of
        level g: one fused LDS launch when the row fits, else fold + four-step."""
        L = g["L"]
        out = torch.empty((B, g["P"], L, 2), device=self.dev)
        tw = _lib.ptr(_tw(L, self.dev))
        if L <= _lib_max_fft():
            _lib.call("vt_scat_mod_spec", _lib.ptr(A), B, a_rows, n_in, _lib.ptr(g["a_idx"]), _lib.ptr(self.pool),
                      _lib.ptr(g["f_off"]), g["P"], g["k"], tw, _lib.ptr(out), _lib.stream())
            return out
        Y = self._filter_sub(A, B, a_rows, n_in, g)
        ws = torch.empty_like(Y)
        rows = B * g["P"]
        _lib.call("vt_fft_large", _lib.ptr(Y), _lib.ptr(out), _lib.ptr(ws), rows, L, 1, tw, _lib.stream())
        _lib.call("vt_modulus_cplx", _lib.ptr(out), _lib.ptr(Y), rows * L, _lib.stream())
        _lib.call("vt_fft_large", _lib.ptr(Y), _lib.ptr(out), _lib.ptr(ws), rows, L, 0, tw, _lib.stream())
        return out

    def _lowpass(self, U, B, P, L, spec, out):
        foff, k, i0, i1, ch = spec
        _lib.call("vt_scat_lowpass", _lib.ptr(U), B, P, L, self.pool.data_ptr() + 4 * foff, k, i0, i1, _lib.ptr(ch),
                  self.C, _lib.ptr(_tw(L // k, self.dev)), _lib.ptr(out), _lib.stream())

    def _filter_sub(self, A, B, a_rows, L_in, g):
        Y = torch.empty((B, g["P"], g["L"], 2), device=self.dev)
        _lib.call("vt_scat_filter_sub", _lib.ptr(A), B, a_rows, L_in, _lib.ptr(g["a_idx"]), _lib.ptr(self.pool),
                  _lib.ptr(g["f_off"]), g["P"], g["k"], _lib.ptr(Y), _lib.stream())
        return Y

    def __call__(self, x2):
        """x2 (B, N) float32 contiguous on device -> S (B, C, S_out)."""
        B, N = x2.shape
        n = self.n
        xp = torch.empty((B, n), device=self.dev)
        _lib.call("vt_pad_reflect", _lib.ptr(x2), _lib.ptr(xp), B, N, self.pad[0], self.pad[1], _lib.stream())
        xc = torch.zeros((B, n, 2), device=self.dev)
        xc[..., 0] = xp
        U0h = TorchHipBackend1D._fft(xc, False)
        out = torch.empty((B, self.C, self.S), device=self.dev)
        self._lowpass(U0h, B, 1, n, self.s0, out)
        for lvl in self.levels:
            U1h = self._spectrum(U0h, B, 1, n, lvl)
            self._lowpass(U1h, B, lvl["P"], lvl["L"], lvl["s1"], out)
            for g in lvl["sub"]:
                U2h = self._spectrum(U1h, B, lvl["P"], lvl["L"], g)
                self._lowpass(U2h, B, g["P"], g["L"], g["s2"], out)
        return out


# ------------------------------------------------------------------ frontend
class Scattering1D(nn.Module):
    """Drop-in for kymatio's (locally modified) ScatteringTorch1D: forward(x)
    returns [S, S] (ref/kymatio/kymatio/scattering1d/frontend/torch_frontend.py:163-255)."""

    def __init__(self, J, shape, Q=1, max_order=2, average=True, oversampling=0, vectorize=True, out_type="array",
                 backend="torch_hip", T=None):
        super().__init__()
        if backend not in ("torch_hip", TorchHipBackend1D):
            raise ImportError("Backend " + str(backend) + " not found!")
        self.backend = TorchHipBackend1D
        self.J, self.Q, self.max_order, self.average = J, Q, max_order, average
        self.oversampling, self.vectorize, self.out_type = oversampling, vectorize, out_type
        if isinstance(shape, int):
            self.N = shape
        elif isinstance(shape, tuple):
            if len(shape) > 1:
                raise ValueError("If shape is specified as a tuple, it must have exactly one element")
            self.N = shape[0]
        else:
            raise ValueError("shape must be an integer or a 1-tuple")
        # T=None: kymatio's documented default 2**J (the reference build() sets it,
        # then its torch frontend resets it to None and crashes)
        self.T = 2 ** J if T is None else T
        if self.T > 2 ** J:
            raise ValueError("The temporal support T of the low-pass filter cannot exceed 2**J (got {} > {})".format(
                self.T, 2 ** J))
        pd = padding(self.N, J, Q, self.T)
        self.J_pad, self.pad_left, self.pad_right = pd.J_pad, pd.pad_left, pd.pad_right
        self.ind_start, self.ind_end = pd.ind_start, pd.ind_end
        bank = build_bank(self.J_pad, J, Q, self.T)
        self._bank = bank
        self._tables = None
        self._fused = None
        self._cascade = None
        self.cascade = True     # False: per-filter generic core over the plugin (the reference's loop)

    def _device_tables(self, device):
        if self._tables is None or self._tables[0] != str(device):
            f = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.float32)).view(-1, 1).to(device)
            b = self._bank
            phi = {"levels": [f(l) for l in b.phi_levels]}
            psi1 = [{"levels": [f(b.psi1[i])], "xi": b.xi1[i], "j": int(b.j1[i])} for i in range(len(b.xi1))]
            psi2 = [{"levels": [f(l) for l in b.psi2_levels[i]], "xi": b.xi2[i], "j": int(b.j2[i])}
                    for i in range(len(b.xi2))]
            self._tables = (str(device), phi, psi1, psi2)
        return self._tables[1:]

    def _fused_ok(self):
        return (self.max_order == 1 and self.average and self.oversampling == 0 and self.vectorize
                and self.out_type == "array" and 2 ** self.J_pad <= 8192)

    def _cascade_ok(self, x):
        """Batched level-grouped cascade: average=True, array output, no autograd
        (the generic core over the plugin keeps the reference's autograd)."""
        return (self.cascade and self.average and self.out_type == "array" and self.vectorize and self.max_order in (1, 2)
                and not (torch.is_grad_enabled() and x.requires_grad) and x.is_cuda)

    def meta(self):
        raise NotImplementedError("meta() is outside the training path")

    def scattering(self, x):
        if len(x.shape) < 1:
            raise ValueError("Input tensor x should have at least one axis, got {}".format(len(x.shape)))
        if self.out_type not in ("array", "list"):
            raise RuntimeError("The out_type must be one of 'array' or 'list'.")
        if not self.average and self.out_type == "array" and self.vectorize:
            raise ValueError("Options average=False, out_type='array' and vectorize=True are mutually incompatible. "
                             "Please set out_type to 'list' or vectorize to False.")
        batch_shape = x.shape[:-1]
        x2 = x.reshape((-1, x.shape[-1])).contiguous()
        if self._fused_ok():
            S = self._fused_forward(x2)
        elif self._cascade_ok(x2):
            if self._cascade is None or self._cascade.dev != x2.device:
                self._cascade = _Cascade(self, x2.device)
            S = self._cascade(x2)
        else:
            phi, psi1, psi2 = self._device_tables(x.device)
            S = scattering1d_core(x2.reshape(-1, 1, x.shape[-1]), self.backend, self.J, self.T, psi1, psi2, phi,
                                  self.pad_left, self.pad_right, self.ind_start, self.ind_end, self.oversampling,
                                  self.max_order, self.average, self.vectorize, self.out_type)
        if self.out_type == "array" and self.vectorize:
            S = S.reshape(batch_shape + S.shape[-2:])
        elif self.out_type == "array":
            S = {k: v.reshape(batch_shape + v.shape[-2:]) for k, v in S.items()}
        else:
            for o in S:
                o["coef"] = o["coef"].reshape(batch_shape + o["coef"].shape[-1:])
        return [S, S]

    def _fused_forward(self, x2):
        from .frontend import FrontEndPlan, launch_lowpass, launch_spectrum, launch_wavelet
        if self._fused is None or self._fused[0].device != x2.device:
            plan = FrontEndPlan(self.J, self.Q, self.T, self.N, device=x2.device)
            self._fused = (plan, plan.tables([], [], scattering=True))
        plan, tab = self._fused
        B = x2.shape[0]
        C = 1 + plan.n_filters
        xhat = torch.empty((B, plan.n_pad, 2), device=x2.device)
        launch_spectrum(plan, x2, B, 0, xhat)
        S = torch.empty((B, C, plan.S), device=x2.device)
        launch_lowpass(plan, x2, B, plan.N, S, C * plan.S)
        launch_wavelet(plan, xhat, B, 1, tab, None, S, C)
        return S

    def forward(self, x):
        self.backend.input_checks(x)
        return self.scattering(x)
