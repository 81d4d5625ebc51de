"""MI355X front-end: Scattering1D + phase harmonics + normalisation, fused.

`FrontEndPlan` is built once on the host (filter bank, padding, pair and
slot tables, twiddles) and uploaded; `FrontEnd.__call__` then turns a batch of
raw windows x (B, 2, N) [ch0 = fhr, ch1 = up] into the model inputs of the
reference's data contract (ref/hdf5_dataset/hdf5_dataset.py:706-779,
ref/model/pytorch_lightning_modules.py:480-483):
    fhr_st (B, S, 43), fhr_ph (B, S, 44), fhr_up_ph (B, S, 130), fhr (B, N)
normalised with the dataset statistics, all in one stream of HIP launches.

Reference semantics reproduced:
  * the two front-end calls of ref/hdf5_dataset/create_hdf5_dataset.py:418-441
    (phase on ch0; cross-phase ch0 x ch1) with the selection masks of
    get_optimal_coefficients_for_fhr (kymatio_phase_scattering.py:635-760);
  * only the selected pairs are computed (the reference computes all 903 per
    call and masks afterwards; pairs are independent, so the result is equal);
  * each analytic signal a_{c,f} is computed once and shared by every pair
    that uses it and by the first-order scattering of ch0.
"""
import math

import numpy as np
import torch

from . import _lib
from .filter_bank import build_bank, lowpass_taps, padding, twiddles

FIELDS = ("fhr_st", "fhr_ph", "fhr_up_ph")


def _i32(a, dev):
    return torch.as_tensor(np.ascontiguousarray(a, dtype=np.int32), device=dev)


def _f32(a, dev):
    return torch.as_tensor(np.ascontiguousarray(a, dtype=np.float32), device=dev)


class FrontEndPlan:
    """Host-built, device-resident tables for one (J, Q, T, N) configuration."""

    def __init__(self, J=11, Q=4, T=16, N=4096, device="cuda", tail_tol=1e-9):
        self.J, self.Q, self.T, self.N = J, Q, T, N
        self.device = torch.device(device)
        pd = padding(N, J, Q, T)
        self.pad = pd
        self.n_pad, self.pad_left, self.pad_right = pd.n_pad, pd.pad_left, pd.pad_right
        if self.n_pad > 8192:
            raise NotImplementedError(f"fused front-end holds one FFT in LDS (n_pad <= 8192), got {self.n_pad}")
        bank = build_bank(pd.J_pad, J, Q, T)
        self.bank = bank
        self.log2T = int(math.floor(math.log2(T)))
        self.step = 2 ** self.log2T
        self.start = pd.ind_start[self.log2T]
        self.S = pd.ind_end[self.log2T] - pd.ind_start[self.log2T]
        self.n_filters = len(bank.xi1)
        self.k1 = np.maximum(np.minimum(bank.j1, self.log2T), 0)

        # pair tables (kymatio_phase_scattering.py:134-160): float32 powers as
        # the reference computes them (xi stored float32, divided in float32)
        xi = bank.xi1.astype(np.float32)
        ii, jj, pw = [], [], []
        for i in range(len(xi)):
            for j in range(len(xi)):
                if xi[j] >= xi[i]:
                    ii.append(i); jj.append(j)
                    pw.append(np.float32(xi[j]) / np.float32(xi[i]) if xi[i] > 1e-8 else np.float32(1.0))
        self.i_idx, self.j_idx = np.array(ii), np.array(jj)
        self.powers = np.array(pw, dtype=np.float32)
        self.autoc_idx = np.array([k for k in range(len(ii)) if ii[k] == jj[k]])
        self.center_freqs = xi
        self.phase_mask, self.cross_mask = self.fhr_masks()

        # phase-path low-pass decimation (kymatio_phase_scattering.py:287-292, :255-268)
        self.dec = max(1, min(N, N // self.S)) if N > self.S else 1
        self.nb = self.n_pad // self.dec
        self.pair_start = self.pad_left // self.dec
        self.pair_len = min(N // self.dec, self.nb - self.pair_start)
        h0, radius = lowpass_taps(bank.phi_levels[0], tail_tol)
        self.radius = radius

        dev = self.device
        self.t_psi = _f32(bank.psi1, dev)
        self.t_h0 = _f32(h0, dev)
        self.t_phi_crop = _f32(bank.phi_levels[0][: self.nb], dev)
        self.t_tw = _f32(twiddles(self.n_pad), dev)

    # ------------------------------------------------------------------ masks
    def fhr_masks(self):
        """get_optimal_coefficients_for_fhr (kymatio_phase_scattering.py:635-760)."""
        xi, pw, ii, jj = self.center_freqs, self.powers, self.i_idx, self.j_idx
        fmin = np.float32(0.006 if self.J >= 11 else 0.003)
        band = xi >= fmin
        auto = np.zeros(len(ii), bool)
        auto[self.autoc_idx] = True
        phase = band[ii] & band[jj] & auto
        for r in (2, 3):
            phase |= band[ii] & band[jj] & (np.abs(pw - np.float32(r)) < np.float32(0.1)) & (pw <= 8)
        up = xi < np.float32(0.02)
        fh = (xi >= np.float32(0.04)) & (xi <= np.float32(0.5))
        cross = up[ii] & fh[jj] & (pw >= 1) & (pw <= 32)
        return phase, cross

    # ------------------------------------------------------------- work tables
    def tables(self, phase_pairs, cross_pairs, scattering=True):
        """Wavelet items, analytic slots and pair tables for the given pair index
        lists (indices into the 903-pair enumeration)."""
        need = set()
        for k in phase_pairs:
            need.add((0, int(self.i_idx[k]))); need.add((0, int(self.j_idx[k])))
        for k in cross_pairs:
            need.add((0, int(self.i_idx[k]))); need.add((1, int(self.j_idx[k])))
        slots = {cf: s for s, cf in enumerate(sorted(need))}
        items = []
        for f in range(self.n_filters):
            s1 = 1 + f if scattering else -1
            slot = slots.get((0, f), -1)
            if s1 >= 0 or slot >= 0:
                items.append((0, f, slot, s1, int(self.k1[f])))
        for f in range(self.n_filters):
            if (1, f) in slots:
                items.append((1, f, slots[(1, f)], -1, 0))
        pi = [slots[(0, int(self.i_idx[k]))] for k in phase_pairs] + \
             [slots[(0, int(self.i_idx[k]))] for k in cross_pairs]
        pj = [slots[(0, int(self.j_idx[k]))] for k in phase_pairs] + \
             [slots[(1, int(self.j_idx[k]))] for k in cross_pairs]
        pw = [self.powers[k] for k in phase_pairs] + [self.powers[k] for k in cross_pairs]
        dev = self.device
        return dict(n_slots=len(slots), items=_i32(np.array(items).reshape(-1, 5), dev), n_items=len(items),
                    slot_i=_i32(pi, dev), slot_j=_i32(pj, dev), power=_f32(pw, dev), n_pairs=len(pi))


PAD_MODES = {"reflect": 0, "constant": 1, "circular": 2}


def launch_spectrum(p, x, rows, pad_mode, xhat):
    """rows of x (each p.N long, contiguous) -> padded spectra xhat (rows, n_pad) complex."""
    _lib.call("vt_fe_spectrum", _lib.ptr(x), rows, p.N, p.n_pad, p.pad_left, pad_mode, _lib.ptr(p.t_tw),
              _lib.ptr(xhat), _lib.stream())


def launch_lowpass(p, x, rows, x_row_stride, out, out_row_stride):
    """S0 (order-0 scattering) of each row, written at out[row * out_row_stride + m]."""
    _lib.call("vt_fe_lowpass", _lib.ptr(x), rows, x_row_stride, p.N, p.n_pad, p.pad_left, _lib.ptr(p.t_h0), p.radius,
              p.step, p.start, p.S, out.data_ptr(), out_row_stride, _lib.stream())


def launch_wavelet(p, xhat, B, C, tab, analytic, s1, s1_channels):
    _lib.call("vt_fe_wavelet", _lib.ptr(xhat), B, C, p.n_pad, _lib.ptr(p.t_psi), tab["n_items"], _lib.ptr(tab["items"]),
              _lib.ptr(p.t_tw), p.N, p.pad_left, _lib.ptr(analytic) if analytic is not None else None,
              max(tab["n_slots"], 1), _lib.ptr(p.t_h0), p.radius, p.step, p.start, p.S,
              _lib.ptr(s1) if s1 is not None else None, s1_channels, _lib.stream())


def launch_pairs(p, analytic, B, tab, out, lowpass=True, pad_mode=0):
    if lowpass:
        _lib.call("vt_fe_pairs", _lib.ptr(analytic), B, tab["n_slots"], p.N, p.n_pad, p.pad_left, tab["n_pairs"],
                  _lib.ptr(tab["slot_i"]), _lib.ptr(tab["slot_j"]), _lib.ptr(tab["power"]), _lib.ptr(p.t_tw),
                  _lib.ptr(p.t_phi_crop), p.dec, p.pair_start, p.pair_len, pad_mode, _lib.ptr(out), _lib.stream())
    else:
        _lib.call("vt_fe_pairs", _lib.ptr(analytic), B, tab["n_slots"], p.N, p.n_pad, p.pad_left, tab["n_pairs"],
                  _lib.ptr(tab["slot_i"]), _lib.ptr(tab["slot_j"]), _lib.ptr(tab["power"]), _lib.ptr(p.t_tw),
                  _lib.ptr(p.t_phi_crop), 0, 0, p.N, pad_mode, _lib.ptr(out), _lib.stream())


class FrontEnd:
    """Fused training-step front-end: raw windows -> normalised model inputs."""

    def __init__(self, plan: FrontEndPlan, stats=None, trim=0):
        """trim: decimated steps dropped at each end of the model inputs — the dataset's
        trim_minutes (ref/hdf5_dataset/hdf5_dataset.py:359-364, :733-741: 2 minutes of a
        4 Hz window = 480 raw samples = 30 steps), fused into the normalisation pass; the
        raw fhr loses trim x 16 samples at each end.  S_out = S - 2 trim, N_out = N - 32 trim."""
        self.plan = p = plan
        if trim < 0 or 2 * trim >= p.S:
            raise ValueError(f"trim {trim} out of range for {p.S} steps")
        self.trim = trim
        self.S_out = p.S - 2 * trim
        self.N_out = p.N - 2 * trim * p.step
        self.phase_pairs = np.nonzero(p.phase_mask)[0]
        self.cross_pairs = np.nonzero(p.cross_mask)[0]
        self.tab = p.tables(self.phase_pairs, self.cross_pairs, scattering=True)
        self.C_st = 1 + p.n_filters
        self.C_ph, self.C_x = len(self.phase_pairs), len(self.cross_pairs)
        self.stats = None
        if stats is not None:
            self.set_stats(stats)
        self._bufs = {}

    def set_stats(self, stats):
        """stats: mapping with '<field>_mean' / '<field>_variance' arrays (the
        layout of vaeteb/data/stats_*.npz, cf. calculate_dataset_stats.py:364-444)."""
        dev = self.plan.device
        s = {}
        for f, n, kind in (("fhr_st", self.C_st, None), ("fhr_ph", self.C_ph, 2), ("fhr_up_ph", self.C_x, 2)):
            m = np.asarray(stats[f + "_mean"], np.float32).reshape(-1)
            v = np.asarray(stats[f + "_variance"], np.float32).reshape(-1)
            assert m.shape[0] == n, (f, m.shape, n)
            k = np.full(n, 2, np.int32) if kind == 2 else np.array([0] + [1] * (n - 1), np.int32)
            s[f] = (_i32(k, dev), _f32(m, dev), _f32(np.sqrt(v), dev))
        s["fhr"] = (float(np.asarray(stats["fhr_mean"])), float(np.sqrt(np.asarray(stats["fhr_variance"]))))
        self.stats = s

    def _buf(self, name, shape, dtype=torch.float32):
        b = self._bufs.get(name)
        if b is None or tuple(b.shape) != tuple(shape):
            b = torch.empty(shape, dtype=dtype, device=self.plan.device)
            self._bufs[name] = b
        return b

    def raw(self, x, side=None):
        """x (B, 2, N) float32 on device -> raw (un-normalised) features
        {'fhr_st': (B,43,S), 'pairs': (B, 44+130, S)} as the reference stores them.
        With a side stream, the cross pairs (the source encoder's input) are
        computed there concurrently with the phase pairs and returned separately
        as 'cross' (B, 130, S); the caller's stream does not wait for them."""
        p, t = self.plan, self.tab
        if x.dim() != 3 or x.shape[1] != 2 or x.shape[2] != p.N:
            raise ValueError(f"expected (B, 2, {p.N}) windows, got {tuple(x.shape)}")
        x = x.contiguous()
        B = x.shape[0]
        xhat = self._buf("xhat", (B, 2, p.n_pad, 2))
        launch_spectrum(p, x, B * 2, 0, xhat)
        s_raw = self._buf("s_raw", (B, self.C_st, p.S))
        launch_lowpass(p, x, B, 2 * p.N, s_raw, self.C_st * p.S)
        an = self._buf("analytic", (B, t["n_slots"], p.N, 2))
        launch_wavelet(p, xhat, B, 2, t, an, s_raw, self.C_st)
        if side is None or not self.C_ph or not self.C_x:
            pr = self._buf("pairs", (B, t["n_pairs"], p.pair_len))
            launch_pairs(p, an, B, t, pr, lowpass=True, pad_mode=0)
            return {"fhr_st": s_raw, "pairs": pr}
        main = torch.cuda.current_stream()
        side.wait_stream(main)               # analytic signals ready
        pr = self._buf("pairs_ph", (B, self.C_ph, p.pair_len))
        launch_pairs(p, an, B, _sub_table(t, 0, self.C_ph), pr, lowpass=True, pad_mode=0)
        with torch.cuda.stream(side):
            px = self._buf("pairs_x", (B, self.C_x, p.pair_len))
            launch_pairs(p, an, B, _sub_table(t, self.C_ph, self.C_x), px, lowpass=True, pad_mode=0)
        return {"fhr_st": s_raw, "pairs": pr, "cross": px}

    def __call__(self, x, out=None, side=None):
        """Normalised model inputs (AttributeDict fields of the reference batch).
        side: optional HIP stream for the source encoder's input (fhr_up_ph is
        then produced on that stream; see SeqVaeTeb(concurrent_encoders))."""
        if self.stats is None:
            raise RuntimeError("FrontEnd needs normalisation statistics (set_stats)")
        p = self.plan
        r = self.raw(x, side)
        B, S, S0, Sl = x.shape[0], p.S, self.trim, self.S_out
        st = _lib.stream()
        out = {} if out is None else out
        get = lambda k, shape: out[k] if k in out else torch.empty(shape, device=p.device)
        y_st = get("fhr_st", (B, Sl, self.C_st))
        y_ph = get("fhr_ph", (B, Sl, self.C_ph))
        x_ph = get("fhr_up_ph", (B, Sl, self.C_x))
        y_raw = get("fhr", (B, self.N_out))
        k, m, s = self.stats["fhr_st"]
        _lib.call("vt_fe_normalize_window", _lib.ptr(r["fhr_st"]), B, self.C_st, self.C_st, S, S0, Sl, _lib.ptr(k),
                  _lib.ptr(m), _lib.ptr(s), 1e-6, _lib.ptr(y_st), self.C_st, 0, st)
        pairs = r["pairs"]
        if self.C_ph:
            k, m, s = self.stats["fhr_ph"]
            _lib.call("vt_fe_normalize_window", pairs.data_ptr(), B, self.C_ph, pairs.shape[1], S, S0, Sl,
                      _lib.ptr(k), _lib.ptr(m), _lib.ptr(s), 1e-6, _lib.ptr(y_ph), self.C_ph, 0, st)
        if self.C_x:
            k, m, s = self.stats["fhr_up_ph"]
            if "cross" in r:
                with torch.cuda.stream(side):
                    _lib.call("vt_fe_normalize_window", r["cross"].data_ptr(), B, self.C_x, self.C_x, S, S0, Sl,
                              _lib.ptr(k), _lib.ptr(m), _lib.ptr(s), 1e-6, _lib.ptr(x_ph), self.C_x, 0,
                              _lib.stream())
                x_ph.record_stream(side)
            else:
                _lib.call("vt_fe_normalize_window", pairs[:, self.C_ph:].data_ptr(), B, self.C_x, pairs.shape[1], S,
                          S0, Sl, _lib.ptr(k), _lib.ptr(m), _lib.ptr(s), 1e-6, _lib.ptr(x_ph), self.C_x, 0, st)
        fm, fs = self.stats["fhr"]
        _lib.call("vt_normalize_raw", _lib.ptr(x) + 4 * S0 * p.step, B, 2 * p.N, self.N_out, fm, fs, _lib.ptr(y_raw),
                  st)
        return {"fhr_st": y_st, "fhr_ph": y_ph, "fhr_up_ph": x_ph, "fhr": y_raw}


def _sub_table(t, first, count):
    """Pair table restricted to pairs [first, first + count) (views, no copy)."""
    s = dict(t)
    s["slot_i"], s["slot_j"], s["power"] = (t[k][first:first + count] for k in ("slot_i", "slot_j", "power"))
    s["n_pairs"] = count
    return s


def load_stats(J=11, Q=4, T=16, N=4096):
    import os
    path = os.path.join(os.path.dirname(__file__), "data", f"stats_j{J}q{Q}t{T}_n{N}.npz")
    return dict(np.load(path, allow_pickle=False))


class KymatioPhaseScattering1D(torch.nn.Module):
    """Drop-in for ref/hdf5_dataset/kymatio_phase_scattering.py:11-811 (module
    API: constructor, forward, masks, selection helpers) on the HIP kernels.
    forward() returns the reference's dict: 'scattering' (B, 1+F, S) and
    'phase_corr' or 'cross_phase_corr' (B, 903, S) over all pairs, plus
    'autoc_idx'.  The fused training path (FrontEnd) computes only the selected
    pairs; this class exists for code written against the reference module."""

    def __init__(self, J, Q, T, shape, device=None, oversampling=0, max_order=2, border_mode="reflect",
                 tukey_alpha=None):
        super().__init__()
        if isinstance(Q, tuple):
            self.Q_scattering, self.Q = Q, Q[0]
        else:
            self.Q_scattering = self.Q = Q
        self.J, self.T, self.oversampling, self.max_order = J, T, oversampling, max_order
        self.border_mode, self.tukey_alpha = border_mode, tukey_alpha
        self.device = device if device is not None else torch.device("cuda")
        self.eps = 1e-14
        self.N = int(shape) if isinstance(shape, (int, float)) else int(shape[0])
        from .scattering import Scattering1D
        self.scattering = Scattering1D(J=J, shape=self.N, Q=self.Q, max_order=max_order, average=True,
                                       oversampling=oversampling, vectorize=True, out_type="array", T=T)
        self.plan = FrontEndPlan(J, self.Q, T, self.N, device=self.device)
        p = self.plan
        self.J_pad, self.pad_left, self.pad_right, self.N_padded = p.pad.J_pad, p.pad_left, p.pad_right, p.n_pad
        self.ind_start, self.ind_end = p.pad.ind_start, p.pad.ind_end
        self.center_freqs = torch.from_numpy(p.center_freqs).to(self.device)
        self.i_idx = torch.from_numpy(p.i_idx).to(self.device)
        self.j_idx = torch.from_numpy(p.j_idx).to(self.device)
        self.powers = torch.from_numpy(p.powers).to(self.device)
        self.autoc_idx = torch.from_numpy(p.autoc_idx).to(self.device)

    # ------------------------------------------------------------ selection
    def get_optimal_coefficients_for_fhr(self, j_config=11, q_config=4, t_config=16):
        """Masks of :635-760 (returned in the reference's dict structure, core keys)."""
        phase, cross = self.plan.fhr_masks()
        pm = torch.from_numpy(phase).to(self.device)
        cm = torch.from_numpy(cross).to(self.device)
        return {"phase_selection": {"optimal_mask": pm}, "cross_selection": {"cross_mask": cm},
                "recommendations": {"use_phase_mask": pm, "use_cross_mask": cm,
                                    "total_selected_features": j_config * q_config + 1 + int(pm.sum()) + int(cm.sum())}}

    # ------------------------------------------------------------ forward
    def _tukey(self, x):
        a, n = self.tukey_alpha, x.shape[-1]
        if a is None or not (0 < a <= 1):
            return x
        if a >= 1.0:
            w = torch.hann_window(n, periodic=False, device=x.device)
        else:
            tl = int(a * (n - 1) / 2.0)
            if tl == 0:
                return x
            taper = torch.hann_window(2 * tl, periodic=False, device=x.device)
            w = torch.ones(n, device=x.device)
            w[:tl] = taper[:tl]
            w[n - tl:] = taper[tl:]
        return x * w

    def forward(self, x, compute_phase=True, compute_cross_phase=False, cross_phase_same_pairs_only=False,
                cross_phase_low_pass=True, scattering_channel=0, phase_channels=None):
        x = x.to(self.device).float()
        if self.tukey_alpha is not None:
            x = self._tukey(x)
        if x.dim() == 3:
            B, C, N = x.shape
            if scattering_channel >= C:
                raise ValueError(f"scattering_channel {scattering_channel} >= {C}")
            s_in = x[:, scattering_channel, :].contiguous()
            if compute_cross_phase:
                if phase_channels is None:
                    if C < 2:
                        raise ValueError("Cross-channel correlation requires at least 2 channels")
                    phase_channels = [0, 1]
                if len(phase_channels) != 2 or any(ch >= C for ch in phase_channels):
                    raise ValueError("Invalid phase_channels for cross-channel correlation")
                ph = x[:, phase_channels, :].contiguous()
            elif phase_channels is not None:
                if len(phase_channels) != 1:
                    raise ValueError("Single-channel phase correlation requires exactly 1 channel")
                if phase_channels[0] >= C:
                    raise ValueError(f"phase_channel {phase_channels[0]} >= {C}")
                ph = x[:, phase_channels[0], :].contiguous()
            else:
                ph = s_in
        elif x.dim() == 2:
            if scattering_channel != 0:
                raise ValueError("scattering_channel must be 0 for single-channel input")
            if compute_cross_phase:
                raise ValueError("Cross-channel correlation requires multi-channel input")
            s_in, ph = x.contiguous(), (x.contiguous() if compute_phase else None)
        else:
            raise ValueError(f"Input must be 2D or 3D, got shape {x.shape}")
        S, _ = self.scattering(s_in)
        res = {"scattering": S}
        if S.shape[-1] == 0:
            raise ValueError(f"Scattering output has zero temporal dimension: {S.shape}")
        if (compute_phase or compute_cross_phase) and ph is not None:
            if ph.dim() == 2:
                ph = ph.unsqueeze(1)
            if compute_cross_phase and ph.shape[1] != 2:
                raise ValueError("Cross-channel correlation requires exactly 2 channels")
            p = self.plan
            B, C = ph.shape[0], ph.shape[1]
            if compute_cross_phase:
                sel = self.autoc_idx.cpu().numpy() if cross_phase_same_pairs_only else np.arange(len(p.i_idx))
                tab = p.tables([], sel, scattering=False)
            else:
                tab = p.tables(np.arange(len(p.i_idx)), [], scattering=False)
            pm = PAD_MODES.get(self.border_mode)
            if pm is None:
                raise ValueError(f"Unsupported border_mode: {self.border_mode}")
            xhat = torch.empty((B, C, p.n_pad, 2), device=x.device)
            launch_spectrum(p, ph, B * C, pm, xhat)
            an = torch.empty((B, tab["n_slots"], p.N, 2), device=x.device)
            launch_wavelet(p, xhat, B, C, tab, an, None, 0)
            low = (not compute_cross_phase) or cross_phase_low_pass
            out = torch.empty((B, tab["n_pairs"], p.pair_len if low else p.N), device=x.device)
            launch_pairs(p, an, B, tab, out, lowpass=low, pad_mode=pm)
            res["cross_phase_corr" if compute_cross_phase else "phase_corr"] = out
            res["autoc_idx"] = self.autoc_idx
        return res
