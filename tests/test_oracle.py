"""The oracle pinned against the reference's own known answers (CPU only).

* kymatio's shipped known-answer vector test_data_1d.npz
  (ref/kymatio/tests/scattering1d/test_torch_scattering1d.py:82-113)
* fixtures produced by running the reference in the build container
  (tools/gen_golden.py): filter banks, Scattering1D, the phase front-end,
  normalisation, the full SeqVaeTeb training step and the tiny config-1 model.
"""
import re

import numpy as np
import pytest
import torch

from oracle import frontend_ref as F
from oracle import model_ref as M
from golden_util import det_fill_


def rel_l2_per_channel(a, b):
    return np.sqrt(((a - b) ** 2).sum(-1) / np.maximum((b ** 2).sum(-1), 1e-30))


def test_kymatio_known_answer(golden):
    d = golden("kymatio_test_data_1d")
    J = int(d["J"])
    S = F.scattering1d(d["x"], J, int(d["Q"]), 2 ** J, max_order=2)
    assert S.shape == d["Sx"].shape
    assert np.allclose(S, d["Sx"], rtol=1e-5, atol=1e-7)   # torch.allclose defaults


@pytest.mark.parametrize("cfg", [(11, 4, 16, 4096), (6, 1, 16, 4096), (8, 12, 256, 16384)])
def test_filter_bank(golden, cfg):
    J, Q, T, N = cfg
    g = golden(f"filters_j{J}q{Q}t{T}_n{N}")
    J_pad, pl, pr, i0, i1 = F.padding_plan(N, J, Q, T)
    assert (J_pad, pl, pr) == (int(g["J_pad"]), int(g["pad_left"]), int(g["pad_right"]))
    assert [i0[k] for k in range(J + 1)] == list(g["ind_start"])
    phi, psi1, psi2, tmax = F.filter_bank(J_pad, J, Q, T)
    assert tmax == int(g["t_max_phi"])
    assert np.allclose([p["xi"] for p in psi1], g["xi1"], rtol=0, atol=1e-15)
    assert [p["j"] for p in psi2] == list(g["j2"])
    psi = np.stack([p["levels"][0] for p in psi1])
    assert np.allclose(psi.sum(1), g["psi1_sum"], rtol=1e-12, atol=1e-12)
    if "psi1" in g.files:
        assert np.abs(psi - g["psi1"]).max() < 1e-13
    assert np.allclose([lv.sum() for lv in phi["levels"]], g["phi_levels_sum"], rtol=1e-12)


@pytest.mark.parametrize("name", ["j6q1t16_n4096_o1", "j6q1t16_n4096_o2", "j11q4t16_n4096_o1",
                                  "j8q12t256_n16384_o2"])
def test_scattering(golden, name):
    g = golden("scattering_" + name)
    J, Q, T, N, o = map(int, re.findall(r"\d+", name))
    S = F.scattering1d(g["x"], J, Q, T, o)
    assert S.shape == g["S"].shape
    assert np.abs(S - g["S"]).max() <= 2e-6 * np.abs(g["S"]).max()
    S64 = F.scattering1d(g["x"], J, Q, T, o, dtype=np.float64)
    assert np.abs(S64 - g["S64"]).max() <= 1e-8 * np.abs(g["S64"]).max()


@pytest.mark.parametrize("J,Q", [(11, 4), (6, 1)])
def test_phase_frontend(golden, J, Q):
    g = golden(f"frontend_j{J}q{Q}t16_n4096")
    fe = F.PhaseFrontEnd(J, Q, 16, 4096)
    pm, cm = fe.masks()
    assert (pm == g["phase_mask"]).all() and (cm == g["cross_mask"]).all()
    x = g["x"]
    rp = fe.forward(x, compute_phase=True, pair_subset=pm)
    rc = fe.forward(x, compute_phase=False, compute_cross_phase=True, pair_subset=cm)
    assert rel_l2_per_channel(rp["scattering"], g["fhr_st"]).max() < 1e-4
    # Phase acceleration (atan2 * power, power <= 32) is ill-conditioned and the
    # low-pass cancels most of the product's energy, so channel errors are
    # measured against the cancellation-free scale ||lowpass(|a_i||a_j|)||
    # (see DESIGN.md "Parity tolerances").  Budget: 2x the reference's own
    # fp32-vs-fp64 error, taken over the channel distribution (max and median):
    # non-integer powers make atan2's branch cut a discontinuity, so two fp32
    # implementations flip at different samples and per-channel agreement is
    # not attainable; the error distribution is.
    fe64 = F.PhaseFrontEnd(J, Q, 16, 4096, dtype=np.float64)
    a64 = fe64.analytic(x[:, [0, 1]])
    for key, out, sel, ai, aj in (("fhr_ph", rp["phase_corr"], pm, a64[:, 0], a64[:, 0]),
                                  ("fhr_up_ph", rc["cross_phase_corr"], cm, a64[:, 0], a64[:, 1])):
        ii, jj = fe64.i_idx[sel], fe64.j_idx[sel]
        scale = np.sqrt((fe64._lowpass(np.abs(ai[:, ii]) * np.abs(aj[:, jj]) + 0j, 256) ** 2).sum(-1))
        err = np.sqrt(((out - g[key + "64"]) ** 2).sum(-1)) / scale
        ref_err = np.sqrt(((g[key] - g[key + "64"]) ** 2).sum(-1)) / scale
        assert err.max() <= 2 * ref_err.max() + 1e-5, key
        assert np.median(err) <= 2 * np.median(ref_err) + 1e-6, key
    r64 = fe64.forward(x, compute_phase=True, pair_subset=pm)
    assert rel_l2_per_channel(r64["phase_corr"], g["fhr_ph64"]).max() < 1e-10
    a = fe.analytic(x[:, [0, 1]])
    ref = g["analytic_ch0_f0"]
    assert np.abs(a[:, 0, 0] - ref).max() <= 1e-4 * np.abs(ref).max()


@pytest.mark.parametrize("J,Q", [(11, 4), (6, 1)])
def test_normalize(golden, J, Q):
    g = golden(f"normalize_j{J}q{Q}t16_n4096")
    for f in ("fhr", "up", "fhr_st", "fhr_ph", "fhr_up_ph"):
        out = F.normalize(g["in_" + f], f, g[f + "_mean"], g[f + "_variance"])
        assert np.allclose(out, g["out_" + f], rtol=1e-5, atol=1e-5), f


@pytest.mark.parametrize("name", ["model_s16_b4", "model_s4_b3", "model_s256_b2"])
def test_model_step(golden, name):
    g = golden(name)
    m = det_fill_(M.SeqVaeTebRef(int(g["S"])))
    names = [k for k, _ in m.named_parameters()]
    assert names == list(g["param_names"])
    T = lambda k: torch.from_numpy(g[k])
    fw, L, grads, gn = M.train_step(m, dict(y_st=T("y_st"), y_ph=T("y_ph"), x_ph=T("x_ph"), y_raw=T("y_raw")),
                                    T("eps"), float(g["beta"]))
    for k in ("total_loss", "nll_loss", "kld_loss", "mse_loss"):
        assert abs(L[k].item() - float(g["loss_" + k])) <= 1e-6 * abs(float(g["loss_" + k])) + 1e-7
    gl2 = np.array([grads[k].double().norm().item() for k in names])
    assert np.allclose(gl2, g["grad_l2"], rtol=1e-5, atol=1e-9)
    for i, k in enumerate(names):
        if f"grad_{i}" in g.files:
            assert np.allclose(grads[k].numpy(), g[f"grad_{i}"], rtol=1e-5, atol=1e-7), k
        elif f"gradrows_{i}" in g.files:
            assert np.allclose(grads[k][:16].numpy(), g[f"gradrows_{i}"], rtol=1e-5, atol=1e-7), k
    if "after_0" in g.files:
        sd = m.state_dict()
        for i, k in enumerate(names):
            assert np.allclose(sd[k].numpy(), g[f"after_{i}"], rtol=1e-6, atol=1e-7), k


def test_transfer_entropy(golden):
    """measure_transfer_entropy (ref/model/vae_teb_model.py:1194-1226) after one
    train-mode forward: eval-mode BatchNorm on the updated running statistics."""
    g, t = golden("model_s16_b4"), golden("te_s16_b4")
    m = det_fill_(M.SeqVaeTebRef(16))
    m.train()
    T = lambda k: torch.from_numpy(g[k])
    with torch.no_grad():
        m(T("y_st"), T("y_ph"), T("x_ph"), T("eps"))
    te = m.measure_transfer_entropy(T("y_st"), T("y_ph"), T("x_ph"))
    assert not m.training
    assert np.allclose(te.numpy(), t["te"], rtol=1e-5, atol=1e-6)
    assert abs(m.measure_transfer_entropy(T("y_st"), T("y_ph"), T("x_ph"), reduce_mean=True).item()
               - float(t["te_mean"])) <= 1e-6 * abs(float(t["te_mean"]))


def test_tiny_c1(golden):
    g = golden("tiny_c1")
    m = det_fill_(M.TinyVaeTebRef())
    r = m(torch.from_numpy(g["x"]), torch.from_numpy(g["eps"]))
    r["total"].backward()
    assert abs(r["total"].item() - float(g["total"])) < 1e-5
    for i, (k, p) in enumerate(m.named_parameters()):
        assert np.allclose(p.grad.numpy(), g[f"grad_{i}"], rtol=1e-5, atol=1e-6), k


def test_classifier(golden):
    """Config 4 head: the oracle vs the reference FHRInceptionTimeClassifier
    (conv_long cropped to L) — logits, CE, dz, every gradient, BN stats."""
    from oracle import classifier_ref as C
    g = golden("classifier_s64_b4")
    m = det_fill_(C.InceptionTimeClassifier(dropout=0.0))
    names = [k for k, _ in m.named_parameters()]
    assert names == list(g["param_names"])
    m.train()
    z = torch.from_numpy(g["z"]).requires_grad_(True)
    logits = m(z)
    loss = torch.nn.functional.cross_entropy(logits, torch.from_numpy(g["labels"]))
    loss.backward()
    assert np.allclose(logits.detach().numpy(), g["logits"], rtol=1e-5, atol=1e-6)
    assert abs(loss.item() - float(g["loss"])) < 1e-6
    assert np.allclose(z.grad.numpy(), g["dz"], rtol=1e-4, atol=1e-7)
    for i, (k, p) in enumerate(m.named_parameters()):
        ref = g[f"grad_{i}"]
        err = np.linalg.norm(p.grad.numpy() - ref) / max(np.linalg.norm(ref), 1e-30)
        assert err < 1e-5, (k, err)
    sd = m.state_dict()
    for i, k in enumerate(g["bn_names"]):
        assert np.allclose(sd[k].numpy(), g[f"bn_{i}"], rtol=1e-5, atol=1e-7), k


def test_seqvae_classifier_loss(golden):
    """SeqVaeTebClassifier.compute_loss (ELBO beta 1 + CE, end to end) at S=16."""
    from oracle import classifier_ref as C
    g = golden("seqvae_classifier_s16_b4")
    S = int(g["S"])
    vae = det_fill_(M.SeqVaeTebRef(S))
    clf = det_fill_(C.InceptionTimeClassifier(dropout=0.0))
    vae.train()
    clf.train()
    T = lambda k: torch.from_numpy(g[k])
    out = C.seqvae_classifier_loss(vae, clf, T("y_st"), T("y_ph"), T("x_ph"), T("labels"), T("y_raw"), T("eps"))
    out["total_loss"].backward()
    for k in ("classification_loss", "vae_loss", "total_loss"):
        assert abs(out[k].item() - float(g[k])) <= 1e-5 * abs(float(g[k])), k
    params = [("vae_model." + k, p) for k, p in vae.named_parameters()] + \
             [("classifier." + k, p) for k, p in clf.named_parameters()]
    assert [k for k, _ in params] == list(g["param_names"])
    gl2 = np.array([p.grad.double().norm().item() for _, p in params])
    assert np.allclose(gl2, g["grad_l2"], rtol=2e-4, atol=1e-8)
