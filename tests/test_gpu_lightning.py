"""Eval-mode BatchNorm paths (validation, frozen VAE, predict), the frozen-VAE
classifier configuration (the reference default) and the LightSeqVaeTeb
mirror's optimisation step on the HIP kernels, vs the torch-CPU oracle
(pinned to the reference by tests/test_oracle.py).  Tolerances as in
test_gpu_model.py (fp32 vs fp32 in different summation orders)."""
import pytest
import torch

from golden_util import det_fill_

pytestmark = pytest.mark.gpu


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def _random_running_stats_(*mods):
    g = torch.Generator().manual_seed(3)
    keys = None
    for m in mods:
        sd = m.state_dict()
        ks = sorted(k for k in sd if k.endswith(("running_mean", "running_var")))
        keys = keys or ks
        assert ks == keys
    for k in keys:
        shape = mods[0].state_dict()[k].shape
        v = (torch.randn(shape, generator=g) * 0.2) if k.endswith("mean") else (1 + torch.rand(shape, generator=g))
        for m in mods:
            m.state_dict()[k].copy_(v)


@pytest.fixture(scope="module")
def batch(golden):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    g = golden("model_s16_b4")
    return {k: torch.from_numpy(g[k]) for k in ("y_st", "y_ph", "x_ph", "y_raw", "eps")}


def test_vae_eval_mode_vs_oracle(batch):
    from oracle import model_ref as M
    from vaeteb.model import SeqVaeTeb
    ref = det_fill_(M.SeqVaeTebRef(16))
    m = det_fill_(SeqVaeTeb(sequence_length=16))
    _random_running_stats_(ref, m)
    m = m.cuda().eval()
    ref.eval()
    with torch.no_grad():
        fr = ref(batch["y_st"], batch["y_ph"], batch["x_ph"], batch["eps"])
        fw = m(*(batch[k].cuda() for k in ("y_st", "y_ph", "x_ph")), eps=batch["eps"].cuda())
    for k in ("z", "mu_pr", "logvar_pr", "linear_output"):
        assert rel(fw[k], fr[k]) < 5e-5, k


def test_classifier_eval_mode_vs_oracle():
    from oracle import classifier_ref as C
    from vaeteb.classifier import FHRInceptionTimeClassifier
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ref = det_fill_(C.InceptionTimeClassifier(dropout=0.2))
    m = det_fill_(FHRInceptionTimeClassifier(dropout=0.2))
    _random_running_stats_(ref, m)
    ref.eval()
    m = m.cuda().eval()
    z = torch.randn(3, 64, 32)
    with torch.no_grad():
        assert rel(m(z.cuda()), ref(z)) < 2e-5


def test_frozen_vae_classifier_vs_oracle(batch):
    """SeqVaeTebClassifier(freeze_vae=True): VAE in eval mode without gradients,
    classifier trained (ref/model/vae_teb_model.py:1296-1320, :1350-1390)."""
    from oracle import classifier_ref as C
    from oracle import model_ref as M
    from vaeteb.classifier import SeqVaeTebClassifier
    ref_vae, ref_clf = det_fill_(M.SeqVaeTebRef(16)), det_fill_(C.InceptionTimeClassifier(dropout=0.0))
    m = SeqVaeTebClassifier(sequence_length=16, freeze_vae=True, classifier_dropout=0.0)
    det_fill_(m.vae_model)
    det_fill_(m.classifier)
    _random_running_stats_(ref_vae, m.vae_model)
    m = m.cuda().train()
    labels = torch.tensor([0, 1, 1, 0])
    out = m.compute_loss(*(batch[k].cuda() for k in ("y_st", "y_ph", "x_ph")), labels.cuda(),
                         y_raw=batch["y_raw"].cuda(), compute_vae_loss=True, eps=batch["eps"].cuda())
    out["total_loss"].backward()
    ref_vae.eval()
    ref_clf.train()
    with torch.no_grad():
        fw = ref_vae(batch["y_st"], batch["y_ph"], batch["x_ph"], batch["eps"])
        vl = ref_vae.compute_loss(fw, batch["y_st"], batch["y_ph"], batch["y_raw"], beta=1.0)["total_loss"]
    ce = torch.nn.functional.cross_entropy(ref_clf(fw["z"]), labels)
    (ce + 0.1 * vl).backward()
    assert abs(out["vae_loss"].item() - vl.item()) <= 2e-5 * abs(vl.item())
    assert abs(out["classification_loss"].item() - ce.item()) <= 2e-5 * abs(ce.item())
    assert all(p.grad is None for p in m.vae_model.parameters())
    rp = dict(ref_clf.named_parameters())
    worst = max((rel(p.grad, rp[k].grad), k) for k, p in m.classifier.named_parameters())
    assert worst[0] < 1e-4, worst
    preds, probs = m.predict(*(batch[k].cuda() for k in ("y_st", "y_ph", "x_ph")))
    assert preds.shape == (4,) and torch.allclose(probs.sum(-1), torch.ones(4, device="cuda"))


def test_light_module_fit_step_vs_oracle(batch):
    """fit(): zero_grad -> training_step -> backward -> clip 0.5 -> AdamW(0.9, 0.999)
    (Lightning settings, ref/model/pytorch_lightning_modules.py:537-564 and the
    gradient_clip_val of ref/model/graph_model.py) vs the oracle step."""
    from oracle import model_ref as M
    from vaeteb.lightning import LightSeqVaeTeb, fit
    from vaeteb.model import SeqVaeTeb
    ref = det_fill_(M.SeqVaeTebRef(16))
    M.train_step(ref, batch, batch["eps"], 1e-5, lr=1e-3, clip=0.5, betas=(0.9, 0.999))
    model = det_fill_(SeqVaeTeb(sequence_length=16)).cuda()
    eps = batch["eps"].cuda()
    fwd = model.forward
    model.forward = lambda a, b, c, eps_=None: fwd(a, b, c, eps=eps)
    lm = LightSeqVaeTeb(model, lr=1e-3, beta_schedule="constant", beta_const_val=1e-5)
    cb = {"fhr_st": batch["y_st"].cuda(), "fhr_ph": batch["y_ph"].cuda(), "fhr_up_ph": batch["x_ph"].cuda(),
          "fhr": batch["y_raw"].cuda()}
    logged = fit(lm, [cb], max_epochs=1, gradient_clip_val=0.5)
    assert set(logged) >= {"kld_beta", "train/total_loss", "train/nll_loss", "train/kld_loss"}
    sd, rsd = model.state_dict(), ref.state_dict()
    worst = max((rel(sd[k], v), k) for k, v in rsd.items() if v.dtype == torch.float32)
    assert worst[0] < 1e-4, worst


def test_fit_validation_runs_in_eval_mode(batch):
    """fit() validates in eval mode (Lightning semantics): BatchNorm running
    statistics are untouched by validation batches, and training mode is
    restored afterwards (advisor round 1)."""
    from vaeteb.lightning import LightSeqVaeTeb, fit
    from vaeteb.model import SeqVaeTeb
    model = det_fill_(SeqVaeTeb(sequence_length=16)).cuda()
    _random_running_stats_(model)
    before = {k: v.clone() for k, v in model.state_dict().items() if k.endswith(("running_mean", "running_var"))}
    lm = LightSeqVaeTeb(model, lr=1e-3, beta_schedule="constant", beta_const_val=1e-5)
    cb = {"fhr_st": batch["y_st"].cuda(), "fhr_ph": batch["y_ph"].cuda(), "fhr_up_ph": batch["x_ph"].cuda(),
          "fhr": batch["y_raw"].cuda()}
    logged = fit(lm, [], max_epochs=1, val_loader=[cb])
    assert "val/total_loss" in logged
    sd = model.state_dict()
    assert all(torch.equal(sd[k], v) for k, v in before.items())
    assert model.training
