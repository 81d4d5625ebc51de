"""Per-parameter gradient-norm deviation of SeqVaeTebClassifier vs the reference golden."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vae-teb_amd"), os.path.join(ROOT, "tests")]
import numpy as np, torch
from golden_util import det_fill_
from vaeteb.classifier import SeqVaeTebClassifier
g = np.load(os.path.join(ROOT, "tests/golden/seqvae_classifier_s16_b4.npz"))
m = SeqVaeTebClassifier(sequence_length=16, freeze_vae=False, classifier_dropout=0.0)
det_fill_(m.vae_model); det_fill_(m.classifier)
m = m.cuda().train()
T = lambda k: torch.from_numpy(g[k]).cuda()
out = m.compute_loss(T("y_st"), T("y_ph"), T("x_ph"), T("labels"), y_raw=T("y_raw"), compute_vae_loss=True, eps=T("eps"))
print({k: (out[k].item(), float(g[k])) for k in ("classification_loss", "vae_loss", "total_loss")})
out["total_loss"].backward()
names = [k for k, _ in m.named_parameters()]
gl2 = np.array([p.grad.norm().item() for _, p in m.named_parameters()])
err = np.abs(gl2 - g["grad_l2"]) / np.maximum(g["grad_l2"], 1e-12)
for i in np.argsort(-err)[:25]:
    print(f"{err[i]:.2e} {gl2[i]:.4e} {g['grad_l2'][i]:.4e} {names[i]}")

# HIP vs the fp64 oracle, beside the reference's own fp32-vs-fp64 deviation
from oracle import model_ref as M, classifier_ref as C
vae = det_fill_(M.SeqVaeTebRef(16)).double().train(); clf = det_fill_(C.InceptionTimeClassifier(dropout=0.0)).double().train()
D = lambda k: torch.from_numpy(g[k]).double() if g[k].dtype != np.int64 else torch.from_numpy(g[k])
o64 = C.seqvae_classifier_loss(vae, clf, D("y_st"), D("y_ph"), D("x_ph"), D("labels"), D("y_raw"), D("eps"))
o64["total_loss"].backward()
ps = [p for _, p in vae.named_parameters()] + [p for _, p in clf.named_parameters()]
g64 = np.array([p.grad.norm().item() for p in ps])
e_hip = np.abs(gl2 - g64) / np.maximum(g64, 1e-12)
e_ref = np.abs(g["grad_l2"] - g64) / np.maximum(g64, 1e-12)
print("HIP vs fp64: max", e_hip.max(), "median", np.median(e_hip), "| ref fp32 vs fp64: max", e_ref.max(), "median", np.median(e_ref))
for i in np.argsort(-e_hip)[:12]:
    print(f"hip {e_hip[i]:.2e} ref {e_ref[i]:.2e} {names[i]}")
