"""Run-to-run determinism of the SeqVaeTebClassifier forward (same process, same inputs)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vae-teb_amd"), os.path.join(ROOT, "tests")]
import numpy as np, torch
from golden_util import det_fill_
from vaeteb.classifier import SeqVaeTebClassifier
g = np.load(os.path.join(ROOT, "tests/golden/seqvae_classifier_s16_b4.npz"))
T = lambda k: torch.from_numpy(g[k]).cuda()
outs = []
for rep in range(3):
    m = SeqVaeTebClassifier(sequence_length=16, freeze_vae=False, classifier_dropout=0.0)
    det_fill_(m.vae_model); det_fill_(m.classifier)
    m = m.cuda().train()
    z, fw = m.extract_latent_features(T("y_st"), T("y_ph"), T("x_ph"), return_all_outputs=True, eps=T("eps"))
    logits = m.classifier(z)
    outs.append((z.detach().clone(), logits.detach().clone()))
    print(rep, logits.flatten().tolist())
for i in (1, 2):
    print("z equal", torch.equal(outs[0][0], outs[i][0]), "logits equal", torch.equal(outs[0][1], outs[i][1]))
# classifier alone on a fixed z, 3 times
from vaeteb.classifier import FHRInceptionTimeClassifier
c = det_fill_(FHRInceptionTimeClassifier(dropout=0.0)).cuda().train()
zz = outs[0][0]
r = [c(zz).detach().clone() for _ in range(3)]
print("classifier alone equal", torch.equal(r[0], r[1]), torch.equal(r[0], r[2]), (r[0] - r[1]).abs().max().item())
