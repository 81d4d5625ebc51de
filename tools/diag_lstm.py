"""LSTM op on the model's real inputs (SeqVaeTebClassifier golden batch) vs torch fp64."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vae-teb_amd"), os.path.join(ROOT, "tests")]
import numpy as np, torch
from golden_util import det_fill_
from vaeteb import ops
from vaeteb.classifier import SeqVaeTebClassifier
g = np.load(os.path.join(ROOT, "tests/golden/seqvae_classifier_s16_b4.npz"))
cap = []
orig = ops.lstm
def hook(x, params):
    y = orig(x, params)
    cap.append((x.detach().clone(), [p.detach().clone() for p in params], y.detach().clone()))
    return y
ops.lstm = hook
import vaeteb.model as VM
VM.ops.lstm = hook
m = SeqVaeTebClassifier(sequence_length=16, freeze_vae=False, classifier_dropout=0.0)
det_fill_(m.vae_model); det_fill_(m.classifier)
m = m.cuda().train()
T = lambda k: torch.from_numpy(g[k]).cuda()
out = m.compute_loss(T("y_st"), T("y_ph"), T("x_ph"), T("labels"), y_raw=T("y_raw"), compute_vae_loss=True, eps=T("eps"))
for x, params, y in cap:
    In = x.shape[-1]
    ref = torch.nn.LSTM(In, 64, 4, batch_first=True).double()
    with torch.no_grad():
        for p, q in zip(ref.parameters(), params):
            p.copy_(q.double().cpu())
        yr, _ = ref(x.double().cpu())
    e = (y.double().cpu() - yr).abs()
    rel_t = ((y.double().cpu() - yr).norm(dim=(0, 2)) / yr.norm(dim=(0, 2)))
    print("In", In, "rel-L2", ((y.double().cpu() - yr).norm() / yr.norm()).item(), "max abs", e.max().item())
    print("  per t:", " ".join(f"{v:.1e}" for v in rel_t.tolist()))
    # unit-wise worst
    idx = torch.nonzero(e == e.max())[0].tolist()
    print("  worst at", idx, y.double().cpu()[tuple(idx)].item(), yr[tuple(idx)].item())
