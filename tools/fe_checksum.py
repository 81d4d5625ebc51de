"""SHA-256 of the training-geometry front-end's features (J=11 Q=4 T=16, N=4096, B=64, seeded
synthetic windows): run under two kernel-selection settings (e.g. VAETEB_WAVELET_LP=0 / 1) to
check that a variant writes the same bits."""
import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vae-teb_amd"))
import torch  # noqa: E402
from vaeteb import synthetic  # noqa: E402
from vaeteb.frontend import FrontEnd, FrontEndPlan, load_stats  # noqa: E402

fe = FrontEnd(FrontEndPlan(11, 4, 16, 4096, device="cuda"), load_stats(11, 4, 16, 4096))
out = fe(torch.from_numpy(synthetic.batch(77, 64, 4096)).cuda())
torch.cuda.synchronize()
h = hashlib.sha256()
for k in sorted(out):
    h.update(out[k].detach().cpu().numpy().tobytes())
print(" ".join(f"{k}{tuple(out[k].shape)}" for k in sorted(out)), h.hexdigest())
