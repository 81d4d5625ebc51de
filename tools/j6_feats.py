"""Diagnostic: the J = 6 end-to-end test's features from the GPU front-end with polar analytic
slots on and off, saved for an oracle comparison on the CPU (gpurun_out/j6_feats.npz)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "vae-teb_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from vaeteb import _lib, synthetic  # noqa: E402
from vaeteb.frontend import FrontEnd, FrontEndPlan, load_stats  # noqa: E402

fns = _lib.lib().fns
fe = FrontEnd(FrontEndPlan(6, 1, 16, 4096, device="cuda"), load_stats(6, 1, 16, 4096))
x = torch.from_numpy(synthetic.batch(4242, 2, 4096)).cuda()
out = {}
for pol in (1, 0):
    fns["vt_fe_set_analytic_polar"](pol)
    for k, v in fe(x).items():
        out[f"p{pol}_{k}"] = v.detach().cpu().numpy()
np.savez(os.path.join(ROOT, "gpurun_out", "j6_feats.npz"), **out)
print("saved", sorted(out))
