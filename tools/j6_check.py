"""Diagnostic (J = 6 end-to-end test): the Trainer step from raw windows vs the same step
from the features a separate front-end call produced (polar analytic slots on)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "vae-teb_amd"), os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from golden_util import det_fill_  # noqa: E402
from vaeteb import synthetic  # noqa: E402
from vaeteb.frontend import FrontEnd, FrontEndPlan, load_stats  # noqa: E402
from vaeteb.model import SeqVaeTeb  # noqa: E402
from vaeteb.train import Trainer  # noqa: E402

st = load_stats(6, 1, 16, 4096)
fe = FrontEnd(FrontEndPlan(6, 1, 16, 4096, device="cuda"), st)
widths = (fe.C_st, fe.C_ph, fe.C_x)
x = torch.from_numpy(synthetic.batch(4242, 2, 4096)).cuda()
eps = torch.from_numpy(np.random.default_rng(6).standard_normal((2, 256, 32)).astype(np.float32)).cuda()
feats = {k: v.clone() for k, v in fe(x).items()}
res = []
for mode in ("raw", "feats", "raw2"):
    m = det_fill_(SeqVaeTeb(sequence_length=256, scattering_channels=widths[0], phase_channels=widths[1],
                            cross_phase_channels=widths[2])).cuda()
    tr = Trainer(m, lr=1e-3, frontend=fe if mode != "feats" else None)
    batch = {"x": x} if mode != "feats" else feats
    L = tr.step(batch, eps=eps)
    torch.cuda.synchronize()
    res.append((mode, float(L["total_loss"]), float(L["grad_norm"]), tr.state.g.clone()))
    print(mode, res[-1][1], res[-1][2], flush=True)
g0 = res[0][3]
for mode, l, gn, g in res[1:]:
    print(f"{mode} vs raw: max |dg| {(g - g0).abs().max().item():.3e}  (max |g| {g0.abs().max().item():.3e})")
