"""Diagnostic: front-end features with polar analytic slots vs complex, per channel (J = 6 and 11)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "vae-teb_amd")]
import torch  # noqa: E402

from vaeteb import _lib, synthetic  # noqa: E402
from vaeteb.frontend import FrontEnd, FrontEndPlan, load_stats  # noqa: E402

fns = _lib.lib().fns
for J, Q in ((6, 1), (11, 4)):
    fe = FrontEnd(FrontEndPlan(J, Q, 16, 4096, device="cuda"), load_stats(J, Q, 16, 4096))
    x = torch.from_numpy(synthetic.batch(4242, 2, 4096)).cuda()
    out = {}
    for pol in (1, 0):
        fns["vt_fe_set_analytic_polar"](pol)
        out[pol] = {k: v.clone() for k, v in fe(x).items()}
        out[pol]["raw"] = fe.raw(x)["pairs"].clone()
    torch.cuda.synchronize()
    for k in ("fhr_ph", "fhr_up_ph", "raw"):
        a, b = out[1][k].double(), out[0][k].double()
        ch = -1 if k != "raw" else 1
        d = (a - b).abs().amax(dim=tuple(i for i in range(a.dim()) if i != (a.dim() - 1 if k != "raw" else 1)))
        m = b.abs().amax(dim=tuple(i for i in range(b.dim()) if i != (b.dim() - 1 if k != "raw" else 1)))
        worst = torch.argsort(d / m.clamp_min(1e-30), descending=True)[:5].tolist()
        print(f"J{J} {k}: max abs diff {d.max().item():.3e}; worst channels (diff, max|v|): " +
              ", ".join(f"{c}: ({d[c].item():.2e}, {m[c].item():.2e})" for c in worst), flush=True)
    fns["vt_fe_set_analytic_polar"](1)
