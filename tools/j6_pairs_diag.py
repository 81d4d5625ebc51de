"""J=6 front-end outputs per pair-kernel form (vt_fe_set_pairs_half 0 / 1 / 3), with and without the
side stream the trainer uses: max |difference| per output field against form 0 without a side
stream.  Usage: python tools/j6_pairs_diag.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vae-teb_amd"))
import torch  # noqa: E402
from vaeteb import _lib, synthetic  # noqa: E402
from vaeteb.frontend import FrontEnd, FrontEndPlan, load_stats  # noqa: E402

fns = _lib.lib().fns
for J, Q in ((6, 1), (11, 4)):
    fe = FrontEnd(FrontEndPlan(J, Q, 16, 4096, device="cuda"), load_stats(J, Q, 16, 4096))
    x = torch.from_numpy(synthetic.batch(4244, 2, 4096)).cuda()
    side = torch.cuda.Stream()
    res = {}
    for form in (0, 1, 3):
        fns["vt_fe_set_pairs_half"](form)
        for sd in (None, side):
            o = {k: v.clone() for k, v in fe(x, side=sd).items()}
            torch.cuda.synchronize()
            res[(form, sd is not None)] = o
    ref = res[(0, False)]
    for key, o in res.items():
        print(f"J={J} form {key[0]} side {int(key[1])}: " +
              " ".join(f"{k} {(o[k] - ref[k]).abs().max().item():.3e}" for k in ref), flush=True)
    for k in ("fhr_ph", "fhr_up_ph"):
        d = (res[(1, True)][k] - ref[k]).abs().amax(dim=(0, 1))
        print(f"J={J} form 1 side 1 {k} per channel:", [f"{v:.1e}" for v in d.tolist()])
    fns["vt_fe_set_pairs_half"](1)
