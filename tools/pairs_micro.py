"""Pair-kernel forms side by side: the front-end at B = 256 run 10 times per form of
vt_fe_set_pairs_half (0 full image, 1 half image at 3 workgroups / CU, 2 at 4), for a rocprofv3
kernel trace or --pmc pass (each form is its own kernel instance).  Prints HIP-event times of
the whole front-end per form too.  Usage: python tools/pairs_micro.py [forms, default 0,1,2]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vae-teb_amd"))
import torch  # noqa: E402
from vaeteb import _lib, synthetic  # noqa: E402
from vaeteb.frontend import FrontEnd, FrontEndPlan, load_stats  # noqa: E402

dev = torch.device("cuda:0")
forms = [int(f) for f in (sys.argv[1] if len(sys.argv) > 1 else "0,1,2").split(",")]
plan = FrontEndPlan(11, 4, 16, 4096, device=dev)
fe = FrontEnd(plan, load_stats(11, 4, 16, 4096))
x = torch.from_numpy(synthetic.batch(0, 256, 4096)).to(dev)
fns = _lib.lib().fns
for f in forms:
    fns["vt_fe_set_pairs_half"](f)
    for _ in range(3):
        fe(x)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(10):
        fe(x)
    b.record()
    torch.cuda.synchronize()
    print(f"form {f}: front-end {a.elapsed_time(b) / 10:.3f} ms per batch of 256", flush=True)
