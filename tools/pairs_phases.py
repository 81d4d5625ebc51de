"""Phase timeline of the training-geometry pair kernel (k_fe_pairs8k): wave 0's
wall clock (100 MHz) at each phase boundary of every workgroup, averaged per
launch (vt_fe_set_pairs_stamps).  Usage: python tools/pairs_phases.py [B]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vae-teb_amd"))
import torch  # noqa: E402
from vaeteb import synthetic  # noqa: E402
from vaeteb._lib import call  # noqa: E402
from vaeteb.frontend import FrontEnd, FrontEndPlan, load_stats  # noqa: E402

dev = torch.device("cuda:0")
B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
plan = FrontEndPlan(11, 4, 16, 4096, device=dev)
fe = FrontEnd(plan, load_stats(11, 4, 16, 4096))
x = torch.from_numpy(synthetic.batch(0, B, 4096)).to(dev)
for _ in range(3):
    fe(x)
torch.cuda.synchronize()
npairs = [int(plan.phase_mask.sum()), int(plan.cross_mask.sum())]
buf = torch.zeros(B * sum(npairs) * 8, dtype=torch.int64, device=dev)
call("vt_fe_set_pairs_stamps", buf.data_ptr())
fe(x)
torch.cuda.synchronize()
call("vt_fe_set_pairs_stamps", None)
st = buf.cpu().double()
names = ["loads+accel", "col read+pass1", "pass2", "pass3+phi", "ifft512", "store"]
off = 0
for k, n in enumerate(npairs):
    s = st[off: off + B * n * 8].view(B * n, 8)
    off += B * n * 8
    if s[:, 0].eq(0).all():
        print("launch", k, "no stamps (other variant)")
        continue
    span = (s[:, 6].max() - s[:, 0].min()) * 10 / 1000
    d = (s[:, 1:7] - s[:, 0:6]) * 10 / 1000   # us
    tot = (s[:, 6] - s[:, 0]) * 10 / 1000
    print(f"launch {k}: {n} pairs x B={B}: span {span:.1f} us, per-WG mean {tot.mean():.2f} us "
          f"(p10 {tot.quantile(0.1):.2f}, p90 {tot.quantile(0.9):.2f})")
    for i, nm in enumerate(names):
        print(f"   {nm:16s} mean {d[:, i].mean():7.3f} us  p90 {d[:, i].quantile(0.9):7.3f}")
