"""Where the step's device-to-device copies (__amd_rocclr_copyBuffer) come from:
torch.profiler over a few eager training steps, aten copy/clone/cat ops grouped
by their Python call site."""
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vae-teb_amd"))
import torch  # noqa: E402
from vaeteb import synthetic  # noqa: E402
from vaeteb.frontend import FrontEnd, FrontEndPlan, load_stats  # noqa: E402
from vaeteb.model import SeqVaeTeb  # noqa: E402
from vaeteb.train import Trainer  # noqa: E402

dev = torch.device("cuda:0")
plan = FrontEndPlan(11, 4, 16, 4096, device=dev)
fe = FrontEnd(plan, load_stats(11, 4, 16, 4096))
torch.manual_seed(1234)
model = SeqVaeTeb(sequence_length=plan.S, scattering_channels=fe.C_st, phase_channels=fe.C_ph,
                  cross_phase_channels=fe.C_x, head_precision="bf16", concurrent_encoders=True).to(dev)
tr = Trainer(model, lr=1e-3, frontend=fe)
x = torch.from_numpy(synthetic.batch(0, 256, 4096)).to(dev)
for _ in range(3):
    tr.step({"x": x})
torch.cuda.synchronize()
STEPS = 2
with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU], with_stack=True) as prof:
    for _ in range(STEPS):
        tr.step({"x": x})
    torch.cuda.synchronize()
cnt = collections.Counter()
names = ("aten::copy_", "aten::clone", "aten::cat", "aten::contiguous", "aten::_to_copy", "aten::index",
         "aten::stack", "aten::where", "aten::zero_", "aten::fill_")
for ev in prof.events():
    if ev.name not in names:
        continue
    st = [f for f in (ev.stack or []) if "vaeteb" in f or "bench" in f or "train" in f]
    cnt[(ev.name, " <- ".join(st[:3]))] += 1
for (n, s), c in cnt.most_common(60):
    print(f"{c / STEPS:6.1f}/step {n:18s} {s}")
