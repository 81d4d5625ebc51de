"""Host/GPU pacing of the eager step: torch sync-debug warnings (any hidden
host synchronisation), per-step host enqueue time and how far the host runs
ahead of the GPU (event query at each step start)."""
import os
import sys
import time
import warnings

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
                  cross_phase_channels=fe.C_x, head_precision="bf16", conv_precision="bf16",
                  concurrent_encoders=True).to(dev)
tr = Trainer(model, lr=1e-3, frontend=fe)
x = torch.from_numpy(synthetic.batch(0, 256, 4096)).to(dev)
for _ in range(3):
    tr.step({"x": x})
torch.cuda.synchronize()
torch.cuda.set_sync_debug_mode("warn")
with warnings.catch_warnings(record=True) as w:
    warnings.simplefilter("always")
    tr.step({"x": x})
    torch.cuda.synchronize()
torch.cuda.set_sync_debug_mode(0)
print("sync warnings:", len(w))
for x_ in w[:10]:
    print("  ", str(x_.message)[:200], x_.filename, x_.lineno)
torch.cuda.synchronize()
evs = []
t0 = time.perf_counter()
marks = []
for i in range(20):
    e = torch.cuda.Event()
    e.record()
    evs.append(e)
    h0 = time.perf_counter()
    tr.step({"x": x})
    h1 = time.perf_counter()
    # how many earlier steps has the GPU finished when the host starts step i?
    done = sum(1 for ev in evs[:-1] if ev.query())
    marks.append((i, (h1 - h0) * 1e3, i - done))
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / 20 * 1e3
for m in marks:
    print(f"step {m[0]:2d}: host {m[1]:6.2f} ms, steps in flight at start {m[2]}")
print(f"wall per step {dt:.2f} ms")
