"""GPU-only time of the eager training step: the main stream sleeps while the
host enqueues n steps, so the GPU then runs them back to back with no host
limit (events around the steps).  usage: gpu_bound_probe.py [n_steps]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vae-teb_amd"))
import torch  # noqa: E402
from vaeteb import synthetic  # noqa: E402
from vaeteb.frontend import FrontEnd, FrontEndPlan, load_stats  # noqa: E402
from vaeteb.model import SeqVaeTeb  # noqa: E402
from vaeteb.train import Trainer  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 2
dev = torch.device("cuda:0")
plan = FrontEndPlan(11, 4, 16, 4096, device=dev)
fe = FrontEnd(plan, load_stats(11, 4, 16, 4096))
torch.manual_seed(1234)
model = SeqVaeTeb(sequence_length=plan.S, scattering_channels=fe.C_st, phase_channels=fe.C_ph,
                  cross_phase_channels=fe.C_x, head_precision="bf16", conv_precision="bf16", mlp_precision="bf16",
                  concurrent_encoders=True).to(dev)
tr = Trainer(model, lr=1e-3, frontend=fe)
x = torch.from_numpy(synthetic.batch(0, 256, 4096)).to(dev)
for _ in range(3):
    tr.step({"x": x})
torch.cuda.synchronize()
for rep in range(3):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda._sleep(int(400e6))        # ~0.2 s of GPU time: covers the host enqueue below
    e0.record()
    t0 = time.perf_counter()
    for _ in range(n):
        tr.step({"x": x})
    e1.record()
    t_host = time.perf_counter() - t0
    torch.cuda.synchronize()
    print(f"{n} steps: GPU {e0.elapsed_time(e1) / n:.3f} ms/step (host enqueue {t_host / n * 1e3:.3f} ms/step)",
          flush=True)
