"""hipGraph capture probe of the c2 training step: capture Trainer's step
(front-end included) at the given head / conv precision, replay it, and time
replay vs eager.  usage: graph_probe.py --heads bf16 --conv fp32 [--B 256]"""
import argparse
import faulthandler
import os
import sys
import time

faulthandler.enable()
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vae-teb_amd"))
import torch  # noqa: E402
from vaeteb import synthetic  # noqa: E402
from vaeteb.frontend import FrontEnd, FrontEndPlan, load_stats  # noqa: E402
from vaeteb.model import SeqVaeTeb  # noqa: E402
from vaeteb.train import Trainer  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--heads", default="bf16")
ap.add_argument("--conv", default="bf16")
ap.add_argument("--B", type=int, default=256)
ap.add_argument("--steps", type=int, default=10)
ap.add_argument("--serial", action="store_true")
a = ap.parse_args()
dev = torch.device("cuda:0")
plan = FrontEndPlan(11, 4, 16, 4096, device=dev)
fe = FrontEnd(plan, load_stats(11, 4, 16, 4096))
torch.manual_seed(1234)
model = SeqVaeTeb(sequence_length=plan.S, scattering_channels=fe.C_st, phase_channels=fe.C_ph,
                  cross_phase_channels=fe.C_x, head_precision=a.heads, conv_precision=a.conv,
                  concurrent_encoders=not a.serial).to(dev)
tr = Trainer(model, lr=1e-3, frontend=fe)
x = torch.from_numpy(synthetic.batch(0, a.B, 4096)).to(dev)
for _ in range(3):
    tr.step({"x": x})
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(a.steps):
    L = tr.step({"x": x})
torch.cuda.synchronize()
eager = (time.perf_counter() - t) / a.steps * 1e3
print(f"eager {eager:.3f} ms/step loss {L['total_loss'].item():.6f}", flush=True)
print("capturing", flush=True)
cap = tr.capture({"x": x}, warmup=2)
print("captured", flush=True)
torch.cuda.synchronize()
for _ in range(2):
    cap.replay()
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(a.steps):
    out = cap.replay()
torch.cuda.synchronize()
rep = (time.perf_counter() - t) / a.steps * 1e3
print(f"replay {rep:.3f} ms/step loss {out['total_loss'].item():.6f}", flush=True)
