"""Host cost of hipGraphLaunch on this ROCm: (1) a captured chain of n tiny
kernels, host time per replay() call vs n; (2) the captured training step,
host time of each replay() call while the GPU is busy.
usage: graph_host_probe.py"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vae-teb_amd"))
import torch  # noqa: E402

x = torch.zeros(1024, device="cuda")
for n in (10, 100, 500):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            for _ in range(n):
                x.add_(1.0)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(n):
            x.add_(1.0)
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    ts = []
    t0 = time.perf_counter()
    for _ in range(20):
        a = time.perf_counter()
        g.replay()
        ts.append(time.perf_counter() - a)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    ts.sort()
    print(f"graph of {n:4d} kernels: replay() host median {1e6 * ts[10]:8.1f} us, max {1e6 * ts[-1]:8.1f}; "
          f"wall per replay {1e6 * (t2 - t0) / 20:8.1f} us", flush=True)
    # eager equivalent
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        x.add_(1.0)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    print(f"   eager {n} launches host {1e6 * (t1 - t0):8.1f} us", flush=True)

from vaeteb import synthetic  # noqa: E402
from vaeteb.frontend import FrontEnd, FrontEndPlan, load_stats  # noqa: E402
from vaeteb.model import SeqVaeTeb  # noqa: E402
from vaeteb.train import Trainer  # noqa: E402
dev = torch.device("cuda:0")
plan = FrontEndPlan(11, 4, 16, 4096, device=dev)
fe = FrontEnd(plan, load_stats(11, 4, 16, 4096))
torch.manual_seed(1234)
model = SeqVaeTeb(sequence_length=plan.S, scattering_channels=fe.C_st, phase_channels=fe.C_ph,
                  cross_phase_channels=fe.C_x).to(dev)
tr = Trainer(model, lr=1e-3, frontend=fe)
xb = torch.from_numpy(synthetic.batch(0, 256, 4096)).to(dev)
cap = tr.capture({"x": xb}, warmup=2)
torch.cuda.synchronize()
cap.replay()
torch.cuda.synchronize()
ts = []
t0 = time.perf_counter()
for _ in range(10):
    a = time.perf_counter()
    cap.replay()
    ts.append(time.perf_counter() - a)
torch.cuda.synchronize()
t2 = time.perf_counter()
print("step graph replay() host ms:", " ".join(f"{1e3 * t:.2f}" for t in ts), f"| wall/step {1e3 * (t2 - t0) / 10:.2f} ms",
      flush=True)
