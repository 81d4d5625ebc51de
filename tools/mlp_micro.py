"""Micro-benchmark of the whole-ResidualMLP kernels on one stack shape:
forward / backward launch times (HIP events) at several row counts."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vae-teb_amd"))
import torch  # noqa: E402
from vaeteb import model as M  # noqa: E402

CFG = {
    "mu33": lambda: M.ResidualMLP(32, M.geometric_schedule(32, 32, 32), final_activation=False),
    "pre64": lambda: M.ResidualMLP(64, M.geometric_schedule(64, 32, 4), final_activation=True),
    "src130": lambda: M.ResidualMLP(130, M.geometric_schedule(130, 32, 5), final_activation=False),
}


def run(name, rows, reps=10, fused=True):
    torch.manual_seed(0)
    m = CFG[name]().cuda()
    m.fused = fused
    x = torch.randn(rows, m.input_norm.weight.shape[0], device="cuda", requires_grad=True)
    for _ in range(3):
        y = m(x)
        y.backward(torch.ones_like(y))
    torch.cuda.synchronize()
    tf = tb = 0.0
    for _ in range(reps):
        e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
        e0.record()
        y = m(x)
        e1.record()
        y.backward(torch.ones_like(y))
        e2.record()
        torch.cuda.synchronize()
        tf += e0.elapsed_time(e1)
        tb += e1.elapsed_time(e2)
    print(f"{name:7s} rows {rows:7d} fused={fused}: fwd {tf / reps * 1e3:8.1f} us  bwd {tb / reps * 1e3:8.1f} us",
          flush=True)


if __name__ == "__main__":
    names = sys.argv[1].split(",") if len(sys.argv) > 1 else list(CFG)
    for n in names:
        for rows in (16384, 65536, 262144):
            run(n, rows)
        run(n, 65536, fused=False)
