"""bf16 whole-ResidualMLP kernels, one stack shape at a time: forward /
backward launch times (HIP events) at 65,536 rows, fp32 and bf16 families.
usage: mlpb_micro.py [names] [--bf16-only]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vae-teb_amd"))
import torch  # noqa: E402
from vaeteb import model as M  # noqa: E402

CFG = {
    "src130": lambda: M.ResidualMLP(130, M.geometric_schedule(130, 32, 5), final_activation=False),
    "mu33": lambda: M.ResidualMLP(32, M.geometric_schedule(32, 32, 32), final_activation=False),
    "pre64": lambda: M.ResidualMLP(64, M.geometric_schedule(64, 32, 4), final_activation=True),
    "scat43": lambda: M.ResidualMLP(43, M.geometric_schedule(43, 16, 4), final_activation=False, activation="gelu"),
    "dec50": lambda: M.ResidualMLP(50, M.geometric_schedule(50, 87, 5)),
}


def run(name, rows, bf16, reps=10):
    torch.manual_seed(0)
    m = CFG[name]().cuda()
    m.bf16 = bf16
    x = torch.randn(rows, m.input_norm.weight.shape[0], device="cuda", requires_grad=True)
    for _ in range(3):
        y = m(x)
        y.backward(torch.ones_like(y))
    torch.cuda.synchronize()
    tf = tb = 0.0
    for _ in range(reps):
        e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
        g = torch.ones(rows, y.shape[-1], device="cuda")
        e0.record()
        y = m(x)
        e1.record()
        y.backward(g)
        e2.record()
        torch.cuda.synchronize()
        tf += e0.elapsed_time(e1)
        tb += e1.elapsed_time(e2)
    print(f"{name:7s} rows {rows:7d} {'bf16' if bf16 else 'fp32'}: fwd {tf / reps * 1e3:8.1f} us  bwd {tb / reps * 1e3:8.1f} us",
          flush=True)


if __name__ == "__main__":
    names = sys.argv[1].split(",") if len(sys.argv) > 1 and not sys.argv[1].startswith("--") else list(CFG)
    for n in names:
        for bf16 in ((True,) if "--bf16-only" in sys.argv else (True, False)):
            run(n, 65536, bf16)
