"""Marginal cost of the step's phases (GPU-bound timing, no profiler): full step,
step on precomputed features (no front-end), front-end alone, forward+loss only."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vae-teb_amd"))
import torch
from vaeteb import synthetic
from vaeteb.frontend import FrontEnd, FrontEndPlan, load_stats
from vaeteb.model import SeqVaeTeb
from vaeteb.train import Trainer

dev = torch.device("cuda:0")
plan = FrontEndPlan(11, 4, 16, 4096, device=dev)
fe = FrontEnd(plan, load_stats(11, 4, 16, 4096))
torch.manual_seed(1234)
model = SeqVaeTeb(sequence_length=plan.S, scattering_channels=fe.C_st, phase_channels=fe.C_ph,
                  cross_phase_channels=fe.C_x, head_precision="bf16", conv_precision="bf16",
                  concurrent_encoders=True).to(dev)
tr = Trainer(model, lr=1e-3, frontend=fe)
x = torch.from_numpy(synthetic.batch(0, 256, 4096)).to(dev)
feats = {k: v.clone() for k, v in fe(x).items()}


def timeit(fn, n=20, w=5):
    for _ in range(w):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n * 1e3


print("full step      %.3f ms" % timeit(lambda: tr.step({"x": x})))
print("step, features %.3f ms" % timeit(lambda: tr.step(feats)))
print("front-end only %.3f ms" % timeit(lambda: fe(x)))
with torch.no_grad():
    print("fwd+loss only  %.3f ms" % timeit(lambda: tr.loss(feats)))
