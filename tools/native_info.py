"""Native executor launch-list statistics per stream count (kernels, memcpy, memset,
cross-stream waits) and the GPU time of replays (events), eager step for reference."""
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
                  cross_phase_channels=fe.C_x, head_precision="bf16", conv_precision="bf16", mlp_precision="bf16",
                  concurrent_encoders=True).to(dev)
tr = Trainer(model, lr=1e-3, frontend=fe)
x = torch.from_numpy(synthetic.batch(0, 256, 4096)).to(dev)
feats = fe(x)
eps = torch.randn(256, plan.S, 32, device=dev)


def timed(fn, n=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    torch.cuda._sleep(int(2e8))   # GPU busy while the host enqueues: GPU-only time
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n


print(f"eager step (model only): {timed(lambda: tr.step(feats, eps=eps)):.3f} ms", flush=True)
caps = {}
for ns in [int(a) for a in (sys.argv[1:] or ["1", "2", "3", "4", "6"])]:
    cap = tr.capture(feats, eps=eps, warmup=1, native=True, n_streams=ns)
    caps[ns] = cap
    k, mc, ms, w = cap.info()
    print(f"streams {ns}: {k} kernels, {mc} memcpy, {ms} memset, {w} waits; "
          f"replay {timed(lambda: cap.replay()):.3f} ms", flush=True)
