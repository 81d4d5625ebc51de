"""Front-end micro-benchmark: the training front-end on one batch, repeated."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vae-teb_amd"))
import torch  # noqa: E402
from vaeteb import synthetic  # noqa: E402
from vaeteb.frontend import FrontEnd, FrontEndPlan, load_stats  # noqa: E402

dev = torch.device("cuda:0")
B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
fe = FrontEnd(FrontEndPlan(11, 4, 16, 4096, device=dev), load_stats(11, 4, 16, 4096))
x = torch.from_numpy(synthetic.batch(0, B, 4096)).to(dev)
for _ in range(3):
    fe(x)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(10):
    fe(x)
e1.record()
torch.cuda.synchronize()
print(f"front-end B={B}: {e0.elapsed_time(e1) / 10:.3f} ms per call", flush=True)
