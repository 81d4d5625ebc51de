"""cProfile of the eager training step's host side (where the ~16 ms of
Python / ctypes dispatch per step goes)."""
import cProfile
import os
import pstats
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
                  cross_phase_channels=fe.C_x, head_precision="bf16", conv_precision="bf16",
                  mlp_precision="bf16", concurrent_encoders=True).to(dev)
tr = Trainer(model, lr=1e-3, frontend=fe)
x = torch.from_numpy(synthetic.batch(0, 256, 4096)).to(dev)
if os.environ.get("SINGLE_THREAD_BACKWARD", "1") == "1":
    # run the autograd backward on this thread, so cProfile sees the ops' backward functions
    torch.autograd.set_multithreading_enabled(False)
for _ in range(3):
    tr.step({"x": x})
torch.cuda.synchronize()
pr = cProfile.Profile()
pr.enable()
for _ in range(5):
    tr.step({"x": x})
pr.disable()
torch.cuda.synchronize()
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(60)
st.sort_stats("cumulative").print_stats(60)
