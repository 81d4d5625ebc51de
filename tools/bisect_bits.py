"""Which library build changes the bf16 training bits (diagnostic): 3 bench-precision steps at
S = 256, B = 2 on the trajectory fixture's batches; prints the losses and a checksum of the
parameters.  Run once per library (VAETEB_LIB=...)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "vae-teb_amd"), os.path.join(ROOT, "tests")]
import torch  # noqa: E402

from golden_util import det_fill_, traj_inputs  # noqa: E402
from vaeteb.model import SeqVaeTeb  # noqa: E402
from vaeteb.train import Trainer  # noqa: E402

m = det_fill_(SeqVaeTeb(sequence_length=256, head_precision="bf16", conv_precision="bf16", mlp_precision="bf16",
                        lstm_precision="16-mixed", concurrent_encoders=True)).cuda()
tr = Trainer(m, lr=1e-3)
B = int(os.environ.get("BISECT_B", "2"))
out = []
for t in range(3):
    y_st, y_ph, x_ph, y_raw, eps = [torch.from_numpy(a).cuda() for a in traj_inputs(256, B, t)]
    L = tr.step({"fhr_st": y_st, "fhr_ph": y_ph, "fhr_up_ph": x_ph, "fhr": y_raw}, eps=eps)
    out.append(float(L["nll_loss"]))
torch.cuda.synchronize()
g = tr.state.g.double()
print(os.environ.get("VAETEB_LIB", "in-tree"), B, out, float(tr.state.p.double().sum()), float(g.abs().sum()))
