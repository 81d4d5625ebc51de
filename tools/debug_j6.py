"""Debug: J6 step after-AdamW mismatch on decoder.linear (no MSE term)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vae-teb_amd"), os.path.join(ROOT, "tests")]
import numpy as np, torch
from golden_util import det_fill_
from vaeteb import synthetic
from vaeteb.frontend import FrontEnd, FrontEndPlan, load_stats
from vaeteb.model import SeqVaeTeb
from vaeteb.train import Trainer
st = load_stats(6, 1, 16, 4096)
fe = FrontEnd(FrontEndPlan(6, 1, 16, 4096, device="cuda"), st)
m = det_fill_(SeqVaeTeb(sequence_length=256, scattering_channels=8, phase_channels=13, cross_phase_channels=7)).cuda()
k = "decoder.linear.1.skip_proj.bias"
before = dict(m.named_parameters())[k].detach().clone()
tr = Trainer(m, lr=1e-3, frontend=fe)
x = synthetic.batch(4242, 2, 4096)
eps = np.random.default_rng(6).standard_normal((2, 256, 32)).astype(np.float32)
L = tr.step({"x": torch.from_numpy(x).cuda()}, eps=torch.from_numpy(eps).cuda())
torch.cuda.synchronize()
p = dict(m.named_parameters())[k]
print("grad absmax", p.grad.abs().max().item(), "norm out", tr.norm_out.tolist())
print("before", before[:6].tolist())
print("after ", p.detach()[:6].tolist())
print("rel change", ((p.detach() - before).norm() / before.norm()).item())
