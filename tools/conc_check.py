"""Serial vs concurrent (two-stream) training step from raw windows, fp32 paths
(tests/test_gpu_model.py::test_concurrent_frontend_and_encoders_bitwise_identical as
a script): prints both losses and whether losses / gradients are bit-identical.
usage: conc_check.py [package_root (default: this tree)] [repeats]"""
import os
import sys

ROOT = os.path.abspath(sys.argv[1]) if len(sys.argv) > 1 else os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vae-teb_amd"))
import torch  # noqa: E402
from vaeteb import synthetic  # noqa: E402
from vaeteb.frontend import FrontEnd, FrontEndPlan, load_stats  # noqa: E402
from vaeteb.model import SeqVaeTeb  # noqa: E402
from vaeteb.train import Trainer  # noqa: E402

plan = FrontEndPlan(11, 4, 16, 4096, device="cuda")
fe = FrontEnd(plan, load_stats(11, 4, 16, 4096))
x = torch.from_numpy(synthetic.batch(5, 4, 4096)).cuda()
for rep in range(int(sys.argv[2]) if len(sys.argv) > 2 else 3):
    res = []
    for conc in (False, True):
        torch.manual_seed(0)
        m = SeqVaeTeb(sequence_length=plan.S, scattering_channels=fe.C_st, phase_channels=fe.C_ph,
                      cross_phase_channels=fe.C_x, concurrent_encoders=conc).cuda()
        tr = Trainer(m, lr=1e-3, frontend=fe)
        eps = torch.randn(4, plan.S, 32, generator=torch.Generator().manual_seed(1)).cuda()
        L = tr.step({"x": x}, eps=eps)
        torch.cuda.synchronize()
        res.append((L["total_loss"].item(), tr.state.g.clone()))
    print(f"{ROOT[-12:]} rep {rep}: serial {res[0][0]:.9f} concurrent {res[1][0]:.9f} "
          f"loss {'==' if res[0][0] == res[1][0] else '!='} grads {'==' if torch.equal(res[0][1], res[1][1]) else '!='}",
          flush=True)
