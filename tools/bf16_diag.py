"""Per-parameter gradient differences of the bf16-conv step vs the fp32 step."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vae-teb_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from golden_util import det_fill_  # noqa: E402
from vaeteb.model import SeqVaeTeb  # noqa: E402


def run(S, B, batch, eps, fill):
    res = {}
    for prec in ("fp32", "bf16"):
        torch.manual_seed(0)
        m = SeqVaeTeb(sequence_length=S)
        if fill:
            det_fill_(m)
        m = m.cuda()
        m.set_conv_precision(prec)
        out = m(batch["y_st"], batch["y_ph"], batch["x_ph"], eps=eps)
        loss = m.compute_loss(out, batch["y_st"], batch["y_ph"], batch["y_raw"], beta=1e-5)
        loss["total_loss"].backward()
        res[prec] = ({k: v.item() for k, v in loss.items() if v is not None},
                     {n: p.grad.detach().double() for n, p in m.named_parameters()})
    print("losses fp32", res["fp32"][0], "\n       bf16", res["bf16"][0])
    errs = sorted(((((res["bf16"][1][n] - g).norm() / g.norm().clamp_min(1e-30)).item(), n, g.norm().item())
                   for n, g in res["fp32"][1].items()), reverse=True)
    for e, n, gn in errs[:12]:
        print(f"  {e:.3e}  |g| {gn:.3e}  {n}")
    ga = torch.cat([v.reshape(-1) for v in res["bf16"][1].values()])
    gb = torch.cat([v.reshape(-1) for v in res["fp32"][1].values()])
    print("  cosine", torch.nn.functional.cosine_similarity(ga, gb, dim=0).item(), flush=True)


g = np.load(os.path.join(ROOT, "tests/golden/model_s16_b4.npz"))
b = {k: torch.from_numpy(g[k]).cuda() for k in ("y_st", "y_ph", "x_ph", "y_raw")}
print("golden S16 B4 (det_fill weights)")
run(16, 4, b, torch.from_numpy(g["eps"]).cuda(), True)
for S, B in ((16, 4), (64, 16)):
    torch.manual_seed(1)
    b = dict(y_st=torch.randn(B, S, 43), y_ph=torch.randn(B, S, 44), x_ph=torch.randn(B, S, 130),
             y_raw=torch.randn(B, 16 * S))
    b = {k: v.cuda() for k, v in b.items()}
    print(f"random init S{S} B{B}")
    run(S, B, b, torch.randn(B, S, 32).cuda(), False)
