import sys, torch
sys.path.insert(0, "tests"); sys.path.insert(0, "vae-teb_amd")
import test_gpu_resmlp_bf16 as B
from vaeteb import model as M
for width, depth, rows in ((32, 12, 64), (32, 16, 64), (32, 20, 64), (32, 33, 64), (64, 20, 64), (32, 33, 1000)):
    torch.manual_seed(0)
    m = M.ResidualMLP(width, tuple([width] * depth), final_activation=False).cuda()
    m.bf16 = True
    x = torch.randn(rows, width, dtype=torch.float64)
    y0, _ = B.ref_step(m, x, None)
    gy = torch.randn_like(y0)
    yr, Gr = B.ref_step(m, x, gy)
    y, Gk = B._gpu(m, x, gy)
    bad = [idx for idx, ln, a in m._plan if B.rel(Gk[f"body.{idx}.weight"], Gr[f"body.{idx}.weight"]) > 0.5]
    print(width, depth, rows, "first bad layer", (bad[-1] // 3 if bad else None), "n bad", len(bad),
          "sizes", m._fused_spec()[0].sizes(rows, True), flush=True)
