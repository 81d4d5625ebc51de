import sys, torch
sys.path.insert(0, "tests"); sys.path.insert(0, "vae-teb_amd")
import test_gpu_resmlp_bf16 as B
for rows in (7, 16, 64, 300):
    m, x = B._setup("target_mu_33", rows, rows + 12)
    y0, _ = B.ref_step(m, x, None)
    gy = torch.randn_like(y0)
    yr, Gr = B.ref_step(m, x, gy)
    y, Gk = B._gpu(m, x, gy)
    m.bf16 = False
    y32, G32 = B._gpu(m, x, gy)
    m.bf16 = True
    line = []
    for k in ("body.96.weight", "body.81.weight", "body.57.weight", "body.54.weight", "body.51.weight", "body.30.weight", "body.0.weight", "x"):
        line.append(f"{k}: k {Gk[k].norm():.2e} r {Gr[k].norm():.2e} f32 {G32[k].norm():.2e} rel {B.rel(Gk[k], Gr[k]):.1e}")
    print(rows, " | ".join(line), flush=True)
