"""bf16 ResidualMLP error budget per stack shape: kernel vs the bf16-rounded fp64
model (max over tensors / aggregate), the rounded model vs exact fp64, and an
exact-fp64 run on inputs perturbed by bf16's rounding step (model sensitivity)."""
import sys, torch
sys.path.insert(0, "tests"); sys.path.insert(0, "vae-teb_amd")
import test_gpu_resmlp_bf16 as B


def agg(G, R):
    num = sum(((G[k].double().cpu() - v) ** 2).sum() for k, v in R.items())
    return (num / sum((v ** 2).sum() for v in R.values())).sqrt().item()


for case in B.CASES:
    for rows in (7, 1000, 65536):
        m, x = B._setup(case, rows, rows + len(case))
        margins = []
        y0, _ = B.ref_step(m, x, None, margins=margins)
        gy = torch.randn_like(y0)
        if margins:
            gy[torch.stack(margins).min(dim=0).values < 1e-4] = 0
        yr, Gr = B.ref_step(m, x, gy)
        y, Gk = B._gpu(m, x, gy)
        ye, Ge = B.ref_step(m, x, gy, rounding=False)
        g = torch.Generator().manual_seed(5)
        yp, Gp = B.ref_step(m, x * (1 + 4e-3 * torch.randn(x.shape, generator=g, dtype=torch.float64)), gy,
                            rounding=False)
        kmax = max((B.rel(Gk[k], v), k) for k, v in Gr.items())
        print(f"{case:22s} {rows:6d} y k-r {B.rel(y, yr):.1e} k-e {B.rel(y, ye):.1e} p-e {B.rel(yp, ye):.1e} | "
              f"grad k-r max {kmax[0]:.1e} ({kmax[1]}) agg {agg(Gk, Gr):.1e} | k-e {agg(Gk, Ge):.1e} "
              f"r-e {agg(Gr, Ge):.1e} p-e {agg(Gp, Ge):.1e}", flush=True)
