"""Locate rows where the fused ResidualMLP backward differs from fp64."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vae-teb_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402
from vaeteb import model as M  # noqa: E402
from test_gpu_resmlp import CASES, _ref_forward  # noqa: E402

case = sys.argv[1] if len(sys.argv) > 1 else "decoder_linear"
for rows in (1000, 4096, 16384, 65536):
    torch.manual_seed(rows + len(case))
    m = CASES[case](M)
    with torch.no_grad():
        for n, p in m.named_parameters():
            if p.dim() == 1:
                p.copy_((1.0 if n.endswith("weight") else 0.0) + 0.1 * torch.randn_like(p))
    m = m.cuda()
    d0 = m.input_norm.weight.shape[0]
    x = torch.randn(rows, d0, dtype=torch.float64)
    xr = x.clone().requires_grad_(True)
    yr, P = _ref_forward(m, xr)
    gy = torch.randn_like(yr)
    (yr * gy).sum().backward()
    for rep in range(2):
        m.zero_grad(set_to_none=True)
        xd = x.float().cuda().requires_grad_(True)
        y = m(xd)
        (y * gy.float().cuda()).sum().backward()
        e = ((xd.grad.double().cpu() - xr.grad).norm(dim=1) / xr.grad.norm(dim=1))
        bad = (e > 1e-4).nonzero().flatten()
        print(f"rows {rows} rep {rep}: max row err {e.max():.2e} bad rows {len(bad)} first {bad[:10].tolist()} "
              f"row%64 {sorted(set((bad % 64).tolist()))[:16]} blocks {sorted(set((bad // 64).tolist()))[:10]}",
              flush=True)


def preacts(m, x):
    """fp64 LayerNorm+affine outputs (pre-activation) of every normalised layer for rows x."""
    import torch.nn.functional as F
    P = {n: p.detach().double().cpu() for n, p in m.named_parameters()}
    h = F.layer_norm(x, (x.shape[-1],), P["input_norm.weight"], P["input_norm.bias"], 1e-5)
    out = []
    for idx, has_ln, a in m._plan:
        h = F.linear(h, P[f"body.{idx}.weight"], P[f"body.{idx}.bias"])
        if has_ln:
            u = F.layer_norm(h, (h.shape[-1],), P[f"body.{idx + 1}.weight"], P[f"body.{idx + 1}.bias"], 1e-5)
            out.append(u)
            h = F.relu(u) if a == "relu" else (F.gelu(u) if a == "gelu" else u)
    return out


for rows, bad in ((4096, 2243), (65536, 63887)):
    torch.manual_seed(rows + len(case))
    m = CASES[case](M)
    with torch.no_grad():
        for n, p in m.named_parameters():
            if p.dim() == 1:
                p.copy_((1.0 if n.endswith("weight") else 0.0) + 0.1 * torch.randn_like(p))
    d0 = m.input_norm.weight.shape[0]
    x = torch.randn(rows, d0, dtype=torch.float64)
    us = preacts(m, x[bad:bad + 1])
    print(rows, bad, "min |u| per layer:", [f"{u.abs().min().item():.1e}" for u in us])
