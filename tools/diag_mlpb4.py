import sys, torch, ctypes
sys.path.insert(0, "tests"); sys.path.insert(0, "vae-teb_amd")
import test_gpu_resmlp_bf16 as B
from vaeteb import model as M, ops, _lib
width, depth, rows = 32, 12, 64
torch.manual_seed(0)
m = M.ResidualMLP(width, tuple([width] * depth), final_activation=False).cuda()
spec, params = m._fused_spec()
x = torch.randn(rows, width, device="cuda")
n_xh, n_rs, n_ws = spec.sizes(rows, True)
out = torch.empty(rows, width, device="cuda"); xh = torch.zeros(n_xh, device="cuda"); rs = torch.zeros(n_rs, device="cuda")
pp = spec.pointers(params)
_lib.call("vt_resmlp_bf16_fwd", spec.L, spec.dims, spec.ln, spec.act, spec.skip, spec.eps, pp, x.data_ptr(), rows,
          out.data_ptr(), xh.data_ptr(), rs.data_ptr(), _lib.stream())
gy = torch.randn(rows, width, device="cuda")
ws = torch.full((n_ws,), 7.0, device="cuda")
grads = [torch.zeros_like(p) if p is not None else None for p in params]
gp = spec.pointers(grads)
dx = torch.empty(rows, width, device="cuda")
_lib.call("vt_resmlp_bf16_bwd", spec.L, spec.dims, spec.ln, spec.act, spec.skip, spec.eps, pp, gy.data_ptr(),
          xh.data_ptr(), rs.data_ptr(), rows, dx.data_ptr(), gp, 0, ws.data_ptr(), ws.numel(), _lib.stream())
torch.cuda.synchronize()
W = ws.cpu()
for l in range(depth):
    s = W[l * 1056:(l + 1) * 1056].view(32, 33)
    print(l, "dW norm", s[:, :32].norm().item(), "db norm", s[:, 32].norm().item(), "n==7", (s == 7).sum().item(),
          "grad", grads[2 + 4 * l].norm().item(), flush=True)
print("xh rows per layer nonzero:", [(xh.view(-1, 256, 32)[i] != 0).sum().item() for i in range(depth)])
print("rs", rs.view(-1, 256)[:, :3])
