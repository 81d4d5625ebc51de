"""Diagnostic: bf16 dW kernel vs direct fp32 dW on small integer inputs."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "vae-teb_amd"))
import torch
from vaeteb import _lib as L
torch.manual_seed(0)
def dw(fn, dy, x, mode, up, Cout, K):
    B, Lin, Cin = x.shape
    d = torch.empty(Cout, Cin, K, device="cuda")
    ws = torch.empty(1 << 24, device="cuda")
    L.call(fn, L.ptr(dy), L.ptr(x), B, Lin, Cin, Cout, K, mode, up, L.ptr(d), 0, L.ptr(ws), ws.numel(), L.stream())
    torch.cuda.synchronize()
    return d
for (B, Lin, Cin, Cout, K, mode, up) in [(1, 64, 16, 16, 1, 0, 0), (1, 64, 16, 16, 2, 0, 0), (4, 64, 16, 16, 5, 0, 0)]:
    Lo = L.lib().fns["vt_conv1d_out_len"](Lin, K, mode, up)
    x = torch.randint(-2, 3, (B, Lin, Cin), device="cuda").float()
    dy = torch.randint(-2, 3, (B, Lo, Cout), device="cuda").float()
    a = dw("vt_conv1d_bwd_weight_bf16", dy, x, mode, up, Cout, K)
    b = dw("vt_conv1d_direct_bwd_weight", dy, x, mode, up, Cout, K)
    print("geo", (B, Lin, Cin, Cout, K), "maxdiff", (a - b).abs().max().item())
    if K <= 2:
        print("bf16 k=0 [:4,:8]\n", a[:4, :8, 0].cpu()); print("ref\n", b[:4, :8, 0].cpu())
        # try to identify: is a == b^T ?
        print("a==b^T", torch.equal(a[:, :, 0], b[:, :, 0].t()))
