"""Skinny fp32 GEMMs of the LSTM projections alone (R = 65,536 rows): forward
X W^T + b (N = 256 gates; K = 64 / 32 / 20), input gradient dG W (-> K), weight
gradient dG^T X (+ bias column); HIP events, mean of 10 launches."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vae-teb_amd"))
import torch  # noqa: E402
from vaeteb._lib import call, ptr, stream  # noqa: E402

R, N = 65536, 256
dev = "cuda"


def timed(fn, n=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


ws = torch.empty(64 << 20, device=dev)
for K in (64, 32, 20):
    x = torch.randn(R, K, device=dev)
    w = torch.randn(N, K, device=dev)
    b = torch.randn(N, device=dev)
    y = torch.empty(R, N, device=dev)
    g = torch.randn(R, N, device=dev)
    dx = torch.empty(R, K, device=dev)
    dw = torch.empty(N, K, device=dev)
    db = torch.empty(N, device=dev)
    tf = timed(lambda: call("vt_linear_fwd", ptr(x), R, K, ptr(w), N, ptr(b), ptr(y), stream()))
    td = timed(lambda: call("vt_linear_bwd_data", ptr(g), R, N, ptr(w), K, ptr(dx), 0, stream()))
    tw = timed(lambda: call("vt_linear_bwd_weight", ptr(g), R, N, ptr(x), K, ptr(dw), ptr(db), 0, ptr(ws),
                            ws.numel(), stream()))
    mb = lambda *ts: sum(t.numel() * 4 for t in ts) / 1e6
    print(f"K={K:3d}: fwd {tf:6.1f} us ({mb(x, y) / tf:5.2f} TB/s)  bwd_data {td:6.1f} us ({mb(g, dx) / td:5.2f} TB/s)  "
          f"bwd_weight {tw:6.1f} us ({mb(g, x) / tw:5.2f} TB/s)", flush=True)
