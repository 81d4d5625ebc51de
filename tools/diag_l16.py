"""Where the 16-bit LSTM differs from its fp64 model (tests/test_gpu_lstm16.py::_emu):
per-layer-count, per-step relative errors of y, dx and the parameter gradients."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "vae-teb_amd"), os.path.join(ROOT, "tests")]
import torch  # noqa: E402
import test_gpu_lstm16 as T  # noqa: E402
from vaeteb import ops  # noqa: E402

for In, B, S, nl in [(8, 4, 5, 1), (8, 4, 5, 2), (64, 4, 5, 1), (8, 4, 21, 1), (16, 4, 5, 1)]:
    torch.manual_seed(7 + In + S)
    ref = torch.nn.LSTM(In, 64, nl, batch_first=True)
    params = [p.detach().clone() for p in ref.parameters()]
    x, gy = torch.randn(B, S, In), torch.randn(B, S, 64)
    ye, dxe, ge = T._emu(x, params, gy)
    pd = [p.cuda().requires_grad_() for p in params]
    xd = x.cuda().requires_grad_()
    y = ops.lstm(xd, pd, half=True)
    (y * gy.cuda()).sum().backward()
    torch.cuda.synchronize()
    print(f"In={In} B={B} S={S} nl={nl}: y {T.rel(y, ye):.2e} dx {T.rel(xd.grad, dxe):.2e} grads",
          " ".join(f"{T.rel(p.grad, e):.1e}" for p, e in zip(pd, ge)))
    d = (xd.grad.double().cpu() - dxe)
    print("   dx err by t:", " ".join(f"{(d[:, t].norm() / dxe[:, t].norm()).item():.1e}" for t in range(S)))
    print("   dx err by col:", " ".join(f"{(d[..., k].norm() / dxe[..., k].norm()).item():.1e}" for k in range(In)))
