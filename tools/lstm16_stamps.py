"""Per-step segment timing of the 16-bit LSTM recurrences from in-kernel s_memtime stamps
(VAETEB_L16_DIAG=2 build variant: lane 0 of each wave of workgroup 0 stamps each step at
(0) the step start after the barrier, (1) the MFMA results in registers, (2) the h / dg
LDS write done; the stamps land in out_hprev (forward) / dx (backward)).
Prints mean cycles per segment: read+MFMA (0->1), VALU+write (1->2), barrier (2->next 0)."""
import os
import sys

os.environ["VAETEB_L16_DIAG"] = "2"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vae-teb_amd"))
import torch  # noqa: E402
from vaeteb._lib import call, ptr, stream  # noqa: E402

B, S, H, In = int(os.environ.get("B", "4")), 256, 64, int(os.environ.get("IN", "64"))
dev = "cuda"
x = torch.randn(B, S, In, device=dev)
wih, whh = torch.randn(4 * H, In, device=dev) * 0.1, torch.randn(4 * H, H, device=dev) * 0.1
bih, bhh = torch.randn(4 * H, device=dev) * 0.1, torch.randn(4 * H, device=dev) * 0.1
h, hp, c = (torch.zeros(B, S, H, device=dev) for _ in range(3))
gates = torch.zeros(B, S, 4 * H, device=dev)
dh, dg = torch.randn(B, S, H, device=dev), torch.zeros(B, S, 4 * H, device=dev)
dx = torch.zeros(max(B * S * In, S * 12 * 2), device=dev)


def seg(buf):
    st = buf.reshape(-1).view(torch.int64)[: S * 12].view(S, 4, 3).cpu().double()
    a = (st[:, :, 1] - st[:, :, 0])[8:-8].mean(0)
    b = (st[:, :, 2] - st[:, :, 1])[8:-8].mean(0)
    step = (st[1:, :, 0] - st[:-1, :, 0])[8:-8].mean(0)
    return a, b, step


for it in range(3):
    call("vt_lstm16_layer_fwd", ptr(x), In, ptr(wih), ptr(bih), ptr(whh), ptr(bhh), B, S, H, ptr(h), ptr(hp), ptr(c),
         ptr(gates), stream())
    torch.cuda.synchronize()
a, b, st = seg(hp)
print(f"fwd B={B} In={In}: read+MFMA {a.tolist()}  VALU+write {b.tolist()}  step {st.tolist()} (cycles, per wave)")
for it in range(3):
    call("vt_lstm16_layer_bwd", ptr(dh), ptr(gates), ptr(c), ptr(whh), ptr(wih), In, B, S, H, ptr(dg), ptr(dx),
         stream())
    torch.cuda.synchronize()
a, b, st = seg(dx)
print(f"bwd B={B} In={In}: read+MFMA {a.tolist()}  VALU+write {b.tolist()}  step {-st[0].item():.0f}.. "
      f"{(-st).tolist()} (cycles, per wave; steps walk t downwards)")
