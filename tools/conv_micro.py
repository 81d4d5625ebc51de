"""Decoder conv blocks (bench geometry, B = 256, bf16 convs) forward + backward
one block at a time on one stream, so a kernel trace shows each kernel's
isolated duration (run under rocprofv3 --kernel-trace --stats)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vae-teb_amd"))
import torch  # noqa: E402
from vaeteb import _lib  # noqa: E402
from vaeteb.model import ConvBlock, Decoder  # noqa: E402

_lib.call("vt_conv_bf16_set_staging", int(os.environ.get("VAETEB_CONV_CL", "1")))   # window staging A/B

B, L = 256, 256
dev = "cuda"
for (a, b, k, u) in Decoder.SPEC:
    blk = ConvBlock(a, b, k, causal=False, up=u).to(dev)
    blk.bf16 = True
    x = torch.randn(B, L, a, device=dev, requires_grad=True)
    for _ in range(3):
        y = blk(x)
        gy = torch.randn_like(y)
        y.backward(gy)
    torch.cuda.synchronize()
    print(f"block {a}->{b} k{k} up{int(u)} L{L}", flush=True)
    L = L * (2 if u else 1)
# encoder blocks (causal, L = S = 256)
for (c, k) in [(32, 3), (32, 5), (32, 7), (16, 3), (16, 5), (16, 7)]:
    blk = ConvBlock(c, c, k, causal=True).to(dev)
    blk.bf16 = True
    x = torch.randn(B, 256, c, device=dev, requires_grad=True)
    for _ in range(3):
        y = blk(x)
        y.backward(torch.randn_like(y))
    torch.cuda.synchronize()
    print(f"encoder block {c} k{k}", flush=True)
