"""Micro-benchmark of the bf16 conv weight-gradient kernel on the decoder's layer
shapes (B 256): per-call time and effective TFLOP/s (for rocprofv3 --pmc passes)."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vae-teb_amd"))
import torch  # noqa: E402
from vaeteb import _lib  # noqa: E402

B = 256
# (L_in, Cin, Cout, K, mode, up) of the decoder conv stack (ref/model/vae_teb_model.py:871-880)
LAYERS = [(256, 87, 77, 11, 1, 0), (256, 77, 66, 9, 1, 1), (512, 66, 55, 7, 1, 1), (1024, 55, 44, 5, 1, 0),
          (1024, 44, 33, 5, 1, 1), (2048, 33, 22, 3, 1, 1), (4096, 22, 11, 3, 1, 0), (4096, 11, 1, 3, 1, 0)]
sel = [int(a) for a in sys.argv[1:]] or list(range(len(LAYERS)))
dev = torch.device("cuda:0")
ws = torch.empty(1 << 25, device=dev)
for li in sel:
    L, Cin, Cout, K, mode, up = LAYERS[li]
    Lo = _lib.lib().fns["vt_conv1d_out_len"](L, K, mode, up)
    x = torch.randn(B, L, Cin, device=dev)
    dy = torch.randn(B, Lo, Cout, device=dev)
    dw = torch.empty(Cout, Cin, K, device=dev)
    args = (_lib.ptr(dy), _lib.ptr(x), B, L, Cin, Cout, K, mode, up, _lib.ptr(dw), 0, _lib.ptr(ws), ws.numel(),
            _lib.stream())
    for _ in range(3):
        _lib.call("vt_conv1d_bwd_weight_bf16", *args)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        _lib.call("vt_conv1d_bwd_weight_bf16", *args)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 10
    fl = 2.0 * B * Lo * Cin * Cout * K
    print(f"layer {li} L_out {Lo} {Cin}->{Cout} K{K} up{up}: {ms * 1e3:8.1f} us  {fl / ms / 1e9:7.1f} TFLOP/s", flush=True)
