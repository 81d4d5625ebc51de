"""LSTM recurrence kernels alone: one layer (B=256, S=256, H=64) forward / backward,
one launch at a time and two launches on two streams (the two encoders' layers)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vae-teb_amd"))
import torch  # noqa: E402
from vaeteb._lib import call, ptr  # noqa: E402

B, S, H = 256, 256, 64
dev = "cuda"
torch.manual_seed(0)


def mk():
    gin = torch.randn(B, S, 4 * H, device=dev)
    whh = torch.randn(4 * H, H, device=dev) / 8
    bhh = torch.randn(4 * H, device=dev) / 8
    h, hp, c = (torch.empty(B, S, H, device=dev) for _ in range(3))
    gates = torch.empty(B, S, 4 * H, device=dev)
    dh = torch.randn(B, S, H, device=dev)
    dg = torch.empty(B, S, 4 * H, device=dev)
    return gin, whh, bhh, h, hp, c, gates, dh, dg


sets = [mk(), mk()]
streams = [torch.cuda.current_stream(), torch.cuda.Stream()]


def fwd(k, st):
    gin, whh, bhh, h, hp, c, gates, dh, dg = sets[k]
    with torch.cuda.stream(st):
        call("vt_lstm_layer_fwd", ptr(gin), ptr(whh), ptr(bhh), B, S, H, ptr(h), ptr(hp), ptr(c), ptr(gates),
             st.cuda_stream)


def bwd(k, st):
    gin, whh, bhh, h, hp, c, gates, dh, dg = sets[k]
    with torch.cuda.stream(st):
        call("vt_lstm_layer_bwd", ptr(dh), ptr(gates), ptr(c), ptr(whh), B, S, H, ptr(dg), st.cuda_stream)


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


def both(f):
    def run():
        streams[1].wait_stream(streams[0])
        f(0, streams[0])
        f(1, streams[1])
        streams[0].wait_stream(streams[1])
    return run


for name, f in (("fwd", fwd), ("bwd", bwd)):
    t1 = timed(lambda: f(0, streams[0]))
    t2 = timed(both(f))
    print(f"lstm {name}: alone {t1:7.1f} us ({t1 / S:5.3f} us/step); two concurrent {t2:7.1f} us", flush=True)
