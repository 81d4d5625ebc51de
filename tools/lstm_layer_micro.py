"""One LSTM layer of the training geometry (B = 256 samples, S = 256 steps,
hidden 64, In = 64) alone: vt_lstm_layer_fwd_x, vt_lstm_layer_bwd_x,
vt_lstm_layer_bwd_weight (HIP events, mean of 10 launches), and the recurrences
of two layers launched together on two streams (the two encoders)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vae-teb_amd"))
import torch  # noqa: E402
from vaeteb._lib import call, ptr, stream  # noqa: E402

B, S, H, In = int(os.environ.get("B", "256")), 256, 64, int(os.environ.get("IN", "64"))
L16 = os.environ.get("L16", "0") == "1"   # the 16-bit MFMA recurrences (vt_lstm16_layer_*)
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


def layer():
    t = {}
    t["x"] = torch.randn(B, S, In, device=dev)
    t["wih"] = torch.randn(4 * H, In, device=dev) * 0.1
    t["whh"] = torch.randn(4 * H, H, device=dev) * 0.1
    t["bih"], t["bhh"] = torch.randn(4 * H, device=dev) * 0.1, torch.randn(4 * H, device=dev) * 0.1
    for k in ("h", "hp", "c"):
        t[k] = torch.empty(B, S, H, device=dev)
    t["gates"], t["dg"] = torch.empty(B, S, 4 * H, device=dev), torch.empty(B, S, 4 * H, device=dev)
    t["dh"], t["dx"] = torch.randn(B, S, H, device=dev), torch.empty(B, S, In, device=dev)
    t["dwih"], t["dwhh"] = torch.empty(4 * H, In, device=dev), torch.empty(4 * H, H, device=dev)
    t["db1"], t["db2"] = torch.empty(4 * H, device=dev), torch.empty(4 * H, device=dev)
    t["ws"] = torch.empty(32 << 20, device=dev)
    return t


def fwd(t):
    call("vt_lstm16_layer_fwd" if L16 else "vt_lstm_layer_fwd_x", ptr(t["x"]), In, ptr(t["wih"]), ptr(t["bih"]), ptr(t["whh"]), ptr(t["bhh"]), B, S, H,
         ptr(t["h"]), None if L16 else ptr(t["hp"]), ptr(t["c"]), ptr(t["gates"]), stream())


def bwd(t):
    call("vt_lstm16_layer_bwd" if L16 else "vt_lstm_layer_bwd_x", ptr(t["dh"]), ptr(t["gates"]), ptr(t["c"]), ptr(t["whh"]), ptr(t["wih"]), In, B, S, H,
         ptr(t["dg"]), ptr(t["dx"]), stream())


def bww(t):
    call("vt_lstm16_layer_bwd_weight" if L16 else "vt_lstm_layer_bwd_weight", ptr(t["dg"]), ptr(t["x"]), In,
         ptr(t["h"] if L16 else t["hp"]), B, S, H, ptr(t["dwih"]),
         ptr(t["dwhh"]), ptr(t["db1"]), ptr(t["db2"]), 0, ptr(t["ws"]), t["ws"].numel(), stream())


a, b = layer(), layer()
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()


def pair(fn):
    def go():
        s1.wait_stream(torch.cuda.current_stream())
        s2.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s1):
            fn(a)
        with torch.cuda.stream(s2):
            fn(b)
        torch.cuda.current_stream().wait_stream(s1)
        torch.cuda.current_stream().wait_stream(s2)
    return go


fwd(a), fwd(b), bwd(a), bwd(b)
for name, fn in (("fwd_x", fwd), ("bwd_x", bwd), ("bwd_weight", bww)):
    one = timed(lambda: fn(a))
    two = timed(pair(fn))
    print(f"{'16' if L16 else '32'} In={In} {name:11s}: alone {one:7.1f} us ({one / S * 1e3:6.1f} ns/step)   two streams {two:7.1f} us",
          flush=True)


def mixed():
    # one encoder's recurrence beside the other encoder's weight gradient (the step's overlap)
    s1.wait_stream(torch.cuda.current_stream())
    s2.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s1):
        bwd(a)
    with torch.cuda.stream(s2):
        bww(b)
    torch.cuda.current_stream().wait_stream(s1)
    torch.cuda.current_stream().wait_stream(s2)


print(f"In={In} bwd_x || bwd_weight: {timed(mixed):7.1f} us", flush=True)
