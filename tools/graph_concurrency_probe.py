"""Does a captured hipGraph run independent branches concurrently?  Two LSTM
recurrences on 64 samples each (64 workgroups = a quarter of the CUs, ~latency
bound) on forked streams: eager-concurrent vs graph replay timings."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "vae-teb_amd"))
from vaeteb._lib import call, ptr  # noqa: E402

B, S, H = 64, 256, 64
dev = "cuda"
bufs = []
for _ in range(2):
    gin = torch.randn(B, S, 4 * H, device=dev)
    w = torch.randn(4 * H, H, device=dev) * 0.1
    b = torch.zeros(4 * H, device=dev)
    outs = [torch.empty(B, S, H, device=dev) for _ in range(3)]
    gates = torch.empty(B, S, 4 * H, device=dev)
    bufs.append((gin, w, b, outs, gates))


def run(i):
    gin, w, b, outs, gates = bufs[i]
    call("vt_lstm_layer_fwd", ptr(gin), ptr(w), ptr(b), B, S, H, ptr(outs[0]), ptr(outs[1]), ptr(outs[2]),
         ptr(gates), torch.cuda.current_stream().cuda_stream)


side = torch.cuda.Stream()


def both():
    main = torch.cuda.current_stream()
    side.wait_stream(main)
    with torch.cuda.stream(side):
        for _ in range(4):
            run(1)
    for _ in range(4):
        run(0)
    main.wait_stream(side)


def timeit(fn, n=5):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n * 1e3


serial = timeit(lambda: [run(0) for _ in range(8)])
eager = timeit(both)
s2 = torch.cuda.Stream()
s2.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s2):
    both()
torch.cuda.current_stream().wait_stream(s2)
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    both()
graph = timeit(g.replay)
print(f"8 recurrences serial {serial:.2f} ms | 4+4 on two streams eager {eager:.2f} ms | same as hipGraph {graph:.2f} ms")
