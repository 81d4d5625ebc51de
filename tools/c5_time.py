"""Config 5 (Scattering1D J=8 Q=12 T=256 order 2, N=16384, B=64): time the generic-core path."""
import os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "vae-teb_amd"))
import torch
from vaeteb.scattering import Scattering1D
from vaeteb import synthetic
sc = Scattering1D(J=8, shape=16384, Q=12, max_order=2, T=256)
x = torch.from_numpy(synthetic.batch(0, 64, 16384)[:, 0]).cuda().contiguous()
for _ in range(2):
    S, _ = sc(x)
torch.cuda.synchronize()
t = time.perf_counter()
n = 5
for _ in range(n):
    S, _ = sc(x)
t_enq = time.perf_counter() - t
torch.cuda.synchronize()
dt = (time.perf_counter() - t) / n
print(f"c5 cascade: {dt*1e3:.2f} ms/batch (enqueue {t_enq/n*1e3:.2f}), {64/dt:.1f} samples/s, out {tuple(S.shape)}")
sc.cascade = False
S2, _ = sc(x)
torch.cuda.synchronize()
t = time.perf_counter()
S2, _ = sc(x)
torch.cuda.synchronize()
print(f"c5 per-filter generic core: {(time.perf_counter() - t) * 1e3:.2f} ms/batch; max |cascade - generic| / max|S| = "
      f"{((S - S2).abs().max() / S2.abs().max()).item():.2e}")
