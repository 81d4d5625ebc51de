"""Phase timeline of the bf16 ResidualMLP backward kernel (k_mlpb_bwd): wave 0's
wall clock (100 MHz) at its phase boundaries, averaged over workgroups.
usage: mlpb_phases.py [stack] (stacks of tools/mlpb_micro.py)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vae-teb_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch  # noqa: E402
from mlpb_micro import CFG  # noqa: E402
from vaeteb._lib import call  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "pre64"
rows = 65536
torch.manual_seed(0)
m = CFG[name]().cuda()
m.bf16 = True
x = torch.randn(rows, m.input_norm.weight.shape[0], device="cuda", requires_grad=True)
for _ in range(3):
    y = m(x)
    y.backward(torch.ones_like(y))
torch.cuda.synchronize()
buf = torch.zeros(4096 * 256, dtype=torch.int64, device="cuda")
y = m(x)
torch.cuda.synchronize()
call("vt_resmlp_bf16_set_stamps", buf.data_ptr())
y.backward(torch.ones_like(y))
torch.cuda.synchronize()
call("vt_resmlp_bf16_set_stamps", None)
st = buf.view(4096, 256).cpu().double()
used = st[:, 0] > 0
st = st[used]
nblk = st.shape[0]
t0 = st[:, 0].min()
us = lambda v: v * 10 / 1000
print(f"{name}: {nblk} workgroups; launch spread {us(st[:, 0].max() - t0):.1f} us; "
      f"kernel span {us(st[:, 255].max() - t0):.1f} us; per-WG mean {us((st[:, 255] - st[:, 0]).mean()):.1f} us")
print(f"  staging          {us((st[:, 1] - st[:, 0]).mean()):7.2f} us")
prev = st[:, 1]
step = 0
names = ["to barrier", "dZ pass", "H pass", "img barrier", "GEMM+dW", "flush"]
while 7 + 6 * step < 255 and (st[:, 7 + 6 * step] > 0).all():
    cols = [st[:, 2 + 6 * step + i] for i in range(6)]
    parts = [cols[0] - prev] + [cols[i] - cols[i - 1] for i in range(1, 6)]
    print(f"  step {step:2d}: " + "  ".join(f"{n} {us(v.mean()):5.2f}" for n, v in zip(names, parts)))
    prev = cols[5]
    step += 1
print(f"  input LN + dx    {us((st[:, 255] - prev).mean()):7.2f} us")
if (st[:, 243] > 0).all():   # step 1, first tile of the dZ pass: LN backward | colsum | dZ image | fragments
    c = [st[:, 2 + 6], st[:, 240], st[:, 241], st[:, 242], st[:, 243]]
    print("  step 1 dZ pass, tile 0: " + "  ".join(f"{n} {us((c[i + 1] - c[i]).mean()):5.2f}" for i, n in
                                                  enumerate(("LN bwd", "colsum", "dZ image", "frags"))))
