"""J=6 window 4244: the HIP fp32 step and the fp64 / fp32 oracle steps on the features of the
full-image (form 0) and the half-image (form 1) pair kernels — which side moves when the features
move by ~1e-6?  Usage: python tools/j6_step_diag.py [window]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "vae-teb_amd"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
import numpy as np  # noqa: E402
import torch  # noqa: E402
from test_gpu_parity_s256 import _model, _oracle_step, rel  # noqa: E402
from vaeteb import _lib, synthetic  # noqa: E402
from vaeteb.frontend import FrontEnd, FrontEndPlan, load_stats  # noqa: E402
from vaeteb.train import Trainer  # noqa: E402

torch.set_num_threads(16)
win = int(sys.argv[1]) if len(sys.argv) > 1 else 4244
fe = FrontEnd(FrontEndPlan(6, 1, 16, 4096, device="cuda"), load_stats(6, 1, 16, 4096))
widths = (fe.C_st, fe.C_ph, fe.C_x)
x = torch.from_numpy(synthetic.batch(win, 2, 4096)).cuda()
eps = np.random.default_rng(6).standard_normal((2, 256, 32)).astype(np.float32)
fns = _lib.lib().fns
F, G, O, O32, FW, OFW = {}, {}, {}, {}, {}, {}
for form in (0, 1):
    fns["vt_fe_set_pairs_half"](form)
    F[form] = {k: v.detach().clone() for k, v in fe(x).items()}
    m = _model(256, scattering_channels=widths[0], phase_channels=widths[1], cross_phase_channels=widths[2])
    m.train()
    with torch.no_grad():
        fw = m(F[form]["fhr_st"], F[form]["fhr_ph"], F[form]["fhr_up_ph"], eps=torch.from_numpy(eps).cuda())
    FW[form] = {k: v.detach().double().cpu() for k, v in fw.items() if torch.is_tensor(v)}
    m = _model(256, scattering_channels=widths[0], phase_channels=widths[1], cross_phase_channels=widths[2])
    tr = Trainer(m, lr=1e-3)
    tr.step(F[form], eps=torch.from_numpy(eps).cuda())
    torch.cuda.synchronize()
    G[form] = {k: p.grad.detach().double().cpu() for k, p in m.named_parameters()}
    feats = {k: v.cpu().double().numpy() for k, v in F[form].items()}
    ofw, _, O[form], _ = _oracle_step(feats, eps, widths)
    OFW[form] = {k: v.detach().double() for k, v in ofw.items() if torch.is_tensor(v)}
    _, _, O32[form], _ = _oracle_step(feats, eps, widths, torch.float32)
fns["vt_fe_set_pairs_half"](1)


def stat(a, b):
    e = np.array([rel(a[k], b[k]) for k in b if b[k].norm() > 0])
    return f"median {np.median(e):.2e} p90 {np.percentile(e, 90):.2e} max {e.max():.2e}"


print("features form1 vs form0:", {k: f"{(F[1][k] - F[0][k]).abs().max().item():.1e}" for k in F[0]})
print("HIP f0 vs oracle64 f0:", stat(G[0], O[0]))
print("HIP f1 vs oracle64 f1:", stat(G[1], O[1]))
print("HIP f1 vs HIP f0     :", stat(G[1], G[0]))
print("oracle64 f1 vs f0    :", stat(O[1], O[0]))
print("oracle32 f1 vs o64 f1:", stat(O32[1], O[1]))
print("oracle32 f0 vs o64 f0:", stat(O32[0], O[0]))
print("HIP f1 vs oracle32 f1:", stat(G[1], O32[1]))

for k in OFW[1]:
    if k in FW[1] and FW[1][k].shape == OFW[1][k].shape:
        print(f"forward {k}: HIP f1 vs o64 f1 {rel(FW[1][k], OFW[1][k]):.2e}  HIP f0 vs o64 f0 "
              f"{rel(FW[0][k], OFW[0][k]):.2e}  max|d| f1 {(FW[1][k] - OFW[1][k]).abs().max().item():.2e}")
e = sorted(((rel(G[1][k], G[0][k]), k) for k in G[0] if G[0][k].norm() > 0), reverse=True)
print("largest HIP f1 vs f0 gradient changes:")
for v, k in e[:40]:
    print(f"  {v:.2e} {k}")
lv = OFW[1].get("logvar_pr")
if lv is not None:
    print("oracle logvar_pr range", lv.min().item(), lv.max().item())

# the oracle's fp32 reproducibility ensemble at f1 (one-ulp perturbed initial weights, as the bench
# batch test) and the HIP step's own one-ulp members at f0: do THEY move mu_layer's gradients too?
from golden_util import det_fill_, perturb_ulp_  # noqa: E402
from oracle import model_ref as M  # noqa: E402
feats1 = {k: v.cpu().double().numpy() for k, v in F[1].items()}
Tf = lambda a: torch.from_numpy(np.asarray(a)).float()
env = {}
for seed in range(1, 5):
    ref = perturb_ulp_(det_fill_(M.SeqVaeTebRef(256, *widths)), seed)
    _, _, g, _ = M.train_step(ref, {"y_st": Tf(feats1["fhr_st"]), "y_ph": Tf(feats1["fhr_ph"]),
                                    "x_ph": Tf(feats1["fhr_up_ph"]), "y_raw": Tf(feats1["fhr"])}, Tf(eps), 1e-5)
    print(f"oracle32 member {seed} f1 vs o64 f1:", stat(g, O[1]))
    for k in O[1]:
        if O[1][k].norm() > 0:
            env[k] = max(env.get(k, 0.0), rel(g[k], O[1][k]))
for seed in range(1, 4):
    m = perturb_ulp_(_model(256, scattering_channels=widths[0], phase_channels=widths[1],
                            cross_phase_channels=widths[2]).cpu(), seed).cuda()
    tr = Trainer(m, lr=1e-3)
    tr.step(F[0], eps=torch.from_numpy(eps).cuda())
    torch.cuda.synchronize()
    gm = {k: p.grad.detach().double().cpu() for k, p in m.named_parameters()}
    print(f"HIP member {seed} f0 vs o64 f0:", stat(gm, O[0]))
for v, k in e[:12]:
    print(f"  {k}: HIP f1 {rel(G[1][k], O[1][k]):.2e}, oracle32 ensemble max {env.get(k, 0):.2e}")
