"""How far does an fp32 implementation of the c2 step at B = 256 land from fp64, run to run?
  The oracle step (oracle/model_ref.py, the checker) in fp64 vs fp32 runs
that differ from each other only at the last bit: the plain fp32 run and fp32 runs whose
initial weights (or input features) are perturbed by one ulp with random signs.  For each run
the whole-gradient rel-L2 to fp64, the pre-clip norm's relative gap and the median / p90 of the
per-gradient rel-L2 (the quantities test_bench_batch_fp32_step_vs_fp64_oracle bounds).  CPU only.

  python tools/b256_ensemble.py [--batch 256] [--members 4] [--out gpurun_out/b256_ensemble.json]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "vae-teb_amd")]


def features(B):
    from oracle import frontend_ref as F
    from vaeteb import synthetic
    from vaeteb.frontend import load_stats
    st = load_stats(11, 4, 16, 4096)
    x = synthetic.batch(777, B, 4096)
    old, F.FFT_ENGINE = F.FFT_ENGINE, "torch"
    ofe = F.PhaseFrontEnd(11, 4, 16, 4096, dtype=np.float32)
    pm, cm = ofe.masks()
    rp = ofe.forward(x, compute_phase=True, pair_subset=pm)
    rc = ofe.forward(x, compute_phase=False, compute_cross_phase=True, pair_subset=cm)
    F.FFT_ENGINE = old
    tt = lambda a: np.ascontiguousarray(np.asarray(a, np.float32).transpose(0, 2, 1))
    return {"fhr_st": tt(F.normalize(rp["scattering"], "fhr_st", st["fhr_st_mean"], st["fhr_st_variance"])),
            "fhr_ph": tt(F.normalize(rp["phase_corr"], "fhr_ph", st["fhr_ph_mean"], st["fhr_ph_variance"])),
            "fhr_up_ph": tt(F.normalize(rc["cross_phase_corr"], "fhr_up_ph", st["fhr_up_ph_mean"],
                                        st["fhr_up_ph_variance"])),
            "fhr": np.asarray(F.normalize(x[:, 0], "fhr", st["fhr_mean"], st["fhr_variance"]), np.float32)}


def ulp_perturb_(t, gen):
    """t *= 1 + s 2^-23 (s = +-1 at random): one ulp of fp32 in the mantissa's units"""
    s = torch.randint(0, 2, t.shape, generator=gen).to(t.dtype) * 2 - 1
    t.mul_(1 + s * 2.0 ** -23)


def step(feats, eps, dtype, wseed=None, fseed=None):
    from golden_util import det_fill_
    from oracle import model_ref as M
    ref = det_fill_(M.SeqVaeTebRef(256, 43, 44, 130)).to(dtype)
    if wseed is not None:
        g = torch.Generator().manual_seed(wseed)
        with torch.no_grad():
            for p in ref.parameters():
                ulp_perturb_(p, g)
    T = lambda a: torch.from_numpy(np.asarray(a)).to(dtype)
    b = {"y_st": T(feats["fhr_st"]), "y_ph": T(feats["fhr_ph"]), "x_ph": T(feats["fhr_up_ph"]), "y_raw": T(feats["fhr"])}
    if fseed is not None:
        g = torch.Generator().manual_seed(fseed)
        for k in b:
            ulp_perturb_(b[k], g)
    _, L, grads, _ = M.train_step(ref, b, T(eps), 1e-5)
    return L, grads


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--members", type=int, default=4)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "b256_ensemble.json"))
    a = ap.parse_args()
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    t0 = time.time()
    feats = features(a.batch)
    eps = np.random.default_rng(8).standard_normal((a.batch, 256, 32)).astype(np.float32)
    print(f"features {time.time() - t0:.1f} s", flush=True)
    L64, g64 = step(feats, eps, torch.float64)
    names = list(g64)
    heads = {k for k in names if g64[k].numel() >= 1 << 20}
    flat = lambda g: torch.cat([g[k].double().reshape(-1) for k in names])
    go = flat(g64)
    gn64 = go.norm().item()
    runs = [("fp32", {})] + [(f"fp32 weights 1-ulp seed {s}", {"wseed": s}) for s in range(a.members - 1)] + \
           [("fp32 features 1-ulp seed 0", {"fseed": 0})]
    out = {"batch": a.batch, "norm_fp64": gn64, "runs": []}
    for name, kw in runs:
        t = time.time()
        L, g = step(feats, eps, torch.float32, **kw)
        v = flat(g)
        per = np.array([((g[k].double() - g64[k]).norm() / g64[k].norm()).item() for k in names
                        if k not in heads and g64[k].norm() > 0])
        r = {"run": name, "whole_rel": ((v - go).norm() / go.norm()).item(), "norm_rel": (v.norm().item() - gn64) / gn64,
             "median": float(np.median(per)), "p90": float(np.percentile(per, 90)), "max": float(per.max()),
             "bias_l3_rel": ((g["target_encoder.lstm.bias_ih_l3"].double() - g64["target_encoder.lstm.bias_ih_l3"]).norm()
                             / g64["target_encoder.lstm.bias_ih_l3"].norm()).item(),
             "total_loss_rel": abs(L["total_loss"].item() - L64["total_loss"].item()) / abs(L64["total_loss"].item())}
        out["runs"].append(r)
        print(json.dumps(r), f"({time.time() - t:.1f} s)", flush=True)
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    json.dump(out, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
