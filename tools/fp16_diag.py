"""Where does the fp16 step's distance from the reference's fp32 step come from?  (round 6)
One forward + backward at S = 256, B = 2 on model_s256_b2.npz's inputs / weights for several
precision mixes (each 16-bit family alone in fp16 / bf16, the LSTM recurrences fp32 or 16-mixed),
printing every loss's relative deviation from the reference fp32 step next to the reference's own
emulated fp16 / bf16 deviations (model_s256_b2_amp.npz).  GPU; usage: python tools/fp16_diag.py"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "vae-teb_amd")]

from test_gpu_parity_s256 import LOSSES, _forward_backward, _model, rel  # noqa: E402

G = np.load(os.path.join(ROOT, "tests", "golden", "model_s256_b2.npz"))
A = np.load(os.path.join(ROOT, "tests", "golden", "model_s256_b2_amp.npz"))
ref = {k: float(G["loss_" + k]) for k in LOSSES}
print("reference deviations (rel):", {m: {k: f"{abs(float(A[f'{m}_loss_{k}']) - ref[k]) / abs(ref[k]):.2e}"
                                          for k in LOSSES} for m in ("emu_fp16", "emu_bf16", "cpu_bf16")})
MIXES = [("fp16 all, lstm 16-mixed", "fp16", "fp16", "fp16", "16-mixed"),
         ("fp16 all, lstm fp32", "fp16", "fp16", "fp16", "fp32"),
         ("fp32 all, lstm 16-mixed", "fp32", "fp32", "fp32", "16-mixed"),
         ("fp16 mlp only", "fp32", "fp32", "fp16", "fp32"),
         ("fp16 conv only", "fp32", "fp16", "fp32", "fp32"),
         ("fp16 heads only", "fp16", "fp32", "fp32", "fp32"),
         ("bf16 all, lstm 16-mixed", "bf16", "bf16", "bf16", "16-mixed")]
for name, h, c, m_, l in MIXES:
    m = _model(256, head_precision=h, conv_precision=c, mlp_precision=m_, lstm_precision=l, concurrent_encoders=True)
    fw, L = _forward_backward(m, G)
    dev = {k: f"{abs(L[k].item() - ref[k]) / abs(ref[k]):.2e}" for k in LOSSES}
    fwd = {k: f"{rel(fw[k], G['fw_' + k]):.2e}" for k in ("z", "mu_prior", "logvar_prior", "mu_post", "logvar_post")}
    print(f"{name:28s} losses {dev}\n{'':28s} forward {fwd}", flush=True)
    del m
    torch.cuda.empty_cache()
