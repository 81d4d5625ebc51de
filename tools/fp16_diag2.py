"""Per ResidualMLP stack: the KL loss / z deviation from the reference fp32 step at S = 256 when ONLY
that stack runs 16-bit (fp16, then bf16), everything else exact fp32 (round 6: which stack carries
the fp16 step's KL shift).  GPU; usage: python tools/fp16_diag2.py"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "vae-teb_amd")]

from test_gpu_parity_s256 import _forward_backward, _model, rel  # noqa: E402
from vaeteb.model import ResidualMLP  # noqa: E402

G = np.load(os.path.join(ROOT, "tests", "golden", "model_s256_b2.npz"))
ref = float(G["loss_kld_loss"])
m = _model(256, concurrent_encoders=True)
stacks = [(n, mod) for n, mod in m.named_modules() if isinstance(mod, ResidualMLP) and mod._fused_spec() is not None]
print(f"{len(stacks)} fused ResidualMLP stacks; reference kld {ref:.6f}", flush=True)
for n, mod in stacks:
    out = []
    for fmt in ("fp16", "bf16"):
        mod.bf16 = fmt
        fw, L = _forward_backward(m, G)
        out.append(((L["kld_loss"].item() - ref) / ref, rel(fw["z"], G["fw_z"]), rel(fw["mu_post"], G["fw_mu_post"])))
        mod.bf16 = False
        m.zero_grad(set_to_none=True)
    dims = mod._fused_spec()[0].dims_l
    print(f"{n:45s} dims {len(dims) - 1} layers {dims[0]}->{dims[-1]}: fp16 kld {out[0][0]:+.2e} z {out[0][1]:.2e} "
          f"mu_post {out[0][2]:.2e} | bf16 kld {out[1][0]:+.2e} z {out[1][1]:.2e}", flush=True)
