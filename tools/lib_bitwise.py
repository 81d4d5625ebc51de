"""Bit-equality of two library builds on the training step: run 2 steps of the
bf16 SeqVaeTeb (S = 64, B = 8, deterministic weights / inputs) and save the flat
gradient, parameters and losses (sha256 digests); `compare` checks two saved runs for equality.
usage: lib_bitwise.py run OUT.json   (with VAETEB_LIB=... for the other build)
       lib_bitwise.py compare A.json B.json"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vae-teb_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402

if sys.argv[1] == "compare":
    import json
    a, b = json.load(open(sys.argv[2])), json.load(open(sys.argv[3]))
    for k in a:
        print(f"{k}: {'bit-identical' if a[k] == b[k] else 'DIFFERENT'} ({a[k][:16]} / {b[k][:16]})")
    sys.exit(0 if a == b else 1)

from golden_util import det_fill_  # noqa: E402
from vaeteb.model import SeqVaeTeb  # noqa: E402
from vaeteb.train import Trainer  # noqa: E402

S, B = int(os.environ.get("LB_S", 64)), int(os.environ.get("LB_B", 8))
g = torch.Generator().manual_seed(7)
batch = {"fhr_st": torch.randn(B, S, 43, generator=g), "fhr_ph": torch.randn(B, S, 44, generator=g),
         "fhr_up_ph": torch.randn(B, S, 130, generator=g), "fhr": torch.randn(B, 16 * S, generator=g)}
eps = torch.randn(B, S, 32, generator=g).cuda()
batch = {k: v.cuda() for k, v in batch.items()}
m = det_fill_(SeqVaeTeb(sequence_length=S, head_precision="bf16", conv_precision="bf16", mlp_precision="bf16",
                        concurrent_encoders=True)).cuda()
tr = Trainer(m, lr=1e-3)
for _ in range(2):
    L = tr.step(batch, eps=eps)
torch.cuda.synchronize()
import hashlib  # noqa: E402
import json  # noqa: E402
digest = lambda t: hashlib.sha256(t.detach().cpu().contiguous().numpy().tobytes()).hexdigest()
json.dump({"loss": digest(L["total_loss"].reshape(1)), "g": digest(tr.state.g), "p": digest(tr.state.p)},
          open(sys.argv[2], "w"))
print("saved", sys.argv[2], L["total_loss"].item())
