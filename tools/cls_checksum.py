"""Per-op SHA-256 of the classifier's element-wise and attention kernels (max-pool forward /
backward, Dropout / Dropout1d, attention forward / backward) on seeded inputs at the c4
geometry: run under two builds (VAETEB_LIB=...) to see which op writes different bits."""
import hashlib
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vae-teb_amd"))
import torch  # noqa: E402
from vaeteb import _lib  # noqa: E402

call, ptr, st = _lib.call, _lib.ptr, _lib.stream


def digest(*ts):
    torch.cuda.synchronize()
    h = hashlib.sha256()
    for t in ts:
        h.update(t.cpu().numpy().tobytes())
    return h.hexdigest()[:16]


g = torch.Generator().manual_seed(5)
B, L, C = 64, 256, 128
x = torch.randn(B, L, C, generator=g).cuda()
x[:, ::7] = x[:, 1::7][:, : x[:, ::7].shape[1]]   # ties between neighbours
gy = torch.randn(B, L, C, generator=g).cuda()
y = torch.empty_like(x)
call("vt_maxpool3_fwd", ptr(x), B, L, C, ptr(y), st())
dx = torch.empty_like(x)
call("vt_maxpool3_bwd", ptr(gy), ptr(x), B, L, C, ptr(dx), 0, st())
print("maxpool fwd", digest(y), "bwd", digest(dx))
d1 = torch.empty_like(x)
call("vt_dropout_apply", ptr(x), x.numel(), C, L, 0.2, 123, None, ptr(d1), st())
d0 = torch.empty_like(x)
call("vt_dropout_apply", ptr(x), x.numel(), C, 0, 0.2, 123, None, ptr(d0), st())
print("dropout1d", digest(d1), "dropout", digest(d0))
H, S, E = 4, 256, 128
qkv = torch.randn(B, S, 3 * E, generator=g).cuda()
dout = torch.randn(B, S, E, generator=g).cuda()
for p in (0.0, 0.1):
    out = torch.empty(B, S, E, device="cuda")
    lse = torch.empty(B * H * S, device="cuda")
    scale = 1.0 / math.sqrt(E // H)
    call("vt_attn_fwd", ptr(qkv), B, S, H, scale, p, 77, None, ptr(out), ptr(lse), st())
    dq = torch.empty_like(qkv)
    call("vt_attn_bwd", ptr(qkv), ptr(out), ptr(dout), ptr(lse), B, S, H, scale, p, 77, None, ptr(dq), st())
    print(f"attn p={p} fwd", digest(out), "lse", digest(lse), "bwd", digest(dq))
    if os.environ.get("CK_SAVE") and p == 0.0:   # for an old / new comparison against fp64
        torch.save({"qkv": qkv.cpu(), "out": out.cpu(), "lse": lse.cpu()}, os.environ["CK_SAVE"])
