"""SHA-256 of vt_layernorm_bwd's outputs (dx, dgamma, dbeta) over seeded inputs at the widths the
model uses (C 16 .. 256, rows up to 256 x 256): run under two builds (VAETEB_LIB=...) to check
that a change to the backward or its column reduction writes the same bits."""
import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vae-teb_amd"))
import torch  # noqa: E402
from vaeteb import _lib  # noqa: E402

h = hashlib.sha256()
for R, C, act in ((65536, 256, 0), (65536, 128, 1), (65536, 64, 2), (65536, 32, 0), (1000, 16, 1), (777, 144, 0)):
    g = torch.Generator().manual_seed(R + C)
    dy = torch.randn(R, C, generator=g).cuda()
    xh = torch.randn(R, C, generator=g).cuda()
    rs = torch.rand(R, generator=g).add_(0.5).cuda()
    gam = torch.randn(C, generator=g).cuda()
    bet = torch.randn(C, generator=g).cuda()
    dx = torch.empty_like(dy)
    dg = torch.empty(C, device="cuda")
    db = torch.empty(C, device="cuda")
    ws = torch.empty(2 * C * 1024 + 2 * R * C, device="cuda")
    _lib.call("vt_layernorm_bwd", _lib.ptr(dy), _lib.ptr(xh), _lib.ptr(rs), R, C, _lib.ptr(gam), _lib.ptr(bet), act,
              _lib.ptr(dx), _lib.ptr(dg), _lib.ptr(db), 0, _lib.ptr(ws), ws.numel(), _lib.stream())
    torch.cuda.synchronize()
    for t in (dx, dg, db):
        h.update(t.cpu().numpy().tobytes())
print(h.hexdigest())
