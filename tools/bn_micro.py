"""BatchNorm backward kernels of the conv blocks at the decoder / encoder shapes (B = 256):
vt_batchnorm_bwd_coef (k_col_partial4 + k_bn_finalize) and vt_batchnorm_bwd_x16
(k_bn_bwd_x16), HIP-event time per launch and HBM GB/s of the compulsory bytes, plus a
checksum of the bf16 rows (compare runs under VAETEB_BNX16_PF=0 / 1: same bits).
usage: bn_micro.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vae-teb_amd"))
import torch  # noqa: E402
from vaeteb._lib import call  # noqa: E402

SHAPES = [(256 * 4096, 22), (256 * 4096, 11), (256 * 4096, 1), (256 * 2048, 33), (256 * 1024, 44),
          (256 * 1024, 55), (256 * 512, 66), (256 * 256, 77), (256 * 256, 32), (256 * 256, 16)]
p = lambda t: t.data_ptr()
st = torch.cuda.current_stream().cuda_stream
for M, C in SHAPES:
    g = torch.Generator(device="cuda").manual_seed(M + C)
    dy = torch.randn(M, C, device="cuda", generator=g)
    x = torch.randn(M, C, device="cuda", generator=g)
    mean, rstd = x.mean(0), x.var(0).add(1e-5).rsqrt()
    gam, bet = torch.rand(C, device="cuda", generator=g) + 0.5, torch.randn(C, device="cuda", generator=g)
    dg, db = torch.zeros(C, device="cuda"), torch.zeros(C, device="cuda")
    bnp = torch.empty(6 * C, device="cuda")
    ws = torch.empty(4096 * C + 2 * C, device="cuda")
    c32 = (C + 31) // 32 * 32
    d16 = torch.empty(M * c32, dtype=torch.bfloat16, device="cuda")
    coef = lambda: call("vt_batchnorm_bwd_coef", p(dy), p(x), M, C, p(mean), p(rstd), p(gam), p(bet), 1, p(dg), p(db),
                        0, p(bnp), p(ws), ws.numel(), st)
    x16 = lambda: call("vt_batchnorm_bwd_x16", p(dy), p(x), p(bnp), 1, M, C, p(d16), st)
    res = []
    for fn, nbytes in ((coef, 2 * M * C * 4), (x16, 2 * M * C * 4 + M * c32 * 2)):
        for _ in range(3):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            fn()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / 20 * 1e3
        res.append(f"{us:7.1f} us {nbytes / us / 1e3:6.0f} GB/s")
    ck = int(d16.view(torch.int16).to(torch.int64).sum().item())
    dg.zero_()
    db.zero_()
    coef()
    cc = hash(tuple(torch.cat([dg, db, bnp]).view(torch.int32).tolist()))
    print(f"M {M:8d} C {C:3d}: coef {res[0]} | x16 {res[1]} | rows checksum {ck} | coef bits {cc}", flush=True)
