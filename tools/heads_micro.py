#!/usr/bin/env python3
"""Decoder-head GEMMs at the bench geometry (R = 256 rows, K = N = 4096), HIP-event timed:
vt_mfma_linear_fwd / _bwd_data / _bwd_weight, each launch averaged over `--iters` calls
(weights and activations resident; the weight shadow written once).  Prints one JSON line."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vae-teb_amd"))

import torch  # noqa: E402

from vaeteb import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--R", type=int, default=256)
    ap.add_argument("--K", type=int, default=4096)
    ap.add_argument("--N", type=int, default=4096)
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args()
    import ctypes
    R, K, N = a.R, a.K, a.N
    L = _lib.lib()
    n = ctypes.c_int64(0)
    L.fns["vt_mfma_workspace_floats"](R, K, N, ctypes.addressof(n))
    ws = torch.empty(n.value + 64, device="cuda")
    X = torch.randn(R, K, device="cuda")
    W = torch.randn(N, K, device="cuda") * 0.01
    b = torch.randn(N, device="cuda")
    Y = torch.empty(R, N, device="cuda")
    dY = torch.randn(R, N, device="cuda")
    dX = torch.empty(R, K, device="cuda")
    dW = torch.empty(N, K, device="cuda")
    w16 = torch.empty(N, K, dtype=torch.bfloat16, device="cuda")
    w16t = torch.empty(K, N, dtype=torch.bfloat16, device="cuda")
    st = _lib.stream()
    L.call("vt_mfma_weight_shadow", W.data_ptr(), N, K, w16.data_ptr(), w16t.data_ptr(), st)
    calls = {
        "fwd": lambda: L.call("vt_mfma_linear_fwd", X.data_ptr(), R, K, w16.data_ptr(), N, b.data_ptr(), Y.data_ptr(),
                              ws.data_ptr(), ws.numel(), st),
        "bwd_data": lambda: L.call("vt_mfma_linear_bwd_data", dY.data_ptr(), R, N, w16t.data_ptr(), K, dX.data_ptr(), 0,
                                   ws.data_ptr(), ws.numel(), st),
        "bwd_weight": lambda: L.call("vt_mfma_linear_bwd_weight", dY.data_ptr(), R, N, X.data_ptr(), K, dW.data_ptr(),
                                     None, 0, ws.data_ptr(), ws.numel(), st),
    }
    out = {"R": R, "K": K, "N": N}
    for name, fn in calls.items():
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / a.iters
        out[name + "_us"] = round(us, 2)
        out[name + "_TFs"] = round(2 * R * K * N / (us * 1e-6) / 1e12, 1)
    # correctness spot check of the forward against torch on the bf16-rounded operands
    ref = (X.bfloat16().double() @ w16.double().t()) + b.double()
    out["fwd_rel_err"] = float((Y.double() - ref).norm() / ref.norm())
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
