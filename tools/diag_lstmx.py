"""Fused vs unfused LSTM layer backward: which dx / dgates rows differ."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vae-teb_amd"))
import torch  # noqa: E402
from vaeteb._lib import call, ptr, stream  # noqa: E402

H = 64
for In, B, S in ((20, 3, 33), (20, 2, 32), (64, 2, 33), (64, 2, 16), (64, 1, 5)):
    torch.manual_seed(In + S)
    dev = "cuda"
    x = torch.randn(B, S, In, device=dev)
    wih, whh = torch.randn(4 * H, In, device=dev) * 0.2, torch.randn(4 * H, H, device=dev) * 0.2
    bih, bhh = torch.randn(4 * H, device=dev) * 0.1, torch.randn(4 * H, device=dev) * 0.1
    h, hp, c = [torch.empty(B, S, H, device=dev) for _ in range(3)]
    gates = torch.empty(B, S, 4 * H, device=dev)
    call("vt_lstm_layer_fwd_x", ptr(x), In, ptr(wih), ptr(bih), ptr(whh), ptr(bhh), B, S, H, ptr(h), ptr(hp), ptr(c),
         ptr(gates), stream())
    dh = torch.randn(B, S, H, device=dev)
    dg0, dg1 = torch.empty(B, S, 4 * H, device=dev), torch.empty(B, S, 4 * H, device=dev)
    dx0, dx1 = torch.empty(B, S, In, device=dev), torch.full((B, S, In), float("nan"), device=dev)
    call("vt_lstm_layer_bwd", ptr(dh), ptr(gates), ptr(c), ptr(whh), B, S, H, ptr(dg0), stream())
    call("vt_linear_bwd_data", ptr(dg0), B * S, 4 * H, ptr(wih), In, ptr(dx0), 0, stream())
    call("vt_lstm_layer_bwd_x", ptr(dh), ptr(gates), ptr(c), ptr(whh), ptr(wih), In, B, S, H, ptr(dg1), ptr(dx1),
         stream())
    torch.cuda.synchronize()
    bad_g = (dg0 != dg1).any(-1)
    bad_x = ~(dx0 == dx1).all(-1)
    print(f"In={In} B={B} S={S}: dgates rows differing {bad_g.sum().item()} {bad_g.nonzero()[:8].tolist()}; "
          f"dx rows differing {bad_x.sum().item()} {bad_x.nonzero()[:8].tolist()} "
          f"max|d| {(dx0 - dx1).abs().nan_to_num(1e9).max().item():.3e}", flush=True)
