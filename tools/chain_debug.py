"""Diagnostic for the chained LSTM launches (round 6): vt_lstm16_quad_bwd against two
vt_lstm16_pair_bwd calls on the same forward state, every output compared separately
(dgates of layers 3, 2, the hand-off dmid, dgates of layers 1, 0, dx), and the same for the
forward's 12 outputs.  Prints one line per tensor: equal or the count / max of differences.

  python tools/chain_debug.py [B] [S] [In]
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vae-teb_amd"))
import torch  # noqa: E402

from vaeteb import _lib  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    S = int(sys.argv[2]) if len(sys.argv) > 2 else 256
    In = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    H = 64
    torch.manual_seed(3)
    ref = torch.nn.LSTM(In, H, 4, batch_first=True)
    params = [p.detach().cuda().contiguous() for p in ref.parameters()]
    x = torch.randn(B, S, In, device="cuda")
    call, ptr, st = _lib.call, _lib.ptr, _lib.stream
    E = lambda *s: torch.empty(*s, device="cuda")

    def outs():
        return [t for _ in range(4) for t in (E(B, S, H), E(B, S, H), E(B, S, 4 * H))]

    # forward: quad vs two pairs
    oq, op = outs(), outs()
    pv = (ctypes.c_void_p * 16)(*[ptr(t) for t in params])
    ov = (ctypes.c_void_p * 12)(*[ptr(t) for t in oq])
    call("vt_lstm16_quad_fwd", ptr(x), In, ctypes.addressof(pv), B, S, H, ctypes.addressof(ov), st())
    P = params
    call("vt_lstm16_pair_fwd", ptr(x), In, ptr(P[0]), ptr(P[2]), ptr(P[1]), ptr(P[3]), ptr(P[4]), ptr(P[6]), ptr(P[5]),
         ptr(P[7]), B, S, H, *[ptr(t) for t in op[:6]], st())
    call("vt_lstm16_pair_fwd", ptr(op[3]), H, ptr(P[8]), ptr(P[10]), ptr(P[9]), ptr(P[11]), ptr(P[12]), ptr(P[14]),
         ptr(P[13]), ptr(P[15]), B, S, H, *[ptr(t) for t in op[6:]], st())
    torch.cuda.synchronize()
    for i, (a, b) in enumerate(zip(oq, op)):
        n = (a != b).sum().item()
        print(f"fwd layer {i // 3} {('h', 'c', 'gates')[i % 3]}: {'equal' if n == 0 else f'{n} differ, max {(a - b).abs().max().item():.3e}'}")
    # backward on the pair-forward state
    h, c, g = op[0::3], op[1::3], op[2::3]
    dh = torch.randn(B, S, H, device="cuda")
    dgq, dgp = [E(B, S, 4 * H) for _ in range(4)], [E(B, S, 4 * H) for _ in range(4)]
    mq, mp = E(B, S, H), E(B, S, H)
    xq, xp = E(B, S, In), E(B, S, In)
    wv = (ctypes.c_void_p * 8)(*[ptr(P[4 * k + i]) for k in range(4) for i in (0, 1)])
    gv = (ctypes.c_void_p * 8)(*[ptr(t) for k in range(4) for t in (g[k], c[k])])
    dv = (ctypes.c_void_p * 4)(*[ptr(t) for t in dgq])
    cnt = ctypes.c_int()
    call("vt_lstm16_chain_errors", ctypes.byref(cnt), 1)
    call("vt_lstm16_quad_bwd", ptr(dh), ctypes.addressof(wv), ctypes.addressof(gv), In, B, S, H, ctypes.addressof(dv),
         ptr(mq), ptr(xq), st())
    call("vt_lstm16_pair_bwd", ptr(dh), ptr(g[3]), ptr(c[3]), ptr(P[13]), ptr(P[12]), ptr(g[2]), ptr(c[2]), ptr(P[9]),
         ptr(P[8]), H, B, S, H, ptr(dgp[3]), ptr(dgp[2]), ptr(mp), st())
    call("vt_lstm16_pair_bwd", ptr(mp), ptr(g[1]), ptr(c[1]), ptr(P[5]), ptr(P[4]), ptr(g[0]), ptr(c[0]), ptr(P[1]),
         ptr(P[0]), In, B, S, H, ptr(dgp[1]), ptr(dgp[0]), ptr(xp), st())
    torch.cuda.synchronize()
    call("vt_lstm16_chain_errors", ctypes.byref(cnt), 1)
    print(f"chain timeouts: {cnt.value}")
    for name, a, b in [("dg3", dgq[3], dgp[3]), ("dg2", dgq[2], dgp[2]), ("dmid", mq, mp), ("dg1", dgq[1], dgp[1]),
                       ("dg0", dgq[0], dgp[0]), ("dx", xq, xp)]:
        d = a != b
        n = d.sum().item()
        if n:
            idx = d.nonzero()
            ts = idx[:, 1]
            print(f"bwd {name}: {n} differ, max {(a - b).abs().max().item():.3e}; steps {ts.min().item()}..{ts.max().item()}, "
                  f"samples {idx[:, 0].min().item()}..{idx[:, 0].max().item()}")
        else:
            print(f"bwd {name}: equal")
        if name == "dmid" and n:
            per_t = d.any(-1).float().mean(0)          # fraction of samples wrong per step
            print("  dmid wrong-sample fraction per step (every 8th):", [round(v, 2) for v in per_t[::8].tolist()])
            per_c = d.any(1).float().mean(0)           # per column
            print("  dmid wrong fraction per column (every 4th):", [round(v, 2) for v in per_c[::4].tolist()])
            for sh in (-16, -8, -1, 1, 8, 16):
                if sh > 0:
                    eq = (a[:, sh:] == b[:, :-sh]).float().mean().item()
                else:
                    eq = (a[:, :sh] == b[:, -sh:]).float().mean().item()
                print(f"  dmid(quad)[t] == dmid(pairs)[t - {sh}] fraction {eq:.3f}")
            print("  quad zeros:", (a == 0).float().mean().item(), "pairs zeros:", (b == 0).float().mean().item())


if __name__ == "__main__":
    main()
