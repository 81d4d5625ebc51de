"""Fused ELBO kernels and the flat AdamW / grad-clip step vs torch fp32/fp64
references of the same formulas (ref/model/vae_teb_model.py:932-1082,
ref/model/graph_model.py:654-660,724).  Tolerances are written per assert."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def L():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from vaeteb import _lib
    return _lib


def _kl_ref(mp, lp, mq, lq):
    return (0.5 * (lp - lq - 1 + (lq.exp() + (mq - mp) ** 2) / lp.exp())).sum(-1).mean()


def test_latent_fwd_bwd(L):
    torch.manual_seed(0)
    B, S, D = 8, 64, 32
    cpu = {k: torch.randn(B, S, D, dtype=torch.float64) for k in ("mu_c", "lv_q", "mu_y", "lv_p", "eps", "gz")}
    cpu["lv_q"] = cpu["lv_q"].clamp(-3, 3)
    cpu["lv_p"] = cpu["lv_p"].clamp(-3, 3)
    beta = 1e-2
    # fp64 autograd reference
    ref = {k: v.clone().requires_grad_(k in ("mu_c", "lv_q", "mu_y", "lv_p")) for k, v in cpu.items()}
    mq = ref["mu_c"] + ref["mu_y"]
    z = mq + ref["eps"] * torch.exp(0.5 * ref["lv_q"])
    kl = _kl_ref(ref["mu_y"], ref["lv_p"], mq, ref["lv_q"])
    ((z * ref["gz"]).sum() + beta * kl).backward()

    d = {k: v.float().cuda().contiguous() for k, v in cpu.items()}
    zt, mpt, klt = torch.empty_like(d["mu_c"]), torch.empty_like(d["mu_c"]), torch.empty(1, device="cuda")
    ws = torch.empty(L.lib().fns["vt_elbo_workspace_floats"](), device="cuda")
    P = L.ptr
    L.call("vt_elbo_latent_fwd", P(d["mu_c"]), P(d["lv_q"]), P(d["mu_y"]), P(d["lv_p"]), P(d["eps"]), B * S, D,
           P(zt), P(mpt), P(klt), P(ws), L.stream())
    assert torch.allclose(zt.cpu().double(), z.detach(), rtol=1e-6, atol=1e-6)
    assert abs(klt.item() - kl.item()) <= 1e-6 * abs(kl.item())
    gk = torch.tensor([beta], device="cuda")
    g = {k: torch.empty_like(d["mu_c"]) for k in ("mu_c", "lv_q", "mu_y", "lv_p")}
    L.call("vt_elbo_latent_bwd", P(d["mu_c"]), P(d["lv_q"]), P(d["mu_y"]), P(d["lv_p"]), P(d["eps"]), B * S, D,
           P(d["gz"]), None, P(gk), P(g["mu_c"]), P(g["lv_q"]), P(g["mu_y"]), P(g["lv_p"]), L.stream())
    for k in g:
        assert torch.allclose(g[k].cpu().double(), ref[k].grad, rtol=1e-5, atol=1e-6), k


@pytest.mark.parametrize("with_mse", [True, False])
def test_output_losses(L, with_mse):
    torch.manual_seed(1)
    B, S = 4, 32
    R = 16 * S
    mu, lv, y = torch.randn(B, R, dtype=torch.float64), torch.randn(B, R, dtype=torch.float64), torch.randn(B, R, dtype=torch.float64)
    lin, ts, tp = torch.randn(B, S, 87, dtype=torch.float64), torch.randn(B, S, 43, dtype=torch.float64), torch.randn(B, S, 44, dtype=torch.float64)
    r = {k: v.clone().requires_grad_(True) for k, v in dict(mu=mu, lv=lv, lin=lin).items()}
    nll = (0.5 * (r["lv"] + (y - r["mu"]) ** 2 / r["lv"].exp())).mean()
    mse = ((r["lin"] - torch.cat([ts, tp], -1)) ** 2).mean()
    (nll + mse).backward()
    d = {k: v.float().cuda() for k, v in dict(mu=mu, lv=lv, y=y, lin=lin, ts=ts, tp=tp).items()}
    g_mu, g_lv, g_lin = torch.empty_like(d["mu"]), torch.empty_like(d["mu"]), torch.empty_like(d["lin"])
    out = torch.zeros(2, device="cuda")
    ws = torch.empty(L.lib().fns["vt_elbo_workspace_floats"](), device="cuda")
    P = L.ptr
    L.call("vt_elbo_output_fwd", P(d["mu"]), P(d["lv"]), P(d["y"]), B * R, P(d["lin"]) if with_mse else None,
           P(d["ts"]), P(d["tp"]), B * S, 43, 44, P(g_mu), P(g_lv), P(g_lin), out.data_ptr(), out.data_ptr() + 4,
           P(ws), L.stream())
    o = out.cpu()
    assert abs(o[0].item() - nll.item()) <= 1e-6 * abs(nll.item())
    assert torch.allclose(g_mu.cpu().double(), r["mu"].grad, rtol=1e-5, atol=1e-10)
    assert torch.allclose(g_lv.cpu().double(), r["lv"].grad, rtol=1e-5, atol=1e-10)
    if with_mse:
        assert abs(o[1].item() - mse.item()) <= 1e-6 * abs(mse.item())
        assert torch.allclose(g_lin.cpu().double(), r["lin"].grad, rtol=1e-5, atol=1e-10)


def test_grad_norm_and_adamw_match_torch(L):
    """3 steps of flat clip+AdamW == torch clip_grad_norm_ + torch.optim.AdamW (fp32 CPU)."""
    torch.manual_seed(2)
    shapes = [(37, 11), (5,), (256, 64), (1000,)]
    params = [torch.randn(s) for s in shapes]
    n = sum(p.numel() for p in params)
    ref = [p.clone().requires_grad_(True) for p in params]
    opt = torch.optim.AdamW(ref, lr=1e-2, weight_decay=1e-4, eps=1e-8, betas=(0.9, 0.98))
    flat_p = torch.cat([p.reshape(-1) for p in params]).cuda()
    m, v = torch.zeros_like(flat_p), torch.zeros_like(flat_p)
    ws = torch.empty(L.lib().fns["vt_grad_norm_workspace_floats"](), device="cuda")
    out2 = torch.empty(2, device="cuda")
    world = 2.0  # emulate an all-reduce SUM over 2 ranks folded into pre_scale
    for step in range(1, 4):
        grads = [torch.randn(s) * 3 for s in shapes]
        for p, g in zip(ref, grads):
            p.grad = g.clone()
        tn = torch.nn.utils.clip_grad_norm_(ref, max_norm=1.0)
        opt.step()
        flat_g = torch.cat([g.reshape(-1) for g in grads]).cuda() * world
        L.call("vt_grad_norm_clip", flat_g.data_ptr(), n, 1.0 / world, 1.0, out2.data_ptr(), ws.data_ptr(), L.stream())
        L.call("vt_adamw_step", flat_p.data_ptr(), flat_g.data_ptr(), m.data_ptr(), v.data_ptr(), n, 1e-2, 0.9, 0.98,
               1e-8, 1e-4, step, out2.data_ptr() + 4, L.stream())
        assert abs(out2[0].item() - tn.item()) <= 1e-5 * tn.item()
    got = flat_p.cpu()
    exp = torch.cat([p.detach().reshape(-1) for p in ref])
    assert torch.allclose(got, exp, rtol=1e-5, atol=1e-6), (got - exp).abs().max()


def test_adamw_vector_equals_scalar(L):
    """The float4 AdamW kernel (aligned buffers) gives the scalar kernel's bits,
    including the < 4 tail elements; a misaligned view takes the scalar kernel."""
    torch.manual_seed(3)
    for n in (4099, 1 << 20):
        p0, g = torch.randn(n + 1, device="cuda"), torch.randn(n + 1, device="cuda") * 3
        m0, v0 = torch.randn(n + 1, device="cuda") * 0.1, torch.rand(n + 1, device="cuda") * 0.1
        gscale = torch.tensor([0.7], device="cuda")
        outs = []
        for vec in (1, 0):
            L.call("vt_adamw_set_vector", vec)
            p, m, v = p0.clone(), m0.clone(), v0.clone()
            for step in (1, 2):
                L.call("vt_adamw_step", p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(), n, 1e-3, 0.9, 0.999,
                       1e-8, 1e-4, step, gscale.data_ptr(), L.stream())
            outs.append((p, m, v))
        L.call("vt_adamw_set_vector", 1)
        for a, b in zip(*outs):
            assert torch.equal(a, b)
        # misaligned (offset by one float): the launcher falls back to the scalar kernel
        p, m, v = p0.clone(), m0.clone(), v0.clone()
        L.call("vt_adamw_step", p.data_ptr() + 4, g.data_ptr() + 4, m.data_ptr() + 4, v.data_ptr() + 4, n, 1e-3, 0.9,
               0.999, 1e-8, 1e-4, 1, gscale.data_ptr(), L.stream())
        assert torch.equal(p[0], p0[0]) and not torch.equal(p[1:], p0[1:])


def test_adamw_writes_bf16_shadows_same_bits():
    """The optimizer step writing the bf16 weight shadows (tiled AdamW over the 4096^2
    heads: vt_adamw_step_dev_shadow; the conv shadows in one batched launch) == the forward
    rewriting them (VAETEB_SHADOW_UPDATE=0), bit for bit over 3 steps at the bench geometry
    (S = 256, bf16 heads / convs / MLP, B = 2): losses, parameters, Adam moments; and a
    load_state_dict between steps (the weights change behind the trainer's back) makes the
    next forward rewrite the shadows (the torch version counter check)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from golden_util import det_fill_
    from vaeteb import ops
    from vaeteb import train as T
    from vaeteb.model import SeqVaeTeb
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "model_s256_b2.npz"), allow_pickle=False)
    C = lambda k: torch.from_numpy(g[k]).cuda()
    batch = {"fhr_st": C("y_st"), "fhr_ph": C("y_ph"), "fhr_up_ph": C("x_ph"), "fhr": C("y_raw")}
    res = []
    prev = T.SHADOW_UPDATE
    try:
        for mode in (0, 1):
            T.SHADOW_UPDATE = mode
            m = det_fill_(SeqVaeTeb(sequence_length=256, head_precision="bf16", conv_precision="bf16",
                                    mlp_precision="bf16", concurrent_encoders=True)).cuda()
            tr = T.Trainer(m, lr=1e-3)
            losses = [tr.step(batch, eps=C("eps"))["total_loss"].item() for _ in range(3)]
            if mode:
                assert tr._shadow_plan()[0] == 4 and tr._shadow_plan()[1] == 17   # 4 heads, 17 convs
                assert len(ops._FRESH) == 21
            torch.cuda.synchronize()
            res.append((losses, tr.state.p.clone(), tr.state.m.clone(), tr.state.v.clone(), m))
    finally:
        T.SHADOW_UPDATE = prev
    assert res[0][0] == res[1][0], (res[0][0], res[1][0])
    for a, b in zip(res[0][1:4], res[1][1:4]):
        assert torch.equal(a, b)
    # weights replaced behind the trainer's back: the fresh shadows must not be used
    m_old, m_new = res[0][4], res[1][4]
    with torch.no_grad():
        m_new.load_state_dict(det_fill_(SeqVaeTeb(sequence_length=256)).state_dict())
        m_old.load_state_dict(m_new.state_dict())
        m_old.train(), m_new.train()
        a = m_new(C("y_st"), C("y_ph"), C("x_ph"), eps=C("eps"))["mu_pr"]
        b = m_old(C("y_st"), C("y_ph"), C("x_ph"), eps=C("eps"))["mu_pr"]
    assert torch.equal(a, b)
