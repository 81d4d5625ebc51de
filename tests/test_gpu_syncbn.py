"""Synchronised BatchNorm (Lightning sync_batchnorm=True, ref/model/graph_model.py:517;
torch.nn.SyncBatchNorm semantics) in the HIP conv blocks, two ranks on one MI355X
over gloo (CUDA tensors; RCCL refuses two ranks on one device): each rank holds half
of a batch; its block output, the running statistics, the input gradient and the
summed parameter gradients must equal the single-process full-batch block
(tolerance rel-L2 1e-5 for y / running stats, 2e-5 for dx / dW / dgamma / dbeta:
different summation orders; 2e-3 for the gradients of the bf16 blocks, see below).  Also the whole SeqVaeTeb step via
convert_sync_batchnorm: both ranks' BatchNorm running statistics agree and equal
the full-batch model's."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CASES = [  # (B per rank, L, Cin, Cout, K, causal, up, bf16)
    (3, 64, 16, 16, 5, True, False, False),
    (2, 40, 87, 77, 11, False, False, True),
    (2, 32, 33, 22, 3, False, True, True),
]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _data(case):
    B, L, Cin, Cout, K, causal, up, bf16 = case
    g = torch.Generator().manual_seed(Cin * 100 + Cout)
    x = torch.randn(2 * B, L, Cin, generator=g)
    w = torch.randn(Cout, Cin, K, generator=g) / (Cin * K) ** 0.5
    gam = 1 + 0.1 * torch.randn(Cout, generator=g)
    bet = 0.1 * torch.randn(Cout, generator=g)
    return x, w, gam, bet


def _block(case, w, gam, bet):
    from vaeteb.model import ConvBlock
    B, L, Cin, Cout, K, causal, up, bf16 = case
    blk = ConvBlock(Cin, Cout, K, causal=causal, up=up).cuda()
    blk.bf16 = bf16
    with torch.no_grad():
        blk.conv.weight.copy_(w)
        blk.bn_layer.weight.copy_(gam)
        blk.bn_layer.bias.copy_(bet)
    return blk


def _run(blk, x, gy):
    xd = x.cuda().requires_grad_(True)
    y = blk(xd)
    (y * gy.cuda()).sum().backward()
    torch.cuda.synchronize()
    return (y.detach().cpu(), xd.grad.cpu(), blk.conv.weight.grad.cpu(), blk.bn_layer.weight.grad.cpu(),
            blk.bn_layer.bias.grad.cpu(), blk.bn_layer.running_mean.cpu(), blk.bn_layer.running_var.cpu())


def _worker(rank, world, port, q):
    sys.path[:0] = [os.path.join(ROOT, "vae-teb_amd"), os.path.join(ROOT, "tests")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from vaeteb.model import SeqVaeTeb, convert_sync_batchnorm
    out = []
    for case in CASES:
        x, w, gam, bet = _data(case)
        B = case[0]
        blk = convert_sync_batchnorm(_block(case, w, gam, bet))
        res = _run(blk, x[rank * B:(rank + 1) * B], _gy(case)[rank * B:(rank + 1) * B])
        out.append(tuple(t.numpy() for t in res))
    # whole model: both ranks' running statistics equal the full-batch model's
    from golden_util import det_fill_
    g = np.load(os.path.join(ROOT, "tests", "golden", "model_s16_b4.npz"), allow_pickle=False)
    m = convert_sync_batchnorm(det_fill_(SeqVaeTeb(sequence_length=16)).cuda())
    T = lambda k: torch.from_numpy(g[k][2 * rank:2 * rank + 2].copy()).cuda()
    fw = m(T("y_st"), T("y_ph"), T("x_ph"), eps=T("eps"))
    L = m.compute_loss(fw, T("y_st"), T("y_ph"), T("y_raw"), beta=float(g["beta"]))
    L["total_loss"].backward()
    torch.cuda.synchronize()
    stats = {k: v.cpu().numpy() for k, v in m.state_dict().items() if "running" in k}
    q.put((rank, out, stats))
    dist.destroy_process_group()


def _gy(case):
    """The upstream gradient of the full batch (the ranks take their halves)."""
    B, L, Cin, Cout, K, causal, up, bf16 = case
    return torch.randn(2 * B, L * (2 if up else 1), Cout, generator=torch.Generator().manual_seed(7))


def test_sync_batchnorm_two_ranks_equals_full_batch():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    sys.path[:0] = [os.path.join(ROOT, "vae-teb_amd")]
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=200) for _ in range(world)], key=lambda o: o[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    rel = lambda a, b: float(np.linalg.norm(np.asarray(a, np.float64) - b) / max(np.linalg.norm(b), 1e-30))
    for ci, case in enumerate(CASES):
        x, w, gam, bet = _data(case)
        full = [t.numpy() for t in _run(_block(case, w, gam, bet), x, _gy(case))]
        r0, r1 = res[0][1][ci], res[1][1][ci]
        assert rel(np.concatenate([r0[0], r1[0]]), full[0]) < 1e-5, (case, "y")
        # bf16 blocks: the full-batch path stages the BN input gradient straight into bf16
        # (fused kernel), the synchronised one from an fp32 buffer formed with the global
        # sums pre-divided by the count: rounding-level differences flip some bf16
        # roundings of the operand (2^-8 each)
        tol = 2e-3 if case[-1] else 2e-5
        assert rel(np.concatenate([r0[1], r1[1]]), full[1]) < tol, (case, "dx")
        for j, n in ((2, "dW"), (3, "dgamma"), (4, "dbeta")):
            assert rel(r0[j] + r1[j], full[j]) < tol, (case, n)      # DDP sums (then averages) them
        for j, n in ((5, "running_mean"), (6, "running_var")):
            assert rel(r0[j], full[j]) < 1e-5 and rel(r1[j], full[j]) < 1e-5, (case, n)
    # whole SeqVaeTeb: synchronised statistics over the 2 + 2 samples == the 4-sample model
    from golden_util import det_fill_
    from vaeteb.model import SeqVaeTeb
    g = np.load(os.path.join(ROOT, "tests", "golden", "model_s16_b4.npz"), allow_pickle=False)
    m = det_fill_(SeqVaeTeb(sequence_length=16)).cuda()
    T = lambda k: torch.from_numpy(g[k]).cuda()
    fw = m(T("y_st"), T("y_ph"), T("x_ph"), eps=T("eps"))
    torch.cuda.synchronize()
    sd = {k: v.cpu().numpy() for k, v in m.state_dict().items() if "running" in k}
    for k, v in sd.items():
        assert rel(res[0][2][k], v) < 1e-5 and rel(res[1][2][k], v) < 1e-5, k


def _fit_worker(rank, world, port, q):
    sys.path[:0] = [os.path.join(ROOT, "vae-teb_amd"), os.path.join(ROOT, "tests")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    q.put((rank,) + _fit(rank, world))
    dist.destroy_process_group()


def _fit(rank, world):
    """One Lightning-style fit step (ref/model/graph_model.py:496-523: DDP, clip 0.5,
    sync_batchnorm on > 1 GPU) on this rank's share of model_s16_b4's 4 samples; returns
    the flat gradient of that step (the all-reduced SUM on several ranks), the loss and
    the running statistics."""
    from golden_util import det_fill_
    from vaeteb.lightning import LightSeqVaeTeb, fit
    from vaeteb.model import SeqVaeTeb
    g = np.load(os.path.join(ROOT, "tests", "golden", "model_s16_b4.npz"), allow_pickle=False)
    n = 4 // world
    sl = slice(rank * n, (rank + 1) * n)
    batch = {"fhr_st": g["y_st"][sl], "fhr_ph": g["y_ph"][sl], "fhr_up_ph": g["x_ph"][sl], "fhr": g["y_raw"][sl]}
    batch = {k: torch.from_numpy(v.copy()).cuda() for k, v in batch.items()}
    eps = torch.from_numpy(g["eps"][sl].copy()).cuda()
    # fp32 blocks (the bf16 synchronised block is checked above): in bf16 the split batch's
    # rounding-level differences flip bf16 roundings that this model amplifies (one bf16
    # step's gradients sit ~50 % from fp32's, tests/test_gpu_parity_s256.py)
    m = det_fill_(SeqVaeTeb(sequence_length=16, concurrent_encoders=True)).cuda()
    if rank > 0:
        # every other rank starts from a different model: fit() must start all ranks from
        # rank 0's parameters and buffers (DDP's construction-time broadcast)
        with torch.no_grad():
            gen = torch.Generator(device="cuda").manual_seed(rank)
            for p_ in m.parameters():
                p_.add_(0.1 * torch.randn(p_.shape, device="cuda", generator=gen))
            for b_ in m.buffers():
                if b_.is_floating_point():
                    b_.add_(1.0)
    fwd = m.forward
    m.forward = lambda *a, **k: fwd(*a, eps=eps)        # the stored reparameterisation noise
    mod = LightSeqVaeTeb(m, lr=1e-3, beta_schedule="constant", beta_const_val=1e-5)
    logged = fit(mod, [batch], max_epochs=1, gradient_clip_val=0.5, sync_batchnorm=world > 1)
    torch.cuda.synchronize()
    flat = mod._optimizer.flat
    stats = {k: v.cpu().numpy() for k, v in m.state_dict().items() if "running" in k}
    return flat.g.cpu().numpy() / world, float(logged["train/total_loss"]), stats, flat.p.cpu().numpy()


def test_lightning_fit_ddp_sync_batchnorm_two_ranks():
    """fit() on 2 ranks (2 samples each, sync_batchnorm=True, bucketed gradient
    all-reduce) == fit() on 1 process with all 4 samples: the loss (1e-5), the averaged
    gradient (rel-L2 over the flat buffer 1e-4: different reduction orders through 17
    BatchNorms and the LSTMs), the BatchNorm running statistics (1e-5) and identical
    parameters on both ranks."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_fit_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=200) for _ in range(world)], key=lambda o: o[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    g1, loss1, stats1, p1 = _fit(0, 1)
    rel = lambda a, b: float(np.linalg.norm(np.asarray(a, np.float64) - b) / max(np.linalg.norm(b), 1e-30))
    assert np.array_equal(res[0][1], res[1][1])                # the all-reduced gradient on both ranks
    assert np.array_equal(res[0][4], res[1][4])                # identical parameters after the step
    assert abs(0.5 * (res[0][2] + res[1][2]) - loss1) <= 1e-5 * abs(loss1), (res[0][2], res[1][2], loss1)
    for k, v in stats1.items():
        assert rel(res[0][3][k], v) < 1e-5 and rel(res[1][3][k], v) < 1e-5, k
    if rel(res[0][1], g1) >= 1e-4:      # name the parameters before failing
        from vaeteb.train import FlatState  # noqa: F401  (layout: reverse registration order)
        from golden_util import det_fill_
        from vaeteb.model import SeqVaeTeb
        names = [k for k, _ in det_fill_(SeqVaeTeb(sequence_length=16)).named_parameters()][::-1]
        shapes = [tuple(p.shape) for _, p in det_fill_(SeqVaeTeb(sequence_length=16)).named_parameters()][::-1]
        o, rep = 0, []
        for n, sh in zip(names, shapes):
            c = int(np.prod(sh))
            rep.append((rel(res[0][1][o:o + c], g1[o:o + c]), n))
            o += c
        print(sorted(rep)[-12:])
    assert rel(res[0][1], g1) < 1e-4, rel(res[0][1], g1)
