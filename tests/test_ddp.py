"""Multi-process data-parallel path on CPU (gloo, world_size 2): the flat
parameter/gradient views and the bucketed all-reduce hooks of vaeteb.train
(the same code that runs over RCCL on the GPUs).  The HIP optimiser kernels
are GPU-only; here the reduced gradients are checked directly."""
import os
import socket
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, bucket_mb, q, reduce_dtype=torch.float32):
    sys.path.insert(0, os.path.join(ROOT, "vae-teb_amd"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from vaeteb.train import FlatState, GradBuckets
    torch.manual_seed(0)  # identical init on every rank
    model = torch.nn.Sequential(torch.nn.Linear(16, 64), torch.nn.ReLU(), torch.nn.Linear(64, 64), torch.nn.ReLU(),
                                torch.nn.Linear(64, 3))
    st = FlatState(model)
    gb = GradBuckets(st, None, bucket_mb=bucket_mb, reduce_dtype=reduce_dtype)
    results = []
    for step in range(2):
        st.zero_grad()
        gb.reset()
        g = torch.Generator().manual_seed(100 * step + rank)  # rank-local data shard
        x = torch.randn(8, 16, generator=g)
        model(x).pow(2).mean().backward()
        fired_before_finish = len(gb.works)
        gb.finish()
        results.append((st.g.clone() / world, fired_before_finish, len(gb.buckets)))
    # every parameter / grad is a view of the flat buffers
    ok_views = all(p.data_ptr() >= st.p.data_ptr() and p.grad.data_ptr() >= st.g.data_ptr() for p in st.params)
    # numpy through the queue: a tensor would be shared by file descriptor, which fails when this
    # process exits before the parent has received it (EOFError in the resource sharer)
    q.put((rank, [r[0].numpy() for r in results], [r[1] for r in results], results[0][2], ok_views))
    dist.destroy_process_group()


def _torch_out(o):
    return (o[0], [torch.from_numpy(a) for a in o[1]], o[2], o[3], o[4])


@pytest.mark.parametrize("bucket_mb", [0.01, 64.0])
def test_bucketed_allreduce_matches_full_batch_average(bucket_mb):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, bucket_mb, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [_torch_out(q.get(timeout=120)) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    out.sort(key=lambda o: o[0])
    # reference: average of the per-rank gradients computed independently
    torch.manual_seed(0)
    ref_model = torch.nn.Sequential(torch.nn.Linear(16, 64), torch.nn.ReLU(), torch.nn.Linear(64, 64),
                                    torch.nn.ReLU(), torch.nn.Linear(64, 3))
    for step in range(2):
        grads = []
        for rank in range(world):
            ref_model.zero_grad()
            g = torch.Generator().manual_seed(100 * step + rank)
            ref_model(torch.randn(8, 16, generator=g)).pow(2).mean().backward()
            grads.append(torch.cat([p.grad.reshape(-1) for p in reversed(list(ref_model.parameters()))]))
        avg = sum(grads) / world
        for rank in range(world):
            assert torch.allclose(out[rank][1][step], avg, atol=1e-6), (rank, step)
    n_buckets = out[0][3]
    if bucket_mb < 1:
        assert n_buckets > 1
        # with several buckets, all but possibly the last were launched from the
        # backward hooks (overlapped), not at finish()
        assert all(f >= n_buckets - 1 for f in out[0][2])
    assert all(o[4] for o in out)


def test_bucketed_allreduce_bf16():
    """GradBuckets(reduce_dtype=bfloat16): each bucket rounded to bf16, reduced in bf16,
    widened back into the fp32 gradient buffer == the sum of the ranks' bf16-rounded
    gradients in bf16 arithmetic (2 ranks: one rounding of the sum), within bf16
    rounding (rel-L2 2^-8) of the fp32 average."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, 0.01, q, torch.bfloat16)) for r in range(world)]
    for p in procs:
        p.start()
    out = sorted([_torch_out(q.get(timeout=120)) for _ in range(world)], key=lambda o: o[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    torch.manual_seed(0)
    ref_model = torch.nn.Sequential(torch.nn.Linear(16, 64), torch.nn.ReLU(), torch.nn.Linear(64, 64),
                                    torch.nn.ReLU(), torch.nn.Linear(64, 3))
    for step in range(2):
        grads = []
        for rank in range(world):
            ref_model.zero_grad()
            g = torch.Generator().manual_seed(100 * step + rank)
            ref_model(torch.randn(8, 16, generator=g)).pow(2).mean().backward()
            grads.append(torch.cat([p.grad.reshape(-1) for p in reversed(list(ref_model.parameters()))]))
        exp = (grads[0].bfloat16() + grads[1].bfloat16()).float() / world
        for rank in range(world):
            assert torch.equal(out[rank][1][step], exp), (rank, step)
        avg = (grads[0] + grads[1]) / world
        # elementwise the sum can cancel; overall the bf16 reduce is within bf16 rounding
        assert ((out[0][1][step] - avg).norm() / avg.norm()).item() < 2 ** -8


def _bcast_worker(rank, world, port, q):
    sys.path.insert(0, os.path.join(ROOT, "vae-teb_amd"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from vaeteb.train import FlatState, broadcast_state
    torch.manual_seed(10 + rank)  # a DIFFERENT initialisation on every rank
    model = torch.nn.Sequential(torch.nn.Linear(16, 32), torch.nn.BatchNorm1d(32), torch.nn.Linear(32, 3))
    model.train()
    model(torch.randn(8, 16))     # rank-local BatchNorm running statistics / counter
    before = [t.detach().numpy().copy() for t in list(model.parameters()) + list(model.buffers())]
    st = FlatState(model)
    broadcast_state(st, model)
    after = [t.detach().numpy().copy() for t in list(model.parameters()) + list(model.buffers())]
    q.put((rank, before, after, st.p.numpy().copy()))
    dist.destroy_process_group()


def test_broadcast_state_starts_every_rank_from_rank0():
    """Trainer(world_size > 1) / lightning.fit: ranks initialised differently end up with
    rank 0's parameters (through the flat buffer) and buffers (BatchNorm running stats and
    counter), as DDP's construction-time sync (ref/model/graph_model.py:644)."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bcast_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = sorted([q.get(timeout=120) for _ in range(world)], key=lambda o: o[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (_, b0, a0, p0), (_, b1, a1, p1) = out
    assert any(not (x == y).all() for x, y in zip(b0, b1))       # they did start apart
    for x0, y0, y1 in zip(b0, a0, a1):
        assert (x0 == y0).all() and (y0 == y1).all()             # rank 0 unchanged, rank 1 = rank 0
    assert (p0 == p1).all()


def _bufsync_worker(rank, world, port, q):
    sys.path.insert(0, os.path.join(ROOT, "vae-teb_amd"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from vaeteb.train import BufferBroadcast
    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.BatchNorm1d(16), torch.nn.ReLU(),
                                torch.nn.Linear(16, 4), torch.nn.BatchNorm1d(4)).train()
    sd0 = {k: v.clone() for k, v in model.state_dict().items()}
    bs = BufferBroadcast(model)
    same_values = all(torch.equal(sd0[k], v) for k, v in model.state_dict().items())
    res = []
    for step in range(3):
        bs()                                   # rank 0's statistics before the forward (DDP)
        before = [b.numpy().copy() for b in model.buffers() if b.is_floating_point()]
        g = torch.Generator().manual_seed(10 * step + rank)
        model(torch.randn(32, 8, generator=g) * (rank + 1)).sum().backward()   # rank-local statistics
        res.append((before, [b.detach().numpy().copy() for b in model.buffers() if b.is_floating_point()]))
    # a replaced buffer (load_state_dict(assign=True)) is rebound on the next call
    model.load_state_dict({k: v.clone() for k, v in model.state_dict().items()}, assign=True)
    bs()
    rebound = bs.bound()
    # numpy, not tensors: shared-memory tensor handles can outlive a worker that exits first
    q.put((rank, same_values, res, rebound, [b.numpy().copy() for b in model.buffers() if b.is_floating_point()]))
    dist.destroy_process_group()


def test_buffer_broadcast_every_step():
    """DDP broadcast_buffers=True (the reference's DDP wrap, graph_model.py:644, and Lightning's
    DDPStrategy): before every step every rank holds rank 0's BatchNorm running statistics, though
    each rank's forward updated them from its own shard; one flat collective per step; state_dict
    values unchanged by the flattening; a replaced buffer is rebound."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bufsync_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = sorted([q.get(timeout=120) for _ in range(world)], key=lambda o: o[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (_, s0, r0, b0, f0), (_, s1, r1, b1, f1) = out
    assert s0 and s1 and b0 and b1
    for step in range(3):
        for a, b in zip(r0[step][0], r1[step][0]):
            assert (a == b).all()                        # synced before the forward
        assert any((a != b).any() for a, b in zip(r0[step][1], r1[step][1]))   # local updates differ
        if step:
            for a, b in zip(r0[step][0], r0[step - 1][1]):
                assert (a == b).all()                    # rank 0 keeps its own statistics
    for a, b in zip(f0, f1):
        assert (a == b).all()
