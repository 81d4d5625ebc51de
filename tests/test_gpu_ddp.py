"""Bucketed gradient all-reduce with the side-stream weight gradients
(concurrent encoders, bf16-MFMA decoder heads whose weight gradients run on a
side stream): two ranks on one MI355X, gloo over CUDA tensors (RCCL refuses two
ranks on one device; the stream ordering under test — the collective's stream
waiting on every stream that wrote the bucket — is the same).  Each rank's
reduced gradient must equal the sum of both ranks' locally computed gradients
bit for bit, and the parameters must stay identical across ranks.
(Advisor round 1: the side streams were snapshotted before the first forward
created them, so the first step's head-weight buckets raced the reduce.)"""
import os
import socket
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _batch(rank):
    import numpy as np
    g = np.load(os.path.join(ROOT, "tests", "golden", "model_s16_b4.npz"), allow_pickle=False)
    b = {"fhr_st": g["y_st"], "fhr_ph": g["y_ph"], "fhr_up_ph": g["x_ph"], "fhr": g["y_raw"]}
    b = {k: torch.from_numpy(v.copy()).cuda() for k, v in b.items()}
    if rank:
        b = {k: v.flip(0).contiguous() for k, v in b.items()}
    return b, torch.from_numpy(g["eps"].copy()).cuda()


def _model():
    from golden_util import det_fill_
    from vaeteb.model import SeqVaeTeb
    return det_fill_(SeqVaeTeb(sequence_length=16, concurrent_encoders=True, head_precision="bf16",
                               conv_precision="bf16")).cuda()


def _worker(rank, world, port, q):
    sys.path[:0] = [os.path.join(ROOT, "vae-teb_amd"), os.path.join(ROOT, "tests")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from vaeteb.train import Trainer
    batch, eps = _batch(rank)
    # this rank's own gradient (no collective)
    loc = Trainer(_model(), lr=1e-3)
    loc._forward_backward(batch, eps, overlap_comm=False)
    torch.cuda.synchronize()
    g_local = loc.state.g.cpu()
    del loc
    # a fresh process-group-wide step; small buckets so several fire from the hooks
    tr = Trainer(_model(), lr=1e-3, world_size=world, bucket_mb=0.5)
    tr._forward_backward(batch, eps, overlap_comm=True)
    fired = len(tr.buckets.works)
    tr.buckets.finish()
    torch.cuda.synchronize()
    g_red = tr.state.g.cpu()
    tr._update()
    tr.step(batch, eps=eps)
    torch.cuda.synchronize()
    # numpy, not tensors: shared-memory tensor handles can outlive a worker that exits first
    q.put((rank, g_local.numpy(), g_red.numpy(), tr.state.p.cpu().numpy(), fired, len(tr.buckets.buckets)))
    dist.destroy_process_group()


def test_bucketed_allreduce_waits_for_side_stream_gradients():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = sorted([q.get(timeout=150) for _ in range(world)], key=lambda o: o[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    out = [(o[0], torch.from_numpy(o[1]), torch.from_numpy(o[2]), torch.from_numpy(o[3]), o[4], o[5]) for o in out]
    expect = out[0][1] + out[1][1]
    assert not torch.equal(out[0][1], out[1][1])          # the ranks' local gradients differ
    for rank in range(world):
        assert torch.equal(out[rank][2], expect), rank
    assert out[0][4] > 1 and out[0][5] > 1                # buckets launched from the backward hooks
    assert torch.equal(out[0][3], out[1][3])


def _seg_worker(rank, world, port, q):
    """Eager DDP steps vs the captured step replayed by the native executor in ranges,
    each bucket's all-reduce issued after the range that ends with its marker."""
    sys.path[:0] = [os.path.join(ROOT, "vae-teb_amd"), os.path.join(ROOT, "tests")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from vaeteb.train import Trainer
    b0, e0 = _batch(rank)
    b1 = {k: v.roll(1, 0).contiguous() for k, v in b0.items()}
    e1 = e0.roll(1, 0).contiguous()
    seq = ((b1, e1), (b0, e0), (b1, e1))
    res, n_mark, n_buckets = [], 0, 0
    for native in (False, True):
        tr = Trainer(_model(), lr=1e-3, world_size=world, bucket_mb=0.5)
        if native:
            cap = tr.capture(b0, eps=e0, warmup=2, native=True)
            n_mark, n_buckets = len(cap.markers), len(tr.buckets.buckets)
            outs = [cap.replay(b, eps=e)["total_loss"].item() for b, e in seq]
        else:
            for _ in range(2):
                tr.step(b0, eps=e0)
            outs = [tr.step(b, eps=e)["total_loss"].item() for b, e in seq]
        torch.cuda.synchronize()
        # numpy, not tensors: shared-memory tensor handles can outlive a worker that exits first
        res.append((outs, tr.state.p.cpu().numpy(), tr.state.m.cpu().numpy(), tr.state.v.cpu().numpy()))
        del tr
    q.put((rank, res, n_mark, n_buckets))
    dist.destroy_process_group()


def test_segmented_native_replay_equals_eager_ddp_step():
    """the data-parallel step on the native executor.  The step is
    captured with a marker where each gradient bucket completes (GradBuckets under
    Trainer.capture), the executor enqueues the replay in ranges split at the markers,
    and each bucket's all-reduce is issued on the comm stream right after its range —
    overlapping the rest of the backward instead of following the whole replay.  Two
    ranks on one GPU (gloo over CUDA tensors): losses, parameters and Adam moments after
    2 + 3 steps equal the eager DDP step's (all-reduces from the backward hooks) bit for
    bit, and the parameters are identical across ranks."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_seg_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = sorted([q.get(timeout=200) for _ in range(world)], key=lambda o: o[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, res, n_mark, n_buckets in out:
        (o_e, p_e, m_e, v_e), (o_n, p_n, m_n, v_n) = res
        assert n_buckets > 4 and n_mark >= n_buckets - 1, (n_mark, n_buckets)   # all but possibly the last
        assert o_e == o_n, (rank, o_e, o_n)
        assert (p_e == p_n).all() and (m_e == m_n).all() and (v_e == v_n).all(), rank
    assert (out[0][1][1][1] == out[1][1][1][1]).all()        # the same model on both ranks


def test_bench_self_launch_two_ranks():
    """`python bench.py --gpus 2` starts its own two ranks (no torchrun),
    here with VAETEB_DIST_BACKEND=gloo so both share this box's one GPU.  Exactly one JSON line
    reaches stdout (rank 0's), it reports the whole job (2 GPUs, global batch 512), the mode
    names the gradient buckets all-reduced from the segmented native replay, and the ELBO of the
    last step is finite; every rank ran the barrier / max-over-ranks timing (else rank 0 hangs)."""
    import json
    import math
    import subprocess
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    env = dict(os.environ, VAETEB_DIST_BACKEND="gloo")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup",
                        "1", "--no-cpu-baseline"], env=env, cwd=ROOT, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["config"]["global_batch"] == 512 and out["config"]["parallelism"] == "dp2"
    assert "gradient buckets" in out["mode"] and out.get("dist_backend") == "gloo", out["mode"]
    assert out["value"] > 0 and all(math.isfinite(v) for v in out["elbo"].values()), out["elbo"]
    assert "cpu_baseline" not in out
