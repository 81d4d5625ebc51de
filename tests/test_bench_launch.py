"""`python bench.py --gpus N` launches its own ranks (vaeteb.train.spawn_local_ranks, the
reference's `mp.spawn(main_pytorch, nprocs=world_size)`, ref/model/graph_model.py:2152-2157):
CPU checks of the launcher with a stub worker — the rank environment, rank 0's stdout as the
only relayed output, failure propagation — and of bench.py's dispatch into it.  The real
two-rank bench run is tests/test_gpu_ddp.py::test_bench_self_launch_two_ranks."""
import io
import json
import os
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

STUB = r"""
import json, os, sys, time
r, n = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
mode = sys.argv[1]
with open(os.path.join(sys.argv[2], f"env{r}.json"), "w") as f:
    json.dump({k: os.environ[k] for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR",
                                          "MASTER_PORT")}, f)
if mode == "fail" and r == 1:
    sys.exit(3)
if mode == "fail":
    time.sleep(60)          # a rank waiting in a collective for the failed one
if r == 0:
    print(json.dumps({"metric": "stub", "n_gpus": n}))
else:
    print("noise from another rank")   # must not reach the launcher's stdout
"""


def _stub(tmp_path):
    p = tmp_path / "stub.py"
    p.write_text(STUB)
    return str(p)


def test_spawn_local_ranks_env_and_single_line(tmp_path):
    from vaeteb.train import spawn_local_ranks
    out = io.StringIO()
    rc = spawn_local_ranks([sys.executable, _stub(tmp_path), "ok", str(tmp_path)], 3, stdout=out)
    assert rc == 0
    lines = out.getvalue().splitlines()
    assert len(lines) == 1 and json.loads(lines[0]) == {"metric": "stub", "n_gpus": 3}
    envs = [json.load(open(tmp_path / f"env{r}.json")) for r in range(3)]
    for r, e in enumerate(envs):
        assert (e["RANK"], e["LOCAL_RANK"], e["WORLD_SIZE"], e["LOCAL_WORLD_SIZE"]) == (str(r), str(r), "3", "3")
        assert e["MASTER_ADDR"] == "127.0.0.1" and e["MASTER_PORT"] == envs[0]["MASTER_PORT"]


def test_spawn_local_ranks_failure_terminates_the_others(tmp_path):
    from vaeteb.train import spawn_local_ranks
    out = io.StringIO()
    t0 = time.time()
    rc = spawn_local_ranks([sys.executable, _stub(tmp_path), "fail", str(tmp_path)], 2, stdout=out)
    assert rc == 3                        # the failing rank's code, not the terminated rank's
    assert time.time() - t0 < 30          # rank 0 (sleeping 60 s) was terminated
    assert out.getvalue() == ""


def test_bench_dispatches_to_the_launcher(monkeypatch):
    """bench.py --gpus 2 without WORLD_SIZE spawns itself twice with the same arguments and
    exits with the launcher's code; with WORLD_SIZE set (torchrun) it does not spawn."""
    sys.path.insert(0, ROOT)
    import bench
    calls = []
    monkeypatch.setattr(bench, "spawn_local_ranks", lambda cmd, n: calls.append((cmd, n)) or 7)
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    argv = ["bench.py", "--gpus", "2", "--steps", "2", "--warmup", "1", "--no-cpu-baseline"]
    monkeypatch.setattr(sys, "argv", argv)
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert e.value.code == 7
    (cmd, n), = calls
    assert n == 2 and cmd[0] == sys.executable and os.path.samefile(cmd[1], os.path.join(ROOT, "bench.py"))
    assert cmd[2:] == argv[1:]


def test_init_distributed_backend_override(monkeypatch):
    from vaeteb.train import init_distributed
    monkeypatch.setenv("VAETEB_DIST_BACKEND", "mpi")
    with pytest.raises(ValueError, match="VAETEB_DIST_BACKEND"):
        init_distributed()
    monkeypatch.setenv("VAETEB_DIST_BACKEND", "gloo")
    monkeypatch.setenv("WORLD_SIZE", "1")
    monkeypatch.setenv("LOCAL_RANK", "0")
    assert init_distributed()[:3] == (0, 1, 0)
