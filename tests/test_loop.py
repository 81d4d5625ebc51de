"""The epoch driver (vaeteb.loop.train_base_model_pytorch, mirroring
ref/model/graph_model.py:612-908) on CPU with gloo, world size 2: the C3 loss-sum
all-reduce, the per-epoch CosineAnnealingLR, rank-0 best checkpoint and the C4
early-stop broadcast.  The training step is a stand-in with the Trainer's interface
(plain torch, AdamW as the reference configures it); the GPU test
(tests/test_gpu_loop.py) runs the driver over the HIP Trainer."""
import os
import socket
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = ("total_loss", "reconstruction_loss", "kld_loss", "mse_loss", "nll_loss")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class StubTrainer:
    """Trainer interface (model, lr, step, eval_losses) over a tiny torch model."""

    def __init__(self, lr):
        torch.manual_seed(0)
        self.model = torch.nn.Sequential(torch.nn.Linear(4, 8), torch.nn.ReLU(), torch.nn.Linear(8, 2))
        self.lr = lr
        self.opt = torch.optim.AdamW(self.model.parameters(), lr=lr, weight_decay=1e-4, eps=1e-8, betas=(0.9, 0.98))
        self.lrs = []
        self.evals = []

    def _losses(self, b):
        out = self.model(b["x"])
        mse = (out[:, 0] - b["y"]).pow(2).mean()
        nll = out[:, 1].pow(2).mean()
        kld = out.abs().mean()
        return {"mse_loss": mse, "nll_loss": nll, "kld_loss": kld, "reconstruction_loss": mse + nll,
                "total_loss": mse + nll + 1e-5 * kld}

    def step(self, b):
        self.lrs.append(self.lr)
        for g in self.opt.param_groups:
            g["lr"] = self.lr
        self.opt.zero_grad()
        L = self._losses(b)
        L["total_loss"].backward()
        for p in self.model.parameters():       # DDP gradient average
            dist.all_reduce(p.grad)
            p.grad /= dist.get_world_size()
        torch.nn.utils.clip_grad_norm_(self.model.parameters(), 1.0)
        self.opt.step()
        return {k: v.detach() for k, v in L.items()}

    def eval_losses(self, b):
        with torch.no_grad():
            L = self._losses(b)
        self.evals.append(float(L["total_loss"]))
        return L


def _loader(rank, n, seed, shift=0.0):
    g = torch.Generator().manual_seed(seed + 17 * rank)
    return [{"x": torch.randn(6, 4, generator=g), "y": torch.randn(6, generator=g) + shift} for _ in range(n)]


def _worker(rank, world, port, tmp, patience, q):
    sys.path.insert(0, os.path.join(ROOT, "vae-teb_amd"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from vaeteb.loop import train_base_model_pytorch
    tr = StubTrainer(lr=0.01)
    # validation drifts away from training so the validation loss rises and early stop fires
    hist = train_base_model_pytorch(tr, _loader(rank, 3, 1), _loader(rank, 2, 2, shift=5.0), epochs=8,
                                    checkpoint_dir=os.path.join(tmp, f"ck{rank}"), early_stop_patience=patience)
    # the epoch-summed losses each rank saw (identical after C3), for the cross-rank check
    q.put((rank, hist, tr.lrs, [p.detach().numpy().copy() for p in tr.model.parameters()],
           os.path.exists(os.path.join(tmp, f"ck{rank}", "base-model-best-pytorch.pt")), tr.evals))
    dist.destroy_process_group()


@pytest.mark.parametrize("patience", [2, 100])
def test_epoch_driver_two_ranks(tmp_path, patience):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, str(tmp_path), patience, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = sorted([q.get(timeout=120) for _ in range(world)], key=lambda o: o[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (_, hist, lrs0, params0, ck0, ev0), (_, hist1, lrs1, params1, ck1, ev1) = out
    assert hist1 is None and hist is not None            # history on rank 0 only
    assert ck0 and not ck1                                # best checkpoint written by rank 0 only
    # identical lr sequence and stop decision on both ranks (same number of steps)
    assert lrs0 == lrs1
    for a, b in zip(params0, params1):
        assert (a == b).all()
    n_epochs = len(hist["epoch"])
    assert len(lrs0) == 3 * n_epochs
    if patience == 2:
        assert n_epochs < 8
        # stopped exactly when the validation loss had not improved for `patience` epochs
        v = hist["val/total_loss"]
        best = min(range(len(v)), key=lambda i: v[i])
        assert n_epochs - 1 - best == patience
    else:
        assert n_epochs == 8
    # CosineAnnealingLR(T_max=epochs, eta_min=0.01 lr), stepped once per epoch
    p = torch.zeros(1, requires_grad=True)
    opt = torch.optim.SGD([p], lr=0.01)
    sch = torch.optim.lr_scheduler.CosineAnnealingLR(opt, T_max=8, eta_min=1e-4)
    exp = []
    for _ in range(n_epochs):
        exp.append(opt.param_groups[0]["lr"])
        sch.step()
    assert hist["lr"] == exp
    assert [lrs0[3 * e] for e in range(n_epochs)] == exp
    # C3: rank 0's epoch averages are the mean over both ranks' batches
    for k in KEYS:
        assert len(hist[f"train/{k}"]) == n_epochs and len(hist[f"val/{k}"]) == n_epochs
    for e in range(n_epochs):
        exp_v = (sum(ev0[2 * e:2 * e + 2]) + sum(ev1[2 * e:2 * e + 2])) / 4
        assert abs(hist["val/total_loss"][e] - exp_v) <= 1e-6 * abs(exp_v), e
