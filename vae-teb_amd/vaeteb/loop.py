"""The epoch driver of the reference's hand-written DDP training loop,
`SeqVAEGraphModel.train_base_model_pytorch` (ref/model/graph_model.py:612-908),
around the MI355X training step (vaeteb.train.Trainer: one process per GPU, RCCL
bucketed gradient all-reduce, clip 1.0 + AdamW(wd 1e-4, eps 1e-8, betas
(0.9, 0.98)) on flat buffers).

Per epoch, in the reference's order:
  train   Trainer.step per batch (zero_grad, forward, compute_loss(beta=kld_beta),
          backward, clip, AdamW: :700-726); the five loss sums accumulate ON THE
          DEVICE in fp64 (the reference reads 5 x .item() per step, :746-755 — a host
          synchronisation per step that the MI355X path does not make)
  val     model.eval(), no_grad, the same losses (:769-815)
  C3      all_reduce(SUM) of the train and validation sums (:822-830)
  sched   CosineAnnealingLR(T_max=epochs, eta_min=0.01 lr).step() (:663-667, :833)
  rank 0  averages over len(loader) x world batches (:838-848), history, best
          validation total -> torch.save(model.state_dict(), base-model-best-pytorch.pt)
          (:872-877), patience counter (:868-880)
  C4      broadcast(stop flag, src=0) (:882-898); every rank stops together
Returns the history dict on rank 0 (the reference's loss_plotter.history, :900-906)
and None elsewhere.  Plotting / logging / the pickle dump are out of scope.

`trainer` is duck-typed: .model, .lr (read by the step), .step(batch) -> loss dict
of device scalars, .eval_losses(batch) -> loss dict (vaeteb.train.Trainer has all).
"""
import math
import os

import torch
import torch.distributed as dist

KEYS = ("total_loss", "reconstruction_loss", "kld_loss", "mse_loss", "nll_loss")   # train_loss_dict order, :692-695


class CosineAnnealingLR:
    """torch.optim.lr_scheduler.CosineAnnealingLR over the trainer's scalar lr: torch's
    own scheduler drives a one-parameter stand-in optimizer, so the lr sequence (its
    recursive closed form) is torch's bit for bit."""

    def __init__(self, trainer, T_max, eta_min=0.0):
        self.trainer = trainer
        self._p = torch.zeros(1, requires_grad=True)
        self._opt = torch.optim.SGD([self._p], lr=float(trainer.lr))
        self._sched = torch.optim.lr_scheduler.CosineAnnealingLR(self._opt, T_max=T_max, eta_min=eta_min)

    def step(self):
        self._opt.step()   # no gradient: a no-op that keeps torch's step-order check quiet
        self._sched.step()
        self.trainer.lr = self._opt.param_groups[0]["lr"]

    def get_last_lr(self):
        return self._sched.get_last_lr()


def _dist():
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def train_base_model_pytorch(trainer, train_loader, validation_loader, epochs, checkpoint_dir=None,
                             early_stop_patience=100, group=None, to_device=None):
    """ref/model/graph_model.py:612-908 (see the module docstring)."""
    rank, world = _dist()
    model = trainer.model
    dev = next(model.parameters()).device
    scheduler = CosineAnnealingLR(trainer, T_max=epochs, eta_min=trainer.lr * 0.01)
    history = {"epoch": [], "lr": []}
    for k in KEYS:
        history[f"train/{k}"] = []
        history[f"val/{k}"] = []
    best_val = float("inf")
    patience = 0
    mv = to_device or (lambda b: b)
    for epoch in range(epochs):
        model.train()
        tr_sum = torch.zeros(len(KEYS), dtype=torch.float64, device=dev)
        for batch in train_loader:
            L = trainer.step(mv(batch))
            tr_sum += torch.stack([L[k].detach().to(torch.float64).reshape(()) for k in KEYS])
        model.eval()
        if getattr(trainer, "buffer_sync", None) is not None:
            trainer.buffer_sync()   # DDP broadcast_buffers applies to the eval forward too (rank 0's stats)
        va_sum = torch.zeros(len(KEYS), dtype=torch.float64, device=dev)
        with torch.no_grad():
            for batch in validation_loader:
                L = trainer.eval_losses(mv(batch))
                va_sum += torch.stack([L[k].detach().to(torch.float64).reshape(()) for k in KEYS])
        if world > 1:                                                     # C3
            dist.all_reduce(tr_sum, op=dist.ReduceOp.SUM, group=group)
            dist.all_reduce(va_sum, op=dist.ReduceOp.SUM, group=group)
        lr_epoch = float(trainer.lr)
        scheduler.step()
        stop = torch.zeros((), dtype=torch.int64, device=dev)
        if rank == 0:
            n_tr = max(len(train_loader) * world, 1)
            n_va = max(len(validation_loader) * world, 1)
            tr = (tr_sum / n_tr).tolist()
            va = (va_sum / n_va).tolist()
            history["epoch"].append(epoch)
            history["lr"].append(lr_epoch)
            for k, a, b in zip(KEYS, tr, va):
                history[f"train/{k}"].append(a)
                history[f"val/{k}"].append(b)
            if va[0] < best_val:
                best_val = va[0]
                patience = 0
                if checkpoint_dir is not None:
                    os.makedirs(checkpoint_dir, exist_ok=True)
                    torch.save({k: v.detach().cpu() for k, v in model.state_dict().items()},
                               os.path.join(checkpoint_dir, "base-model-best-pytorch.pt"))
            else:
                patience += 1
            if patience >= early_stop_patience:
                stop.fill_(1)
        if world > 1:                                                     # C4
            dist.broadcast(stop, src=0, group=group)
        if int(stop.item()) == 1:
            break
    return history if rank == 0 else None


def best_val_loss(history):
    return min(history["val/total_loss"]) if history and history["val/total_loss"] else math.inf
