"""Lightning-compatible training module and checkpoint interchange, without
Lightning (not installed here, and not needed on the MI355X path).

  LightSeqVaeTeb            ref/model/pytorch_lightning_modules.py:401-564
      same constructor (hparams), forward, KLD-beta schedules, _common_step /
      training_step / validation_step (same logged names), configure_optimizers
      (AdamW lr, wd 1e-4, eps 1e-8, betas (0.9, 0.999); CosineAnnealingWarmRestarts
      with T_0 = max(lr_milestones) // 4, eta_min = lr / 100, stepped per batch)
  load_from_checkpoint      Lightning .ckpt files: state_dict under "model."
                            (the module attribute), hyper_parameters restored
  load_pytorch_checkpoint   ref/model/graph_model.py:381-390 ("seqvae_model."
                            prefix stripped)
  fit                       the epoch loop of Trainer.fit as configured in
                            ref/model/graph_model.py:404-610 (gradient_clip_val
                            0.5, per-step scheduler)

The optimizer is `FlatAdamW`: parameters, gradients and moments live in flat
fp32 buffers (vaeteb.train.FlatState), the HIP ops write gradients in place,
and clip + AdamW are two launches (vt_grad_norm_clip, vt_adamw_step_dev) with
no host synchronisation.  `param_groups[0]["lr"]` is read at every step, so any
schedule that edits it applies.
"""
import math

import torch
import torch.nn as nn

from . import _lib
from .train import FlatState


class AttributeDict(dict):
    """Lightning's AttributeDict (hparams): keys readable as attributes."""

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e

    def __setattr__(self, k, v):
        self[k] = v


class FlatAdamW:
    """torch.optim.AdamW (decoupled weight decay) + optional clip_grad_norm_
    over flat buffers; duck-types the torch optimizer surface used here
    (param_groups, zero_grad, step, state_dict)."""

    def __init__(self, module, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2, max_norm=None):
        self.flat = FlatState(module)
        dev = self.flat.p.device
        self.param_groups = [dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, initial_lr=lr)]
        self.max_norm = max_norm
        self.pre_scale = 1.0      # 1 / world under data parallelism: the all-reduced SUM becomes the mean
        self.norm_out = torch.zeros(2, device=dev)
        self.step_dev = torch.zeros(1, dtype=torch.int32, device=dev)
        self.coef = torch.zeros(2, device=dev)
        self.norm_ws = torch.empty(_lib.lib().fns["vt_grad_norm_workspace_floats"](), device=dev)

    def zero_grad(self, set_to_none=False):
        self.flat.zero_grad()

    def clip_grad_norm_(self, max_norm):
        """clip_grad_norm_(parameters, max_norm) on the flat gradient; the total
        norm stays on the device (returned as a 0-d tensor view)."""
        s = self.flat
        _lib.call("vt_grad_norm_clip", s.g.data_ptr(), s.numel, 1.0, float(max_norm), self.norm_out.data_ptr(),
                  self.norm_ws.data_ptr(), _lib.stream())
        _lib.call("vt_scale_by_device_scalar", s.g.data_ptr(), s.numel, self.norm_out.data_ptr() + 4, _lib.stream())
        return self.norm_out[0]

    def step(self, closure=None):
        g = self.param_groups[0]
        s = self.flat
        gscale = 0
        if self.max_norm is not None or self.pre_scale != 1.0:
            # clip_grad_norm_ on the averaged gradient (max_norm <= 0: scale only)
            _lib.call("vt_grad_norm_clip", s.g.data_ptr(), s.numel, float(self.pre_scale),
                      float(self.max_norm) if self.max_norm is not None else 0.0,
                      self.norm_out.data_ptr(), self.norm_ws.data_ptr(), _lib.stream())
            gscale = self.norm_out.data_ptr() + 4
        b1, b2 = g["betas"]
        _lib.call("vt_adamw_step_dev", s.p.data_ptr(), s.g.data_ptr(), s.m.data_ptr(), s.v.data_ptr(), s.numel,
                  float(g["lr"]), float(b1), float(b2), float(g["eps"]), float(g["weight_decay"]),
                  self.step_dev.data_ptr(), self.coef.data_ptr(), gscale, _lib.stream())
        from . import ops
        ops._FRESH.clear()   # the weights moved without their bf16 shadows: the next forward rewrites them

    def state_dict(self):
        return {"param_groups": [dict(g) for g in self.param_groups], "step": self.step_dev.clone(),
                "exp_avg": self.flat.m.clone(), "exp_avg_sq": self.flat.v.clone()}

    def load_state_dict(self, sd):
        """The flat moments as saved, or as saved before round 4 added the 64-float alignment of
        the >= 2^20-element parameters (the same parameters back to back, no padding): those are
        remapped parameter by parameter.  Any other length raises."""
        s = self.flat
        n_old = sd["exp_avg"].numel()
        if n_old == s.numel:
            remap = None
        elif n_old == sum(n for _, n in s.offsets):
            remap = s.offsets
        else:
            raise ValueError(f"FlatAdamW.load_state_dict: {n_old} moments for {s.numel} flat elements "
                             f"({sum(n for _, n in s.offsets)} parameters)")
        self.param_groups = [dict(g) for g in sd["param_groups"]]
        self.step_dev.copy_(sd["step"])
        for dst, src in ((s.m, sd["exp_avg"]), (s.v, sd["exp_avg_sq"])):
            src = src.to(dst.device)
            if remap is None:
                dst.copy_(src)
                continue
            dst.zero_()   # the padding elements hold zero moments (zero gradient, zero update)
            o_old = 0
            for o, n in remap:
                dst[o:o + n].copy_(src[o_old:o_old + n])
                o_old += n


class CosineAnnealingWarmRestarts:
    """torch.optim.lr_scheduler.CosineAnnealingWarmRestarts (integer steps):
    lr = eta_min + (base - eta_min) * (1 + cos(pi * T_cur / T_i)) / 2,
    T_i *= T_mult at each restart."""

    def __init__(self, optimizer, T_0, T_mult=1, eta_min=0.0):
        if T_0 <= 0 or not isinstance(T_0, int):
            raise ValueError(f"Expected positive integer T_0, but got {T_0}")
        if T_mult < 1 or not isinstance(T_mult, int):
            raise ValueError(f"Expected integer T_mult >= 1, but got {T_mult}")
        self.optimizer, self.T_0, self.T_i, self.T_mult, self.eta_min = optimizer, T_0, T_0, T_mult, eta_min
        self.base_lrs = [g["initial_lr"] for g in optimizer.param_groups]
        self.T_cur = 0
        self.last_epoch = 0
        self._apply()

    def _apply(self):
        for g, base in zip(self.optimizer.param_groups, self.base_lrs):
            g["lr"] = self.eta_min + (base - self.eta_min) * (1 + math.cos(math.pi * self.T_cur / self.T_i)) / 2

    def get_last_lr(self):
        return [g["lr"] for g in self.optimizer.param_groups]

    def step(self):
        self.last_epoch += 1
        self.T_cur += 1
        if self.T_cur >= self.T_i:
            self.T_cur -= self.T_i
            self.T_i *= self.T_mult
        self._apply()


def _field(batch, name):
    return getattr(batch, name) if hasattr(batch, name) else batch[name]


class LightSeqVaeTeb(nn.Module):
    """ref/model/pytorch_lightning_modules.py:401-564 without Lightning."""

    def __init__(self, seqvae_teb_model, lr=1e-4, lr_milestones=None, beta_schedule="linear", beta_start=0.0,
                 beta_end=1.0, beta_anneal_epochs=100, beta_cycle_len=1000, beta_const_val=1.0):
        super().__init__()
        self.hparams = AttributeDict(lr=lr, lr_milestones=lr_milestones, beta_schedule=beta_schedule,
                                     beta_start=beta_start, beta_end=beta_end, beta_anneal_epochs=beta_anneal_epochs,
                                     beta_cycle_len=beta_cycle_len, beta_const_val=beta_const_val)
        self.model = seqvae_teb_model
        self.current_epoch = 0
        self.global_step = 0
        self.logged = {}
        self._optimizer = None

    def forward(self, y_st, y_ph, x_ph):
        return self.model(y_st, y_ph, x_ph)

    def log(self, name, value, **kwargs):
        """Keeps the last value per name (device tensors stay on the device)."""
        self.logged[name] = value

    def _calculate_beta(self):
        hp, epoch = self.hparams, self.current_epoch
        if hp.beta_schedule == "linear":
            progress = min(1.0, epoch / hp.beta_anneal_epochs)
            return hp.beta_start + (hp.beta_end - hp.beta_start) * progress
        if hp.beta_schedule == "cyclic":
            progress = (epoch % hp.beta_cycle_len) / hp.beta_cycle_len
            return hp.beta_start + (hp.beta_end - hp.beta_start) * progress
        if hp.beta_schedule == "constant":
            return hp.beta_const_val
        raise ValueError(f"Unknown beta schedule: {hp.beta_schedule}")

    def on_train_epoch_start(self):
        self.hparams.beta = self._calculate_beta()
        self.log("kld_beta", self.hparams.beta)
        if self._optimizer is not None:
            self.log("lr", self._optimizer.param_groups[0]["lr"])

    def _common_step(self, batch, batch_idx=0):
        y_st, y_ph, x_ph, y_raw = (_field(batch, k) for k in ("fhr_st", "fhr_ph", "fhr_up_ph", "fhr"))
        fw = self.model(y_st, y_ph, x_ph)
        beta = self.hparams.get("beta", self._calculate_beta())
        return self.model.compute_loss(fw, y_st, y_ph, y_raw, compute_kld_loss=True, beta=beta)

    def _log_losses(self, prefix, d):
        self.log(f"{prefix}/total_loss", d["total_loss"])
        self.log(f"{prefix}/recon_loss", d["reconstruction_loss"])
        for k in ("mse_loss", "nll_loss", "kld_loss"):
            self.log(f"{prefix}/{k}", d[k])

    def training_step(self, batch, batch_idx=0):
        d = self._common_step(batch, batch_idx)
        self._log_losses("train", d)
        return d["total_loss"]

    def validation_step(self, batch, batch_idx=0):
        d = self._common_step(batch, batch_idx)
        self._log_losses("val", d)
        return d["total_loss"]

    def configure_optimizers(self):
        hp = self.hparams
        opt = FlatAdamW(self, lr=hp.lr, weight_decay=1e-4, eps=1e-8, betas=(0.9, 0.999))
        self._optimizer = opt
        if hp.lr_milestones:
            sched = CosineAnnealingWarmRestarts(opt, T_0=max(hp.lr_milestones) // 4, T_mult=1, eta_min=hp.lr * 0.01)
            return {"optimizer": opt, "lr_scheduler": {"scheduler": sched, "interval": "step", "frequency": 1}}
        return opt

    # ------------------------------------------------------ checkpoints
    def lightning_state_dict(self):
        return {"model." + k: v for k, v in self.model.state_dict().items()}

    def save_checkpoint(self, path, epoch=None):
        """A Lightning-format checkpoint (state_dict under "model.", epoch,
        global_step, hyper_parameters) that the reference's
        LightSeqVaeTeb.load_from_checkpoint reads."""
        torch.save({"state_dict": {k: v.detach().cpu() for k, v in self.lightning_state_dict().items()},
                    "epoch": self.current_epoch if epoch is None else epoch, "global_step": self.global_step,
                    "hyper_parameters": dict(self.hparams)}, path)

    @classmethod
    def load_from_checkpoint(cls, checkpoint_path, seqvae_teb_model=None, strict=True, map_location="cpu", **hp):
        """LightningModule.load_from_checkpoint as used at ref/model/graph_model.py:338-342:
        the model instance is passed in (its weights are overwritten)."""
        ck = torch.load(checkpoint_path, map_location=map_location, weights_only=True)
        hparams = dict(ck.get("hyper_parameters", {}))
        hparams.pop("beta", None)
        hparams.update(hp)
        if seqvae_teb_model is None:
            raise TypeError("load_from_checkpoint needs seqvae_teb_model= (it is not saved in hyper_parameters)")
        obj = cls(seqvae_teb_model, **hparams)
        sd = {k[len("model."):]: v for k, v in ck["state_dict"].items() if k.startswith("model.")}
        obj.model.load_state_dict(sd, strict=strict)
        obj.current_epoch = int(ck.get("epoch", 0))
        obj.global_step = int(ck.get("global_step", 0))
        return obj


def load_pytorch_checkpoint(model, path, map_location="cpu"):
    """ref/model/graph_model.py:381-390: checkpoint['state_dict'] with the
    'seqvae_model.' prefix stripped, loaded strictly; returns the epoch."""
    ck = torch.load(path, map_location=map_location, weights_only=True)
    sd = {k.replace("seqvae_model.", ""): v for k, v in ck["state_dict"].items()}
    model.load_state_dict(sd)
    return ck.get("epoch")


def _join_side_streams():
    """The HIP ops write some gradients in place on side streams (no AccumulateGrad, so
    autograd does not join them): the optimizer's stream waits for them."""
    if torch.cuda.is_available():
        from . import ops
        for st in ops.SIDE_STREAMS:
            _lib.wait_for(_lib.stream(), st)


def fit(module, train_loader, max_epochs=1, gradient_clip_val=0.5, val_loader=None, to_device=None,
        sync_batchnorm=False, group=None):
    """Lightning Trainer.fit as configured at ref/model/graph_model.py:404-610
    (gradient_clip_val 0.5, step-interval scheduler).  Returns the module's
    last logged values.  No host synchronisation inside an epoch.

    Under torch.distributed with world size > 1 (one process per GPU, as Lightning's
    DDPStrategy, :470-471): the gradients are all-reduced in buckets from the backward
    (vaeteb.train.GradBuckets) and averaged (1 / world folded into the clip), and with
    sync_batchnorm=True (Lightning's flag, :517) every conv block's BatchNorm takes its
    statistics over all ranks (vaeteb.model.convert_sync_batchnorm)."""
    import torch.distributed as dist
    world = dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1
    if sync_batchnorm and world > 1:
        from .model import convert_sync_batchnorm
        convert_sync_batchnorm(module.model, group)
    conf = module.configure_optimizers()
    opt, sched = (conf["optimizer"], conf["lr_scheduler"]["scheduler"]) if isinstance(conf, dict) else (conf, None)
    opt.max_norm = gradient_clip_val
    buckets = None
    if world > 1:
        from .train import BufferBroadcast, GradBuckets, broadcast_state
        broadcast_state(opt.flat, module.model, group)   # DDP: every rank starts from rank 0's model
        buckets = GradBuckets(opt.flat, group)
        # DDPStrategy's broadcast_buffers=True: rank 0's BatchNorm statistics before every step
        # (SyncBatchNorm keeps them identical already)
        bsync = None if sync_batchnorm else BufferBroadcast(module.model, group)
        opt.pre_scale = 1.0 / world
    mv = lambda b: to_device(b) if to_device else b
    for epoch in range(module.current_epoch, max_epochs):
        module.current_epoch = epoch
        module.train()
        module.on_train_epoch_start()
        for i, batch in enumerate(train_loader):
            opt.zero_grad()
            if buckets is not None:
                buckets.reset()
                if bsync is not None:
                    bsync()
            loss = module.training_step(mv(batch), i)
            loss.backward()
            _join_side_streams()
            if buckets is not None:
                buckets.finish()
            opt.step()
            if sched is not None:
                sched.step()
            module.global_step += 1
        if val_loader is not None:
            # Lightning validates in eval mode: BatchNorm uses (and does not update)
            # its running statistics
            module.eval()
            if buckets is not None and bsync is not None:
                bsync()   # DDP broadcasts buffers before an eval forward too: rank 0's statistics
            for i, batch in enumerate(val_loader):
                with torch.no_grad():
                    module.validation_step(mv(batch), i)
            module.train()
    return module.logged
