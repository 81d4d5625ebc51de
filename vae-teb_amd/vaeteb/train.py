"""Thin training-step module: the MI355X replacement for the reference's
PyTorch-Lightning / hand-written DDP loops (ref/model/graph_model.py:404-908,
ref/model/pytorch_lightning_modules.py:401-564).

One process per GPU (torchrun), RCCL (torch backend "nccl") over xGMI.
Per step (ref/model/graph_model.py:700-726 order, no host synchronisation):
  zero grads -> [front-end] -> forward -> loss -> backward
  (bucketed gradient all-reduce launched from post-accumulate hooks, overlapped
  with the rest of the backward) -> grad-norm clip -> AdamW
All parameters, gradients and Adam moments are views into four flat fp32
buffers, so zeroing, clipping and the optimiser are single launches over
contiguous memory and the all-reduce buckets are plain slices.
"""
import ctypes
import math
import os

import torch
import torch.distributed as dist

from . import _lib

# run the autograd backward on the calling thread instead of autograd's device worker thread
# (measured: ~1 ms/step less host enqueue; 0 = torch default)
BWD_SAME_THREAD = int(os.environ.get("VAETEB_BWD_SAME_THREAD", "1"))
# the optimizer step writes the bf16 shadows of the MFMA heads (tiled AdamW) and of the bf16
# convs (one batched launch) for the next forward, which then launches no shadow kernels
# (0 = shadows rewritten by every forward, as before; same bits either way)
SHADOW_UPDATE = int(os.environ.get("VAETEB_SHADOW_UPDATE", "1"))


BIG_ALIGN = 64          # floats: start of every parameter with >= BIG_PARAM elements in the flat buffers
BIG_PARAM = 1 << 20
# Trainer steps leave the decoder heads' gradient ranges unzeroed and let their weight-gradient
# kernel overwrite them (FlatState.first_writer; VAETEB_FIRST_WRITER=0: zero everything)
FIRST_WRITER = os.environ.get("VAETEB_FIRST_WRITER", "1") == "1"


class FlatState:
    """Flat parameter / gradient / moment storage for a module's parameters.
    Layout is reverse registration order (≈ the order gradients become ready
    in backward), so the all-reduce buckets fill front to back.  Parameters of
    >= 2^20 elements (the decoder's R x R heads) start on a 64-float boundary (a few
    zero padding elements before them: zero gradient, zero update), so the AdamW pass
    can update them as 2-D tiles and write their bf16 shadows (vt_adamw_step_dev_shadow)
    while the rest stays 16-byte aligned."""

    def __init__(self, module):
        params = [p for p in module.parameters() if p.requires_grad]
        self.params = list(reversed(params))
        dev = self.params[0].device
        self.offsets = []
        o = 0
        for p in self.params:
            n = p.numel()
            if n >= BIG_PARAM:
                o = (o + BIG_ALIGN - 1) // BIG_ALIGN * BIG_ALIGN
            self.offsets.append((o, n))
            o += n
        self.numel = o
        self.p = torch.zeros(self.numel, device=dev)
        self.g = torch.zeros(self.numel, device=dev)
        self.m = torch.zeros(self.numel, device=dev)
        self.v = torch.zeros(self.numel, device=dev)
        with torch.no_grad():
            for p, (o, n) in zip(self.params, self.offsets):
                self.p[o:o + n].copy_(p.reshape(-1))
                p.data = self.p[o:o + n].view_as(p)
                p.grad = self.g[o:o + n].view_as(p)
                p._vt_sink = True  # HIP ops accumulate this gradient in place (vaeteb.ops._ParamGrads)
        self._grad_ptrs = [self.g.data_ptr() + 4 * o for o, _ in self.offsets]
        # first-writer gradients: the weight (>= BIG_PARAM elements, 2-D) and bias of each
        # linear module whose backward writes them with one kernel call (the decoder heads):
        # zero_grad(first_writer=True) leaves their ranges alone and that call overwrites
        # instead of accumulating (ops.FIRST_WRITER), saving the fill and the kernel's read of
        # the old gradient (2 x 268 MB per step at R = 4096)
        ids = {id(p): i for i, p in enumerate(self.params)}
        self.first_writer = []
        for m in module.modules():
            w, b = getattr(m, "weight", None), getattr(m, "bias", None)
            if isinstance(w, torch.nn.Parameter) and id(w) in ids and w.dim() == 2 and w.numel() >= BIG_PARAM and \
                    (b is None or id(b) in ids):
                self.first_writer.append([w] + ([b] if b is not None else []))
        skip = sorted(ids[id(q)] for grp in self.first_writer for q in grp)
        self._zero_ranges = []   # the complement of the first-writer ranges
        o0 = 0
        for i in skip:
            o, n = self.offsets[i]
            if o > o0:
                self._zero_ranges.append((o0, o))
            o0 = max(o0, o + n)
        if o0 < self.numel:
            self._zero_ranges.append((o0, self.numel))
        self._fw_ok, self._fw_bad = set(), set()   # groups confirmed / seen written by another op
        # a gradient of a first-writer weight that reaches it through autograd (AccumulateGrad:
        # LinearF without its in-place path, or another op using the weight) while the group's
        # range is still unzeroed: the group is zeroed right before that accumulation
        for grp in self.first_writer:
            for q in grp:
                q.register_hook(lambda grad, key=id(grp[0]): FlatState._fw_before_accumulate(key, grad))

    @staticmethod
    def _fw_before_accumulate(key, grad):
        from . import ops
        ent = ops.FIRST_WRITER.get(key)
        if ent is not None and ent[1]:
            with torch.no_grad():
                for q in ent[0]:
                    q.grad.zero_()
            ent[1] = False   # now zeroed: later writers of this step accumulate, nothing is dropped
        return grad

    def zero_grad(self, first_writer=False):
        """first_writer (Trainer steps: one forward / backward per zero_grad): a first-writer
        group is left unzeroed once a step has shown that its weight gradient comes from one
        first-writer-aware kernel call (vaeteb.ops.LinearF); until then it is zeroed like the
        rest (and any group the step does not write is zeroed after the backward,
        finish_first_writer).  A gradient that reaches an unzeroed group through autograd
        instead zeroes the group first (_fw_before_accumulate) and demotes it, so an op that
        accumulates into it never sees stale values and no gradient is dropped."""
        if first_writer and self.first_writer:
            from . import ops
            ranges = self._zero_ranges if len(self._fw_ok) == len(self.first_writer) else None
            if ranges is None:
                self.g.zero_()
            elif self.g.is_cuda and ranges:
                for i in range(0, len(ranges), 16):   # one launch per 16 ranges (was one Fill each)
                    chunk = ranges[i:i + 16]
                    st = (ctypes.c_int64 * len(chunk))(*[a for a, _ in chunk])
                    en = (ctypes.c_int64 * len(chunk))(*[b for _, b in chunk])
                    _lib.call("vt_zero_ranges", _lib.ptr(self.g), len(chunk), st, en, _lib.stream())
            else:
                for a, b in ranges:
                    self.g[a:b].zero_()
            ops.FIRST_WRITER.clear()
            ops.FIRST_WRITER_HIT.clear()
            for gi, grp in enumerate(self.first_writer):
                # [group, overwrite?]: overwrite only when the whole buffer was not zeroed
                ops.FIRST_WRITER[id(grp[0])] = [grp, ranges is not None, gi]
        else:
            self.g.zero_()
            if self.first_writer:
                from . import ops
                ops.FIRST_WRITER.clear()
                ops.FIRST_WRITER_HIT.clear()
        for p, (o, n), gp in zip(self.params, self.offsets, self._grad_ptrs):
            g = p.grad
            if g is None or g.data_ptr() != gp:
                p.grad = self.g[o:o + n].view_as(p)

    def finish_first_writer(self):
        """After the backward: a group its first-writer kernel handled is confirmed; a group no
        such kernel wrote is zeroed if it was left unzeroed, and never confirmed."""
        if not self.first_writer:
            return
        from . import ops
        for gi in ops.FIRST_WRITER_HIT:
            self._fw_ok.add(gi)
        for grp, overwrite, gi in ops.FIRST_WRITER.values():
            self._fw_bad.add(gi)
            self._fw_ok.discard(gi)
            if overwrite:
                for q in grp:
                    q.grad.zero_()
        self._fw_ok -= self._fw_bad
        ops.FIRST_WRITER.clear()
        ops.FIRST_WRITER_HIT.clear()


def broadcast_state(state, module, group=None, src=0):
    """DistributedDataParallel's construction-time module-state sync (the reference wraps
    the model in DDP: ref/model/graph_model.py:644, Lightning DDPStrategy :470-471): rank
    `src`'s parameters (the flat buffer: one collective) and buffers (BatchNorm running
    statistics and step counters) are copied to every rank, so all ranks start from the
    same model whatever their local initialisation was."""
    dist.broadcast(state.p, src=src, group=group)
    for b in module.buffers():
        dist.broadcast(b, src=src, group=group)


class BufferBroadcast:
    """DistributedDataParallel's `broadcast_buffers=True` — the default of the reference's DDP
    wrap (ref/model/graph_model.py:644) and of Lightning's DDPStrategy (:470-471): before every
    training forward, rank `src`'s floating buffers (BatchNorm running mean / variance) overwrite
    every other rank's, so ranks never drift apart.  DDP broadcasts before an eval forward as well:
    the epoch driver (loop.train_base_model_pytorch) and lightning.fit call it before their
    validation passes, so eval-mode validation sees rank 0's statistics on every rank; after the
    last training step each rank holds its own step's update until the next call (a checkpoint is
    written by rank 0, whose statistics these are).  One collective per call: the buffers are rebound as views
    of one flat tensor (state_dict keys and values unchanged; rebound again if a buffer is
    replaced, e.g. by .to() or load_state_dict(assign=True)).  The step counters
    (num_batches_tracked) advance identically on every rank and are not sent."""

    def __init__(self, module, group=None, src=0):
        self.module, self.group, self.src = module, group, src
        self.flat, self.views = None, []
        self._bind()

    def _bind(self):
        ents = [(m, n, b) for m in self.module.modules() for n, b in m._buffers.items()
                if b is not None and b.is_floating_point()]
        self.views = []
        if not ents:
            self.flat = None
            return
        with torch.no_grad():
            self.flat = torch.cat([b.detach().reshape(-1).float() for _, _, b in ents])
            o = 0
            for m, n, b in ents:
                v = self.flat[o:o + b.numel()].view(b.shape)
                o += b.numel()
                if b.dtype != torch.float32:
                    raise ValueError(f"BufferBroadcast: buffer {n} is {b.dtype}, only float32 buffers are flattened")
                m._buffers[n] = v
                self.views.append((m, n, v))

    def bound(self):
        return all(m._buffers.get(n) is v for m, n, v in self.views)

    def __call__(self):
        if self.flat is None:
            return
        if not self.bound():
            if self.flat.is_cuda and torch.cuda.is_current_stream_capturing():
                raise RuntimeError("BufferBroadcast: buffers were replaced after a step was captured")
            self._bind()
        dist.broadcast(self.flat, src=self.src, group=self.group)


class GradBuckets:
    """Bucketed all-reduce (SUM) of the flat gradient buffer, launched from
    post-accumulate-grad hooks as soon as every parameter of a bucket has its
    gradient, on RCCL's stream (overlaps the remaining backward).  Buckets are
    >= bucket_mb of contiguous gradient memory (xGMI rings are per-link bound:
    fewer, larger collectives)."""

    def __init__(self, state: FlatState, group=None, bucket_mb=64.0, reduce_dtype=torch.float32):
        """reduce_dtype=torch.bfloat16: each bucket is rounded to bf16 (vt_cast_bf16), reduced
        in bf16 (half the bytes over xGMI) and widened back into the fp32 gradient buffer
        (vt_cast_bf16_to_f32) before clip + AdamW, which keep fp32 master gradients and
        moments.  The default fp32 reduce is the reference's DDP semantics."""
        self.state, self.group = state, group
        if reduce_dtype not in (torch.float32, torch.bfloat16):
            raise ValueError(f"reduce_dtype must be float32 or bfloat16, got {reduce_dtype}")
        self.reduce_dtype = reduce_dtype
        self.g16 = (torch.empty(state.numel, dtype=torch.bfloat16, device=state.g.device)
                    if reduce_dtype == torch.bfloat16 else None)
        limit = int(bucket_mb * (1 << 20) / 4)
        self.buckets = []  # (start, end, n_params)
        self.param_bucket = {}
        start, count, cur = 0, 0, 0
        for i, (p, (o, n)) in enumerate(zip(state.params, state.offsets)):
            self.param_bucket[id(p)] = len(self.buckets)
            count += 1
            cur = o + n
            if cur - start >= limit or i == len(state.params) - 1:
                self.buckets.append((start, cur, count))
                start, count = cur, 0
        self.pending = [0] * len(self.buckets)
        self.works = []
        self.launched = []
        self.ready = set()
        self.enabled = True   # False while a hipGraph is captured: no collective inside the graph
        # while a step is captured for the native executor: a marker kernel on `comm` (joined
        # with every gradient writer) where each bucket completes, so the replay can issue the
        # bucket's all-reduce mid-backward (CapturedStep.replay, vt_stepgraph_launch_range)
        self.mark_capture = False
        self.comm = None
        # torch ops reach the flat gradient through AccumulateGrad (hook); the HIP
        # ops write it in place and report through vaeteb.ops.GRAD_READY
        self.handles = [p.register_post_accumulate_grad_hook(self._hook) for p in state.params]
        from . import ops
        ops.GRAD_READY = self._hook

    def reset(self):
        self.pending = [b[2] for b in self.buckets]
        self.works = []
        self.launched = []
        self.ready = set()
        # the stream the step's forward / backward is issued on: a bucket's writers may be on it
        # even when the hook that completes the bucket runs on a side stream (the encoders'
        # backward runs on the streams their forward ran on)
        self.base = torch.cuda.current_stream() if self.state.g.is_cuda else None

    def launch_bucket(self, b):
        """Bucket b's all-reduce, issued on the current stream (the replay of a captured
        step: the comm stream, after the executor range ending with b's marker)."""
        if self.pending[b] > 0:
            s, e, _ = self.buckets[b]
            self._launch(s, e)
            self.pending[b] = 0

    def reduce_all(self):
        """All buckets at once (after a graph replay of the backward)."""
        for b, (s, e, _) in enumerate(self.buckets):
            self._launch(s, e)
            self.pending[b] = 0

    def _hook(self, p):
        if not (self.enabled or self.mark_capture) or id(p) in self.ready or id(p) not in self.param_bucket:
            return  # each parameter counts once per step
        self.ready.add(id(p))
        b = self.param_bucket[id(p)]
        self.pending[b] -= 1
        if self.pending[b] == 0 and self.mark_capture:
            # the comm stream joins every stream that may have written the bucket (the
            # current one and the side streams), then the marker: a graph node that depends
            # on exactly the bucket's writers and that nothing in the step waits for
            cur = _lib.stream()
            from . import ops
            _lib.wait_for(self.comm, cur)
            if self.base is not None and self.base.cuda_stream != cur:
                _lib.wait_for(self.comm, self.base)
            for st in ops.SIDE_STREAMS:
                if st.cuda_stream != self.comm.cuda_stream:
                    _lib.wait_for(self.comm, st)
            _lib.call("vt_bucket_marker", b, self.comm.cuda_stream)
        elif self.pending[b] == 0:
            # a bucket's gradients may have been written on several streams (the
            # concurrent encoders, the side-stream weight gradients): the collective
            # waits for all of them.  The side streams are read here, not at
            # reset(): the model creates them lazily during the first forward, and
            # a head weight gradient queued on one just before this hook must be
            # covered by the wait
            self._join_side_streams()
            s, e, _ = self.buckets[b]
            self._launch(s, e)

    def _join_side_streams(self):
        """The collective's stream waits for every stream that may have written gradients
        (the concurrent encoders, the side-stream weight gradients)."""
        if self.state.g.is_cuda:
            from . import ops
            cur = torch.cuda.current_stream()
            base = getattr(self, "base", None)
            if base is not None and base != cur:
                cur.wait_stream(base)
            for st in ops.SIDE_STREAMS:
                if st != cur:
                    cur.wait_stream(st)

    def finish(self):
        # parameters that received no gradient this step still have to be reduced (after
        # every gradient writer: a caller's backward may leave side-stream work in flight)
        if any(left > 0 for left in self.pending):
            self._join_side_streams()
        for b, left in enumerate(self.pending):
            if left > 0:
                s, e, _ = self.buckets[b]
                self._launch(s, e)
                self.pending[b] = 0
        for w in self.works:
            w.wait()  # orders the compute stream after the collective; no host wait for RCCL
        if self.g16 is not None:
            for s, e in self.launched:
                self._cast(s, e, back=True)
        self.works = []
        self.launched = []

    def _cast(self, s, e, back=False):
        g, h = self.state.g, self.g16
        if not g.is_cuda:   # the CPU (gloo) path: torch casts, same rounding (round to nearest even)
            if back:
                g[s:e].copy_(h[s:e])
            else:
                h[s:e].copy_(g[s:e])
            return
        if back:
            _lib.call("vt_cast_bf16_to_f32", h[s:].data_ptr(), g[s:].data_ptr(), e - s, _lib.stream())
        else:
            _lib.call("vt_cast_bf16", g[s:].data_ptr(), h[s:].data_ptr(), e - s, _lib.stream())

    def _launch(self, s, e):
        """all_reduce(SUM) of the flat gradient slice [s, e) (through its bf16 copy when
        reduce_dtype is bfloat16)."""
        if self.g16 is None:
            self.works.append(dist.all_reduce(self.state.g[s:e], op=dist.ReduceOp.SUM, group=self.group,
                                              async_op=True))
            return
        self._cast(s, e)
        self.works.append(dist.all_reduce(self.g16[s:e], op=dist.ReduceOp.SUM, group=self.group, async_op=True))
        self.launched.append((s, e))


class Trainer:
    """AdamW(lr, weight_decay=1e-4, eps=1e-8, betas) + clip_grad_norm_(max_norm)
    over flat buffers (ref/model/graph_model.py:654-660, :724)."""

    def __init__(self, model, lr=1e-3, betas=(0.9, 0.98), eps=1e-8, weight_decay=1e-4, max_norm=1.0, beta_kld=1e-5,
                 frontend=None, world_size=1, group=None, bucket_mb=64.0, vae_loss_weight=0.1,
                 reduce_dtype=torch.float32, ddp=None, broadcast_buffers=True, loss_scale=None, init_scale=2.0 ** 16,
                 growth_factor=2.0, backoff_factor=0.5, growth_interval=2000):
        """ddp: the bucketed gradient all-reduce (GradBuckets) on (True) / off (False);
        default on exactly when world_size > 1.  ddp=True with one rank (an initialised
        single-rank process group) runs the data-parallel step's whole machinery — buckets,
        the world > 1 stream budget, the segmented native replay — at N = 1 (bench.py
        --ddp-probe).  broadcast_buffers (DDP's flag, default True as in the reference):
        with several ranks, rank 0's BatchNorm running statistics are broadcast before every
        step (BufferBroadcast).
        loss_scale: torch.amp.GradScaler('cuda') around the step (ref/model/graph_model.py:670,
        718-726) — the backward runs on loss * scale, the clip sees the unscaled norm, a step
        whose gradients overflow (inf / NaN) is skipped and the scale backs off, growth_interval
        clean steps double it; all on device state (self.scaler = {scale, growth tracker,
        found_inf, skipped steps}), no host sync.  Default: on exactly when the model trains
        fp16 operands (SeqVaeTeb.loss_scaling); bf16 keeps fp32's range and needs none."""
        self.model = model
        self.vae_loss_weight = vae_loss_weight
        self.frontend = frontend
        self.state = FlatState(model)
        self.lr, self.betas, self.eps, self.wd, self.max_norm = lr, betas, eps, weight_decay, max_norm
        self.beta_kld = beta_kld
        self.world = world_size
        self.steps = 0
        dev = self.state.p.device
        vae = getattr(model, "vae_model", model)
        self.loss_scale = bool(getattr(vae, "loss_scaling", False)) if loss_scale is None else bool(loss_scale)
        self.scaler_cfg = (float(growth_factor), float(backoff_factor), int(growth_interval))
        self.scaler = torch.tensor([float(init_scale), 0.0, 0.0, 0.0], device=dev) if self.loss_scale else None
        self.norm_out = torch.zeros(4, device=dev)   # pre-clip norm, AdamW gradient factor, found_inf
        self.step_dev = torch.zeros(1, dtype=torch.int32, device=dev)   # AdamW step counter (device side)
        self.adam_coef = torch.zeros(2, device=dev)
        self.graph = None
        self.norm_ws = torch.empty(_lib.lib().fns["vt_grad_norm_workspace_floats"](), device=dev)
        ddp = world_size > 1 if ddp is None else bool(ddp)
        self.buckets = GradBuckets(self.state, group, bucket_mb, reduce_dtype) if ddp else None
        if ddp:
            broadcast_state(self.state, model, group)   # every rank starts from rank 0's model (DDP)
        self.buffer_sync = BufferBroadcast(model, group) if (ddp and world_size > 1 and broadcast_buffers) else None
        if ddp and torch.cuda.is_available():
            # hardware-queue budget: a process's streams map onto GPU_MAX_HW_QUEUES = 4 queues;
            # the model uses main + 3 side streams on one GPU, and RCCL's stream would be a 5th
            # sharing (and serialising behind) one of them — with several ranks the model keeps
            # main + 2 side streams so RCCL owns a queue (VAETEB_* environment overrides)
            from . import model as _model
            if "VAETEB_MAX_SIDE_STREAMS" not in os.environ:
                _model.MAX_SIDE = min(_model.MAX_SIDE, 2)
            if "VAETEB_GRAD_SIDE_STREAM" not in os.environ:
                _model.GRAD_SIDE = min(_model.GRAD_SIDE, 2)

    def loss(self, batch, eps=None):
        """Forward + loss for an AttributeDict-like batch with fields fhr_st,
        fhr_ph, fhr_up_ph (B,S,C) and fhr (B,R) (the reference batch contract,
        ref/model/graph_model.py:702-705), or raw windows under key 'x'."""
        vae = getattr(self.model, "vae_model", self.model)   # SeqVaeTebClassifier (config 4) wraps the VAE
        labels = batch.get("labels") if hasattr(batch, "get") else None
        if "x" in batch:
            if hasattr(vae, "prepass"):
                vae.prepass()   # weight-only forward work on a side stream, overlapping the front-end
            side = None
            if getattr(vae, "concurrent_encoders", False) and batch["x"].is_cuda:
                from .model import side_stream
                side = side_stream(batch["x"].device.index if batch["x"].device.index is not None else
                                   torch.cuda.current_device(), 1)  # the source encoder's stream
            batch = self.frontend(batch["x"], side=side)
        if vae is not self.model:
            # SeqVaeTebClassifier.compute_loss (ref/model/vae_teb_model.py:1440-1498): CE + w * ELBO(beta 1)
            return self.model.compute_loss(batch["fhr_st"], batch["fhr_ph"], batch["fhr_up_ph"], labels,
                                           y_raw=batch["fhr"], compute_vae_loss=True,
                                           vae_loss_weight=self.vae_loss_weight, eps=eps)
        fw = self.model(batch["fhr_st"], batch["fhr_ph"], batch["fhr_up_ph"], eps=eps)
        return self.model.compute_loss(fw, batch["fhr_st"], batch["fhr_ph"], batch["fhr"], compute_kld_loss=True,
                                       beta=self.beta_kld)

    def eval_losses(self, batch, eps=None):
        """Validation losses (ref/model/graph_model.py:769-815): the model in eval mode
        (BatchNorm on its running statistics), no gradients, the training loss terms."""
        if self.model.training:
            self.model.eval()
        with torch.no_grad():
            out = self.loss(batch, eps)
        return {k: (v.detach() if isinstance(v, torch.Tensor) else v) for k, v in out.items()}

    def step(self, batch, eps=None, before_update=None):
        """One optimisation step; returns the loss dict (device scalars, no sync).
        before_update(): optional host callback between the backward and the
        clip + AdamW launches (e.g. to enqueue the next batch's front-end on
        another stream, so it overlaps the memory-bound optimizer)."""
        losses = self._forward_backward(batch, eps, overlap_comm=True)
        if self.buckets:
            self.buckets.finish()
        if before_update is not None:
            before_update()
        self._update()
        losses["grad_norm"] = self.norm_out[0]
        return losses

    def _forward_backward(self, batch, eps, overlap_comm):
        if not self.model.training:
            self.model.train()
        self.state.zero_grad(first_writer=FIRST_WRITER)
        if self.state.g.is_cuda:
            # every side stream joins the step at its start: under hipGraph capture a
            # stream the step never forked to would otherwise be joined at the end
            # from outside the capture
            from . import ops
            for st in ops.SIDE_STREAMS:
                _lib.wait_for(st)
        if self.buckets:
            self.buckets.reset()
            self.buckets.enabled = overlap_comm
        if self.buffer_sync is not None and not (self.state.p.is_cuda and torch.cuda.is_current_stream_capturing()):
            self.buffer_sync()   # DDP broadcast_buffers (under capture: CapturedStep.replay issues it)
        losses = self.loss(batch, eps)
        # GradScaler.scale: the backward seeds carry the scale (device scalar, no sync)
        root = losses["total_loss"] * self.scaler[0] if self.loss_scale else losses["total_loss"]
        if BWD_SAME_THREAD:
            # the backward on this thread instead of autograd's device worker thread
            with torch.autograd.set_multithreading_enabled(False):
                root.backward()
        else:
            root.backward()
        if torch.cuda.is_available():
            # gradients written in place on side streams (no AccumulateGrad, so
            # autograd does not join those streams for us)
            from . import ops
            cur = _lib.stream()
            for st in ops.SIDE_STREAMS:
                _lib.wait_for(cur, st)
        self.state.finish_first_writer()
        # detached: a returned loss must not keep this step's autograd graph (and
        # with it the parameters' AccumulateGrad nodes, bound to this step's
        # stream) alive into the next step or a hipGraph capture
        return {k: (v.detach() if isinstance(v, torch.Tensor) else v) for k, v in losses.items()}

    def _shadow_plan(self):
        """The model's bf16 shadows the optimizer step can write: up to 4 2-D weights
        (64-float aligned in the flat buffers, both dims multiples of 64: the MFMA heads) for
        the tiled AdamW, up to 24 conv weights for the batched shadow launch — those whose
        shadows a forward has created (ops._SHADOW / ops._CONV_SHADOW).  Cached until new
        shadows appear."""
        import ctypes
        from . import ops
        sig = (len(ops._SHADOW), len(ops._CONV_SHADOW), _lib._H16[0],
               tuple(v[0].data_ptr() for v in list(ops._SHADOW.values())[:8]))
        if getattr(self, "_splan_sig", None) == sig:
            return self._splan
        heads, convs = [], []
        for p, (o, n) in zip(self.state.params, self.state.offsets):
            key = (p.data_ptr(), *p.shape)
            if p.dim() == 2 and key in ops._SHADOW and len(heads) < 4:
                N, K = p.shape
                if o % 64 == 0 and N % 64 == 0 and K % 64 == 0:
                    heads.append((o, N, K, ops._SHADOW[key], key, p))
            elif p.dim() == 3 and key in ops._CONV_SHADOW and len(convs) < 24:
                convs.append((p, ops._CONV_SHADOW[key], key))
        I64, I32 = ctypes.c_int64, ctypes.c_int
        arrs = {
            "h_off": (I64 * 4)(*[h[0] for h in heads]), "h_N": (I32 * 4)(*[h[1] for h in heads]),
            "h_K": (I32 * 4)(*[h[2] for h in heads]), "h_w16": (I64 * 4)(*[h[3][0].data_ptr() for h in heads]),
            "h_w16t": (I64 * 4)(*[h[3][1].data_ptr() for h in heads]),
            "c_w": (I64 * 24)(*[c[0].data_ptr() for c in convs]), "c_co": (I32 * 24)(*[c[0].shape[0] for c in convs]),
            "c_ci": (I32 * 24)(*[c[0].shape[1] for c in convs]), "c_k": (I32 * 24)(*[c[0].shape[2] for c in convs]),
            "c_w16": (I64 * 24)(*[c[1][0].data_ptr() for c in convs]),
            "c_w16t": (I64 * 24)(*[c[1][1].data_ptr() for c in convs])}
        addr = {k: ctypes.addressof(v) for k, v in arrs.items()}
        keys = [(h[4], h[5]) for h in heads] + [(c[2], c[0]) for c in convs]
        self._splan = (len(heads), len(convs), arrs, addr, keys) if (heads or convs) else None
        self._splan_sig = sig
        return self._splan

    def _update(self, adam_stream=None):
        """clip_grad_norm_ + AdamW over the flat buffers.  adam_stream: run the AdamW pass
        (memory-bound) on that stream, forked after the norm, so the caller can overlap it
        with work that does not read the parameters (the next batch's front-end); the
        caller joins it before the next forward."""
        self.steps += 1
        st = _lib.stream()
        s = self.state
        vae = getattr(self.model, "vae_model", self.model)
        fmt = getattr(vae, "h16_format", None)
        if fmt and s.p.is_cuda:
            _lib.set_h16(fmt == "fp16")     # the shadows below are written in the model's format
        skip = None
        if self.loss_scale:
            # GradScaler: unscale + inf check + clip coefficient + scale update in one finalise;
            # an overflowing step is skipped on the device (skip = found_inf)
            g, b, n = self.scaler_cfg
            _lib.call("vt_grad_norm_clip_scaled", s.g.data_ptr(), s.numel, 1.0 / self.world, float(self.max_norm),
                      self.norm_out.data_ptr(), self.norm_ws.data_ptr(), self.scaler.data_ptr(), g, b, n, st)
            skip = self.norm_out.data_ptr() + 8
        else:
            _lib.call("vt_grad_norm_clip", s.g.data_ptr(), s.numel, 1.0 / self.world, float(self.max_norm),
                      self.norm_out.data_ptr(), self.norm_ws.data_ptr(), st)
        if adam_stream is not None:
            _lib.wait_for(adam_stream, st)
            st = adam_stream.cuda_stream
        from . import ops
        plan = self._shadow_plan() if (SHADOW_UPDATE and s.p.is_cuda) else None
        ops._FRESH.clear()
        if plan is None:
            _lib.call("vt_adamw_step_dev_skip", s.p.data_ptr(), s.g.data_ptr(), s.m.data_ptr(), s.v.data_ptr(),
                      s.numel, float(self.lr), float(self.betas[0]), float(self.betas[1]), float(self.eps),
                      float(self.wd), self.step_dev.data_ptr(), self.adam_coef.data_ptr(), self.norm_out.data_ptr() + 4,
                      skip, st)
            return
        n_heads, n_convs, _, a, keys = plan
        _lib.call("vt_adamw_step_dev_shadow_skip", s.p.data_ptr(), s.g.data_ptr(), s.m.data_ptr(), s.v.data_ptr(),
                  s.numel, float(self.lr), float(self.betas[0]), float(self.betas[1]), float(self.eps),
                  float(self.wd), self.step_dev.data_ptr(), self.adam_coef.data_ptr(), self.norm_out.data_ptr() + 4,
                  n_heads, a["h_off"], a["h_N"], a["h_K"], a["h_w16"], a["h_w16t"], skip, st)
        if n_convs:
            _lib.call("vt_conv1d_bf16_shadow_batch", n_convs, a["c_w"], a["c_co"], a["c_ci"], a["c_k"], a["c_w16"],
                      a["c_w16t"], st)
        for key, w in keys:
            ops.mark_fresh(key, w)           # the next forward uses these shadows as they are

    def scaler_state(self):
        """The dynamic loss scale (host copy, syncs): {scale, growth_tracker, found_inf (last step),
        skipped_steps} — GradScaler.get_scale() / _growth_tracker; None without loss scaling."""
        if not self.loss_scale:
            return None
        v = self.scaler.tolist()
        return {"scale": v[0], "growth_tracker": int(v[1]), "found_inf": bool(v[2]), "skipped_steps": int(v[3])}

    # ------------------------------------------------------------ hipGraph
    def capture(self, batch, eps=None, warmup=2, pre_capture=None, native=False, n_streams=4, update=True):
        """Record the training step as a hipGraph over static input buffers and
        return it as a `CapturedStep` (also kept as the trainer's default for
        `replay`).  A replay is one launch instead of ~1200 host-side op
        dispatches (the eager step is host-bound: ~20 ms of Python/ctypes
        dispatch for ~22 ms of GPU work).  Every op is stream-ordered, host-sync
        free and allocation-stable after the first steps, so a replay is the same
        computation as an eager step (tests/test_gpu_model.py checks bit
        equality).  Single GPU: the whole step (forward, backward, clip, AdamW)
        is one graph.  Several GPUs: the graph ends after the backward; the
        bucketed RCCL all-reduce, clip and AdamW are issued after each replay (a
        handful of launches), so no collective is captured.  `warmup` eager
        steps run first (on the capture side stream, as torch requires) and do
        update the model.  Capture more than once for double-buffered inputs.

        native=True: the replay is the library's multi-stream executor
        (vt_stepgraph_*, csrc/stepgraph.cpp) over the captured graph instead of
        hipGraphLaunch — the eager step's stream concurrency at graph-replay host
        cost.  It does not advance in-graph RNG offsets, so `eps` (the
        reparameterisation noise) must be given: the caller draws each step's
        noise into `CapturedStep.static_eps` before the replay."""
        if native and eps is None:
            raise ValueError("native replay needs an explicit eps buffer (in-graph RNG is not advanced)")
        if any(getattr(m, "sync_bn", False) for m in self.model.modules()):
            raise ValueError("a model with SyncBatchNorm blocks (convert_sync_batchnorm) cannot be captured: its "
                             "BatchNorm statistics are all-reduced inside the step; use Trainer.step")
        static_in = {k: v.clone() for k, v in batch.items()}
        static_eps = None if eps is None else eps.clone()
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(warmup):
                self.step(static_in, eps=static_eps)
        torch.cuda.current_stream().wait_stream(side)
        if pre_capture is not None:
            pre_capture()
        # the bf16 shadows the captured forward will trust instead of rewriting (written by the
        # warmup steps' optimizer pass, ops._FRESH): CapturedStep.replay re-checks their weights'
        # version counters, so a load_state_dict / copy_ between replays cannot leave the heads and
        # convs computing with stale bf16 copies (advisor r04)
        from . import ops
        shadow_watch = [[ref, ver] for ref, ver in ops._FRESH.values()]
        graph = torch.cuda.CUDAGraph(keep_graph=native)
        comm = None
        if self.buckets is not None and native:
            # several ranks: the executor runs the model's streams (main + MAX_SIDE) plus a
            # comm stream on which each bucket's marker joins that bucket's writers; the
            # replay issues the bucket's all-reduce there as soon as its range is enqueued
            from . import model as _model
            n_streams = min(n_streams, 1 + _model.MAX_SIDE)
            comm = _model.side_stream(torch.cuda.current_device(), n_streams)
            self.buckets.comm = comm
            self.buckets.mark_capture = True
        # several ranks: torch's process-group watchdog thread queries the warmup steps'
        # collective events while this thread captures; a global-mode capture forbids that
        # (hipErrorStreamCaptureUnsupported, the watchdog aborts the process), a thread-local
        # one restricts only this thread
        mode = "thread_local" if self.buckets is not None else "global"
        try:
            with torch.cuda.graph(graph, capture_error_mode=mode):
                out = self._forward_backward(static_in, static_eps, overlap_comm=False)
                if not self.buckets and update:
                    self._update()
                if CAPTURE_JOIN:
                    _join_side_streams()
                if os.environ.get("VAETEB_CAPTURE_TRACE", "0") == "1":   # diagnostic (capture_probe.py)
                    import sys
                    from . import ops
                    from ._lib import capture_info
                    for st in [torch.cuda.current_stream(), *ops.SIDE_STREAMS]:
                        print(f"[capture] before end, {'capture' if st == torch.cuda.current_stream() else 'side'} "
                              f"stream:\n{capture_info(st)}", file=sys.stderr, flush=True)
        finally:
            if self.buckets is not None:
                self.buckets.mark_capture = False
        out["grad_norm"] = self.norm_out[0]
        self.captured = CapturedStep(self, graph, static_in, static_eps, out, native=native, n_streams=n_streams,
                                     comm=comm)
        self.captured.update = update
        self.captured.shadow_watch = shadow_watch
        return self.captured

    def replay(self, batch=None, eps=None):
        """One step of the last captured graph on `batch` (copied into its static inputs)."""
        return self.captured.replay(batch, eps)


CAPTURE_JOIN = os.environ.get("VAETEB_CAPTURE_JOIN", "1") == "1"
DDP_DIAG = int(os.environ.get("VAETEB_DDP_DIAG", "0"))   # segmented-replay diagnostics (tools/gpu_ddp_ab.sh)


def _join_side_streams():
    """before a capture ends, the capture stream waits for every side
    stream the model forked into it (ops.SIDE_STREAMS, the comm stream included), so no
    branch can be left unjoined whatever a future fork does.  Streams not in the capture are
    skipped (a wait on them would be an external dependency)."""
    from . import ops
    from ._lib import wait_for
    cur = torch.cuda.current_stream()
    for s in ops.SIDE_STREAMS:
        if s.device != cur.device or s.cuda_stream == cur.cuda_stream:
            continue
        with torch.cuda.stream(s):
            capturing = torch.cuda.is_current_stream_capturing()
        if capturing:
            wait_for(cur, s)


class CapturedStep:
    """A training step recorded as a hipGraph (Trainer.capture)."""

    def __init__(self, trainer, graph, static_in, static_eps, out, native=False, n_streams=4, comm=None):
        self.trainer, self.graph, self.static_in, self.static_eps, self.out = trainer, graph, static_in, static_eps, out
        self.handle = None
        self.markers, self.comm = [], comm
        if native:
            import ctypes
            from .model import side_stream
            h = ctypes.c_void_p()
            _lib.call("vt_stepgraph_build", graph.raw_cuda_graph(), n_streams, ctypes.addressof(h))
            self.handle = h.value
            # the executor runs on the caller's stream plus the eager step's side streams
            # (each bound to its own hardware queue)
            dev = torch.cuda.current_device()
            self.side = [side_stream(dev, i) for i in range(1, n_streams)]
            n_ops, n_mark = ctypes.c_int(), ctypes.c_int()
            _lib.call("vt_stepgraph_markers", self.handle, ctypes.addressof(n_ops), ctypes.addressof(n_mark), None,
                      None, 0)
            if n_mark.value:
                ends, bks = (ctypes.c_int * n_mark.value)(), (ctypes.c_int * n_mark.value)()
                _lib.call("vt_stepgraph_markers", self.handle, ctypes.addressof(n_ops), ctypes.addressof(n_mark),
                          ctypes.addressof(ends), ctypes.addressof(bks), n_mark.value)
                self.markers = list(zip(list(ends), list(bks)))
                if comm is None:
                    raise RuntimeError("captured step holds bucket markers but no comm stream")
                self.side.append(comm)          # streams[n_streams]: the markers' stream
            self.n_ops = n_ops.value
            self.streams = (ctypes.c_void_p * len(self.side + [None]))()
            self._st_addr = ctypes.addressof(self.streams)
            self._destroy = _lib.lib().fns["vt_stepgraph_destroy"]

    shadow_watch = ()

    def _refresh_shadows(self):
        """The captured forward reads the bf16 shadows of the heads / convs as the optimizer
        pass left them (the replay's own AdamW rewrites them, which does not touch torch's
        version counters).  A weight changed from torch since (load_state_dict, copy_, another
        optimizer) has a new version: its shadows are rewritten here, on the current stream,
        before the launch."""
        from . import ops
        for e in self.shadow_watch:
            w = e[0]()
            if w is not None and w._version != e[1]:
                (ops._weight_shadow if w.dim() == 2 else ops._conv_shadow)(w, prepass=True)
                e[1] = w._version

    def _launch_range(self, begin, end, flags):
        _lib.call("vt_stepgraph_launch_range", self.handle, self._st_addr, begin, end, flags)

    def info(self):
        """(kernels, memcpys, memsets, cross-stream waits) of the native executor's launch list."""
        import ctypes
        v = [ctypes.c_int() for _ in range(4)]
        _lib.call("vt_stepgraph_info", self.handle, *[ctypes.addressof(x) for x in v])
        return tuple(x.value for x in v)

    def __del__(self):
        if getattr(self, "handle", None):
            self._destroy(self.handle)   # bound at build time: safe during interpreter shutdown
            self.handle = None

    def replay(self, batch=None, eps=None, adam_stream=None):
        """One step.  A step captured with update=False issues clip + AdamW after the
        replay (adam_stream: the AdamW pass on that stream, see Trainer._update)."""
        tr = self.trainer
        self._refresh_shadows()
        if tr.buffer_sync is not None:
            tr.buffer_sync()     # DDP broadcast_buffers: rank 0's BatchNorm statistics before the step
        if batch is not None:
            for k, v in batch.items():
                if v.data_ptr() != self.static_in[k].data_ptr():
                    self.static_in[k].copy_(v, non_blocking=True)
        if eps is not None:
            self.static_eps.copy_(eps, non_blocking=True)
        if self.handle is not None:
            st = self.streams
            st[0] = _lib.stream()
            for i, sd in enumerate(self.side, 1):
                st[i] = sd.cuda_stream
            if tr.buckets and self.markers:
                # DDP overlap: the launch list in ranges; after the range that ends with a
                # bucket's marker, that bucket's all-reduce on the comm stream, which has
                # waited for exactly the bucket's gradient writers (the rest of the backward
                # keeps running on the model's streams)
                tr.buckets.reset()
                pos = 0
                for end, b in self.markers:
                    self._launch_range(pos, end, 1 if pos == 0 else 0)
                    with torch.cuda.stream(self.comm):
                        if DDP_DIAG == 1:   # diagnostic: the comm stream waits for every executor stream
                            _lib.wait_for(self.comm, st[0])
                            for sd in self.side:
                                if sd.cuda_stream != self.comm.cuda_stream:
                                    _lib.wait_for(self.comm, sd)
                        tr.buckets.launch_bucket(b)
                        if DDP_DIAG == 2 and tr.buckets.works:   # diagnostic: each collective completes here
                            tr.buckets.works[-1].wait()
                    pos = end
                self._launch_range(pos, self.n_ops, (1 if pos == 0 else 0) | 2)
            else:
                _lib.call("vt_stepgraph_launch", self.handle, self._st_addr)
        else:
            self.graph.replay()
        if tr.buckets:
            if not (self.handle is not None and self.markers):
                tr.buckets.reduce_all()
            tr.buckets.finish()
            tr._update()
        elif not getattr(self, "update", True):
            tr._update(adam_stream)
        else:
            tr.steps += 1
        return self.out


def init_distributed():
    """torchrun environment -> (rank, world, local_rank, device); RCCL on GPUs,
    gloo on CPU-only hosts (the multi-process CPU tests).

    VAETEB_DIST_BACKEND=gloo|nccl overrides the backend.  With gloo on a GPU host the
    ranks may outnumber the GPUs: rank r runs on cuda:(local_rank mod device_count),
    so several ranks can share one GPU (RCCL refuses two ranks on one device) — the
    one-GPU rehearsal of the multi-rank bench (tests/test_gpu_ddp.py)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    override = os.environ.get("VAETEB_DIST_BACKEND", "")
    if override not in ("", "gloo", "nccl"):
        raise ValueError(f"VAETEB_DIST_BACKEND must be gloo or nccl, got {override!r}")
    cuda = torch.cuda.is_available()
    if cuda and override == "gloo":
        local = local % max(1, torch.cuda.device_count())
    if world > 1 and not dist.is_initialized():
        backend = override or ("nccl" if cuda else "gloo")
        if cuda:
            torch.cuda.set_device(local)
        dist.init_process_group(backend=backend)
    dev = torch.device(f"cuda:{local}") if cuda else torch.device("cpu")
    return rank, world, local, dev


def free_port():
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def spawn_local_ranks(cmd, n, env=None, poll_s=0.2, stdout=None):
    """Start `n` ranks of `cmd` on this node, one process per GPU, and wait for them — the
    reference's own launcher for its DDP loop (`mp.spawn(main_pytorch, nprocs=world_size)`,
    ref/model/graph_model.py:2152-2157; torchrun in ref/run_train_ddp.sh:11-17) as fresh
    processes, so the caller never touches the GPU itself (a process that has initialised
    HIP must not fork / exec GPU workers).

    Each rank gets RANK = LOCAL_RANK = r, WORLD_SIZE = LOCAL_WORLD_SIZE = n and a free
    MASTER_PORT on MASTER_ADDR 127.0.0.1.  Rank 0's stdout is relayed line by line to
    `stdout` (default sys.stdout) after it exits; the other ranks' stdout goes to this
    process's stderr.  When one rank fails, the others are terminated (they would wait in a
    collective forever).  Returns the exit code of the rank that failed first (the ones
    terminated because of it are not counted), else 0."""
    import subprocess
    import sys
    import threading
    import time
    port = free_port()
    procs, out0, failed, reader = [], [], None, None
    try:
        for r in range(n):
            e = dict(os.environ if env is None else env, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                     LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
            procs.append(subprocess.Popen(cmd, env=e, stdout=subprocess.PIPE if r == 0 else sys.stderr.fileno()))
            if r == 0:   # rank 0's pipe drained while it runs (never blocks on a full pipe)
                reader = threading.Thread(target=lambda p=procs[0]: out0.extend(p.stdout), daemon=True)
                reader.start()
        while failed is None and None in [p.poll() for p in procs]:   # every rank polled
            time.sleep(poll_s)
            failed = next((p.returncode for p in procs if p.returncode not in (None, 0)), None)
        if failed is None:
            failed = next((p.returncode for p in procs if p.returncode != 0), None)
    finally:
        for p in procs:
            if p.poll() is None:
                p.terminate()
        for p in procs:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
    if reader is not None:
        reader.join(timeout=10)
    sink = stdout or sys.stdout
    for line in out0:
        sink.write(line.decode())
    sink.flush()
    return failed or 0
