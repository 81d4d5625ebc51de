"""SeqVaeTeb on MI355X: same constructor / forward / compute_loss contract and
the same state_dict key names as the reference (ref/model/vae_teb_model.py:982-1192),
so checkpoints interchange (ref/model/graph_model.py:338-342,381-390), with
every op routed to the HIP kernels in libvaeteb.so (vaeteb.ops).

Activations stay (B, S, C) / (B, L, C) row-major end to end; the conv stacks
read that layout directly (their kernels fuse the reference's transposes,
padding and upsampling).  Widths follow the reference exactly (geometric
schedules, SURVEY.md §8(a) "Exact ResidualMLP widths"); the encoder input
widths and the decoder head size R = 16*S are constructor parameters so the
J=6/Q=1 front-end variant and other sequence lengths work unchanged.
"""
import math
import os

import torch
import torch.nn as nn

from . import _lib, ops


# ----------------------------------------------------------- stream forks
# SeqVaeTeb(concurrent_encoders=True) runs independent branches of the graph
# (source / target encoder, the target encoder's scattering / phase branches,
# the conditional encoder's and the decoder's mu / logvar heads) on side HIP
# streams.  Every reduction has a fixed order, so results are bit-identical
# to the serial run (tests/test_gpu_model.py).
_PAR = {"on": False, "next": 1}
MAX_SIDE = int(__import__("os").environ.get("VAETEB_MAX_SIDE_STREAMS", "3"))
GRAD_SIDE = int(__import__("os").environ.get("VAETEB_GRAD_SIDE_STREAM", "3"))  # conv weight-gradient stream (measured: 3 < 2 < 1)
HEAD_GRAD_SIDE = int(__import__("os").environ.get("VAETEB_HEAD_GRAD_SIDE_STREAM", "1"))  # 0: inline
# LSTM parameter gradients (deferred after the recurrence chain, ops.LSTM_GRAD_DEFER) on this side
# stream; 0: in line after the chain (measured fastest: GPU-only step 10.22 vs 10.42 ms on stream 3
# and 10.45 ms per layer in line)
LSTM_GRAD_SIDE = int(__import__("os").environ.get("VAETEB_LSTM_GRAD_SIDE_STREAM", "0"))
# DIAGNOSTIC (tools/capture_probe.py): keep the head / LSTM weight-gradient side-stream branches
# under hipGraph capture too (they are dropped there: DESIGN.md §9, the capture segfault)
CAPTURE_BRANCHES = __import__("os").environ.get("VAETEB_CAPTURE_BRANCHES", "0") == "1"
# weight-only forward work (bf16 shadows, BatchNorm counters) on this side stream ahead of a
# concurrent training forward; 0 (default): shadows in line, counters in one launch
PREPASS = int(__import__("os").environ.get("VAETEB_PREPASS", "0"))   # measured: GPU-neutral, +1 ms host
PREPASS_SIDE = 3
_SIDE = {}


def side_stream(device, i):
    s = _SIDE.get((device, i))
    if s is None:
        s = _SIDE[(device, i)] = torch.cuda.Stream(device=device)
        ops.SIDE_STREAMS.append(s)
    return s


def fork(*thunks):
    """Run thunks[0] on the current stream and thunks[i] on side stream i; the
    current stream waits for all of them.  Serial unless a concurrent model is
    running on a GPU."""
    if not _PAR["on"]:
        return [t() for t in thunks]
    dev = torch.cuda.current_device()
    main = torch.cuda.current_stream()
    outs = [None] * len(thunks)
    sides = []
    for i, t in enumerate(thunks[1:], 1):
        # fork k of a forward pass runs on side stream min(k, MAX_SIDE): with HIP's
        # default 4 hardware queues per process, main + 3 side streams each own a
        # queue (a 5th stream would share one and serialise behind its work)
        st = side_stream(dev, min(_PAR["next"], MAX_SIDE))
        _PAR["next"] += 1
        _lib.wait_for(st, main)
        with torch.cuda.stream(st):
            outs[i] = t()
        sides.append(st)
    outs[0] = thunks[0]()
    for st in sides:
        _lib.wait_for(main, st)
    for o in outs[1:]:
        for t in (o if isinstance(o, (tuple, list)) else (o,)):
            if isinstance(t, torch.Tensor) and t.is_cuda:
                t.record_stream(main)
    return outs


LOCKSTEP = os.environ.get("VAETEB_LOCKSTEP", "1") != "0"
# which branch creates its autograd nodes first in each lockstep stage: "enc" = the main
# branch first in the encoder fork only (its side branch's nodes then outrank the main
# branch's in every stage of the backward), "all" = in every fork, "none" = side first
LOCKSTEP_MAIN_FIRST = os.environ.get("VAETEB_LOCKSTEP_MAIN_FIRST", "enc")


def _drain(gen):
    """Run a stage generator to completion; its return value."""
    try:
        while True:
            next(gen)
    except StopIteration as e:
        return e.value


def fork_lockstep(*gens, main_first=False):
    """fork() for stage generators: the branches advance one stage at a time in
    turn (side branches first), so their autograd nodes are created interleaved.
    The backward replays nodes in reverse creation order, so it then alternates
    between the branches and the two streams' backward kernels overlap, instead
    of one branch's whole backward being enqueued before the other's starts
    (what a plain fork gives: every node of the later branch outranks every
    node of the earlier one).  Same kernels on the same streams; serial runs
    each generator to completion.  main_first: the main branch advances first in every
    stage, so in the backward the side branch's node of a stage is enqueued first (the
    side branch's long first-stage backward then overlaps the main branch's tail)."""
    if not _PAR["on"]:
        return [_drain(g) for g in gens]
    if not LOCKSTEP:   # A/B switch: plain fork() order (each branch whole, side branches first)
        return fork(*[(lambda g=g: _drain(g)) for g in gens])
    dev = torch.cuda.current_device()
    main = torch.cuda.current_stream()
    streams = [main]
    for _ in gens[1:]:
        st = side_stream(dev, min(_PAR["next"], MAX_SIDE))
        _PAR["next"] += 1
        _lib.wait_for(st, main)
        streams.append(st)
    outs = [None] * len(gens)
    live = list(range(len(gens) - 1, -1, -1))        # side branches first, as fork()
    if main_first:
        live.reverse()
    while live:
        for i in list(live):
            with torch.cuda.stream(streams[i]):
                try:
                    next(gens[i])
                except StopIteration as e:
                    outs[i] = e.value
                    live.remove(i)
    for st in streams[1:]:
        _lib.wait_for(main, st)
    for o in outs[1:]:
        for t in (o if isinstance(o, (tuple, list)) else (o,)):
            if isinstance(t, torch.Tensor) and t.is_cuda:
                t.record_stream(main)
    return outs


def geometric_schedule(input_size, output_size, n_hidden, round_fn=round):
    """ref/model/vae_teb_model.py:11-44 (repeated-multiplication ratio, as there)."""
    r = (output_size / input_size) ** (1 / (n_hidden + 1))
    sizes, cur = [], r
    for _ in range(n_hidden):
        sizes.append(int(round_fn(input_size * cur)))
        cur *= r
    return tuple(sizes + [output_size])


# ------------------------------------------------------------- parameter holders
class Linear(nn.Module):
    def __init__(self, din, dout):
        super().__init__()
        self.in_features, self.out_features = din, dout
        self.weight = nn.Parameter(torch.empty(dout, din))
        self.bias = nn.Parameter(torch.zeros(dout))
        nn.init.xavier_uniform_(self.weight)          # initialization(), vae_teb_model.py:55-59
        self.mfma = False                             # bf16 MFMA GEMMs (set on the decoder heads)

    def forward(self, x):
        return ops.linear(x, self.weight, self.bias, self.mfma)


class LayerNorm(nn.Module):
    def __init__(self, c, eps=1e-5):
        super().__init__()
        self.eps = eps
        self.weight = nn.Parameter(torch.ones(c))
        self.bias = nn.Parameter(torch.zeros(c))

    def forward(self, x, act="none"):
        return ops.layer_norm_act(x, self.weight, self.bias, act, self.eps)


class Activation(nn.Module):
    """Parameter-free marker keeping the reference's Sequential indices."""

    def __init__(self, kind):
        super().__init__()
        self.kind = kind


class ResidualMLP(nn.Module):
    """LN(in) -> [Linear -> LN -> act]* -> Linear (-> LN -> act) (+ skip);
    ref/model/vae_teb_model.py:336-403."""

    def __init__(self, input_dim, hidden_dims, final_activation=True, activation="relu", use_skip_connection=True):
        super().__init__()
        self.input_norm = LayerNorm(input_dim)
        self.final_activation = final_activation
        self.act = activation
        mods, self._plan, d = [], [], input_dim
        for i, h in enumerate(hidden_dims):
            last = i == len(hidden_dims) - 1
            lin = Linear(d, h)
            idx = len(mods)
            mods.append(lin)
            ln = None
            if not (last and not final_activation):
                ln = LayerNorm(h)
                mods.append(ln)
            if not last:
                mods.append(Activation(activation))
            # fused: Linear, then LN + (act for hidden layers; final act for the last with final_activation)
            act = activation if (not last or final_activation) else "none"
            self._plan.append((idx, ln is not None, act))
            d = h
        self.body = nn.Sequential(*mods)
        self.fused = True   # whole-stack kernels (vt_resmlp_*); False: one launch sequence per layer
        self.bf16 = False   # whole-stack kernels on bf16 MFMA (vt_resmlp_bf16_*; the reference's fp16 autocast in bf16)
        self.use_skip_connection = use_skip_connection
        if use_skip_connection:
            self.skip_proj = Linear(input_dim, hidden_dims[-1]) if input_dim != hidden_dims[-1] else nn.Identity()
        else:
            self.skip_proj = None

    def _fused_spec(self):
        """MlpSpec + parameter list for the whole-stack kernels (vt_resmlp_*),
        or None when a width / depth / the bf16 heads rule them out.  Cached;
        rebuilt when a parameter tensor is replaced (its storage moves)."""
        c = getattr(self, "_fs_cache", None)
        if c is not None and all(p is None or p.data_ptr() == q for p, q in zip(c[1], c[2])):
            return c[0], c[1]
        fs = self._build_fused_spec()
        self._fs_cache = None if fs is None else (fs[0], fs[1], [p.data_ptr() if p is not None else 0
                                                                  for p in fs[1]])
        if fs is not None:
            fs[0].param_ptrs = ops.MlpSpec.pointers(fs[1])
        return fs

    def _build_fused_spec(self):
        dims, lns, acts, params = [self.input_norm.weight.shape[0]], [], [], [self.input_norm.weight,
                                                                               self.input_norm.bias]
        eps = {self.input_norm.eps}
        for (idx, has_ln, act) in self._plan:
            lin = self.body[idx]
            if lin.mfma:
                return None
            ln = self.body[idx + 1] if has_ln else None
            dims.append(lin.out_features)
            lns.append(has_ln)
            acts.append(act if has_ln else "none")
            params += [lin.weight, lin.bias, ln.weight if ln else None, ln.bias if ln else None]
            if ln is not None:
                eps.add(ln.eps)
        if len(eps) != 1 or not ops.MlpSpec.supported(dims):
            return None
        skip = 0
        if self.use_skip_connection:
            skip = 1 if isinstance(self.skip_proj, nn.Identity) else 2
        params += [self.skip_proj.weight, self.skip_proj.bias] if skip == 2 else [None, None]
        key = (tuple(dims), tuple(lns), tuple(acts), skip)
        if getattr(self, "_spec_key", None) != key:
            self._spec = ops.MlpSpec(dims, lns, acts, skip, eps.pop())
            self._spec_key = key
        return self._spec, params

    def forward(self, x):
        return _drain(self.stages(x))

    def stages(self, x):
        """forward() as a stage generator (fork_lockstep): one stage per layer."""
        if x.is_cuda and self.fused:
            fs = self._fused_spec()
            if fs is not None:
                return ops.resmlp(x, *fs, bf16=self.bf16)
        x0 = self.input_norm(x)
        h = x0
        for (idx, has_ln, act) in self._plan:
            yield
            lin = self.body[idx]
            if has_ln and not lin.mfma and ops.linear_ln_fused_ok(lin.in_features, lin.out_features):
                ln = self.body[idx + 1]   # Linear -> LN -> act in one pass (vt_linear_ln_fwd)
                h = ops.linear_ln_act(h, lin.weight, lin.bias, ln.weight, ln.bias, act, ln.eps)
                continue
            h = lin(h)
            if has_ln:
                h = self.body[idx + 1](h, act)
        if self.use_skip_connection:
            s = x0 if isinstance(self.skip_proj, nn.Identity) else self.skip_proj(x0)
            h = h + s
        return h


class _ConvWeight(nn.Module):
    def __init__(self, cin, cout, k):
        super().__init__()
        self.in_channels, self.out_channels, self.kernel_size = cin, cout, k
        self.weight = nn.Parameter(torch.empty(cout, cin, k))
        nn.init.xavier_uniform_(self.weight)


class _BatchNorm(nn.Module):
    def __init__(self, c, momentum=0.9, eps=1e-5):
        super().__init__()
        self.momentum, self.eps = momentum, eps
        self.weight = nn.Parameter(torch.ones(c))
        self.bias = nn.Parameter(torch.zeros(c))
        self.register_buffer("running_mean", torch.zeros(c))
        self.register_buffer("running_var", torch.ones(c))
        self.register_buffer("num_batches_tracked", torch.tensor(0, dtype=torch.long))


class ConvBlock(nn.Module):
    """Conv1d(bias=False) -> BatchNorm1d(momentum 0.9) -> ReLU/tanh on (B, L, C).
    causal=True: CausalMultiChannelConvBlock (ref/model/vae_teb_model.py:128-212);
    causal=False: MultiChannelConvBlock with reflect/replicate padding and the
    optional x2 linear upsample (:214-253)."""

    def __init__(self, cin, cout, k, causal, up=False, tanh=False):
        super().__init__()
        self.causal, self.up, self.tanh = causal, up, tanh
        self.bf16 = False  # bf16-MFMA conv (the reference's fp16 autocast, in bf16); BatchNorm stays fp32
        self.conv = _ConvWeight(cin, cout, k)
        self.bn_layer = _BatchNorm(cout)
        self.sync_bn = False      # cross-rank BatchNorm statistics (convert_sync_batchnorm)
        self.sync_group = None    # process group of the synchronised statistics (None: the default group)

    def forward(self, x, xin=None, vout=False):
        """xin / vout: ConvStack's BatchNorm fold (ops.ConvBNActF) — x is the previous block's
        pre-BN output with its BatchNorm xin, and vout returns (pre-BN output, its BatchNorm)."""
        bn = self.bn_layer
        if xin is not None or vout:
            out = ops.conv_bn_act(x, self.conv.weight, bn.weight, bn.bias, bn.running_mean, bn.running_var,
                                  mode=0 if self.causal else 1, up=self.up, act="tanh" if self.tanh else "relu",
                                  momentum=bn.momentum, eps=bn.eps, bf16=self.bf16, xin=xin, vout=vout)
            if not getattr(bn, "_vt_batched", False):
                bn.num_batches_tracked.add_(1)
            return out
        if not self.training:   # model.eval(): running statistics (validation, frozen VAE, predict)
            return ops.conv_bn_eval(x, self.conv.weight, bn.weight, bn.bias, bn.running_mean, bn.running_var,
                                    mode=0 if self.causal else 1, up=self.up, act="tanh" if self.tanh else "relu",
                                    eps=bn.eps, bf16=self.bf16)
        if self.sync_bn:
            y = ops.sync_conv_bn_act(x, self.conv.weight, bn.weight, bn.bias, bn.running_mean, bn.running_var,
                                     mode=0 if self.causal else 1, up=self.up, act="tanh" if self.tanh else "relu",
                                     momentum=bn.momentum, eps=bn.eps, bf16=self.bf16, group=self.sync_group)
        else:
            y = ops.conv_bn_act(x, self.conv.weight, bn.weight, bn.bias, bn.running_mean, bn.running_var,
                                mode=0 if self.causal else 1, up=self.up, act="tanh" if self.tanh else "relu",
                                momentum=bn.momentum, eps=bn.eps, bf16=self.bf16)
        if not getattr(bn, "_vt_batched", False):   # else counted by SeqVaeTeb in one launch
            bn.num_batches_tracked.add_(1)
        return y


# the conv-stack BatchNorm fold (ConvStack): 1 hands inner blocks' pre-BN outputs to the next
# block's staging; off by default — with the apply's exact expression the staging costs more in
# the weight-gradient kernels than the apply passes it removes (7.88 vs 7.77 ms/step)
CONV_FOLD = int(os.environ.get("VAETEB_CONV_FOLD", "0"))


class ConvStack(nn.Sequential):
    """nn.Sequential of ConvBlocks (same children / state_dict keys).  Training with the bf16
    conv kernels: each inner block hands the next its pre-BN output and BatchNorm instead of
    y = act(BN(conv)) — the next block applies them while staging its windows, forward and
    weight gradient (ops.ConvBNActF) — so the inner outputs never round-trip through HBM and
    the separate BatchNorm-apply pass of every inner block is gone.  Same values as the
    unfolded stack (the staged operand is the y the apply pass would have written)."""

    def forward(self, x):
        blocks = list(self)
        if not (CONV_FOLD and len(blocks) > 1 and x.is_cuda and
                all(isinstance(b, ConvBlock) and b.training and b.bf16 == "bf16" and not b.sync_bn for b in blocks) and
                not any(b.tanh for b in blocks[:-1]) and   # the staging applies the inner blocks' ReLU
                # a folded block's backward needs its input's gradient (the fused bf16 path): every
                # inner output must require grad, else the unfolded stack runs (checked here, before
                # the forward updates the running statistics, not as an error in the backward)
                torch.is_grad_enabled() and all(b.conv.weight.requires_grad for b in blocks[:-1])):
            return super().forward(x)
        xin = None
        for i, blk in enumerate(blocks):
            if i == len(blocks) - 1:
                return blk(x, xin=xin)
            x, xin = blk(x, xin=xin, vout=True)


def convert_sync_batchnorm(module, process_group=None):
    """torch.nn.SyncBatchNorm.convert_sync_batchnorm for the HIP conv blocks: every
    ConvBlock's train-mode BatchNorm takes its statistics over all ranks of
    `process_group` (Lightning's sync_batchnorm=True, ref/model/graph_model.py:517).
    Same parameters / buffers / state_dict keys; returns the module."""
    for m in module.modules():
        if isinstance(m, ConvBlock):
            m.sync_bn = True
            m.sync_group = process_group
    return module


class LSTM(nn.Module):
    """nn.LSTM(input_size, hidden, num_layers, batch_first=True) parameters
    (same names), run by the HIP recurrence kernels."""

    def __init__(self, input_size, hidden_size=64, num_layers=4):
        super().__init__()
        self.input_size, self.hidden_size, self.num_layers = input_size, hidden_size, num_layers
        self.half = False   # 16-bit MFMA recurrences (SeqVaeTeb.set_lstm_precision)
        for l in range(num_layers):
            din = input_size if l == 0 else hidden_size
            w_ih = nn.Parameter(torch.empty(4 * hidden_size, din))
            w_hh = nn.Parameter(torch.empty(4 * hidden_size, hidden_size))
            nn.init.orthogonal_(w_ih)
            nn.init.orthogonal_(w_hh)                      # initialization(), vae_teb_model.py:60-70
            b_ih = nn.Parameter(torch.zeros(4 * hidden_size))
            b_hh = nn.Parameter(torch.zeros(4 * hidden_size))
            with torch.no_grad():
                b_hh[hidden_size:2 * hidden_size].fill_(1.0)
            setattr(self, f"weight_ih_l{l}", w_ih)
            setattr(self, f"weight_hh_l{l}", w_hh)
            setattr(self, f"bias_ih_l{l}", b_ih)
            setattr(self, f"bias_hh_l{l}", b_hh)

    def flat(self):
        out = []
        for l in range(self.num_layers):
            out += [getattr(self, f"weight_ih_l{l}"), getattr(self, f"weight_hh_l{l}"),
                    getattr(self, f"bias_ih_l{l}"), getattr(self, f"bias_hh_l{l}")]
        return out

    def forward(self, x):
        return ops.lstm(x, self.flat(), half=self.half)


def _seq1(m):
    s = nn.Sequential()
    s.add_module("0", m)
    return s


# ---------------------------------------------------------------- encoders
class SourceEncoder(nn.Module):
    """ref/model/vae_teb_model.py:589-721."""

    def __init__(self, input_channels=130):
        super().__init__()
        self.mlp = ResidualMLP(input_channels, geometric_schedule(130, 32, 5), final_activation=False)
        self.conv = ConvStack(*[ConvBlock(32, 32, k, causal=True) for k in (3, 5, 7)])
        self.fused_norm = LayerNorm(32)
        self.lstm_norm = LayerNorm(64)
        self.lstm = LSTM(32, 64, 4)
        self.pre_output = ResidualMLP(64, geometric_schedule(64, 32, 4), final_activation=True)
        self.mu_layer = ResidualMLP(32, geometric_schedule(32, 32, 4), final_activation=False)

    def forward(self, x):
        return _drain(self.stages(x))

    def stages(self, x):
        """forward() as a stage generator (fork_lockstep)."""
        h = self.mlp(x)
        yield
        h = self.conv(h)
        yield
        h = self.lstm(self.fused_norm(h))
        yield
        h = self.pre_output(self.lstm_norm(h))
        yield
        return self.mu_layer(h)


class TargetEncoder(nn.Module):
    """ref/model/vae_teb_model.py:406-575."""

    def __init__(self, scattering_channels=43, phase_channels=44):
        super().__init__()
        self.mlp_scattering = _seq1(ResidualMLP(scattering_channels, geometric_schedule(43, 16, 4),
                                                final_activation=False, activation="gelu"))
        self.mlp_phase = ResidualMLP(phase_channels, geometric_schedule(44, 16, 4), final_activation=False)
        self.conv_scattering = ConvStack(*[ConvBlock(16, 16, k, causal=True) for k in (3, 5, 7)])
        self.conv_phase = ConvStack(*[ConvBlock(16, 16, k, causal=True) for k in (3, 5, 7)])
        self.scatter_fused_norm = LayerNorm(16)
        self.phase_fused_norm = LayerNorm(16)
        self.lstm_norm = LayerNorm(64)
        self.cross_modal_fusion = ResidualMLP(32, geometric_schedule(32, 20, 5), final_activation=False)
        self.lstm = LSTM(20, 64, 4)
        self.pre_output = ResidualMLP(64, geometric_schedule(64, 32, 5), final_activation=True)
        self.mu_layer = ResidualMLP(32, geometric_schedule(32, 32, 32), final_activation=False)
        self.logvar_layer = ResidualMLP(32, geometric_schedule(32, 64, 4), final_activation=False)

    def forward(self, y_st, y_ph):
        return _drain(self.stages(y_st, y_ph))

    def stages(self, y_st, y_ph):
        """forward() as a stage generator (fork_lockstep)."""
        a, b = fork(lambda: self.scatter_fused_norm(self.conv_scattering(self.mlp_scattering(y_st))),
                    lambda: self.phase_fused_norm(self.conv_phase(self.mlp_phase(y_ph))))
        yield
        h = self.cross_modal_fusion(ops.cat_last([a, b]))
        yield
        h = self.lstm(h)
        yield
        h = self.pre_output(self.lstm_norm(h))
        yield
        return self.mu_layer(h), ops.clamp(self.logvar_layer(h), -10, 10)


class ConditionalEncoder(nn.Module):
    """ref/model/vae_teb_model.py:743-820."""

    def __init__(self, dim_hx=32, dim_hy=32):
        super().__init__()
        hd = geometric_schedule(dim_hx + dim_hy, 32, 8)
        self.mlp = ResidualMLP(dim_hx + dim_hy, hd[0:5], final_activation=True)
        self.fc_mu = ResidualMLP(hd[4], hd[5:], final_activation=False, use_skip_connection=False)
        self.fc_logvar = ResidualMLP(hd[4], hd[5:], final_activation=False, use_skip_connection=False)

    def forward(self, h_x, h_y):
        h = self.mlp(ops.cat_last([h_x, h_y]))
        mu, lv = fork(lambda: self.fc_mu(h), lambda: self.fc_logvar(h))
        return mu, lv


PRECISIONS = ("fp32", "bf16", "fp16")


class Decoder(nn.Module):
    """ref/model/vae_teb_model.py:823-929 with the head width R = 16*S."""

    SPEC = [(87, 77, 11, False), (77, 66, 9, True), (66, 55, 7, True), (55, 44, 5, False),
            (44, 33, 5, True), (33, 22, 3, True), (22, 11, 3, False), (11, 1, 3, False)]

    def __init__(self, latent_dim=32, sequence_length=300, head_precision="fp32"):
        super().__init__()
        self.sequence_length = sequence_length
        R = 16 * sequence_length
        self.linear = nn.Sequential(ResidualMLP(latent_dim, geometric_schedule(latent_dim, 50, 5)),
                                    ResidualMLP(50, geometric_schedule(50, 87, 5)))
        self.conv = ConvStack(*[ConvBlock(a, b, k, causal=False, up=u) for a, b, k, u in self.SPEC])
        self.output_mu = ResidualMLP(R, (R, R), final_activation=False, use_skip_connection=False)
        self.output_logvar = ResidualMLP(R, (R, R), final_activation=False, use_skip_connection=False)
        self.set_head_precision(head_precision)

    def set_head_precision(self, precision):
        """"fp32": every GEMM on the fp32 kernels (parity mode); "bf16" / "fp16": the
        R x R head GEMMs on 16-bit MFMA with fp32 accumulation — "fp16" is the reference's
        own autocast width (ref/model/graph_model.py:510,710; trained with the dynamic loss
        scale), "bf16" the MI355X default (no loss scale)."""
        if precision not in PRECISIONS:
            raise ValueError(f"head_precision must be one of {PRECISIONS}, got {precision!r}")
        self.head_precision = precision
        for head in (self.output_mu, self.output_logvar):
            for m in head.modules():
                if isinstance(m, Linear):
                    m.mfma = ops.h16_flag(precision != "fp32" and precision)

    def forward(self, z):
        lin = self.linear(z)                       # (B, S, 87)
        x = self.conv(lin)                         # (B, 16S, 1)
        x = x.reshape(x.shape[0], -1)              # flatten (B, 16S)
        mu, lv = fork_lockstep(self.output_mu.stages(x), self.output_logvar.stages(x),
                               main_first=LOCKSTEP_MAIN_FIRST == "all")
        return lin, mu, lv


class SeqVaeTeb(nn.Module):
    """Drop-in for ref/model/vae_teb_model.py:982-1192 (training path)."""

    def __init__(self, input_channels=76, sequence_length=300, latent_dim_source=32, latent_dim_target=32,
                 latent_dim_z=32, decimation_factor=16, warmup_period=30, scattering_channels=43,
                 phase_channels=44, cross_phase_channels=130, head_precision="fp32", concurrent_encoders=False,
                 conv_precision="fp32", mlp_precision="fp32", lstm_precision="fp32"):
        super().__init__()
        # the source and target encoders are independent until the conditional
        # encoder: on a GPU they can run on two HIP streams (their LSTM
        # recurrences use one workgroup per sample, a quarter of the chip each)
        self.concurrent_encoders = concurrent_encoders
        self.latent_dim_source, self.latent_dim_target, self.latent_dim_z = latent_dim_source, latent_dim_target, \
            latent_dim_z
        self.decimation_factor, self.warmup_period = decimation_factor, warmup_period
        self.source_encoder = SourceEncoder(cross_phase_channels)
        self.target_encoder = TargetEncoder(scattering_channels, phase_channels)
        self.conditional_encoder = ConditionalEncoder(latent_dim_source, latent_dim_target)
        self.decoder = Decoder(latent_dim_z, sequence_length, head_precision)
        self.set_conv_precision(conv_precision)
        self.set_mlp_precision(mlp_precision)
        self.set_lstm_precision(lstm_precision)

    def set_lstm_precision(self, precision):
        """"fp32": the exact-fp32 recurrences (parity mode); "16-mixed": the reference's
        own LSTM width under Lightning precision="16-mixed" / torch.amp autocast
        (ref/model/graph_model.py:510, :709-711) — f16 forward operands, bf16 backward
        operands (no loss scale needed), fp32 accumulation, cell state and outputs, on
        MFMA over 4-sample tiles (vt_lstm16_layer_*)."""
        if precision not in ("fp32", "16-mixed"):
            raise ValueError(f"lstm_precision must be 'fp32' or '16-mixed', got {precision!r}")
        self.lstm_precision = precision
        for m in self.modules():
            if isinstance(m, LSTM):
                m.half = precision == "16-mixed"

    def set_mlp_precision(self, precision):
        """"fp32": the ResidualMLP stacks on exact-fp32 MFMA (parity mode); "bf16" / "fp16":
        their Linear layers on 16-bit MFMA with fp32 accumulation, LayerNorm and reductions
        fp32 — the reference trains in fp16 autocast (ref/model/graph_model.py:510, :709-711);
        "fp16" is that width (with the trainer's loss scale), "bf16" the default."""
        if precision not in PRECISIONS:
            raise ValueError(f"mlp_precision must be one of {PRECISIONS}, got {precision!r}")
        self.mlp_precision = precision
        for m in self.modules():
            if isinstance(m, ResidualMLP):
                m.bf16 = ops.h16_flag(precision != "fp32" and precision)
        self._check_h16()

    def set_conv_precision(self, precision):
        """"fp32": exact-fp32 MFMA convs (parity mode); "bf16" / "fp16": 16-bit-MFMA convs
        with fp32 accumulation and fp32 BatchNorm — the reference trains in fp16 autocast
        (ref/model/graph_model.py:510, :709-711); "fp16" is that width, "bf16" the default."""
        if precision not in PRECISIONS:
            raise ValueError(f"conv_precision must be one of {PRECISIONS}, got {precision!r}")
        self.conv_precision = precision
        for m in self.modules():
            if isinstance(m, ConvBlock):
                m.bf16 = ops.h16_flag(precision != "fp32" and precision)
        self._check_h16()

    def set_head_precision(self, precision):
        """The decoder heads' precision (Decoder.set_head_precision), kept to one 16-bit format."""
        self.decoder.set_head_precision(precision)
        self._check_h16()

    def _check_h16(self):
        """One 16-bit operand format per model (the library's format is selected per op, but the
        optimizer writes every shadow of a step in one format): bf16 and fp16 do not mix."""
        fams = {p for p in (self.decoder.head_precision, getattr(self, "conv_precision", "fp32"),
                            getattr(self, "mlp_precision", "fp32")) if p != "fp32"}
        if len(fams) > 1:
            raise ValueError(f"head / conv / MLP precisions mix bf16 and fp16: {sorted(fams)}")
        self.h16_format = fams.pop() if fams else None

    @property
    def loss_scaling(self):
        """True when the model trains 16-bit fp16 operands: the trainer then runs GradScaler's
        dynamic loss scale (ref/model/graph_model.py:670, 718-726)."""
        return getattr(self, "h16_format", None) == "fp16"

    def forward(self, y_st, y_ph, x_ph, eps=None):
        if getattr(self, "h16_format", None) and x_ph.is_cuda:
            _lib.set_h16(self.h16_format == "fp16")   # the prepass shadows below are written in it
        prev = dict(_PAR)
        _PAR["on"], _PAR["next"] = bool(self.concurrent_encoders and x_ph.is_cuda), 1
        # conv weight gradients of this step's backward go to side stream GRAD_SIDE (off the
        # data-gradient chain; bit-identical, only their timing moves)
        ops.GRAD_STREAM = side_stream(torch.cuda.current_device(), GRAD_SIDE) if _PAR["on"] else None
        # the head weight gradients go to side stream 1 (the source encoder's, idle
        # until the encoders' backward, long after the heads')
        # (not under hipGraph capture: with that extra branch, ROCm 7's graph
        # instantiation segfaults in hipStreamEndCapture — measured)
        cap_ok = CAPTURE_BRANCHES or not torch.cuda.is_current_stream_capturing()
        ops.HEAD_GRAD_STREAM = (side_stream(torch.cuda.current_device(), HEAD_GRAD_SIDE)
                                if _PAR["on"] and HEAD_GRAD_SIDE > 0 and cap_ok else None)
        ops.LSTM_GRAD_STREAM = (side_stream(torch.cuda.current_device(), LSTM_GRAD_SIDE)
                                if _PAR["on"] and LSTM_GRAD_SIDE > 0 and cap_ok else None)
        # (not under hipGraph capture: an extra side-stream branch at the start of the graph
        # makes ROCm 7's hipStreamEndCapture segfault, as the head-gradient branch below)
        if getattr(self, "_prepassed", False):
            self._prepassed = False            # done ahead of this forward (prepass())
            if not self.training:
                # the prepass counted a training step, but this forward runs in eval mode
                # (e.g. a frozen VAE switched by its classifier wrapper): take it back
                self._bn_counters().sub_(1)
        elif _PAR["on"] and self.training and PREPASS and not torch.cuda.is_current_stream_capturing():
            self._prepass()
        else:
            ops._PREPARED.clear()   # no stale shadow events outlive the forward they were made for
            if self.training:
                self._count_bn()
        if ops.MLP_PREP_BATCH and x_ph.is_cuda:
            self._mlp_prep(y_st.shape[0] * y_st.shape[1])
        try:
            return self._forward(y_st, y_ph, x_ph, eps)
        finally:
            _PAR.update(prev)
            for bn in getattr(self, "_bn_list", ()):
                bn._vt_batched = False   # counted by this forward's prepass only

    def _mlp_prep(self, rows):
        """The 16-bit weight images of every fused 16-bit ResidualMLP stack of this model (all run on
        the B*S rows) in one launch at the start of the forward (ops.mlp_prep_batch): each stack's
        forward then skips its own image pass.  Same images, same bits."""
        key = (self.mlp_precision, rows)
        if getattr(self, "_mlp_prep_key", None) != key:   # the module walk once per setting
            self._mlp_prep_key = key
            self._mlp_prep_mods = [m for m in self.modules() if isinstance(m, ResidualMLP) and m.bf16 and m.fused]
        stacks = [fs for fs in (m._fused_spec() for m in self._mlp_prep_mods) if fs is not None]
        ops._MLP_PREPPED.clear()   # images of an earlier forward that never ran are stale
        ops.mlp_prep_batch(stacks, rows)

    def _bn_counters(self):
        """The num_batches_tracked buffers of every BatchNorm as views of one int64
        vector (state_dict keys and values unchanged), so a training forward counts
        all 17 in one launch instead of one add per block.  Rebound whenever a
        buffer was replaced (.to(), load_state_dict(assign=True))."""
        bns = getattr(self, "_bn_list", None)
        if bns is None:
            bns = self._bn_list = [m.bn_layer for m in self.modules() if isinstance(m, ConvBlock)]
        flat, views = getattr(self, "_bn_flat", None), getattr(self, "_bn_views", None)
        if flat is None or len(views) != len(bns) or any(
                bn._buffers["num_batches_tracked"] is not v for bn, v in zip(bns, views)):
            dev = bns[0].num_batches_tracked.device
            flat = torch.stack([bn.num_batches_tracked.detach().to(dev) for bn in bns])
            views = [flat[i] for i in range(len(bns))]
            for bn, v in zip(bns, views):
                bn._buffers["num_batches_tracked"] = v
            self._bn_flat, self._bn_views = flat, views
        return flat

    def _count_bn(self):
        """All BatchNorm step counters of this training forward in one launch."""
        self._bn_counters().add_(1)
        for bn in self._bn_list:
            bn._vt_batched = True    # the blocks of this forward skip their own count

    def prepass(self):
        """Run the weight-only prepass now, ahead of the next training forward (the
        trainer calls it before the front-end, so it overlaps that); the forward
        then skips its own."""
        if getattr(self, "_prepassed", False):
            return   # already done for the coming forward (counted once)
        if (self.concurrent_encoders and self.training and PREPASS and torch.cuda.is_available()
                and next(self.parameters()).is_cuda and not torch.cuda.is_current_stream_capturing()):
            self._prepass()
            self._prepassed = True

    def _prepass(self):
        """Weight-only work of the forward on a side stream at its start: the bf16
        shadows of the MFMA heads and bf16 convs, and the BatchNorm step counters
        (ops.prepare_shadows)."""
        key = (self.decoder.head_precision, self.conv_precision)
        if getattr(self, "_prep_key", None) != key:   # module lists walked once per precision setting
            self._prep_key = key
            self._prep_heads = [m for h in (self.decoder.output_mu, self.decoder.output_logvar)
                                for m in h.modules() if isinstance(m, Linear) and m.mfma
                                and ops.mfma_ok(m.in_features, m.out_features)]
            self._prep_convs = [m for m in self.modules() if isinstance(m, ConvBlock) and m.bf16]
        heads = [m.weight for m in self._prep_heads]
        convs = [m.conv.weight for m in self._prep_convs]
        flat = self._bn_counters()
        ops.prepare_shadows(heads, convs, side_stream(torch.cuda.current_device(), PREPASS_SIDE),
                            extra=lambda: flat.add_(1))
        for bn in self._bn_list:
            bn._vt_batched = True    # the blocks of the next forward skip their own count

    def _forward(self, y_st, y_ph, x_ph, eps):
        (mu_y, logvar_y_full), mu_x = fork_lockstep(self.target_encoder.stages(y_st, y_ph),
                                                    self.source_encoder.stages(x_ph),
                                                    main_first=LOCKSTEP_MAIN_FIRST in ("enc", "all"))
        logvar_y_prior, c_logvar = torch.split(logvar_y_full, self.latent_dim_target, dim=-1)
        mu_c, logvar_post = self.conditional_encoder(mu_x, c_logvar)
        if eps is None:
            eps = torch.randn_like(mu_c)            # reparameterize, vae_teb_model.py:1046-1050
        lvp = logvar_y_prior.contiguous()
        z, mu_post, kld = ops.latent(mu_c, logvar_post, mu_y, lvp, eps)
        linear_output, mu_pr, logvar_pr = self.decoder(z)
        return {"z": z, "linear_output": linear_output, "mu_pr": mu_pr, "logvar_pr": logvar_pr,
                "mu_prior": mu_y, "logvar_prior": lvp, "mu_post": mu_post, "logvar_post": logvar_post,
                "_kld": kld}

    def compute_loss(self, forward_outputs, y_st, y_ph, y_raw, compute_kld_loss=True, beta=1.0):
        """ref/model/vae_teb_model.py:1133-1192 (same keys)."""
        if y_raw.dim() == 3 and y_raw.size(-1) == 1:
            y_raw = y_raw.squeeze(-1)
        nll, mse = ops.output_losses(forward_outputs["mu_pr"], forward_outputs["logvar_pr"], y_raw,
                                     forward_outputs["linear_output"], y_st, y_ph)
        kld = forward_outputs["_kld"] if compute_kld_loss else torch.zeros((), device=y_raw.device)
        rec = mse + nll
        return {"reconstruction_loss": rec, "mse_loss": mse, "nll_loss": nll, "kld_loss": kld,
                "total_loss": rec + beta * kld, "classification_loss": None}

    @staticmethod
    def kld_elementwise(mu_prior, logvar_prior, mu_post, logvar_post):
        """_kld_loss(reduce_mean=False), ref/model/vae_teb_model.py:1071-1082."""
        return 0.5 * (logvar_prior - logvar_post - 1 + (logvar_post.exp() + (mu_post - mu_prior) ** 2)
                      / logvar_prior.exp())

    def _kld_loss(self, mu_prior, logvar_prior, mu_post, logvar_post, reduce_mean=True):
        """ref/model/vae_teb_model.py:1052-1082: KL(q || p) per (sample, step, latent);
        reduce_mean: summed over the latent dimension, averaged over (sample, step)."""
        kld = self.kld_elementwise(mu_prior, logvar_prior, mu_post, logvar_post)
        return kld.sum(dim=-1).mean() if reduce_mean else kld

    def encode(self, y_st, y_ph, x_ph):
        """The posterior / prior half of forward() (encoders + conditional encoder,
        ref/model/vae_teb_model.py:1097-1115): (mu_prior, logvar_prior, mu_post,
        logvar_post).  The reparameterisation and the decoder do not influence these."""
        prev = dict(_PAR)
        _PAR["on"], _PAR["next"] = bool(self.concurrent_encoders and x_ph.is_cuda), 1
        try:
            (mu_y, logvar_y_full), mu_x = fork_lockstep(self.target_encoder.stages(y_st, y_ph),
                                                        self.source_encoder.stages(x_ph))
            logvar_y_prior, c_logvar = torch.split(logvar_y_full, self.latent_dim_target, dim=-1)
            mu_c, logvar_post = self.conditional_encoder(mu_x, c_logvar)
        finally:
            _PAR.update(prev)
        return mu_y, logvar_y_prior.contiguous(), mu_c + mu_y, logvar_post

    def measure_transfer_entropy(self, y_st, y_ph, x_ph, reduce_mean=False):
        """ref/model/vae_teb_model.py:1194-1226: transfer entropy x -> z as the KL
        divergence between the posterior q(z | x, y) and the prior p(z | y), with the
        model put in eval mode (BatchNorm on its running statistics; the model stays
        in eval mode afterwards, as in the reference) and no gradients.  Same values
        as the reference's full forward: the decoder it also runs there does not enter
        the KL, so only the encoders and the conditional encoder run here.  Returns
        (B, S, latent) (reduce_mean=False) or the scalar mean of the latent sums.
        The reference's forward also draws the reparameterisation noise (torch.randn_like,
        :1046-1050); one draw of that shape is made and discarded here, so the device's
        random stream advances exactly as in the reference and every later draw (noise,
        dropout, sampling) stays aligned with it."""
        self.eval()
        with torch.no_grad():
            mu_p, lv_p, mu_q, lv_q = self.encode(y_st, y_ph, x_ph)
            torch.randn_like(lv_q)
            return self._kld_loss(mu_p, lv_p, mu_q, lv_q, reduce_mean=reduce_mean)

    @staticmethod
    def get_predictions(x, stride=16, new_C=4800):
        """ref/model/vae_teb_model.py:1228-1246: overlapping per-step windows x (B, N, C)
        placed at offsets i * stride of a (B, N, new_C) canvas (NaN elsewhere) and their
        NaN-mean over the steps (B, new_C)."""
        B, N, C = x.shape
        y = x.new_full((B, N, new_C), float("nan"))
        for i in range(N):
            start = i * stride
            if start >= new_C:
                break
            end = min(start + C, new_C)
            y[:, i, start:end] = x[:, i, :end - start]
        return y, torch.nanmean(y, dim=1)


class TinyVaeTeb(nn.Module):
    """Config 1 (BASELINE.json configs[0]): 2-layer causal conv
    encoder, latent 8, 2-layer reflect conv decoder on 256-pt windows."""

    def __init__(self):
        super().__init__()
        self.enc = ConvStack(ConvBlock(1, 16, 3, causal=True), ConvBlock(16, 16, 5, causal=True))
        self.mu = ResidualMLP(16, (8,), final_activation=False)
        self.logvar = ResidualMLP(16, (8,), final_activation=False)
        self.dec = ConvStack(ConvBlock(8, 16, 3, causal=False), ConvBlock(16, 2, 3, causal=False, tanh=True))

    def forward(self, x, eps):
        """x (B, 1, L) (reference layout) -> losses dict (NLL + KL with a
        standard-normal prior)."""
        xb = x.transpose(1, 2).contiguous()         # (B, L, 1)
        h = self.enc(xb)
        mu, lv = self.mu(h), self.logvar(h)
        zero = torch.zeros_like(mu)
        z, _, kld = ops.latent(mu, lv, zero, zero, eps)
        out = self.dec(z)                           # (B, L, 2)
        mu_r, lv_r = out[..., 0].contiguous(), out[..., 1].contiguous()
        nll, _ = ops.output_losses(mu_r, lv_r, x[:, 0].contiguous())
        return {"mu": mu, "logvar": lv, "mu_r": mu_r, "lv_r": lv_r, "kld": kld, "nll": nll, "total": nll + kld}
