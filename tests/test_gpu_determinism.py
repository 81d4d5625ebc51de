"""Results must not depend on what earlier work left in memory (MI355X).

Two training runs of the same model from the same weights, the second after every cached
workspace (ops.WS), every cached bf16 weight shadow and the torch caching allocator's free
blocks were filled with NaN: losses, parameters and Adam moments must be equal bit for bit.
A kernel that reads workspace it did not write (a partial slab assumed zero, an unwritten
padding lane) or a shadow skipped as fresh when it was not, shows up here as a difference
or a NaN — the kind of fault that makes a fresh process and a long-running one disagree.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _poison():
    from vaeteb import ops
    for b in ops.WS.buf.values():
        b.fill_(float("nan"))
    for d in (ops._SHADOW, ops._CONV_SHADOW):
        for sh in d.values():
            for t in sh:
                t.fill_(float("nan"))
    # the allocator's free blocks: grab most of the cached free memory, fill it, release it
    torch.cuda.synchronize()
    free = torch.cuda.memory_reserved() - torch.cuda.memory_allocated()
    blocks = []
    size = 1 << 26
    while free > size and len(blocks) < 256:
        try:
            t = torch.empty(size // 4, device="cuda")
        except RuntimeError:
            break
        t.fill_(float("nan"))
        blocks.append(t)
        free -= size
    del blocks
    torch.cuda.synchronize()


def _run(precision, S, B, steps):
    from golden_util import det_fill_, traj_inputs
    from vaeteb.model import SeqVaeTeb
    from vaeteb.train import Trainer
    kw = dict(head_precision=precision, conv_precision=precision, mlp_precision=precision,
              lstm_precision="16-mixed" if precision == "bf16" else "fp32", concurrent_encoders=True)
    m = det_fill_(SeqVaeTeb(sequence_length=S, **kw)).cuda()
    tr = Trainer(m, lr=1e-3)
    losses = []
    for t in range(steps):
        y_st, y_ph, x_ph, y_raw, eps = [torch.from_numpy(a).cuda() for a in traj_inputs(S, B, t)]
        L = tr.step({"fhr_st": y_st, "fhr_ph": y_ph, "fhr_up_ph": x_ph, "fhr": y_raw}, eps=eps)
        losses.append(float(L["total_loss"]))
    torch.cuda.synchronize()
    return losses, tr.state.p.clone(), tr.state.m.clone(), tr.state.v.clone()


@pytest.mark.parametrize("precision", ["bf16", "fp32"])
def test_step_independent_of_memory_contents(precision):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    a = _run(precision, 256, 2, 3)
    _poison()
    b = _run(precision, 256, 2, 3)
    assert all(np.isfinite(b[0])), b[0]
    assert a[0] == b[0], (a[0], b[0])
    for x, y in zip(a[1:], b[1:]):
        assert torch.equal(x, y), ((x != y).sum().item(), x.numel())
