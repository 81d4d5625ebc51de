"""LightSeqVaeTeb mirror (ref/model/pytorch_lightning_modules.py:401-564) and
checkpoint interchange (ref/model/graph_model.py:338-342, :381-390): host-side
checks, no GPU needed."""
import math

import pytest
import torch

from golden_util import det_fill_


def _light(**kw):
    from vaeteb.lightning import LightSeqVaeTeb
    from vaeteb.model import SeqVaeTeb
    return LightSeqVaeTeb(SeqVaeTeb(sequence_length=4), **kw)


@pytest.mark.parametrize("sched,epoch,expect", [
    ("linear", 0, 0.0), ("linear", 50, 0.5), ("linear", 500, 1.0), ("cyclic", 250, 0.25), ("cyclic", 1250, 0.25),
    ("constant", 7, 1e-5)])
def test_beta_schedules(sched, epoch, expect):
    m = _light(beta_schedule=sched, beta_const_val=1e-5)
    m.current_epoch = epoch
    m.on_train_epoch_start()
    assert math.isclose(m.hparams.beta, expect, rel_tol=1e-12, abs_tol=1e-15)
    assert m.logged["kld_beta"] == m.hparams.beta
    with pytest.raises(ValueError):
        _light(beta_schedule="bogus")._calculate_beta()


def test_cosine_warm_restarts_matches_torch():
    from vaeteb.lightning import CosineAnnealingWarmRestarts

    class _Opt:
        param_groups = [dict(lr=3e-4, initial_lr=3e-4)]
    ours = CosineAnnealingWarmRestarts(_Opt(), T_0=7, T_mult=2, eta_min=3e-6)
    p = torch.nn.Parameter(torch.zeros(1))
    topt = torch.optim.AdamW([p], lr=3e-4)
    ref = torch.optim.lr_scheduler.CosineAnnealingWarmRestarts(topt, T_0=7, T_mult=2, eta_min=3e-6)
    for _ in range(40):
        assert math.isclose(ours.get_last_lr()[0], ref.get_last_lr()[0], rel_tol=1e-12)
        topt.step()
        ref.step()
        ours.step()


def test_lightning_checkpoint_round_trip(tmp_path):
    """save_checkpoint writes the Lightning layout (state_dict under 'model.',
    epoch, hyper_parameters); load_from_checkpoint restores weights and hparams."""
    from vaeteb.lightning import LightSeqVaeTeb, load_pytorch_checkpoint
    from vaeteb.model import SeqVaeTeb
    a = _light(lr=2e-4, lr_milestones=[40, 80], beta_schedule="constant", beta_const_val=1e-5)
    det_fill_(a.model)
    a.current_epoch = 3
    path = tmp_path / "base.ckpt"
    a.save_checkpoint(path)
    ck = torch.load(path, weights_only=True)
    assert all(k.startswith("model.") for k in ck["state_dict"]) and ck["epoch"] == 3
    assert len(ck["state_dict"]) == len(a.model.state_dict())
    b = LightSeqVaeTeb.load_from_checkpoint(path, seqvae_teb_model=SeqVaeTeb(sequence_length=4), strict=True)
    assert b.hparams.lr == 2e-4 and b.hparams.lr_milestones == [40, 80] and b.current_epoch == 3
    for k, v in a.model.state_dict().items():
        assert torch.equal(v, b.model.state_dict()[k]), k
    # graph_model.load_pytorch_checkpoint layout: 'seqvae_model.' prefix
    p2 = tmp_path / "pt.ckpt"
    torch.save({"state_dict": {"seqvae_model." + k: v for k, v in a.model.state_dict().items()}, "epoch": 9}, p2)
    c = SeqVaeTeb(sequence_length=4)
    assert load_pytorch_checkpoint(c, p2) == 9
    for k, v in a.model.state_dict().items():
        assert torch.equal(v, c.state_dict()[k]), k


def test_reference_oracle_state_dict_loads_into_hip_model():
    """A state_dict with the reference's 594-key layout (the oracle carries the
    same names) loads strictly into the HIP SeqVaeTeb."""
    import sys
    from oracle import model_ref as M
    from vaeteb.model import SeqVaeTeb
    ref = det_fill_(M.SeqVaeTebRef(4))
    m = SeqVaeTeb(sequence_length=4)
    m.load_state_dict(ref.state_dict(), strict=True)
    assert len(ref.state_dict()) == len(m.state_dict())
    assert "torch" in sys.modules


def test_flat_adamw_loads_unpadded_moments():
    """Advisor r04: optimizer checkpoints written before the 64-float alignment of the >= 2^20
    element parameters (flat moments back to back) still load, remapped per parameter; the
    current layout round-trips; any other length raises."""
    from vaeteb.lightning import FlatAdamW
    torch.manual_seed(0)
    net = torch.nn.Sequential(torch.nn.Linear(1024, 1024), torch.nn.Linear(1024, 3))
    opt = FlatAdamW(net)
    s = opt.flat
    n_par = sum(n for _, n in s.offsets)
    assert s.numel > n_par                     # the 2^20-element weight was padded to 64 floats
    old_m, old_v = torch.randn(n_par), torch.randn(n_par)
    sd = {"param_groups": opt.param_groups, "step": torch.tensor([5], dtype=torch.int32), "exp_avg": old_m,
          "exp_avg_sq": old_v}
    opt.load_state_dict(sd)
    o_old = 0
    for (o, n), p in zip(s.offsets, s.params):
        assert torch.equal(s.m[o:o + n], old_m[o_old:o_old + n]) and torch.equal(s.v[o:o + n], old_v[o_old:o_old + n])
        o_old += n
    assert int(opt.step_dev.item()) == 5
    cur = opt.state_dict()
    opt2 = FlatAdamW(net)
    opt2.load_state_dict(cur)
    assert torch.equal(opt2.flat.m, s.m) and torch.equal(opt2.flat.v, s.v)
    with pytest.raises(ValueError, match="moments"):
        opt2.load_state_dict(dict(sd, exp_avg=torch.zeros(7), exp_avg_sq=torch.zeros(7)))
