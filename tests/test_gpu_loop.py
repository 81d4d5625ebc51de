"""The epoch driver over the HIP Trainer (MI355X): vaeteb.loop.train_base_model_pytorch
(ref/model/graph_model.py:612-908) with vaeteb.train.Trainer as the step — train steps
(clip 1.0 + AdamW on the flat buffers), eval-mode validation (BatchNorm on its running
statistics after the train steps), the device-side fp64 loss sums and the per-epoch
CosineAnnealingLR — vs the same loop written out over the oracle model
(oracle/model_ref.py) with torch's AdamW / clip_grad_norm_ / CosineAnnealingLR, at the
golden S = 16 geometry in fp32.

Tolerance per epoch and loss: |ours - oracle fp64| <= 3 x the largest distance from the
fp64 loop of three fp32 oracle loops (the base run and two from one-ulp perturbed initial
weights) + 1e-4 relative.  AdamW makes this model's trajectory chaotic (rounding-level
gradient differences near 0 become lr-sized steps), so one fp32 run's distance from fp64
is luck: it measured 0.05 % on one host and 1.7 % on another for the same epoch."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

KEYS = ("total_loss", "reconstruction_loss", "kld_loss", "mse_loss", "nll_loss")
S, B, EPOCHS = 16, 4, 2


def _batches(seed, n):
    rng = np.random.Generator(np.random.PCG64(seed))
    out = []
    for _ in range(n):
        out.append({"fhr_st": rng.standard_normal((B, S, 43)).astype(np.float32),
                    "fhr_ph": rng.standard_normal((B, S, 44)).astype(np.float32),
                    "fhr_up_ph": rng.standard_normal((B, S, 130)).astype(np.float32),
                    "fhr": rng.standard_normal((B, 16 * S)).astype(np.float32),
                    "eps": rng.standard_normal((B, S, 32)).astype(np.float32)})
    return out


def _oracle_history(train, val, dtype, perturb=None):
    """ref/model/graph_model.py:612-908 over the oracle model (per-epoch averages)."""
    from golden_util import det_fill_, perturb_ulp_
    from oracle import model_ref as M
    ref = det_fill_(M.SeqVaeTebRef(S))
    if perturb is not None:
        perturb_ulp_(ref, perturb)
    ref = ref.to(dtype)
    opt = torch.optim.AdamW(ref.parameters(), lr=1e-3, weight_decay=1e-4, eps=1e-8, betas=(0.9, 0.98))
    sched = torch.optim.lr_scheduler.CosineAnnealingLR(opt, T_max=EPOCHS, eta_min=1e-3 * 0.01)
    T = lambda a: torch.from_numpy(a).to(dtype)
    hist = {f"{s}/{k}": [] for s in ("train", "val") for k in KEYS}

    def losses(b):
        fw = ref(T(b["fhr_st"]), T(b["fhr_ph"]), T(b["fhr_up_ph"]), T(b["eps"]))
        return ref.compute_loss(fw, T(b["fhr_st"]), T(b["fhr_ph"]), T(b["fhr"]), 1e-5)

    for _ in range(EPOCHS):
        ref.train()
        sums = np.zeros(len(KEYS))
        for b in train:
            opt.zero_grad()
            L = losses(b)
            L["total_loss"].backward()
            torch.nn.utils.clip_grad_norm_(ref.parameters(), 1.0)
            opt.step()
            sums += [float(L[k].detach()) for k in KEYS]
        ref.eval()
        vsums = np.zeros(len(KEYS))
        with torch.no_grad():
            for b in val:
                L = losses(b)
                vsums += [float(L[k]) for k in KEYS]
        sched.step()
        for i, k in enumerate(KEYS):
            hist[f"train/{k}"].append(sums[i] / len(train))
            hist[f"val/{k}"].append(vsums[i] / len(val))
    return hist


def test_epoch_driver_over_hip_trainer_vs_oracle_loop():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from golden_util import det_fill_
    from vaeteb.loop import train_base_model_pytorch
    from vaeteb.model import SeqVaeTeb
    from vaeteb.train import Trainer

    class EpsTrainer(Trainer):
        """The stored reparameterisation noise of each batch (the reference draws it with randn)."""

        def step(self, batch):
            return super().step(batch, eps=batch["eps"])

        def eval_losses(self, batch):
            return super().eval_losses(batch, eps=batch["eps"])

    train, val = _batches(31, 2), _batches(32, 1)
    to_dev = lambda b: {k: torch.from_numpy(v).cuda() for k, v in b.items()}
    m = det_fill_(SeqVaeTeb(sequence_length=S)).cuda()
    tr = EpsTrainer(m, lr=1e-3)
    hist = train_base_model_pytorch(tr, train, val, epochs=EPOCHS, to_device=to_dev)
    assert np.allclose(hist["lr"], [1e-3, 1e-3 * 0.01 + (1e-3 - 1e-3 * 0.01) * 0.5], rtol=1e-12, atol=0)
    h64 = _oracle_history(train, val, torch.float64)
    h32 = [_oracle_history(train, val, torch.float32, perturb=p) for p in (None, 1, 2)]
    for key in h64:
        for e in range(EPOCHS):
            a, x = hist[key][e], h64[key][e]
            spread = max(abs(h[key][e] - x) for h in h32)
            print(f"{key} epoch {e}: ours {a:.8f} oracle64 {x:.8f} oracle32 spread {spread:.3e}")
            assert abs(a - x) <= 3 * spread + 1e-4 * abs(x) + 1e-8, (key, e, a, x, spread)
