"""Shared helpers for golden fixtures (test infrastructure, not product code).

`det_fill_` is the deterministic weight fill used by ``tools/gen_golden.py``
(which runs the *reference* ``SeqVaeTeb`` in the build container) and by the
parity tests (which load the same weights into the oracle and into the HIP
model).  Weights are regenerated from the state_dict key names, so fixtures do
not have to store the 67.8 M parameters of the S=256 model.

Rule per key (state_dict order is irrelevant, every key has its own stream):
  rng = numpy PCG64(seed = crc32(key))
  * ``running_mean`` -> 0, ``running_var`` -> 1, ``num_batches_tracked`` -> 0
  * LSTM ``weight_ih_l*/weight_hh_l*`` -> U(-1/sqrt(H), 1/sqrt(H))
  * LSTM ``bias_ih_l*/bias_hh_l*``     -> U(-0.05, 0.05); bias_hh[H:2H] += 1
    (forget-gate bias 1 as in ref/model/vae_teb_model.py:60-70)
  * other >=2-D ``weight`` (Linear/Conv1d) -> Xavier-uniform bound
    sqrt(6/(fan_in+fan_out)) (ref/model/vae_teb_model.py:55-59)
  * 1-D ``weight`` (LayerNorm/BatchNorm gamma) -> 1 + U(-0.1, 0.1)
  * 1-D ``bias`` -> U(-0.05, 0.05)
  * MultiheadAttention ``in_proj_weight`` -> Xavier-uniform over (3E, E),
    ``in_proj_bias`` -> U(-0.05, 0.05)
"""
import zlib

import numpy as np


def _fans(shape):
    if len(shape) == 2:
        return shape[1], shape[0]
    rf = int(np.prod(shape[2:]))
    return shape[1] * rf, shape[0] * rf


def det_value(key, shape, lstm_hidden=None):
    rng = np.random.Generator(np.random.PCG64(zlib.crc32(key.encode())))
    base = key.rsplit(".", 1)[-1]
    if base == "running_mean":
        return np.zeros(shape)
    if base == "running_var":
        return np.ones(shape)
    if base == "num_batches_tracked":
        return np.zeros(shape)
    if base.startswith("weight_ih_l") or base.startswith("weight_hh_l"):
        h = shape[1] if base.startswith("weight_hh") else shape[0] // 4
        b = 1.0 / np.sqrt(h)
        return rng.uniform(-b, b, size=shape)
    if base.startswith("bias_ih_l") or base.startswith("bias_hh_l"):
        v = rng.uniform(-0.05, 0.05, size=shape)
        if base.startswith("bias_hh_l"):
            h = shape[0] // 4
            v[h:2 * h] += 1.0
        return v
    if base == "in_proj_weight":          # nn.MultiheadAttention packed q|k|v projection
        b = np.sqrt(6.0 / (shape[0] + shape[1]))
        return rng.uniform(-b, b, size=shape)
    if base == "in_proj_bias":
        return rng.uniform(-0.05, 0.05, size=shape)
    if base == "weight" and len(shape) >= 2:
        fi, fo = _fans(shape)
        b = np.sqrt(6.0 / (fi + fo))
        return rng.uniform(-b, b, size=shape)
    if base == "weight":
        return 1.0 + rng.uniform(-0.1, 0.1, size=shape)
    if base == "bias":
        return rng.uniform(-0.05, 0.05, size=shape)
    raise KeyError(f"no deterministic rule for {key}")


def det_state_dict(shapes):
    """shapes: ordered mapping key -> tuple shape.  Returns key -> float64 array."""
    return {k: det_value(k, tuple(s)) for k, s in shapes.items()}


def det_fill_(module):
    """Fill a torch module's state in place (works for the reference model,
    the oracle restatement and the HIP model: identical key names)."""
    import torch
    with torch.no_grad():
        for k, t in module.state_dict().items():
            v = det_value(k, tuple(t.shape))
            t.copy_(torch.from_numpy(np.asarray(v)).to(t.dtype))
    return module
