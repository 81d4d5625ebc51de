"""Synthetic fetal-monitoring windows (SURVEY.md §8(d) "Synthetic inputs").

The reference trains on HDF5 windows built from clinical CTG records
(ref/hdf5_dataset/create_hdf5_dataset.py:380-418: ch0 = fhr, ch1 = up, 4 Hz).
Those records are not available, so every benchmark and parity case uses this
generator.  Each window depends only on its *global* sample index, so the data a
rank sees is independent of the number of GPUs (DistributedSampler-style
sharding, ref/hdf5_dataset/hdf5_dataset.py:879-887).
"""
import numpy as np

FS_HZ = 4.0
SEED_BASE = 20250808


def window(global_index, n=4096):
    """One (2, n) float32 window: row 0 = fhr (bpm), row 1 = up (mmHg)."""
    rng = np.random.Generator(np.random.PCG64(SEED_BASE + int(global_index)))
    t = np.arange(n, dtype=np.float64) / FS_HZ
    a1, f1, p1 = rng.uniform(5, 15), rng.uniform(0.003, 0.02), rng.uniform(0, 2 * np.pi)
    a2, f2, p2 = rng.uniform(1, 5), rng.uniform(0.05, 0.3), rng.uniform(0, 2 * np.pi)
    fhr = (140.0 + a1 * np.sin(2 * np.pi * f1 * t + p1) + a2 * np.sin(2 * np.pi * f2 * t + p2)
           + 1.5 * rng.standard_normal(n))
    up = np.full(n, 10.0)
    c = rng.uniform(0, 240)
    while c < t[-1] + 120:
        h, w = rng.uniform(20, 60), rng.uniform(15, 30)
        up += h * np.exp(-((t - c) ** 2) / (2 * w * w))
        c += rng.uniform(120, 240)
    up += 0.5 * rng.standard_normal(n)
    return np.stack([fhr, up]).astype(np.float32)


def batch(start, count, n=4096):
    """Windows [start, start+count) as a (count, 2, n) float32 array."""
    return np.stack([window(start + i, n) for i in range(count)])


def tiny_batch(count=8, n=256, seed=0):
    """Config-1 input: (count, 1, n) noisy sines, k ~ U{1..8}."""
    rng = np.random.Generator(np.random.PCG64(seed))
    t = np.arange(n, dtype=np.float64)
    out = np.empty((count, 1, n), np.float32)
    for i in range(count):
        k = rng.integers(1, 9)
        ph = rng.uniform(0, 2 * np.pi)
        out[i, 0] = np.sin(2 * np.pi * k * t / n + ph) + 0.05 * rng.standard_normal(n)
    return out
