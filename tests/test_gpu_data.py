"""GpuNormalizer (vt_fe_normalize / vt_normalize_raw on the device) vs the
REFERENCE's normalize_tensor_data outputs (tests/golden/normalize_*.npz, made by
executing ref/hdf5_dataset/hdf5_dataset.py:18-137 in tools/gen_golden.py), and the
normalising DataLoader end to end."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", ["normalize_j11q4t16_n4096", "normalize_j6q1t16_n4096"])
def test_gpu_normalizer_vs_reference(golden, name):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from vaeteb.data import GpuNormalizer
    g = golden(name)
    stats = {k: g[k] for k in g.files if k.endswith(("_mean", "_variance"))}
    norm = GpuNormalizer(stats, "cuda")
    batch = {f: torch.from_numpy(g["in_" + f]) for f in ("fhr", "up", "fhr_st", "fhr_ph", "fhr_up_ph")}
    out = norm(batch)
    for f in ("fhr", "up"):
        assert np.allclose(out[f].cpu().numpy(), g["out_" + f], rtol=1e-5, atol=1e-5), f
    for f in ("fhr_st", "fhr_ph", "fhr_up_ph"):
        got = out[f].cpu().numpy().transpose(0, 2, 1)      # (B, S, C) -> the reference's (B, C, S)
        assert np.allclose(got, g["out_" + f], rtol=1e-5, atol=1e-5), f


def test_normalizing_loader(tmp_path):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import os
    from test_data_cpu import _write
    from oracle import frontend_ref as F
    from vaeteb.data import create_optimized_dataloader
    files = [_write(tmp_path / "a.npz", 6, 1)]
    stats = os.path.join(os.path.dirname(__file__), "..", "vae-teb_amd", "vaeteb", "data", "stats_j11q4t16_n4096.npz")
    dl = create_optimized_dataloader(files, batch_size=4, num_workers=0, stats_path=stats)
    st = np.load(stats)
    raw = np.load(files[0])
    b = next(iter(dl))
    idx = [int(x.split("_")[1]) for x in b.guid]
    assert b.fhr_ph.is_cuda and b.fhr_ph.shape == (4, 256, 44)
    exp = F.normalize(raw["fhr_ph"][idx], "fhr_ph", st["fhr_ph_mean"], st["fhr_ph_variance"]).transpose(0, 2, 1)
    assert np.allclose(b.fhr_ph.cpu().numpy(), exp, rtol=1e-5, atol=1e-5)
