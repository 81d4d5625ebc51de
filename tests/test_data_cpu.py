"""Data-path drop-in (ref/hdf5_dataset/hdf5_dataset.py:284-900) on .npz files with
the reference's field names: filters, trimming, collate, DistributedSampler
sharding.  (The HDF5 reader needs h5py, absent here: file-format parity unpinned.)"""
import numpy as np
import pytest
import torch


def _write(path, n, seed, epoch0=0.0):
    rng = np.random.default_rng(seed)
    np.savez(path, fhr=rng.standard_normal((n, 4096)).astype(np.float32) + 140,
             up=rng.standard_normal((n, 4096)).astype(np.float32) + 10,
             fhr_st=np.abs(rng.standard_normal((n, 43, 256))).astype(np.float32),
             fhr_ph=rng.standard_normal((n, 44, 256)).astype(np.float32),
             fhr_up_ph=rng.standard_normal((n, 130, 256)).astype(np.float32),
             guid=np.array([f"g{seed}_{i}" for i in range(n)]), epoch=epoch0 + np.arange(n, dtype=np.float32),
             cs_label=(np.arange(n) % 2 == 0), bg_label=(np.arange(n) % 3 == 0),
             target=np.stack([np.full(256, i % 4) for i in range(n)]).astype(np.int64))
    return str(path)


@pytest.fixture
def files(tmp_path):
    return [_write(tmp_path / "a.npz", 10, 1), _write(tmp_path / "b.npz", 6, 2, epoch0=100.0)]


def test_filters_and_fields(files):
    from vaeteb.data import CombinedHDF5Dataset
    ds = CombinedHDF5Dataset(files, cache_size=0)
    assert len(ds) == 16
    s = ds[0]
    assert s.fhr.shape == (4096,) and s.fhr_st.shape == (256, 43) and s.fhr_up_ph.shape == (256, 130)
    assert s.guid == "g1_0" and s.cs_label is True and isinstance(s.bg_label, bool)
    assert len(CombinedHDF5Dataset(files, cs_label=True)) == 5 + 3
    assert len(CombinedHDF5Dataset(files, epoch_min=3, epoch_max=101)) == 7 + 2
    assert len(CombinedHDF5Dataset(files, allowed_guids=["g2_1", "g1_4"])) == 2
    assert len(CombinedHDF5Dataset(files, label=3)) == 2 + 1
    with pytest.raises(ValueError):
        CombinedHDF5Dataset(files, epoch_min=1e9)


def test_trim_and_collate(files):
    from vaeteb.data import CombinedHDF5Dataset, attribute_dict_collate
    ds = CombinedHDF5Dataset(files, trim_minutes=1, load_fields=["fhr", "fhr_ph", "guid"])
    s = ds[3]
    assert s.fhr.shape == (4096 - 2 * 240,) and s.fhr_ph.shape == (256 - 2 * 15, 44)
    raw = np.load(files[0])["fhr"][3]
    assert np.array_equal(s.fhr.numpy(), raw[240:-240])
    b = attribute_dict_collate([ds[i] for i in range(4)])
    assert b.fhr.shape == (4, 3616) and b.guid == ["g1_0", "g1_1", "g1_2", "g1_3"]


def test_distributed_sharding(files):
    from vaeteb.data import create_optimized_dataloader
    seen = []
    for rank in range(2):
        dl = create_optimized_dataloader(files, batch_size=3, num_workers=0, rank=rank, world_size=2,
                                         load_fields=["guid", "epoch"])
        dl.sampler.set_epoch(0)
        g = [x for b in dl for x in b.guid]
        assert len(g) == 8   # 16 samples, drop_last sharding
        seen.append(set(g))
    assert not (seen[0] & seen[1]) and len(seen[0] | seen[1]) == 16


def test_deferred_normalisation_keeps_file_layout(files, tmp_path):
    from vaeteb.data import CombinedHDF5Dataset
    stats = tmp_path / "stats.npz"
    d = dict(np.load(__import__("os").path.join(__import__("os").path.dirname(__file__), "..", "vae-teb_amd",
                                                "vaeteb", "data", "stats_j11q4t16_n4096.npz")))
    np.savez(stats, **d)
    ds = CombinedHDF5Dataset(files, stats_path=str(stats))
    assert ds.is_normalization_enabled() and ds[0].fhr_st.shape == (43, 256)   # (C, S): the GPU transposes
    ds2 = CombinedHDF5Dataset(files, stats_path=str(stats), normalize_on_gpu=False)
    assert ds2[0].fhr_st.shape == (256, 43)


def _stats(tmp_path):
    import os
    d = dict(np.load(os.path.join(os.path.dirname(__file__), "..", "vae-teb_amd", "vaeteb", "data",
                                  "stats_j11q4t16_n4096.npz")))
    p = tmp_path / "stats.npz"
    np.savez(p, **d)
    return str(p)


def test_fields_not_normalised_on_gpu_are_transposed(files, tmp_path):
    """A feature field that GpuNormalizer leaves alone (excluded by
    normalize_fields) still reaches the batch as (S, C), as in the reference
    (hdf5_dataset.py:758-759 transposes whether or not it normalises)."""
    from vaeteb.data import CombinedHDF5Dataset
    ds = CombinedHDF5Dataset(files, stats_path=_stats(tmp_path), normalize_fields={"fhr_st"})
    s = ds[0]
    assert s.fhr_st.shape == (43, 256)                 # normalised + transposed on the device
    assert s.fhr_ph.shape == (256, 44) and s.fhr_up_ph.shape == (256, 130)
    raw = np.load(files[0])["fhr_ph"][0]
    assert np.array_equal(s.fhr_ph.numpy(), raw.T)


def test_dataset_pickles_and_loads_with_workers(files, tmp_path):
    """The dataset holds no open handles or locks across pickling, so the
    default spawn DataLoader workers start (advisor round 1)."""
    import pickle
    from vaeteb.data import CombinedHDF5Dataset, create_optimized_dataloader
    ds = CombinedHDF5Dataset(files, cache_size=4)
    ds2 = pickle.loads(pickle.dumps(ds))
    assert len(ds2) == 16 and ds2[5].guid == ds[5].guid
    dl = create_optimized_dataloader(files, batch_size=4, num_workers=2, load_fields=["guid", "fhr_ph"])
    got = [b for b in dl]
    assert sum(len(b.guid) for b in got) == 16 and got[0].fhr_ph.shape == (4, 256, 44)
