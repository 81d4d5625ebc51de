"""Data-path drop-in for ref/hdf5_dataset/hdf5_dataset.py:
AttributeDict, CombinedHDF5Dataset, attribute_dict_collate and
create_optimized_dataloader with the reference's arguments, filters
(guid / cs_label / bg_label / epoch range / target label), trimming and
DistributedSampler sharding — with the normalisation moved out of the CPU
workers onto the GPU: GpuNormalizer runs normalize_tensor_data (:18-137) and
the (C, S) -> (S, C) transpose (:758-759) as one HIP kernel per field
(vt_fe_normalize / vt_normalize_raw), on the batch after it reaches HBM.

Storage back ends, same field names and per-sample layout as the reference's
files (create_hdf5_dataset.py / append_sample, hdf5_dataset.py:140-282):
  * HDF5 via h5py when it is importable.  h5py is NOT installed in this build
    image, so that reader is untested here (parity unpinned for the file format);
  * .npz files with the same fields (tests, environments without h5py).
Normalisation statistics: the stats_*.npz layout of vaeteb/data/ (the fields of
calculate_dataset_stats.py:364-444), or the reference's HDF5 stats file via h5py.
"""
import os
import threading
import warnings

import numpy as np
import torch
from torch.utils.data import DataLoader, Dataset

FEATURE_FIELDS = ("fhr_st", "fhr_ph", "fhr_up_ph")
RAW_FIELDS = ("fhr", "up")


class AttributeDict(dict):
    """ref/hdf5_dataset/hdf5_dataset.py:284-293."""

    def __getattr__(self, name):
        try:
            return self[name]
        except KeyError as e:
            raise AttributeError(name) from e

    def __setattr__(self, name, value):
        self[name] = value


def _have_h5py():
    try:
        import h5py  # noqa: F401
        return True
    except ImportError:
        return False


def _open_store(path):
    """Mapping field -> array-like indexed by sample (lazy for HDF5)."""
    if path.endswith(".npz"):
        return np.load(path, allow_pickle=False)
    if not _have_h5py():
        raise ImportError(f"reading {path} needs h5py, which is not installed (use .npz files with the same fields)")
    import h5py
    return h5py.File(path, "r", libver="latest", swmr=True)


def load_stats_file(path):
    """Normalisation statistics as {'<field>_mean': ..., '<field>_variance': ...}."""
    if path.endswith(".npz"):
        return dict(np.load(path, allow_pickle=False))
    if not _have_h5py():
        raise ImportError(f"reading the stats file {path} needs h5py (or pass the .npz stats layout)")
    import h5py
    out = {}
    with h5py.File(path, "r") as f:
        for field in RAW_FIELDS + FEATURE_FIELDS:
            if field in f:
                g = f[field]
                out[field + "_mean"] = np.asarray(g["mean"][()])
                out[field + "_variance"] = np.asarray(g["variance"][()] if "variance" in g else g["std"][()] ** 2)
    return out


class CombinedHDF5Dataset(Dataset):
    """ref/hdf5_dataset/hdf5_dataset.py:295-829 (same constructor, filters and
    sample fields).  Samples are returned UN-normalised with features in the
    file layout (C, S); GpuNormalizer (applied by create_optimized_dataloader)
    normalises and transposes the whole batch on the device.  Pass
    normalize_on_gpu=False to get raw features transposed to (S, C) instead."""

    def __init__(self, paths, load_fields=None, allowed_guids=None, cs_label=None, bg_label=None, epoch_min=None,
                 epoch_max=None, label=None, cache_size=2000, pin_memory=True, dtype=torch.float32, stats_path=None,
                 normalize_fields=None, trim_minutes=None, normalize_on_gpu=True):
        self.paths = [paths] if isinstance(paths, str) else list(paths)
        self.load_fields = None if load_fields is None else set(load_fields)
        self.allowed_guids = set(allowed_guids) if allowed_guids is not None else None
        self.cs_label, self.bg_label = cs_label, bg_label
        self.epoch_min, self.epoch_max, self.label = epoch_min, epoch_max, label
        self.cache_size, self.pin_memory, self.dtype = cache_size, pin_memory, dtype
        self.stats_path = stats_path
        self.normalize_fields = set(normalize_fields) if normalize_fields is not None else None
        self.normalize_on_gpu = normalize_on_gpu
        self.trim_minutes = trim_minutes
        self.trim_samples_raw = int(4 * 60 * trim_minutes) if trim_minutes is not None else 0
        self.trim_samples_decimated = self.trim_samples_raw // 16
        self.normalization_stats = load_stats_file(stats_path) if stats_path is not None else None
        self.normalization_enabled = self.normalization_stats is not None
        self._stores = [None] * len(self.paths)
        self._locks = [threading.Lock() for _ in self.paths]
        self._cache, self._cache_lock = {}, threading.Lock()
        self.index_map = []
        self._build_index()
        self._close_stores()   # the reference closes its file after indexing (ref :593-643)
        if not self.index_map:
            raise ValueError("No samples match the specified filters.")

    def _close_stores(self):
        for i, f in enumerate(self._stores):
            if f is not None and hasattr(f, "close"):
                f.close()
            self._stores[i] = None

    def __getstate__(self):
        # picklable for DataLoader workers (spawn): no open file handles, locks or cache
        st = dict(self.__dict__)
        st["_stores"] = [None] * len(self.paths)
        st["_locks"] = None
        st["_cache"], st["_cache_lock"] = {}, None
        return st

    def __setstate__(self, st):
        self.__dict__.update(st)
        self._locks = [threading.Lock() for _ in self.paths]
        self._cache_lock = threading.Lock()

    def gpu_normalizes(self, name):
        """True when `name` is normalised (and transposed) by GpuNormalizer on the
        device instead of here: the same condition GpuNormalizer applies."""
        return (self.normalization_enabled and self.normalize_on_gpu and name + "_mean" in self.normalization_stats
                and (self.normalize_fields is None or name in self.normalize_fields))

    def _store(self, i):
        with self._locks[i]:
            if self._stores[i] is None:
                self._stores[i] = _open_store(self.paths[i])
            return self._stores[i]

    def _build_index(self):
        """ref :593-643 (same filters, same order)."""
        for fidx, path in enumerate(self.paths):
            if not os.path.exists(path):
                warnings.warn(f"HDF5 file not found: {path}")
                continue
            f = self._store(fidx)
            guids = np.asarray(f["guid"][()] if not isinstance(f, np.lib.npyio.NpzFile) else f["guid"])
            epochs = np.asarray(f["epoch"][()] if not isinstance(f, np.lib.npyio.NpzFile) else f["epoch"])
            cs = np.asarray(f["cs_label"][()] if not isinstance(f, np.lib.npyio.NpzFile) else f["cs_label"])
            bg = np.asarray(f["bg_label"][()] if not isinstance(f, np.lib.npyio.NpzFile) else f["bg_label"])
            valid = np.ones(len(guids), dtype=bool)
            if self.epoch_min is not None:
                valid &= epochs >= self.epoch_min
            if self.epoch_max is not None:
                valid &= epochs <= self.epoch_max
            if self.cs_label is not None:
                valid &= cs == self.cs_label
            if self.bg_label is not None:
                valid &= bg == self.bg_label
            for i in np.nonzero(valid)[0]:
                g = guids[i].decode("utf-8") if isinstance(guids[i], bytes) else str(guids[i])
                if self.allowed_guids and g not in self.allowed_guids:
                    continue
                if self.label is not None and not np.any(np.asarray(f["target"][i]) == self.label):
                    continue
                self.index_map.append((fidx, int(i)))

    def __len__(self):
        return len(self.index_map)

    def get_normalization_stats(self):
        return self.normalization_stats

    def is_normalization_enabled(self):
        return self.normalization_enabled

    def __getitem__(self, idx):
        """ref :706-779; normalisation deferred to the GPU (see class doc)."""
        if self.cache_size > 0:
            with self._cache_lock:
                if idx in self._cache:
                    return self._cache[idx]
        fidx, si = self.index_map[idx]
        f = self._store(fidx)
        keys = list(f.files if isinstance(f, np.lib.npyio.NpzFile) else f.keys())
        fields = keys if self.load_fields is None else [k for k in self.load_fields if k in keys]
        out = {}
        tr, td = self.trim_samples_raw, self.trim_samples_decimated
        for name in fields:
            data = np.asarray(f[name][si])
            if self.trim_minutes is not None:
                if name in RAW_FIELDS:
                    data = data[tr:(-tr if tr > 0 else None)]
                elif name in FEATURE_FIELDS:
                    data = data[:, td:(-td if td > 0 else None)]
            if name == "guid":
                out[name] = data.item().decode("utf-8") if isinstance(data.item(), bytes) else str(data.item())
            elif name in ("cs_label", "bg_label"):
                out[name] = bool(data)
            else:
                t = torch.from_numpy(np.ascontiguousarray(data, dtype=np.float32)).to(self.dtype)
                if name in FEATURE_FIELDS and t.dim() == 2 and not self.gpu_normalizes(name):
                    # (C, S) -> (S, C) as the reference returns it (ref :758-759, normalised
                    # or not); GpuNormalizer transposes the fields it normalises
                    t = t.transpose(0, 1).contiguous()
                out[name] = t
        sample = AttributeDict(out)
        if self.cache_size > 0:
            with self._cache_lock:
                if len(self._cache) >= self.cache_size:
                    del self._cache[next(iter(self._cache))]
                self._cache[idx] = sample
        return sample


def attribute_dict_collate(batch):
    """ref :831-836: tensors stacked, other fields as lists."""
    out = AttributeDict()
    for k in batch[0]:
        vals = [b[k] for b in batch]
        out[k] = torch.stack(vals) if isinstance(vals[0], torch.Tensor) else vals
    return out


class GpuNormalizer:
    """normalize_tensor_data (ref :18-137) with the dataset's channel config
    (:385-393) + the (C, S) -> (S, C) transpose, on the device: one HIP launch
    per field (vt_fe_normalize for fhr_st / fhr_ph / fhr_up_ph, vt_normalize_raw
    for fhr / up).  Batches from CombinedHDF5Dataset(normalize_on_gpu=True)."""

    def __init__(self, stats, device=None, fields=None, log_eps=1e-6):
        from . import _lib
        self._lib = _lib
        self.device = torch.device(device) if device is not None else torch.device("cuda")
        self.log_eps = log_eps
        self.fields = set(fields) if fields is not None else None
        self.feat, self.raw = {}, {}
        for f in FEATURE_FIELDS:
            if f + "_mean" not in stats or not self._on(f):
                continue
            m = np.asarray(stats[f + "_mean"], np.float32).reshape(-1)
            v = np.asarray(stats[f + "_variance"], np.float32).reshape(-1)
            n = m.shape[0]
            kind = np.array([0] + [1] * (n - 1), np.int32) if f == "fhr_st" else np.full(n, 2, np.int32)
            self.feat[f] = (torch.from_numpy(kind).to(self.device), torch.from_numpy(m).to(self.device),
                            torch.from_numpy(np.sqrt(v)).to(self.device))
        for f in RAW_FIELDS:
            if f + "_mean" in stats and self._on(f):
                self.raw[f] = (float(np.asarray(stats[f + "_mean"])), float(np.sqrt(np.asarray(stats[f + "_variance"]))))

    def _on(self, f):
        return self.fields is None or f in self.fields

    def __call__(self, batch):
        L, st = self._lib, self._lib.stream()
        out = AttributeDict(batch)
        for f, (kind, m, s) in self.feat.items():
            if f not in batch:
                continue
            x = batch[f].to(self.device, torch.float32, non_blocking=True).contiguous()
            B, C, S = x.shape
            if C != m.numel():
                raise ValueError(f"{f}: {C} channels, stats for {m.numel()}")
            y = torch.empty((B, S, C), device=self.device)
            L.call("vt_fe_normalize", L.ptr(x), B, C, C, S, L.ptr(kind), L.ptr(m), L.ptr(s), self.log_eps, L.ptr(y),
                   C, 0, st)
            out[f] = y
        for f, (mean, std) in self.raw.items():
            if f not in batch:
                continue
            x = batch[f].to(self.device, torch.float32, non_blocking=True).contiguous()
            y = torch.empty_like(x)
            L.call("vt_normalize_raw", L.ptr(x), x.shape[0], x.shape[-1], x.shape[-1], mean, std, L.ptr(y), st)
            out[f] = y
        for k, v in batch.items():   # untouched tensor fields follow to the device
            if k not in out or out[k] is v:
                out[k] = v.to(self.device, non_blocking=True) if isinstance(v, torch.Tensor) else v
        return out


class _NormalizingLoader:
    """Iterates a DataLoader and normalises each batch on the device."""

    def __init__(self, loader, normalizer):
        self.loader, self.normalizer = loader, normalizer
        self.dataset, self.sampler, self.batch_size = loader.dataset, loader.sampler, loader.batch_size

    def __len__(self):
        return len(self.loader)

    def __iter__(self):
        for b in self.loader:
            yield self.normalizer(b)


def create_optimized_dataloader(hdf5_files, batch_size=32, num_workers=4, rank=0, world_size=1, stats_path=None,
                                normalize_fields=None, device=None, **dataset_kwargs):
    """ref :839-900 (same arguments, DistributedSampler(shuffle, drop_last) for
    world_size > 1).  With statistics, batches are normalised on `device`
    (default cuda) by GpuNormalizer instead of in the CPU workers."""
    from torch.utils.data.distributed import DistributedSampler
    ds = CombinedHDF5Dataset(paths=hdf5_files, stats_path=stats_path, normalize_fields=normalize_fields,
                             **dataset_kwargs)
    sampler, shuffle = None, True
    if world_size > 1:
        sampler = DistributedSampler(ds, num_replicas=world_size, rank=rank, shuffle=True, drop_last=True)
        shuffle = False
    loader = DataLoader(ds, batch_size=batch_size, shuffle=shuffle, sampler=sampler, num_workers=num_workers,
                        drop_last=False, prefetch_factor=2 if num_workers > 0 else None,
                        multiprocessing_context="spawn" if num_workers > 0 else None,
                        collate_fn=attribute_dict_collate)
    if ds.normalization_enabled and ds.normalize_on_gpu:
        return _NormalizingLoader(loader, GpuNormalizer(ds.normalization_stats, device, normalize_fields))
    return loader
