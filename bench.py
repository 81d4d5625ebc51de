#!/usr/bin/env python3
"""VAE-TEB training-step benchmark (BASELINE.json metric: train samples/sec + ELBO,
4096-pt windows, batch 256 per GPU, 1/2/4/8 MI355X).

A step = one pass of the north-star hot path over one batch resident in HBM:
raw windows x (B, 2, 4096) -> HIP front-end (Scattering1D + phase harmonics +
normalisation) -> SeqVaeTeb forward -> ELBO -> backward -> RCCL bucketed
gradient all-reduce (N > 1) -> grad-norm clip -> AdamW.  Data are synthetic
fetal-monitoring windows (vaeteb.synthetic; the clinical HDF5 records are not
available), weights are the reference architecture's random init.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--frontend j11|j6] [--batch B] [--workload c2|c4|c5]
  N > 1: either form works —
    python bench.py --gpus N          (starts N rank processes itself, vaeteb.train.spawn_local_ranks)
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N
  VAETEB_DIST_BACKEND=gloo: gloo instead of RCCL, ranks share the visible GPUs (one-GPU rehearsal)

Rank 0 prints ONE JSON line.  `roofline` is for the dominant kernel, timed
live with HIP events on its own stream inside the timed region; `cpu_baseline`
is the oracle (faithful CPU restatement) on a bounded sample, rank 0 / N = 1 only.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "vae-teb_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from vaeteb import _lib, synthetic  # noqa: E402
from vaeteb.frontend import FrontEnd, FrontEndPlan, load_stats  # noqa: E402
from vaeteb.model import SeqVaeTeb  # noqa: E402
from vaeteb.train import Trainer, init_distributed, spawn_local_ranks  # noqa: E402

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md, chip table)
FRONTENDS = {"j11": (11, 4, 16), "j6": (6, 1, 16)}


class KernelTimer:
    """HIP events around every launch of the named C-ABI entry points, recorded
    on the stream the kernels are launched on (the current stream); `flops`
    maps a name to a function of the call's arguments (MFMA accounting)."""

    def __init__(self, names, flops=None):
        self.names, self.pairs, self.enabled = set(names), {n: [] for n in names}, False
        self.flops, self.total_flops = flops or {}, {n: 0 for n in names}
        lib = _lib.lib()
        self._orig = lib.call

        def call(fname, *args):
            if self.enabled and fname in self.names:
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                rc = self._orig(fname, *args)
                e.record()
                self.pairs[fname].append((s, e))
                if fname in self.flops:
                    self.total_flops[fname] += self.flops[fname](*args)
                return rc
            return self._orig(fname, *args)
        lib.call = call

    def reset(self, enabled):
        self.pairs = {n: [] for n in self.names}
        self.total_flops = {n: 0 for n in self.names}
        self.enabled = enabled

    def mean_ms(self, name):
        ts = [s.elapsed_time(e) for s, e in self.pairs[name]]
        return sum(ts) / len(ts) if ts else float("nan"), len(ts)

    def total_ms(self, names):
        return sum(s.elapsed_time(e) for n in names for s, e in self.pairs[n])


# bf16 MFMA head GEMMs: 2*R*K*N flops per call (arguments as in include/vaeteb.h)
MFMA_CALLS = {
    "vt_mfma_linear_fwd": lambda X, R, K, W, N, *a: 2 * R * K * N,
    "vt_mfma_linear_bwd_data": lambda dY, R, N, W, K, *a: 2 * R * K * N,
    "vt_mfma_linear_bwd_weight": lambda dY, R, N, X, K, *a: 2 * R * K * N,
}
MFMA_PEAK_TFLOPS = 2500.0   # dense bf16 (MI355X_MICROARCH.md; no sparsity)


def profile_mfma(workload="c2"):
    """Decoder-head MFMA kernel time per step from the latest committed rocprofv3
    kernel-stats summary of this bench and workload (profiles/r*/kernel_stats_timed.csv for
    c2, kernel_stats_c4_timed.csv for c4): the sum of k_mfma_gemm + k_mfma_dw (+ the split
    reduce k_mfma_reduce of rounds <= 5) over the profiled steps (one k_adamw4 per step).
    Returns (ms per step, csv path) or (None, None)."""
    import csv
    import glob
    # latest round first (profiles/rNN); within a round, the file named in profiles/rNN/LATEST
    # when present, else the most recently written
    def key(f):
        d = os.path.dirname(f)
        latest = os.path.join(d, "LATEST")
        pinned = os.path.exists(latest) and open(latest).read().strip() == os.path.basename(f)
        return (os.path.basename(d), pinned, os.path.getmtime(f))
    if workload == "c4":
        files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "kernel_stats_c4_timed.csv")), key=key)
    else:
        files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "kernel_stats_step*.csv")) +
                       glob.glob(os.path.join(ROOT, "profiles", "r*", "kernel_stats_timed.csv")), key=key)
    for f in reversed(files):
        rows = list(csv.DictReader(open(f)))
        steps = sum(int(r["Calls"]) for r in rows if "k_adamw4" in r["Name"])
        ns = sum(float(r["TotalDurationNs"]) for r in rows if "k_mfma_" in r["Name"])
        if steps and ns:
            return ns / steps / 1e6, os.path.relpath(f, ROOT)
    return None, None


LSTM_KERNELS = {"recurrence": ("k_lstm16_fwd", "k_lstm16_bwd", "k_lstm_fwd", "k_lstm_bwd"),
                "weight gradient": ("k_sk_dw16", "k_sk_sum", "k_lstm_dw")}


def profile_lstm(ROOT_=None):
    """SURVEY.md §8(d) / BASELINE.md §4: the encoders' LSTMs are latency-bound and reported
    separately.  From the latest committed timed-step profile of this bench
    (profiles/rNN/kernel_stats_timed.csv: kernel time per step of every LSTM kernel) and its
    critical chain (critchain_timed.txt, tools/critchain.py: the LSTM recurrences' share of the
    step's longest dependent chain of kernels).  Returns a dict or None."""
    import csv
    import glob
    import re
    for d in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*")), reverse=True):
        ks, cc = os.path.join(d, "kernel_stats_timed.csv"), os.path.join(d, "critchain_timed.txt")
        if not (os.path.exists(ks) and os.path.exists(cc)):
            continue
        fam = {f: 0.0 for f in LSTM_KERNELS}
        per = {}
        for r in csv.DictReader(open(ks)):
            for f, pats in LSTM_KERNELS.items():
                if any(p in r["Name"] for p in pats):
                    fam[f] += float(r["PerStepNs"]) / 1e3
                    short = re.sub(r"\(.*", "", r["Name"].replace("(anonymous namespace)::", "")).replace("void ", "")
                    short = short.split("::")[-1]
                    per[short] = round(per.get(short, 0.0) + float(r["PerStepNs"]) / 1e3, 1)
        lines = open(cc).read().splitlines()
        m = re.search(r"critical chain \d+ kernels, ([\d.]+) us busy of ([\d.]+) us", "\n".join(lines[:3]))
        chain = [re.match(r"\s*([\d.]+) us\s+(.*)", l) for l in lines[2:]]
        on_chain = sum(float(c.group(1)) for c in chain if c and "lstm" in c.group(2))
        if not m or not any(fam.values()):
            continue
        busy = float(m.group(1))
        return {"bound": "latency (sequential recurrence: S = 256 dependent steps x 4 layers x 2 encoders, fwd + bwd)",
                "kernel_us_per_step": {f: round(v, 1) for f, v in fam.items()},
                "per_kernel_us_per_step": per,
                "critical_chain_us": round(on_chain, 1), "critical_chain_busy_us": busy,
                "critical_chain_share": round(on_chain / busy, 4),
                "source": os.path.relpath(ks, ROOT) + " + " + os.path.relpath(cc, ROOT)}
    return None


# algorithmic HBM bytes per sample of the whole step (c2, S = 256):
# front-end raw read + analytic-signal write and read + feature write, VAE activations
# (4,161,024 leaf activation elements per sample x 2 B x 4 passes, measured with hooks on
# the J11 model) and parameter / optimizer traffic 46 B x P per step over the batch.
ACT_ELEMS_PER_SAMPLE = 4_161_024


def step_bytes_per_sample(plan, fe, n_params, batch):
    N, F = plan.N, plan.n_filters
    front = 2 * N * 4 + 2 * (2 * F * N * 8) + (fe.C_st + fe.C_ph + fe.C_x) * plan.S * 4
    return front + ACT_ELEMS_PER_SAMPLE * 2 * 4 + 46 * n_params / batch


def pmc_traffic(kernel, fname="pmc_traffic.json"):
    """HBM bytes per launch of the roofline kernel from the latest committed
    rocprofv3 PMC measurement (profiles/r*/pmc_traffic.json — pmc_traffic_c5.json for the
    c5 workload — written by tools/pmc_traffic.py from separate FETCH_SIZE / WRITE_SIZE
    passes of this same bench command), or None."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", fname)))
    for f in reversed(files):
        d = json.load(open(f))
        if d.get("kernel") == kernel:
            return d["traffic_bytes_per_launch"], os.path.relpath(f, ROOT)
    return None, None


# kernel families of SURVEY.md §8(d)'s "rocprof-reported HBM GB/s for the scattering / conv kernels"
PMC_FAMILIES = {"conv fwd (k_cfw16, k_conv_bf16)": ("k_cfw16", "k_conv_bf16<"),
                "conv bwd-data (k_cbd16)": ("k_cbd16",),
                "conv weight grad (k_cdw16, k_conv_dw_bf16, split sums)": ("k_cdw16", "k_conv_dw_bf16", "k_sum_splits"),
                "BatchNorm (k_bn_*, k_col_partial4)": ("k_bn_", "k_col_partial4"),
                "scattering / wavelets (k_fe_wavelet8k, k_fe_spectrum, k_fe_lowpass)": ("k_fe_wavelet8k", "k_fe_spectrum",
                                                                                         "k_fe_lowpass"),
                "phase pairs (k_fe_pairs8k*)": ("k_fe_pairs8k",)}


def pmc_kernels():
    """Per-family HBM GB/s of the step's kernels from the latest committed per-kernel PMC file
    (profiles/r*/pmc_kernels.json: tools/pmc_traffic.py --kernels over separate FETCH_SIZE /
    WRITE_SIZE passes of this bench; durations = average launches in the timed steps of a
    kernel trace of the same command, tools/step_stats.py): bytes per step / kernel time per
    step, and that as a fraction of 8 TB/s."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "pmc_kernels.json")))
    if not files:
        return None
    d = json.load(open(files[-1]))
    out = {}
    for fam, pats in PMC_FAMILIES.items():
        byt = ns = 0.0
        for name, e in d["kernels"].items():
            if any(p in name for p in pats) and e.get("avg_launch_ns") and e.get("ms_per_step"):
                launches = e["ms_per_step"] * 1e6 / e["avg_launch_ns"]
                byt += e["traffic_bytes_per_launch"] * launches
                ns += e["ms_per_step"] * 1e6
        if ns:
            out[fam] = {"hbm_bytes_per_step": round(byt), "kernel_ms_per_step": round(ns / 1e6, 4),
                        "hbm_GBps": round(byt / ns, 1), "frac": round(byt / ns / HBM_PEAK_GBS, 4)}
    return {"families": out, "source": os.path.relpath(files[-1], ROOT),
            "method": "PMC FETCH_SIZE x2 + WRITE_SIZE per launch x launches per timed step / kernel time per step"}


def cpu_baseline(frontend_cfg, batch=8, threads=None, classifier=False):
    """Faithful CPU restatement (oracle): front-end called twice per window with
    all 903 pairs then masked (create_hdf5_dataset.py:418-441), torch.fft as in
    the reference, + SeqVaeTeb(S=256) fwd/bwd/clip/AdamW on torch-CPU fp32."""
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle import frontend_ref as F
    from oracle import model_ref as M
    threads = threads or min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    J, Q, T = frontend_cfg
    F.FFT_ENGINE = "torch"
    fe = F.PhaseFrontEnd(J, Q, T, 4096)
    pm, cm = fe.masks()
    x = synthetic.batch(10_000_000, batch, 4096)
    model = M.SeqVaeTebRef(256)
    t0 = time.perf_counter()
    rp = fe.forward(x, compute_phase=True)
    rc = fe.forward(x, compute_phase=False, compute_cross_phase=True)
    st = load_stats(J, Q, T)
    y_st = F.normalize(rp["scattering"], "fhr_st", st["fhr_st_mean"], st["fhr_st_variance"])
    y_ph = F.normalize(rp["phase_corr"][:, pm], "fhr_ph", st["fhr_ph_mean"], st["fhr_ph_variance"])
    x_ph = F.normalize(rc["cross_phase_corr"][:, cm], "fhr_up_ph", st["fhr_up_ph_mean"], st["fhr_up_ph_variance"])
    y_raw = F.normalize(x[:, 0], "fhr", st["fhr_mean"], st["fhr_variance"])
    tt = lambda a: torch.from_numpy(np.ascontiguousarray(a.transpose(0, 2, 1)))
    b = dict(y_st=tt(y_st), y_ph=tt(y_ph), x_ph=tt(x_ph), y_raw=torch.from_numpy(y_raw))
    if classifier:
        from oracle import classifier_ref as C
        clf = C.InceptionTimeClassifier(dropout=0.2).train()
        params = list(model.parameters()) + list(clf.parameters())
        out = C.seqvae_classifier_loss(model, clf, b["y_st"], b["y_ph"], b["x_ph"],
                                       torch.randint(0, 2, (batch,)), b["y_raw"], torch.randn(batch, 256, 32))
        out["total_loss"].backward()
        torch.nn.utils.clip_grad_norm_(params, 1.0)
        torch.optim.AdamW(params, lr=1e-3, weight_decay=1e-4, eps=1e-8, betas=(0.9, 0.98)).step()
    else:
        M.train_step(model, b, torch.randn(batch, 256, 32), 1e-5)
    dt = time.perf_counter() - t0
    F.FFT_ENGINE = "numpy"
    return {"value": round(batch / dt, 4), "unit": "samples/s", "cores": threads, "kind": "port",
            "sample": f"1 faithful CPU step at batch {batch}: front-end x2 calls with all 903 pairs + "
                      f"SeqVaeTeb(S=256){' + classifier' if classifier else ''} fwd/bwd/clip/AdamW, "
                      f"torch threads={threads}, {dt:.1f} s"}


OUT = sys.stdout


def _json_stdout():
    """The bench prints ONE JSON line on stdout (rank 0), but native libraries write there too
    (RCCL's init banner on the first collective): fd 1 is pointed at stderr for the run and the
    JSON line goes to a duplicate of the original stdout."""
    sys.stdout.flush()
    saved = os.dup(1)
    os.dup2(2, 1)
    return os.fdopen(saved, "w")


def run_c5(args, rank, world, dev):
    """Config 5 (BASELINE.json configs[4]): long-sequence stress, front-end only —
    Scattering1D(J=8, Q=12, T=256, order 2) on 16384-point windows, batch 64 per
    GPU; samples are independent, so N GPUs run N replicas on disjoint samples
    with no collective (weak scaling).  A step = one batch x (B, 16384) resident
    in HBM -> S (B, 337, 64) through the level-grouped HIP cascade."""
    from vaeteb.scattering import Scattering1D
    B, N = args.batch if args.batch != 256 else 64, 16384
    sc = Scattering1D(J=8, shape=N, Q=12, max_order=2, T=256)
    pool = [torch.from_numpy(synthetic.batch((rank * 2 + i) * B, B, N)[:, 0].copy()).to(dev) for i in range(2)]
    # dominant kernel: vt_scat_mod_spec (fold + ifft -> |.| -> fft per (sample, filter) row);
    # algorithmic bytes = distinct source rows read once (B x a_rows x n c64) + spectra written (B x P x n/k c64)
    work = {"vt_scat_mod_spec": lambda A, Bb, a_rows, n, a_idx, pool_, f_off, P, k, *a: 8 * Bb * (a_rows * n + P * n // k)}
    timer = KernelTimer(list(work), flops=work)
    for i in range(args.warmup):
        sc(pool[i % 2])
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    _lib.call("vt_bucket_marker", 0, _lib.stream())   # timed-region markers (tools/step_stats.py)
    torch.cuda.synchronize()
    timer.reset(True)
    t0 = time.perf_counter()
    for i in range(args.steps):
        S, _ = sc(pool[i % 2])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    _lib.call("vt_bucket_marker", 0, _lib.stream())
    timer.enabled = False
    if world > 1:
        t = torch.tensor([dt], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = t.item()
    k_ms, k_n = timer.mean_ms("vt_scat_mod_spec")
    k_bytes = timer.total_flops["vt_scat_mod_spec"] / max(k_n, 1)
    achieved = k_bytes / (k_ms * 1e-3) / 1e9
    # PMC traffic of the same kernel from separate FETCH_SIZE / WRITE_SIZE passes of this command
    # (profiles/rNN/pmc_traffic_c5.json): an average over the launches of the cascade's levels,
    # quoted for the default geometry only
    traffic, traffic_src = pmc_traffic("k_scat_mod_spec", "pmc_traffic_c5.json") if B == 64 else (None, None)
    out = {"metric": "scattering samples/sec, Scattering1D(J=8, Q=12) 16384-pt windows, batch 64/GPU",
           "value": round(args.steps * B * world / dt, 3), "unit": "samples/s", "n_gpus": world, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 3), "higher_is_better": True,
           "scaling": "weak", "vs_baseline": None, "dtype": "fp32 (complex64)", "data": "synthetic",
           "config": {"workload": "c5: Scattering1D J=8 Q=12 T=256 order 2, N=16384 (n_pad 32768) -> (B, 337, 64), "
                                  f"batch {B}/GPU, replicas (no collective)", "global_batch": B * world,
                      "seq_len": N, "parallelism": f"replicas{world}"},
           "roofline": {"bound": "hbm", "kernel": "vt_scat_mod_spec (k_scat_mod_spec)", "achieved": round(achieved, 1),
                        "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                        "traffic": traffic, "traffic_unit": "bytes/launch (PMC FETCH_SIZE x2 + WRITE_SIZE)",
                        "traffic_source": traffic_src, "avg_launch_ms": round(k_ms, 4), "launches": k_n,
                        "algorithmic_bytes": round(k_bytes)},
           "checksum": float(S.double().abs().sum().item())}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        sys.path.insert(0, ROOT)
        from oracle import frontend_ref as F
        xs = pool[0].cpu().numpy()   # the whole batch
        # the reference's own engine (torch.fft, kymatio's torch backend) on the box's host cores
        threads = min(16, os.cpu_count() or 1)
        torch.set_num_threads(threads)
        F.FFT_ENGINE = "torch"
        t0 = time.perf_counter()
        F.scattering1d(xs, 8, 12, 256, max_order=2)
        dtc = time.perf_counter() - t0
        F.FFT_ENGINE = "numpy"
        out["cpu_baseline"] = {"value": round(len(xs) / dtc, 4), "unit": "samples/s", "cores": threads,
                               "kind": "port",
                               "sample": f"oracle Scattering1D order 2 (torch.fft engine, {threads} threads) on "
                                         f"{len(xs)} of the same windows, {dtc:.1f} s"}
    if rank == 0:
        print(json.dumps(out), file=OUT, flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", choices=["c2", "c4", "c5"], default="c2",
                    help="c2: the training step (BASELINE.json metric, default); c4: the same step with the "
                         "classification head trained jointly (CE + 0.1 ELBO); c5: long-sequence scattering front-end")
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=256, help="per-GPU batch")
    ap.add_argument("--frontend", choices=list(FRONTENDS), default="j11")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-batch", type=int, default=32)
    ap.add_argument("--graph", action="store_true",
                    help="= --mode graph: the model step replayed as a captured hipGraph (double-buffered, "
                         "front-end one step ahead)")
    ap.add_argument("--mode", choices=["auto", "eager", "native", "graph"], default="auto",
                    help="auto (default): native for c2 at any GPU count (the eager step's ~190 C-ABI calls from "
                         "Python take about as long as the GPU work; with several GPUs the replay is enqueued in "
                         "ranges split at the gradient buckets' markers, each bucket's RCCL all-reduce issued as "
                         "soon as its writers are enqueued, overlapping the rest of the backward), eager for c4 "
                         "(host-side dropout seeds); native: the step captured once and replayed by the library's "
                         "multi-stream executor (vt_stepgraph_*); graph: hipGraphLaunch; eager: every op from Python")
    ap.add_argument("--ddp-probe", action="store_true",
                    help="N = 1 with the data-parallel machinery: a single-rank RCCL process group, gradient "
                         "buckets and their all-reduces, the world > 1 stream budget (main + 2 side streams) and "
                         "the segmented replay -- the per-GPU cost of the DDP step without the exchange itself")
    ap.add_argument("--reduce-bf16", action="store_true",
                    help="reduce the gradient buckets in bf16 (fp32 master gradients; the reference reduces fp32)")
    ap.add_argument("--native", action="store_true", help="= --mode native")
    ap.add_argument("--streams", type=int, default=4, help="--native: executor streams")
    ap.add_argument("--fe-in-graph", type=int, default=0,
                    help="native: 1 = the front-end is captured into the step too (raw windows are the "
                         "static input), so the executor runs the cross pairs beside the target encoder as the eager "
                         "step does; the roofline kernel is then timed in eager steps after the timed region")
    ap.add_argument("--overlap-adam", type=int, default=0,
                    help="native: 1 = the step captured without AdamW, which runs after each replay on a side "
                         "stream, overlapping the next batch's front-end (independent of the weights)")
    ap.add_argument("--overlap-fe", action="store_true",
                    help="--native: run the next batch's front-end one step ahead on its own stream (as --graph) "
                         "instead of inline before each replay")
    ap.add_argument("--prefetch", action="store_true",
                    help="eager mode: overlap the next batch's front-end with the current step on its own streams "
                         "(measured slower on MI355X: the front-end's LDS-heavy workgroups delay the latency-bound "
                         "step; default off)")
    ap.add_argument("--overlap-update", action="store_true",
                    help="eager mode: start the next batch's front-end after the backward, overlapping the "
                         "memory-bound clip + AdamW of the current step")
    ap.add_argument("--serial-encoders", action="store_true",
                    help="run the source / target encoders on one stream (default: two HIP streams)")
    ap.add_argument("--precision", choices=["bf16", "fp16"], default="bf16",
                    help="16-bit operand format of the heads / conv blocks / ResidualMLP linears left at their "
                         "default: bf16 (MI355X default, no loss scale) or fp16 (the reference's own autocast width, "
                         "ref/model/graph_model.py:510,709-726, trained with the device-side dynamic loss scale)")
    ap.add_argument("--heads", choices=["bf16", "fp16", "fp32"], default="bf16",
                    help="decoder R x R head GEMMs: bf16 MFMA (the reference trains in fp16 autocast; bf16 is the documented deviation, DESIGN.md §5) or fp32")
    ap.add_argument("--conv", choices=["bf16", "fp16", "fp32"], default="bf16",
                    help="conv blocks: bf16 MFMA with fp32 accumulation / BatchNorm (bf16 for the reference's fp16 autocast) or exact fp32")
    ap.add_argument("--mlp", choices=["bf16", "fp16", "fp32"], default="bf16",
                    help="ResidualMLP stacks: Linear layers on bf16 MFMA with fp32 accumulation, LayerNorm fp32 "
                         "(bf16 for the reference's fp16 autocast) or exact fp32")
    ap.add_argument("--lstm", choices=["16-mixed", "fp32"], default="16-mixed",
                    help="encoder LSTMs: 16-bit MFMA recurrences over 4-sample tiles (f16 forward / bf16 backward "
                         "operands, fp32 state: the reference's own 16-mixed LSTM width) or exact fp32")
    args = ap.parse_args()
    for k in ("heads", "conv", "mlp"):
        if getattr(args, k) == "bf16":
            setattr(args, k, args.precision)
    assert not (args.workload == "c4" and "fp16" in (args.heads, args.conv, args.mlp)), \
        "fp16 operands: c2 only (the classifier's convolutions have bf16 / fp32 kernels)"
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # `python bench.py --gpus N` without torchrun: N fresh rank processes (before this
        # process touches the GPU), rank 0's JSON line relayed, the first failure's exit code
        sys.exit(spawn_local_ranks([sys.executable, os.path.abspath(__file__), *sys.argv[1:]], args.gpus))
    global OUT
    OUT = _json_stdout()

    if args.ddp_probe and "WORLD_SIZE" not in os.environ:
        import socket
        sk = socket.socket()
        sk.bind(("127.0.0.1", 0))
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(sk.getsockname()[1]), WORLD_SIZE="1", RANK="0",
                          LOCAL_RANK="0")
        sk.close()
    rank, world, local, dev = init_distributed()
    if args.ddp_probe and not dist.is_initialized():
        torch.cuda.set_device(dev)
        dist.init_process_group(backend="nccl")
    ddp = world > 1 or args.ddp_probe
    mode = "native" if args.native else ("graph" if args.graph else args.mode)
    if mode == "auto":
        mode = "native" if not (args.prefetch or args.overlap_update) else "eager"
    args.native, args.graph = mode == "native", mode == "graph"
    assert world == args.gpus, f"--gpus {args.gpus} but WORLD_SIZE {world}"
    torch.cuda.set_device(dev)
    if args.workload == "c5":
        return run_c5(args, rank, world, dev)
    J, Q, T = FRONTENDS[args.frontend]
    N, B = 4096, args.batch
    plan = FrontEndPlan(J, Q, T, N, device=dev)
    fe = FrontEnd(plan, load_stats(J, Q, T, N))
    S = plan.S
    torch.manual_seed(1234)  # same initial weights on every rank (DDP semantics)
    vae_kw = dict(scattering_channels=fe.C_st, phase_channels=fe.C_ph, cross_phase_channels=fe.C_x,
                  head_precision=args.heads, conv_precision=args.conv, mlp_precision=args.mlp,
                  lstm_precision=args.lstm, concurrent_encoders=not args.serial_encoders)
    c4 = args.workload == "c4"
    if c4:
        # config 4: SeqVaeTebClassifier end to end (freeze_vae=False), the reference's default classifier
        # (filters 32, depth 6, dropout 0.2, attention), total = CE + 0.1 * ELBO(beta 1)
        from vaeteb.classifier import SeqVaeTebClassifier
        # a captured step replays new dropout masks: the classifier advances a device-side seed
        # offset every training forward (vt_dropout_seed_advance), added to the capture's host seeds
        assert not args.graph, "--graph is not wired for the classifier workload (use --mode native)"
        model = SeqVaeTebClassifier(sequence_length=S, freeze_vae=False, **vae_kw).to(dev)
    else:
        model = SeqVaeTeb(sequence_length=S, **vae_kw).to(dev)
    trainer = Trainer(model, lr=1e-3, frontend=fe, world_size=world, ddp=ddp,
                      reduce_dtype=torch.bfloat16 if args.reduce_bf16 else torch.float32)

    # synthetic windows resident in HBM before timing; global sample index ->
    # rank sharding as DistributedSampler (each rank its own B windows per step)
    pool = [torch.from_numpy(synthetic.batch((rank + world * i) * B, B, N)).to(dev) for i in range(2)]
    labels = [torch.from_numpy(np.random.default_rng(rank + world * i).integers(0, 2, B)).to(dev) for i in range(2)]
    torch.cuda.synchronize()

    # vt_fe_pairs compulsory HBM bytes per launch: every analytic-signal slot the launch's pairs use, read
    # once (N complex64), and the pair features written (pair_len fp32) — SURVEY.md §8(d)'s analytic-signal
    # read + feature write for the pairs of that launch (phase: ch0 slots of the 44 phase pairs; cross: the
    # ch0 i-slots and ch1 j-slots of the 130 cross pairs).  The phase and cross launches run concurrently
    # on two streams; each call's events span its own launch.
    p_ = plan
    ph_slots = {(0, int(p_.i_idx[k])) for k in fe.phase_pairs} | {(0, int(p_.j_idx[k])) for k in fe.phase_pairs}
    x_slots = {(0, int(p_.i_idx[k])) for k in fe.cross_pairs} | {(1, int(p_.j_idx[k])) for k in fe.cross_pairs}
    slots_of = {fe.C_ph: len(ph_slots), fe.C_x: len(x_slots)}
    work = dict(MFMA_CALLS)
    work["vt_fe_pairs"] = lambda an, B, n_slots, N, n_pad, pad_left, n_pairs, *a: \
        B * (slots_of.get(n_pairs, n_slots) * N * 8 + n_pairs * a[7] * 4)
    timer = KernelTimer(["vt_fe_pairs", *MFMA_CALLS], flops=work)
    graph = args.graph or args.native
    fe_in_graph = False
    if graph:
        # The model step (forward, backward, clip, AdamW) is replayed as a
        # hipGraph.  The front-end (~10 launches, independent of the weights)
        # runs eagerly on its own stream, one step ahead, writing into the other
        # of two graphs' static inputs (double buffering), so it overlaps the
        # previous step's replay; the roofline kernel is still timed live with
        # HIP events in every step.
        fe_stream = torch.cuda.Stream()
        if args.native:
            eps_shape = (B, S, model.latent_dim_z)
            fe_in_graph = bool(args.fe_in_graph) and not args.overlap_fe
            lab = (lambda j: {"labels": labels[j]}) if c4 else (lambda j: {})
            caps = [trainer.capture({"x": pool[j], **lab(j)} if fe_in_graph else {**fe(pool[j]), **lab(j)},
                                    eps=torch.randn(eps_shape, device=dev), native=True,
                                    n_streams=args.streams, update=not args.overlap_adam)
                    for j in range(2 if args.overlap_fe else 1)]
            if args.overlap_adam:
                from vaeteb.model import side_stream
                adam_side = side_stream(dev.index or 0, 1)
        else:
            caps = [trainer.capture(fe(pool[0])), trainer.capture(fe(pool[1]))]
        main = torch.cuda.current_stream()
        ready = [torch.cuda.Event(), torch.cuda.Event()]
        done = [torch.cuda.Event(), torch.cuda.Event()]
        for e in done:
            e.record(main)

        def frontend_into(i):
            slot = i % 2
            fe_stream.wait_event(done[slot])        # the graph that last read these inputs is done
            with torch.cuda.stream(fe_stream):
                fe(pool[i % 2], out=caps[slot].static_in)
            ready[slot].record(fe_stream)

        def step(i, last=False):
            slot = i % 2
            if args.native and fe_in_graph:
                # this step's windows into the graph's static input, its noise, the replay
                # (front-end + model step)
                caps[0].static_eps.normal_()   # in place: no temporary + copy (randn(out=) made one)
                if args.overlap_adam:
                    _lib.wait_for(torch.cuda.current_stream(), adam_side)
                    return caps[0].replay({"x": pool[i % 2]}, adam_stream=adam_side)
                return caps[0].replay({"x": pool[i % 2]})
            if args.native and not args.overlap_fe:
                # the step's own front-end first, on the same stream (as the eager step), then
                # this step's noise (drawn outside the graph) and the replay
                fe(pool[i % 2], out=caps[0].static_in)
                caps[0].static_eps.normal_()   # in place: no temporary + copy (randn(out=) made one)
                if args.overlap_adam:
                    # the previous step's AdamW (side stream) ran beside this front-end: join it
                    _lib.wait_for(torch.cuda.current_stream(), adam_side)
                    return caps[0].replay(adam_stream=adam_side)
                return caps[0].replay()
            if i == 0 or step.first:
                frontend_into(i)
                step.first = False
            main.wait_event(ready[slot])
            if args.native:                         # this step's noise, drawn outside the graph
                caps[slot].static_eps.normal_()
            out = caps[slot].replay()
            done[slot].record(main)
            if not last:
                frontend_into(i + 1)                # next batch's front-end overlaps this replay
            return out
        step.first = True
    elif args.prefetch or args.overlap_update:
        # Eager model step, front-end of the NEXT batch prefetched on its own streams:
        # the features of batch i+1 (independent of the weights) are computed while
        # step i runs, into the other of two feature buffers (a GPU-side input
        # pipeline; every step still runs its own batch's front-end inside the
        # timed region, the last step prefetches nothing).
        # reuse the model's side streams: HIP maps a process's streams onto 4 hardware
        # queues, and a 5th / 6th stream would share (and serialise behind) one of them
        from vaeteb.model import side_stream
        fe_stream, fe_side = side_stream(dev.index or 0, 1), side_stream(dev.index or 0, 2)
        bufs = [{k: v.clone() for k, v in fe(pool[j]).items()} for j in range(2)]
        main = torch.cuda.current_stream()
        ready = [torch.cuda.Event(), torch.cuda.Event()]
        done = [torch.cuda.Event(), torch.cuda.Event()]
        for e in done:
            e.record(main)

        def frontend_into(i):
            slot = i % 2
            fe_stream.wait_event(done[slot])        # the step that last read these features is done
            with torch.cuda.stream(fe_stream):
                fe(pool[i % 2], out=bufs[slot], side=fe_side)
                fe_stream.wait_stream(fe_side)
            ready[slot].record(fe_stream)

        def step(i, last=False):
            slot = i % 2
            if step.first:
                frontend_into(i)
                step.first = False
            main.wait_event(ready[slot])
            if not last and not args.overlap_update:
                frontend_into(i + 1)                # overlaps this whole step
            nxt = None
            if not last and args.overlap_update:
                def nxt():                          # overlaps only this step's clip + AdamW
                    done_bwd = torch.cuda.Event()
                    done_bwd.record(main)
                    fe_stream.wait_event(done_bwd)
                    frontend_into(i + 1)
            out = trainer.step({**bufs[slot], "labels": labels[slot]}, before_update=nxt)
            done[slot].record(main)
            return out
        step.first = True
    else:
        step = lambda i, last=False: trainer.step({"x": pool[i % 2], "labels": labels[i % 2]})
    for i in range(args.warmup):
        step(i, last=i == args.warmup - 1)
    if hasattr(step, "first"):
        step.first = True
    if dist.is_initialized():
        dist.barrier()
    torch.cuda.synchronize()
    # timed-region marker for profiles (tools/step_stats.py): a no-op kernel launched right
    # before the timed loop and right after its synchronize, outside the timed interval
    _lib.call("vt_bucket_marker", 0, _lib.stream())
    torch.cuda.synchronize()
    timer.reset(True)
    t0 = time.perf_counter()
    last = None
    for i in range(args.steps):
        last = step(i, last=i == args.steps - 1)
    t_enq = time.perf_counter() - t0   # host time to enqueue the K steps (launch-bound if ~= dt)
    torch.cuda.synchronize()
    if dist.is_initialized():
        dist.barrier()
    dt = time.perf_counter() - t0
    _lib.call("vt_bucket_marker", 0, _lib.stream())   # end of the timed region (profiles only)
    timer.enabled = False
    if world > 1:
        t = torch.tensor([dt], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = t.item()
    keys = ("total_loss", "classification_loss", "vae_loss") if c4 else ("total_loss", "nll_loss", "mse_loss",
                                                                          "kld_loss")
    elbo = {k: round(float(last[k].item()), 6) for k in keys}
    samples = args.steps * B * world
    value = samples / dt
    n_params = sum(p.numel() for p in model.parameters())
    step_bytes = step_bytes_per_sample(plan, fe, n_params, B)
    fe_timed_in = "timed region"
    if graph and args.native and fe_in_graph:
        # the front-end runs inside the replay: time its kernel in two eager steps after the
        # timed region (the same kernels and shapes; profiles/ holds the in-replay durations)
        timer.reset(True)
        for i in range(2):
            trainer.step({"x": pool[i % 2], **({"labels": labels[i % 2]} if c4 else {})})
        torch.cuda.synchronize()
        timer.enabled = False
        fe_timed_in = "eager steps after the timed region (front-end captured in the replayed step)"
    k_ms, k_n = timer.mean_ms("vt_fe_pairs")
    k_bytes = timer.total_flops["vt_fe_pairs"] / max(k_n, 1)   # mean algorithmic bytes per launch
    # the PMC passes ran the default command (native replay, one launch of all pairs per step):
    # only a run with that launch shape quotes their traffic
    traffic, traffic_src = (pmc_traffic("k_fe_pairs8k") if (J, Q, T, B) == (11, 4, 16, 256) and args.native
                            else (None, None))
    achieved = k_bytes / (k_ms * 1e-3) / 1e9
    out = {
        "metric": "train samples/sec + ELBO, 4096-pt windows, batch 256, 1/2/4/8 MI355X",
        "value": round(value, 3), "unit": "samples/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(dt / args.steps * 1e3, 3), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None,
        "dtype": "fp32" if (args.heads, args.conv, args.mlp, args.lstm) == ("fp32", "fp32", "fp32", "fp32") else
                 f"{args.precision} MFMA (" + " + ".join(
                     n for n, v in (("decoder heads", args.heads), ("conv blocks", args.conv),
                                    ("ResidualMLP linears", args.mlp),
                                    ("classifier convolutions", args.conv if c4 else "")) if v in ("bf16", "fp16"))
                 + (", LSTM recurrences f16 fwd / bf16 bwd" if args.lstm == "16-mixed" else "")
                 + "), fp32 accumulation; fp32 LayerNorm / BatchNorm / LSTM state / front-end / optimizer"
                 + ("; dynamic loss scale (GradScaler semantics, device-side)" if trainer.loss_scale else ""),
        "data": "synthetic",
        "config": {"workload": (f"c4: front-end J={J} Q={Q} T={T} (N=4096, S={S}) + SeqVaeTebClassifier("
                                f"R={16 * S}, FHRInceptionTimeClassifier d6 attention, "
                                f"{'bf16-MFMA' if args.conv == 'bf16' else 'exact-fp32'} convolutions, fp32-MFMA "
                                f"attention, dropout 0.2) end-to-end "
                                f"train step, CE + 0.1 ELBO, batch {B}/GPU") if c4 else
                               (f"c2: front-end J={J} Q={Q} T={T} (N=4096, S={S}) + SeqVaeTeb(R={16 * S}) "
                                f"train step, batch {B}/GPU"), "global_batch": B * world, "seq_len": N,
                   "parallelism": f"dp{world}"},
        "elbo": elbo,
        **({"loss_scale": trainer.scaler_state()} if trainer.loss_scale else {}),
        "host_enqueue_ms_per_step": round(t_enq / args.steps * 1e3, 3),
        "mode": (f"step captured once, replayed by the native "
                 f"{len(caps[0].side) + 1 - bool(caps[0].markers)}-stream executor (vt_stepgraph); "
                 + ("front-end inside the captured step" if fe_in_graph else
                    "front-end eager " + ("one step ahead on its own stream" if args.overlap_fe else
                                          "before each replay on the same stream"))
                 + (f"; {len(trainer.buckets.buckets)} gradient buckets "
                    f"({'bf16' if args.reduce_bf16 else 'fp32'}), each all-reduced on a comm stream as soon as its "
                    f"writers are enqueued ({len(caps[0].markers)} markers in the replay)"
                    + (" [ddp probe: single-rank RCCL group]" if args.ddp_probe and world == 1 else "")
                    if trainer.buckets else "")) if args.native else
                "model step replayed as a hipGraph (double-buffered), front-end eager one step ahead on its own stream"
                if graph else ("eager, next batch's front-end overlapped with clip + AdamW (own streams, "
                               "double-buffered features)" if args.overlap_update else
                               "eager, next batch's front-end overlapped with the whole step" if args.prefetch
                               else "eager"),
        "roofline": {"bound": "hbm", "kernel": "vt_fe_pairs (k_fe_pairs8k_h)", "achieved": round(achieved, 1),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": traffic, "traffic_unit": "bytes/launch (PMC FETCH_SIZE x2 + WRITE_SIZE)",
                     "traffic_source": traffic_src, "avg_launch_ms": round(k_ms, 4), "launches": k_n,
                     "algorithmic_bytes": round(k_bytes),
                     "algorithmic_bytes_def": "compulsory: the launch's analytic-signal slots read once + pair "
                                              "features written (SURVEY.md §8(d))",
                     "limiter": "issue stalls and waits, not HBM (profiles/r05/pmc_sq.json: of the wave cycles "
                                "0.46 issue-stall, 0.33 waitcnt / barrier, 0.22 issuing, 0.13 VALU; DESIGN.md §5)",
                     "launches_per_step": k_n / (2 if fe_timed_in != "timed region" else args.steps),
                     "timed_in": fe_timed_in},
        # SURVEY.md §8(d)'s step-level roofline: samples/s x algorithmic bytes per sample / (GPUs x 8 TB/s)
        "roofline_step": {"bound": "hbm", "bytes_per_sample": round(step_bytes),
                          "achieved": round(value * step_bytes / world / 1e9, 1), "peak": HBM_PEAK_GBS,
                          "unit": "GB/s", "frac": round(value * step_bytes / world / (HBM_PEAK_GBS * 1e9), 4),
                          "formula": "value x bytes_per_sample / (n_gpus x 8e12); bytes_per_sample = front-end "
                                     "+ 4,161,024 activation elements x 2 B x 4 + 46 B x params / batch"},
    }
    if dist.is_initialized():
        out["dist_backend"] = dist.get_backend()   # "nccl" = RCCL on ROCm
    hbm = pmc_kernels() if (J, Q, T, B) == (11, 4, 16, 256) and not c4 else None
    if hbm:
        out["hbm_kernels"] = hbm
    lstm = profile_lstm() if (J, Q, T, B) == (11, 4, 16, 256) and not c4 and args.lstm == "16-mixed" else None
    if lstm:
        out["lstm"] = lstm
    mfma_steps = args.steps
    if graph:
        # the MFMA head GEMMs run inside the graph: time them with HIP events in
        # two extra eager steps after the timed region (same kernels, same shapes)
        timer.reset(True)
        for i in range(2):
            trainer.step({**fe(pool[i % 2]), **({"labels": labels[i % 2]} if c4 else {})})   # eager, default stream
        torch.cuda.synchronize()
        timer.enabled = False
        mfma_steps = 2
    mfma_ms = timer.total_ms(list(MFMA_CALLS))
    if mfma_ms > 0:
        # MFMA utilisation of the decoder heads from KERNEL time: the committed rocprofv3 summary of this
        # bench and workload (k_mfma_gemm + k_mfma_dw per step); the live HIP-event span around the
        # C-ABI calls (which also covers the split-K reduces' launch gaps) is kept as call_span_ms
        flops_step = sum(timer.total_flops[n] for n in MFMA_CALLS) / mfma_steps
        k_mfma_ms, k_src = profile_mfma(args.workload) if (J, Q, T, B) == (11, 4, 16, 256) else (None, None)
        tf = flops_step / (k_mfma_ms * 1e-3) / 1e12 if k_mfma_ms else None
        out["mfma"] = {"kernels": "k_mfma_gemm (split-K sums in its last-arriving workgroups) + k_mfma_dw "
                                  "(decoder heads, bf16)",
                       "flop_per_step": flops_step, "kernel_ms_per_step": k_mfma_ms and round(k_mfma_ms, 4),
                       "source": k_src, "achieved": tf and round(tf, 1), "peak": MFMA_PEAK_TFLOPS,
                       "unit": "TFLOP/s", "frac": tf and round(tf / MFMA_PEAK_TFLOPS, 4),
                       "call_span_ms_per_step": round(mfma_ms / mfma_steps, 3),
                       "timed_in": ("call span: eager steps after the timed region" if graph else "timed region")
                                   + "; kernel time: the source's rocprofv3 trace"}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline((J, Q, T), batch=args.cpu_batch, classifier=c4)
    if rank == 0:
        print(json.dumps(out), file=OUT, flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
