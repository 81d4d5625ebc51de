"""HBM traffic per launch from two rocprofv3 --pmc passes (FETCH_SIZE and WRITE_SIZE,
collected separately: they do not fit one TCC pass on gfx950), corrected as
MI355X_MICROARCH.md §HBM prescribes: FETCH_SIZE / WRITE_SIZE are in KiB; on gfx950
FETCH_SIZE reports half the bytes of wide coalesced reads, so it is doubled (exact for
16-B-per-lane streaming reads; other widths are uncalibrated, the guide says so — the
doubled figure is then an upper bound).

  roofline kernel (bench.py reads profiles/rNN/pmc_traffic.json):
    python tools/pmc_traffic.py gpurun_out/pmc k_fe_pairs8k profiles/r04/pmc_traffic.json
  per-kernel HBM GB/s (every template instance whose name contains one of the patterns;
  durations = the average launch of that instance in the timed steps of a kernel trace,
  tools/step_stats.py output):
    python tools/pmc_traffic.py gpurun_out/pmc --kernels k_cfw16 k_cbd16 ... \\
        --durations profiles/r04/kernel_stats_stepX.csv --out profiles/r04/pmc_kernels.json
"""
import argparse
import collections
import csv
import json
import os

HBM_PEAK = 8.0e12


def per_instance(path, pats, counter):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter and any(p in r["Kernel_Name"] for p in pats):
            acc[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return acc


def roofline_kernel(d, kernel, out, command=None):
    f = per_instance(os.path.join(d, "fetch_counter_collection.csv"), [kernel], "FETCH_SIZE")
    w = per_instance(os.path.join(d, "write_counter_collection.csv"), [kernel], "WRITE_SIZE")
    fv = [x for v in f.values() for x in v]
    wv = [x for v in w.values() for x in v]
    fetch_b, write_b = 2 * sum(fv) / len(fv) * 1024, sum(wv) / len(wv) * 1024
    res = {"kernel": kernel, "launches": [len(fv), len(wv)], "FETCH_SIZE_kib_raw": sum(fv) / len(fv),
           "WRITE_SIZE_kib_raw": sum(wv) / len(wv), "fetch_bytes": fetch_b, "write_bytes": write_b,
           "traffic_bytes_per_launch": fetch_b + write_b,
           "correction": "FETCH_SIZE x2 (gfx950 half-counts wide reads), KiB -> bytes",
           "command": command or "rocprofv3 --pmc FETCH_SIZE|WRITE_SIZE --kernel-trace -- python3 bench.py --steps 2 "
                                 "--warmup 1 --no-cpu-baseline (tools/gpu_prof.sh)"}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


def kernels(d, pats, durations, out):
    f = per_instance(os.path.join(d, "fetch_counter_collection.csv"), pats, "FETCH_SIZE")
    w = per_instance(os.path.join(d, "write_counter_collection.csv"), pats, "WRITE_SIZE")
    dur = {r["Name"]: float(r["AverageNs"]) for r in csv.DictReader(open(durations))}
    per_step = {r["Name"]: float(r["PerStepNs"]) for r in csv.DictReader(open(durations))}
    res = {"source": {"pmc": d, "durations": durations}, "peak_GBps": HBM_PEAK / 1e9,
           "correction": "FETCH_SIZE x2 (gfx950 half-counts 16-B-per-lane reads; other widths uncalibrated, "
                         "so the read half is an upper bound), WRITE_SIZE exact for 16-B stores, KiB -> bytes",
           "kernels": {}}
    for name in sorted(set(f) & set(w)):
        fb = 2 * sum(f[name]) / len(f[name]) * 1024
        wb = sum(w[name]) / len(w[name]) * 1024
        ns = dur.get(name)
        e = {"launches_pmc": len(f[name]), "fetch_bytes_per_launch": fb, "write_bytes_per_launch": wb,
             "traffic_bytes_per_launch": fb + wb, "avg_launch_ns": ns,
             "ms_per_step": per_step.get(name, 0.0) / 1e6}
        if ns:
            e["hbm_GBps"] = (fb + wb) / ns
            e["hbm_frac"] = (fb + wb) / ns / (HBM_PEAK / 1e9)
        res["kernels"][name] = e
        print(f"{name[:90]:90s} {(fb + wb) / 1e6:9.2f} MB  {ns or 0:9.0f} ns  {e.get('hbm_GBps', 0):7.1f} GB/s")
    json.dump(res, open(out, "w"), indent=1)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("kernel", nargs="?")
    ap.add_argument("out_json", nargs="?")
    ap.add_argument("--kernels", nargs="*")
    ap.add_argument("--durations")
    ap.add_argument("--out")
    ap.add_argument("--command", help="the profiled command, recorded in the roofline-kernel JSON")
    a = ap.parse_args()
    if a.kernels:
        kernels(a.dir, a.kernels, a.durations, a.out)
    else:
        roofline_kernel(a.dir, a.kernel, a.out_json, a.command)
