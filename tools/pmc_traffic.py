"""HBM traffic per launch of one kernel from two rocprofv3 --pmc passes
(FETCH_SIZE and WRITE_SIZE, collected separately: they do not fit one TCC
pass on gfx950), corrected as MI355X_MICROARCH.md §HBM prescribes:
FETCH_SIZE/WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports half the bytes
of wide coalesced reads, so it is doubled.

  python tools/pmc_traffic.py gpurun_out/pmc k_fe_pairs8k profiles/r01/pmc_traffic.json
"""
import csv
import json
import os
import sys


def per_launch(path, kernel, counter):
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
            if kernel in r["Kernel_Name"] and r["Counter_Name"] == counter]
    return sum(vals) / len(vals), len(vals)


def main(d, kernel, out):
    fetch_kb, nf = per_launch(os.path.join(d, "fetch_counter_collection.csv"), kernel, "FETCH_SIZE")
    write_kb, nw = per_launch(os.path.join(d, "write_counter_collection.csv"), kernel, "WRITE_SIZE")
    fetch_b = 2 * fetch_kb * 1024
    write_b = write_kb * 1024
    res = {"kernel": kernel, "launches": [nf, nw], "FETCH_SIZE_kib_raw": fetch_kb, "WRITE_SIZE_kib_raw": write_kb,
           "fetch_bytes": fetch_b, "write_bytes": write_b, "traffic_bytes_per_launch": fetch_b + write_b,
           "correction": "FETCH_SIZE x2 (gfx950 half-counts wide reads), KiB -> bytes",
           "command": "rocprofv3 --pmc FETCH_SIZE|WRITE_SIZE --kernel-trace -- python3 bench.py --steps 2 --warmup 1 "
                      "--no-cpu-baseline (tools/gpu_pmc.sh)"}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main(*sys.argv[1:4])
