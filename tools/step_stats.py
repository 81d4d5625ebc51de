"""Per-kernel GPU time of the TIMED steps only, from a rocprofv3 kernel trace of bench.py:
bench.py launches the no-op marker kernel k_bucket_mark once right before its timed loop and
once right after it (after the synchronize), so the launches whose start lies between the
first and the last marker are exactly the K timed steps (no setup, capture, warmup or
post-timing kernels).  Writes a kernel-stats CSV in rocprofv3's column layout (Name, Calls,
TotalDurationNs, AverageNs, Percentage, MinNs, MaxNs) plus a per-step column.

  python tools/step_stats.py <run>_kernel_trace.csv K out.csv
"""
import collections
import csv
import sys


def main(trace, steps, out):
    rows = sorted(csv.DictReader(open(trace)), key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows) if "k_bucket_mark" in r["Kernel_Name"]]
    if len(marks) < 2:
        raise SystemExit(f"{trace}: need the two timed-region markers, found {len(marks)}")
    t0, t1 = int(rows[marks[0]]["Start_Timestamp"]), int(rows[marks[-1]]["Start_Timestamp"])
    agg = collections.defaultdict(list)
    for r in rows[marks[0] + 1:marks[-1]]:
        if "k_bucket_mark" in r["Kernel_Name"]:
            continue
        agg[r["Kernel_Name"]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    total = sum(sum(v) for v in agg.values())
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "PerStepNs"])
        for name, d in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
            w.writerow([name, len(d), sum(d), sum(d) / len(d), 100.0 * sum(d) / total, min(d), max(d),
                        sum(d) / steps])
    print(f"{len(agg)} kernels, {sum(len(v) for v in agg.values())} launches in {steps} timed steps: "
          f"{total / steps / 1e6:.3f} ms of kernel time per step, wall {(t1 - t0) / steps / 1e6:.3f} ms per step")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]), sys.argv[3])
