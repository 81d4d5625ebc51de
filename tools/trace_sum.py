"""Per-kernel durations from a rocprofv3 --kernel-trace CSV (min / mean / count per
kernel name, in first-seen order): python tools/trace_sum.py <run_kernel_trace.csv> [filter]"""
import csv
import sys
from collections import OrderedDict

rows = list(csv.DictReader(open(sys.argv[1])))
flt = sys.argv[2] if len(sys.argv) > 2 else ""
agg = OrderedDict()
for r in rows:
    agg.setdefault(r["Kernel_Name"], []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000)
for n, v in agg.items():
    if flt in n:
        print(f"{min(v):8.1f} {sum(v) / len(v):8.1f} {len(v):4d}  {n[:110]}")
