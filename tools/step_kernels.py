"""Per-kernel-family GPU time of one profiled step (between two k_fe_spectrum
launches) from a rocprofv3 kernel trace.  usage: step_kernels.py trace.csv"""
import collections
import csv
import re
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if "k_fe_spectrum" in r["Kernel_Name"]]
st = rows[starts[-2]:starts[-1]]
agg, cnt = collections.Counter(), collections.Counter()
for r in st:
    n = r["Kernel_Name"].replace("vt::", "").replace("(anonymous namespace)::", "")
    n = re.sub(r"\(.*", "", n).replace("void ", "")
    agg[n] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    cnt[n] += 1
tot = sum(agg.values())
print(f"kernel time {tot / 1e3:.2f} ms, {len(st)} launches")
for k, v in agg.most_common(int(sys.argv[2]) if len(sys.argv) > 2 else 60):
    print(f"{v:8.1f} us {cnt[k]:4d} {100 * v / tot:5.1f}%  {k[:90]}")
