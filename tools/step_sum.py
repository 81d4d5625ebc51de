"""Per-step kernel time by kernel name (all streams) from a rocprofv3 kernel trace:
the last complete step between the optimizer launches.  usage: step_sum.py trace.csv [top]"""
import csv
import re
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
top = int(sys.argv[2]) if len(sys.argv) > 2 else 30
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "adamw" in r["Kernel_Name"]]
# steps end with the optimizer launches (consecutive adamw launches belong to one step)
ends = [i for k, i in enumerate(idx) if k + 1 == len(idx) or idx[k + 1] != i + 1]
a, b = ends[-2] + 1, ends[-1] + 1
tot = defaultdict(float)
cnt = defaultdict(int)
for r in rows[a:b]:
    n = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("vt::", "")
    n = re.sub(r"\(.*", "", n)
    n = re.sub(r"^void ", "", n)[:60]
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000
    tot[n] += d
    cnt[n] += 1
span = (int(rows[b - 1]["End_Timestamp"]) - int(rows[a]["Start_Timestamp"])) / 1000
print(f"step: {b - a} kernels, span {span:.0f} us, kernel time sum {sum(tot.values()):.0f} us")
for n, v in sorted(tot.items(), key=lambda kv: -kv[1])[:top]:
    print(f"{v:8.1f} us {cnt[n]:4d}x  {n}")
