"""Main-stream view of one profiled step (rocprofv3 --kernel-trace CSV):
every main-stream kernel with its start, duration and the gap before it
(gaps = waits on side streams or on the host), grouped runs of short kernels.
usage: critpath.py trace.csv [stream] [min_us]"""
import collections
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
sid = sys.argv[2] if len(sys.argv) > 2 else "0"
min_us = float(sys.argv[3]) if len(sys.argv) > 3 else 20
starts = [i for i, r in enumerate(rows) if "k_fe_spectrum" in r["Kernel_Name"]]
st = rows[starts[-2]:starts[-1]]
t0 = int(st[0]["Start_Timestamp"])
prev_end = t0
gaps = 0.0
agg = collections.Counter()
for r in st:
    if r["Stream_Id"] != sid:
        continue
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev_end) / 1e3
    d = (e - s) / 1e3
    gaps += max(gap, 0)
    name = r["Kernel_Name"].replace("vt::", "").replace("(anonymous namespace)::", "")[:70]
    agg[name.split("(")[0]] += d
    if d >= min_us or gap >= min_us:
        print(f"{(s - t0) / 1e3:8.1f} gap {gap:7.1f} dur {d:7.1f}  {name}")
    prev_end = max(prev_end, e)
print(f"stream {sid}: gaps {gaps / 1e3:.2f} ms")
for k, v in agg.most_common(25):
    print(f"{v / 1e3:7.3f} ms  {k}")
