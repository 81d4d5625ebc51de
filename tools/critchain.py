"""Approximate critical path of one step from a rocprofv3 kernel trace taken
with the host out of the way (tools/gpu_bound_probe.py): walk back from the
step's last kernel; a kernel's predecessor is the kernel on its own stream
that ended right before it started, else (a wait) the kernel on another
stream whose end is the latest before that start.  usage: critchain.py trace.csv"""
import collections
import csv
import re
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if "k_fe_spectrum" in r["Kernel_Name"]]
seg = rows[starts[-2]:starts[-1]]
K = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"],
      re.sub(r"\(.*", "", r["Kernel_Name"].replace("(anonymous namespace)::", "")).replace("void ", "").replace("vt::", ""))
     for r in seg]
t0 = K[0][0]
print(f"step span {(int(rows[starts[-1]]['Start_Timestamp']) - t0) / 1e3:.1f} us, {len(K)} kernels")
cur = max(range(len(K)), key=lambda i: K[i][1])
path = []
while True:
    s, e, q, n = K[cur]
    path.append(cur)
    same = [i for i in range(len(K)) if K[i][2] == q and K[i][1] <= s + 1000 and i != cur and K[i][0] < s]
    prev_same = max(same, key=lambda i: K[i][1]) if same else None
    if prev_same is not None and s - K[prev_same][1] < 8000:   # back to back on its queue (< 8 us)
        cur = prev_same
        continue
    other = [i for i in range(len(K)) if K[i][1] <= s + 1000 and K[i][0] < s and i != cur]
    if not other:
        break
    cur = max(other, key=lambda i: K[i][1])
path.reverse()
agg = collections.Counter()
busy = 0
for i in path:
    s, e, q, n = K[i]
    agg[n] += (e - s) / 1e3
    busy += e - s
end = K[path[-1]][1]
print(f"critical chain {len(path)} kernels, {busy / 1e3:.1f} us busy of {(end - K[path[0]][0]) / 1e3:.1f} us")
for n, v in agg.most_common(30):
    print(f"{v:8.1f} us  {n[:80]}")
if len(sys.argv) > 2 and sys.argv[2] == "timeline":
    # the chain in order: runs of kernels with their span (us from the step start)
    print("\ntimeline (start us, duration us, kernel)")
    for i in path:
        s, e, q, n = K[i]
        print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f}  q{q} {n[:70]}")
