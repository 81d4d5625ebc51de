"""Per-stream view of the last profiled step: for each HIP stream, busy time
and its kernels in phases, plus the union of busy intervals (GPU has work)."""
import collections
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if "k_fe_spectrum" in r["Kernel_Name"]]
st = rows[starts[-2]:starts[-1]] if len(starts) > 1 else rows[starts[-1]:]
t0 = int(st[0]["Start_Timestamp"])
t1 = max(int(r["End_Timestamp"]) for r in st)
print(f"step span {(t1 - t0) / 1e6:.2f} ms, {len(st)} kernels")
by = collections.defaultdict(list)
for r in st:
    by[r["Stream_Id"]].append(r)
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in st)
union, cs, ce = 0, iv[0][0], iv[0][1]
for a, b in iv[1:]:
    if a > ce:
        union += ce - cs
        cs, ce = a, b
    else:
        ce = max(ce, b)
union += ce - cs
print(f"GPU busy (union) {union / 1e6:.2f} ms; idle {(t1 - t0 - union) / 1e6:.2f} ms")
for sid, rs in sorted(by.items(), key=lambda kv: -len(kv[1])):
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rs) / 1e6
    first = (int(rs[0]["Start_Timestamp"]) - t0) / 1e6
    last = (int(rs[-1]["End_Timestamp"]) - t0) / 1e6
    print(f"stream {sid}: {len(rs)} kernels, busy {busy:.2f} ms, active {first:.2f}..{last:.2f} ms")
    if len(sys.argv) > 2:
        for r in rs:
            s = (int(r["Start_Timestamp"]) - t0) / 1e6
            d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            if d > float(sys.argv[2]):
                print(f"   {s:7.2f} ms  {d:7.1f} us  {r['Kernel_Name'][:60]}")
