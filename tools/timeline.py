"""Stream timeline of one training step from a rocprofv3 kernel trace:
per-stream busy time, idle gaps, long kernels.  usage: timeline.py trace.csv [min_us]"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
min_us = float(sys.argv[2]) if len(sys.argv) > 2 else 60
ad = [i for i, r in enumerate(rows) if "k_adamw" in r["Kernel_Name"]]
a, b = ad[-3], ad[-1]
seg = rows[a + 1: b + 1]
t0 = int(seg[0]["Start_Timestamp"])
print("span us %.0f" % ((int(seg[-1]["End_Timestamp"]) - t0) / 1e3))
for sid in sorted({r["Stream_Id"] for r in seg}):
    s = [r for r in seg if r["Stream_Id"] == sid]
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in s)
    print("stream", sid, len(s), "kernels, busy us %.0f" % (busy / 1e3))
for r in seg:
    st = (int(r["Start_Timestamp"]) - t0) / 1e3
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    if d > min_us:
        print("%8.0f %7.1f s%s %s" % (st, d, r["Stream_Id"], r["Kernel_Name"][:60]))
