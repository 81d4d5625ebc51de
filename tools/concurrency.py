"""Fraction of a trace window with 0, 1, 2, ... kernels running (rocprofv3 kernel trace).
usage: concurrency.py trace.csv [n_last_kernels]"""
import csv
import sys
from collections import Counter

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 514
last = rows[-n:]
ev = sorted([(int(r["Start_Timestamp"]), 1) for r in last] + [(int(r["End_Timestamp"]), -1) for r in last])
cur, prev, acc = 0, ev[0][0], Counter()
for t, d in ev:
    acc[cur] += t - prev
    prev, cur = t, cur + d
tot = sum(acc.values())
print(f"window {tot / 1000:.0f} us over {n} kernels; time fraction by running-kernel count:",
      {k: round(v / tot, 3) for k, v in sorted(acc.items())})
