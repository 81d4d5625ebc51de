"""Per-step GPU busy time / span / idle gaps from a rocprofv3 kernel trace
(steps delimited by the front-end's first kernel, k_fe_spectrum)."""
import collections
import csv
import sys

path = sys.argv[1]
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if "k_fe_spectrum" in r["Kernel_Name"]]
starts.append(len(rows))
for s, e in zip(starts, starts[1:]):
    st = rows[s:e]
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in st) / 1e6
    span = (int(st[-1]["End_Timestamp"]) - int(st[0]["Start_Timestamp"])) / 1e6
    gaps = collections.Counter()
    for a, b in zip(st, st[1:]):
        g = int(b["Start_Timestamp"]) - int(a["End_Timestamp"])
        if g > 5000:
            gaps[a["Kernel_Name"][:40] + " -> " + b["Kernel_Name"][:40]] += g / 1e6
    print(f"step: kernels {len(st)} busy {busy:.2f} ms span {span:.2f} ms idle>5us {sum(gaps.values()):.2f} ms")
    for k, v in gaps.most_common(8):
        print(f"   {v:.2f} ms  {k}")
if len(sys.argv) > 2:  # top kernels of the last step
    agg = collections.defaultdict(list)
    for r in rows[starts[-2]:starts[-1]]:
        agg[r["Kernel_Name"][:70]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1]))[: int(sys.argv[2])]:
        print(f"{sum(v) / 1e3:7.3f} ms {len(v):4d} x {sum(v) / len(v):8.1f} us  {k}")
