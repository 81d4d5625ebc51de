"""Per-kernel GPU time inside one window of a rocprofv3 kernel trace: the
launches between the i-th and (i+1)-th launch of a marker kernel.
  python tools/prof_window.py trace.csv marker i"""
import collections, csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
marker, i = sys.argv[2], int(sys.argv[3])
idx = [j for j, r in enumerate(rows) if marker in r["Kernel_Name"]]
win = rows[idx[i]:idx[i + 1]]
agg, cnt = collections.Counter(), collections.Counter()
for r in win:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    agg[r["Kernel_Name"][:70]] += d
    cnt[r["Kernel_Name"][:70]] += 1
span = (int(win[-1]["End_Timestamp"]) - int(win[0]["Start_Timestamp"])) / 1e3
for k, v in agg.most_common():
    print(f"{v:9.1f} us {cnt[k]:5d}  {k}")
print(f"busy {sum(agg.values()):.1f} us, span {span:.1f} us, {len(win)} launches")
