"""Static instruction mix per kernel of a gfx950 .s file (hipcc --save-temps).
Usage: python tools/isa_count.py file.s [kernel-substring ...]"""
import re
import sys
from collections import Counter

src = open(sys.argv[1]).read().splitlines()
pats = sys.argv[2:]
cur, counts, meta = None, {}, {}
for ln in src:
    m = re.match(r"^(\S+):\s*(;.*)?$", ln)
    if m and not m.group(1).startswith(".") and "@" not in m.group(1):
        cur = m.group(1)
        counts[cur] = Counter()
        continue
    if cur is None:
        continue
    if ln.startswith(".Lfunc_end"):
        cur = None
        continue
    s = ln.strip()
    if not s or s.startswith((";", ".")):
        continue
    op = s.split()[0]
    if op.startswith("v_pk_"):
        k = "valu_pk"
    elif op.startswith("v_mfma"):
        k = "mfma"
    elif op.startswith("v_"):
        k = "valu"
    elif op.startswith("s_waitcnt") or op.startswith("s_barrier"):
        k = op
    elif op.startswith("s_"):
        k = "salu"
    elif op.startswith("ds_"):
        k = "lds"
    elif op.startswith(("global_", "buffer_", "flat_")):
        k = "vmem"
    elif op.startswith("scratch_"):
        k = "scratch"
    else:
        k = "other"
    counts[cur][k] += 1
for ln in src:
    m = re.match(r"\s*;\s*(NumVgprs|ScratchSize|Occupancy|NumAgprs):\s*(\d+)", ln)
for name, c in counts.items():
    if pats and not any(p in name for p in pats):
        continue
    print(name[:90])
    print("   ", dict(sorted(c.items())))
