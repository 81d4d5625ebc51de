"""Wave-state split per kernel from a rocprofv3 --pmc pass of the SQ counters (tools/gpu_prof.sh:
SQ_WAVE_CYCLES, SQ_WAIT_ANY, SQ_WAIT_INST_ANY, SQ_ACTIVE_INST_ANY, SQ_ACTIVE_INST_VALU,
SQ_ACTIVE_INST_LDS).  Per MI355X_MICROARCH.md's PMC table: WAIT_ANY (wave parked on s_waitcnt /
barrier) + WAIT_INST_ANY (issue stall) + ACTIVE_INST_ANY ≈ WAVE_CYCLES; all count quad-cycles, so
the fractions below are unit-free.  Counters summed over every launch of a kernel instance.

  python tools/pmc_sq.py gpurun_out/pmc/sq_counter_collection.csv profiles/r05/pmc_sq.json [pattern ...]
"""
import collections
import csv
import json
import sys

COUNTERS = ("SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
            "SQ_ACTIVE_INST_LDS")


def main(path, out, pats):
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    launches = collections.defaultdict(set)
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        if pats and not any(p in name for p in pats):
            continue
        if r["Counter_Name"] in COUNTERS:
            acc[name][r["Counter_Name"]] += float(r["Counter_Value"])
            launches[name].add(r["Dispatch_Id"])
    res = {}
    for name, c in sorted(acc.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0.0)):
        wc = c.get("SQ_WAVE_CYCLES", 0.0)
        if wc <= 0:
            continue
        res[name[:160]] = {
            "launches": len(launches[name]),
            **{k: c.get(k, 0.0) for k in COUNTERS},
            "frac_wait_any": c.get("SQ_WAIT_ANY", 0.0) / wc,
            "frac_wait_inst_any": c.get("SQ_WAIT_INST_ANY", 0.0) / wc,
            "frac_active_inst_any": c.get("SQ_ACTIVE_INST_ANY", 0.0) / wc,
            "frac_active_valu": c.get("SQ_ACTIVE_INST_VALU", 0.0) / wc,
            "frac_active_lds": c.get("SQ_ACTIVE_INST_LDS", 0.0) / wc,
        }
    json.dump({"source": path, "note": __doc__.split("\n\n")[0], "kernels": res}, open(out, "w"), indent=1)
    for name, v in list(res.items())[:12]:
        print(f"{name[:70]:70s} wait {v['frac_wait_any']:.2f} stall {v['frac_wait_inst_any']:.2f} "
              f"active {v['frac_active_inst_any']:.2f} valu {v['frac_active_valu']:.2f} lds {v['frac_active_lds']:.2f}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3:])
