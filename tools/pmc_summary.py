"""Per-kernel summary of rocprofv3 --pmc csv output directories given on the command line."""
import collections
import csv
import glob
import sys

agg = collections.defaultdict(lambda: collections.defaultdict(float))
for d in sys.argv[1:]:
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"][:40]
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            agg[k]["_vgpr"] = float(r.get("VGPR_Count") or 0)
            agg[k]["_scratch"] = float(r.get("Scratch_Size") or 0)
for k, v in agg.items():
    if "gic" not in k or v.get("SQ_WAVES", 0) < 100:
        continue
    w = v["SQ_WAVES"]
    cyc = v.get("SQ_WAVE_CYCLES", 1) or 1
    print(f"{k:40s} waves {w:9.0f} vgpr {v['_vgpr']:.0f} scratch {v['_scratch']:.0f}")
    print("   per wave: " + " ".join(f"{c[3:]}={v[c] / w:.0f}" for c in sorted(v) if c.startswith("SQ_INSTS")))
    print(f"   active {v.get('SQ_ACTIVE_INST_ANY', 0) / cyc:.2f} waitinst {v.get('SQ_WAIT_INST_ANY', 0) / cyc:.2f} "
          f"wait {v.get('SQ_WAIT_ANY', 0) / cyc:.2f} cyc/wave {cyc / w:.0f} GRBM_GUI_ACTIVE {v.get('GRBM_GUI_ACTIVE', 0):.3g}")
