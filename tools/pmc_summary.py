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
    if "SQC_ICACHE_MISSES" in v:
        h, m = v.get("SQC_ICACHE_HITS", 0), v["SQC_ICACHE_MISSES"]
        print(f"   icache hits {h:.3g} misses {m:.3g} miss rate {m / max(h + m, 1):.4f} ifetch/wave "
              f"{v.get('SQ_IFETCH', 0) / w:.0f}")
    if "SQ_INSTS_VALU" in v and "SQ_BUSY_CYCLES" in v:
        print(f"   totals: VALU {v['SQ_INSTS_VALU']:.4g} SALU {v.get('SQ_INSTS_SALU', 0):.4g} "
              f"wave-cycles {v.get('SQ_WAVE_CYCLES', 0):.4g} busy-cycles {v['SQ_BUSY_CYCLES']:.4g}")
