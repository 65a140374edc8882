"""Per-kernel time (rocprofv3 --stats csv) joined with the SQ issue counters
(--pmc csv) of the same workload: VALU issue fraction against the gfx950 peak
(one wave64 VALU instruction per SIMD every 2 cycles at 2.4 GHz), SALU/VALU,
wait-inst share.   python tools/kstats_pmc.py <dir with trace/ and pmc/>"""
import collections
import csv
import glob
import sys

PEAK = 256 * 4 * 2.4e9 / 2

d = sys.argv[1]
stats = {}
for f in glob.glob(d + "/trace/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        stats[r["Name"]] = (int(r["Calls"]), float(r["TotalDurationNs"]) / 1e6, float(r["AverageNs"]) / 1e6)
cnt = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(d + "/pmc/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        cnt[r["Kernel_Name"]][r["Counter_Name"]] += float(r["Counter_Value"])
tot = sum(v[1] for v in stats.values())
print(f"total kernel time {tot:.2f} ms")
for name, (calls, ms, avg) in sorted(stats.items(), key=lambda kv: -kv[1][1]):
    if ms < 0.005 * tot:
        continue
    c = cnt.get(name, {})
    v, sa = c.get("SQ_INSTS_VALU", 0), c.get("SQ_INSTS_SALU", 0)
    wc, wi = c.get("SQ_WAVE_CYCLES", 0), c.get("SQ_WAIT_INST_ANY", 0)
    frac = v / (ms * 1e-3) / PEAK if ms else 0
    print(f"{name.split('(')[0][-34:]:34s} {calls:4d} calls {ms:9.2f} ms ({100 * ms / tot:5.1f}%)  VALU {v:.3g} "
          f"issue {100 * frac:5.1f}%  SALU/VALU {sa / v if v else 0:.2f}  wait/wave-cyc {wi / wc if wc else 0:.2f}  "
          f"waves {c.get('SQ_WAVES', 0):.3g}")
