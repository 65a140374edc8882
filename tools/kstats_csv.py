"""Top kernels of a rocprofv3 --kernel-trace --stats csv directory: name, calls, total / average ms."""
import csv
import glob
import sys

f = sorted(glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True))[0]
rows = list(csv.DictReader(open(f)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:int(sys.argv[2]) if len(sys.argv) > 2 else 12]:
    name = r["Name"]
    k = name[name.find("k_"):name.find("(")] if "k_" in name else name[:40]
    print(f"{k:28s} {int(r['Calls']):5d} {float(r['TotalDurationNs']) / 1e6:10.3f} ms {float(r['AverageNs']) / 1e3:10.1f} us "
          f"{100 * float(r['TotalDurationNs']) / tot:5.1f} %")
print(f"total {tot / 1e6:.3f} ms")
