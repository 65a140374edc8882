"""Collect a round-3 profile set (tools/profile_r03.sh <tag>) into profiles/:
everything tools/collect_r02.py copies, plus the exact BC7 search's per-kernel
issue counters (64 block rows of 8K G1, one stream) with their launch times from
the kernel trace of the same command -> profiles/valu_bc7_<kernel>.json and
profiles/<tag>_pmc_valu_bc7.csv, profiles/<tag>_bc7_kernel_stats_single_stream.csv.

    python tools/collect_r03.py <tag>
"""
import collections
import csv
import glob
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    tag = sys.argv[1]
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "collect_r02.py"), tag], check=True)
    pr = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    P = os.path.join(ROOT, "profiles")
    stats = os.path.join(pr, "trace_bc7", "run_kernel_stats.csv")
    shutil.copy(stats, os.path.join(P, f"{tag}_bc7_kernel_stats_single_stream.csv"))
    vj = os.path.join(ROOT, "tools", "valu_json.py")
    for kern, out in (("k_shake_wave<8>", "valu_bc7_shake8.json"), ("k_shake_wave<4>", "valu_bc7_shake4.json"),
                      ("k_dual_wave", "valu_bc7_dual_wave.json"), ("k_quant_sub", "valu_bc7_quant_sub.json")):
        subprocess.run([sys.executable, vj, os.path.join(pr, "valu_bc7"), kern, os.path.join(pr, "bench.json"),
                        os.path.join(P, out), "--stats", stats, "--rows", "64"], check=True)
    per = collections.defaultdict(dict)
    for fn in glob.glob(os.path.join(pr, "valu_bc7", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(fn)):
            d = int(r["Dispatch_Id"])
            per[d]["Kernel_Name"] = r["Kernel_Name"]
            per[d][r["Counter_Name"]] = per[d].get(r["Counter_Name"], 0) + float(r["Counter_Value"])
    keys = sorted({k for d in per for k in per[d] if k != "Kernel_Name"})
    with open(os.path.join(P, f"{tag}_pmc_valu_bc7.csv"), "w") as fo:
        wr = csv.writer(fo)
        wr.writerow(["Dispatch_Id", "Kernel_Name"] + keys)
        for d in sorted(per):
            wr.writerow([d, per[d]["Kernel_Name"]] + [int(per[d].get(k, 0)) for k in keys])


if __name__ == "__main__":
    main()
