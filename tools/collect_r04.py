"""Collect the round-4 profile set into profiles/: tools/profile_r04.sh <tag> prof
(bench under --kernel-trace, SQ counters of the bench legs and of the exact BC7
search) plus the default bench line gpurun_out/<bench dir>/bench.json of the same
tree.  Regenerates profiles/valu_bc1.json, valu_bc7enc16*.json, valu_bc7_*.json and
writes <tag>_kernel_stats.csv, <tag>_bench_under_rocprof.json, <tag>_pmc_valu.csv,
<tag>_pmc_valu_bc7.csv, <tag>_bc7_kernel_stats_single_stream.csv.

    python tools/collect_r04.py <tag> <bench dir under gpurun_out>
"""
import collections
import csv
import glob
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def flatten(src_glob, out, keep="gic::"):
    per = collections.defaultdict(dict)
    for fn in glob.glob(src_glob, recursive=True):
        for r in csv.DictReader(open(fn)):
            d = int(r["Dispatch_Id"])
            per[d]["Kernel_Name"] = r["Kernel_Name"]
            per[d][r["Counter_Name"]] = per[d].get(r["Counter_Name"], 0) + float(r["Counter_Value"])
    keys = sorted({k for d in per for k in per[d] if k != "Kernel_Name"})
    with open(out, "w") as fo:
        wr = csv.writer(fo)
        wr.writerow(["Dispatch_Id", "Kernel_Name"] + keys)
        for d in sorted(per):
            if keep in per[d]["Kernel_Name"]:
                wr.writerow([d, per[d]["Kernel_Name"]] + [int(per[d].get(k, 0)) for k in keys])


def main():
    tag, bdir = sys.argv[1], sys.argv[2]
    pr = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    P = os.path.join(ROOT, "profiles")
    b = os.path.join(ROOT, "gpurun_out", bdir, "bench.json")
    vj = os.path.join(ROOT, "tools", "valu_json.py")
    for kern, out, extra in (("bc1_image_kernel", "valu_bc1.json", ["--take", "4"]),
                             ("bc7enc_image_kernel", "valu_bc7enc16.json", ["--take", "4", "--leg", "bc7enc16"]),
                             ("bc7enc_image_kernel", "valu_bc7enc16_fast.json",
                              ["--skip", "4", "--take", "4", "--leg", "bc7enc16_fast"])):
        subprocess.run([sys.executable, vj, os.path.join(pr, "valu"), kern, b, os.path.join(P, out)] + extra, check=True)
    stats = os.path.join(pr, "trace_bc7", "run_kernel_stats.csv")
    for kern, out in (("k_shake_wave<8>", "valu_bc7_shake8.json"), ("k_shake_wave<4>", "valu_bc7_shake4.json"),
                      ("k_dual_wave(", "valu_bc7_dual_wave.json"), ("k_quant_sub", "valu_bc7_quant_sub.json")):
        subprocess.run([sys.executable, vj, os.path.join(pr, "valu_bc7"), kern, b, os.path.join(P, out), "--stats",
                        stats, "--rows", "64"], check=True)
    shutil.copy(stats, os.path.join(P, f"{tag}_bc7_kernel_stats_single_stream.csv"))
    shutil.copy(os.path.join(pr, "trace", "run_kernel_stats.csv"), os.path.join(P, f"{tag}_kernel_stats.csv"))
    shutil.copy(os.path.join(pr, "bench_under_rocprof.json"), os.path.join(P, f"{tag}_bench_under_rocprof.json"))
    flatten(os.path.join(pr, "valu", "**", "*counter_collection.csv"), os.path.join(P, f"{tag}_pmc_valu.csv"))
    flatten(os.path.join(pr, "valu_bc7", "**", "*counter_collection.csv"), os.path.join(P, f"{tag}_pmc_valu_bc7.csv"))


if __name__ == "__main__":
    main()
