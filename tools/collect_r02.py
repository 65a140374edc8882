"""Copy a round-2 profile set (tools/profile_r02b.sh <tag> + tools/pmc_traffic_bc1.sh
<tag>) from gpurun_out/prof_<tag>/ into profiles/ and regenerate the VALU and
traffic summaries the bench reads.

    python tools/collect_r02.py <tag>
"""
import collections
import csv
import glob
import json
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
from refresh_profiles import per_launch   # noqa: E402


def main():
    tag = sys.argv[1]
    pr = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    P = os.path.join(ROOT, "profiles")
    vj = os.path.join(ROOT, "tools", "valu_json.py")
    b = os.path.join(pr, "bench.json")
    for kern, out, extra in (("bc1_image_kernel", "valu_bc1.json", ["--take", "4"]),
                             ("bc7enc_image_kernel", "valu_bc7enc16.json", ["--take", "4", "--leg", "bc7enc16"]),
                             ("bc7enc_image_kernel", "valu_bc7enc16_fast.json",
                              ["--skip", "4", "--take", "4", "--leg", "bc7enc16_fast"])):
        subprocess.run([sys.executable, vj, os.path.join(pr, "valu"), kern, b, os.path.join(P, out)] + extra, check=True)
    f, nf = per_launch(os.path.join(pr, "pmc_fetch", "run_counter_collection.csv"), "bc1_image_kernel", "FETCH_SIZE")
    w, _ = per_launch(os.path.join(pr, "pmc_write", "run_counter_collection.csv"), "bc1_image_kernel", "WRITE_SIZE")
    tj = os.path.join(P, "traffic_bc1.json")
    t = json.load(open(tj))
    t.update({"fetch_size_kb_per_launch": f, "write_size_kb_per_launch": w,
              "hbm_bytes_per_launch": int(round((2 * f + w) * 1024)),
              "source": f"gpurun_out/prof_{tag}/pmc_{{fetch,write}}/run_counter_collection.csv, {nf} launches "
                        f"averaged (tools/pmc_traffic_bc1.sh)"})
    json.dump(t, open(tj, "w"), indent=1)
    print("traffic / algorithmic", t["hbm_bytes_per_launch"] / t["alg_bytes_per_launch"])
    for src, dst in (("bench.json", "bench.json"), ("bench_under_rocprof.json", "bench_under_rocprof.json"),
                     ("trace/run_kernel_stats.csv", "kernel_stats.csv"),
                     ("pmc_fetch/run_counter_collection.csv", "pmc_fetch_size.csv"),
                     ("pmc_write/run_counter_collection.csv", "pmc_write_size.csv")):
        shutil.copy(os.path.join(pr, src), os.path.join(P, f"{tag}_{dst}"))
    per = collections.defaultdict(dict)
    for fn in glob.glob(os.path.join(pr, "valu", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(fn)):
            d = int(r["Dispatch_Id"])
            per[d]["Kernel_Name"] = r["Kernel_Name"]
            per[d][r["Counter_Name"]] = per[d].get(r["Counter_Name"], 0) + float(r["Counter_Value"])
    keys = sorted({k for d in per for k in per[d] if k != "Kernel_Name"})
    with open(os.path.join(P, f"{tag}_pmc_valu.csv"), "w") as fo:
        wr = csv.writer(fo)
        wr.writerow(["Dispatch_Id", "Kernel_Name"] + keys)
        for d in sorted(per):
            if "gic::" in per[d]["Kernel_Name"]:
                wr.writerow([d, per[d]["Kernel_Name"]] + [int(per[d].get(k, 0)) for k in keys])
    d = json.loads(open(b).read().strip().splitlines()[-1])
    print("BC1", d["value"], d["ms_per_step"], d["cpu_baseline"]["value"], d["cpu_baseline"]["gpu_parity"])
    for k in ("bc7", "bc7_pruned", "bc7_bounded", "bc7_bounded_pruned", "bc7enc16", "bc7enc16_fast", "bc4", "bc5"):
        v = d.get(k)
        if v:
            print(k, v["value"], v.get("ms_per_pass", v.get("ms_per_step")), v.get("cpu_baseline", {}).get("value"),
                  v.get("gpu_parity"))


if __name__ == "__main__":
    main()
