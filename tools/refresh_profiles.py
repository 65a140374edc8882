"""Copy a round's GPU profile outputs into profiles/ (the committed evidence).

    python tools/refresh_profiles.py <prof tag> <valu tag> <bc7 single-stream dir> [round]
e.g. python tools/refresh_profiles.py r01d r01c prof_r01c_bc7 r01

Inputs (under gpurun_out/, written by tools/profile_round.sh, tools/pmc_valu.sh
and tools/profile_round2.sh on the GPU box): the default bench line, the same
command under rocprofv3 --kernel-trace --stats, the separate FETCH_SIZE /
WRITE_SIZE PMC passes of the BC1 kernel, the VALU PMC passes, and a
single-stream BC7 kernel-trace run.
"""
import collections
import csv
import json
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
G = os.path.join(ROOT, "gpurun_out")
P = os.path.join(ROOT, "profiles")


def per_launch(path, kernel, ctr):
    d = collections.defaultdict(float)
    for r in csv.DictReader(open(path)):
        if kernel in r["Kernel_Name"] and r["Counter_Name"] == ctr:
            d[r.get("Dispatch_Id") or r.get("Correlation_Id")] += float(r["Counter_Value"])
    return sum(d.values()) / len(d), len(d)


def main():
    tag, vtag, bc7dir = sys.argv[1], sys.argv[2], sys.argv[3]
    rnd = sys.argv[4] if len(sys.argv) > 4 else "r01"
    pr = os.path.join(G, f"prof_{tag}")
    f, nf = per_launch(os.path.join(pr, "pmc_fetch", "run_counter_collection.csv"), "bc1_image_kernel", "FETCH_SIZE")
    w, _ = per_launch(os.path.join(pr, "pmc_write", "run_counter_collection.csv"), "bc1_image_kernel", "WRITE_SIZE")
    tj = os.path.join(P, "traffic_bc1.json")
    out = json.load(open(tj))
    out.update({"fetch_size_kb_per_launch": f, "write_size_kb_per_launch": w,
                "hbm_bytes_per_launch": int(round((2 * f + w) * 1024)),
                "source": f"gpurun_out/prof_{tag}/pmc_{{fetch,write}}/run_counter_collection.csv, {nf} launches averaged"})
    json.dump(out, open(tj, "w"), indent=1)
    print("traffic / algorithmic", out["hbm_bytes_per_launch"] / out["alg_bytes_per_launch"])
    for src, dst in (("bench.json", f"{rnd}_bench.json"), ("bench_under_rocprof.json", f"{rnd}_bench_under_rocprof.json"),
                     ("trace/run_kernel_stats.csv", f"{rnd}_kernel_stats.csv"),
                     ("pmc_fetch/run_counter_collection.csv", f"{rnd}_pmc_fetch_size.csv"),
                     ("pmc_write/run_counter_collection.csv", f"{rnd}_pmc_write_size.csv")):
        shutil.copy(os.path.join(pr, src), os.path.join(P, dst))
    shutil.copy(os.path.join(G, bc7dir, "run_kernel_stats.csv"), os.path.join(P, f"{rnd}_bc7_kernel_stats_single_stream.csv"))
    shutil.copy(os.path.join(G, bc7dir + ".json"), os.path.join(P, f"{rnd}_bc7_single_stream_bench.json"))
    v = os.path.join(G, f"valu_{vtag}")
    vj = os.path.join(ROOT, "tools", "valu_json.py")
    subprocess.run([sys.executable, vj, os.path.join(v, "bc1"), "bc1_image_kernel", os.path.join(v, "bc1.json"),
                    os.path.join(P, "valu_bc1.json"), "--stats", os.path.join(P, f"{rnd}_kernel_stats.csv")], check=True)
    subprocess.run([sys.executable, vj, os.path.join(v, "bc7"), "k_shake_wave<8>", os.path.join(v, "bc7.json"),
                    os.path.join(P, "valu_bc7_shake8.json"), "--rows", "128", "--stats",
                    os.path.join(P, f"{rnd}_bc7_kernel_stats_single_stream.csv")], check=True)
    d = json.loads(open(os.path.join(P, f"{rnd}_bench.json")).read().strip().splitlines()[-1])
    print(d["value"], d["ms_per_step"], d["roofline"], d["bc7"]["value"], d["bc7"]["ms_per_pass"], d["bc7"]["gpu_parity"])
    for r in list(csv.DictReader(open(os.path.join(P, f"{rnd}_bc7_kernel_stats_single_stream.csv"))))[:8]:
        print(r["Name"][:50], r["Calls"], round(float(r["AverageNs"]) / 1e6, 3), r["Percentage"])


if __name__ == "__main__":
    main()
