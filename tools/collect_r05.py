"""Collect the round-5 profile set (tools/profile_r05.sh <tag> bench|pmc) into profiles/.

    python tools/collect_r05.py <tag>

Writes <tag>_bench.json, <tag>_bench_under_rocprof.json, <tag>_kernel_stats.csv,
<tag>_pmc_valu.csv, <tag>_pmc_valu_bc7.csv, <tag>_bc7_kernel_stats_single_stream.csv,
<tag>_pmc_{fetch,write}_size.csv and regenerates valu_bc1.json, valu_bc7enc16*.json,
valu_bc7_{shake8,shake4,dual_wave,quant_sub}.json, valu_bc7*_pass.json, valu_bc6h_shake*.json,
traffic_bc1.json.
"""
import csv
import json
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
from collect_r04 import flatten          # noqa: E402
from refresh_profiles import per_launch  # noqa: E402


def main():
    tag = sys.argv[1]
    pr = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    P = os.path.join(ROOT, "profiles")
    b = os.path.join(pr, "bench.json")
    vj = os.path.join(ROOT, "tools", "valu_json.py")
    py = sys.executable
    for kern, out, extra in (("bc1_image_kernel", "valu_bc1.json", ["--take", "4"]),
                             ("bc7enc_image_kernel", "valu_bc7enc16.json", ["--take", "4", "--leg", "bc7enc16"]),
                             ("bc7enc_image_kernel", "valu_bc7enc16_fast.json",
                              ["--skip", "4", "--take", "4", "--leg", "bc7enc16_fast"])):
        subprocess.run([py, vj, os.path.join(pr, "valu"), kern, b, os.path.join(P, out)] + extra, check=True)
    stats = os.path.join(pr, "trace_bc7", "run_kernel_stats.csv")
    for kern, out in (("k_shake_wave<8>", "valu_bc7_shake8.json"), ("k_shake_wave<4>", "valu_bc7_shake4.json"),
                      ("k_dual_wave(", "valu_bc7_dual_wave.json"), ("k_quant_sub", "valu_bc7_quant_sub.json")):
        subprocess.run([py, vj, os.path.join(pr, "valu_bc7"), kern, b, os.path.join(P, out), "--stats", stats,
                        "--rows", "64"], check=True)
    for leg, k, bound in (("bc7", 0, 0), ("bc7_pruned", 2, 0), ("bc7_bounded", 0, 0.5), ("bc7_bounded_pruned", 2, 0.5)):
        subprocess.run([py, os.path.join(ROOT, "tools", "valu_pass.py"), os.path.join(pr, f"pass_{leg}"),
                        os.path.join(P, f"valu_{leg}_pass.json"), "--label",
                        f"{leg}: 8K G1 one pass, shake ranks {k}, bound {bound}", "--command",
                        f"tools/time_bc7_bounded.py --rows 2048 --shake-ranks {k} --bound {bound} --no-warm"],
                       check=True)
    p6 = os.path.join(ROOT, "gpurun_out", f"p6_{tag}")
    for k, out in (("unsigned", "valu_bc6h_shake.json"), ("signed", "valu_bc6h_shake_signed.json")):
        if os.path.isdir(os.path.join(p6, k)):
            subprocess.run([py, os.path.join(ROOT, "tools", "valu_bc6h_json.py"), os.path.join(p6, k),
                            os.path.join(P, out), "--size", "1024"], check=True)
    f, nf = per_launch(os.path.join(pr, "pmc_fetch", "run_counter_collection.csv"), "bc1_image_kernel", "FETCH_SIZE")
    w, _ = per_launch(os.path.join(pr, "pmc_write", "run_counter_collection.csv"), "bc1_image_kernel", "WRITE_SIZE")
    tj = os.path.join(P, "traffic_bc1.json")
    out = json.load(open(tj))
    out.update({"fetch_size_kb_per_launch": f, "write_size_kb_per_launch": w,
                "hbm_bytes_per_launch": int(round((2 * f + w) * 1024)),
                "source": f"gpurun_out/prof_{tag}/pmc_{{fetch,write}}/run_counter_collection.csv, {nf} launches averaged "
                          f"(tools/profile_r05.sh)"})
    json.dump(out, open(tj, "w"), indent=1)
    print("traffic / algorithmic", out["hbm_bytes_per_launch"] / out["alg_bytes_per_launch"])
    for src, dst in (("bench.json", f"{tag}_bench.json"), ("bench_under_rocprof.json", f"{tag}_bench_under_rocprof.json"),
                     ("trace/run_kernel_stats.csv", f"{tag}_kernel_stats.csv"),
                     ("pmc_fetch/run_counter_collection.csv", f"{tag}_pmc_fetch_size.csv"),
                     ("pmc_write/run_counter_collection.csv", f"{tag}_pmc_write_size.csv"),
                     ("trace_bc7/run_kernel_stats.csv", f"{tag}_bc7_kernel_stats_single_stream.csv"),
                     ("block_latency.txt", f"{tag}_block_latency.txt")):
        if os.path.exists(os.path.join(pr, src)):
            shutil.copy(os.path.join(pr, src), os.path.join(P, dst))
    flatten(os.path.join(pr, "valu", "**", "*counter_collection.csv"), os.path.join(P, f"{tag}_pmc_valu.csv"))
    flatten(os.path.join(pr, "valu_bc7", "**", "*counter_collection.csv"), os.path.join(P, f"{tag}_pmc_valu_bc7.csv"))
    d = json.loads(open(b).read().strip().splitlines()[-1])
    print(d["value"], d["ms_per_step"], d["bc7"]["value"], d["bc7"]["ms_per_pass"], d["bc7"]["roofline"].get("valu"))


if __name__ == "__main__":
    main()
