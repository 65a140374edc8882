"""Per-step VALU issue figures of the BC6H encoder (all its kernels) from a
tools/prof_bc6h_r04.sh directory (trace/ = --kernel-trace --stats, pmc/ = the
SQ counters of the same workload, run separately).

    python tools/valu_bc6h_json.py <dir> <out json> [--size 1024] [--steps 3]

valu_insts_per_step = SQ_INSTS_VALU summed over the chip and over every
gic::bc6h kernel, / the number of encoder calls (steps) the run made;
bench.py's bc6h legs divide it by their own measured step duration.  The
per-kernel rows keep the time split and the issue fraction against the gfx950
peak (256 CUs x 4 SIMDs, one wave64 VALU instruction per SIMD every 2 cycles at
2.4 GHz).
"""
import argparse
import collections
import csv
import glob
import json

PEAK = 256 * 4 * 2.4e9 / 2


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("out")
    ap.add_argument("--size", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=3)
    a = ap.parse_args()
    stats = {}
    for f in glob.glob(a.dir + "/trace/**/*kernel_stats.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "bc6h" in r["Name"]:
                stats[r["Name"]] = (int(r["Calls"]), float(r["TotalDurationNs"]) / 1e6)
    cnt = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(a.dir + "/pmc/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "bc6h" in r["Kernel_Name"]:
                cnt[r["Kernel_Name"]][r["Counter_Name"]] += float(r["Counter_Value"])
    if not stats or not cnt:
        raise SystemExit(f"no gic::bc6h kernels in {a.dir}")
    kernels = {}
    for name, (calls, ms) in sorted(stats.items(), key=lambda kv: -kv[1][1]):
        c = cnt.get(name, {})
        v = c.get("SQ_INSTS_VALU", 0.0)
        kernels[name.split("(")[0]] = {
            "calls": calls, "total_ms": round(ms, 4),
            "counters": {k: c[k] for k in sorted(c)},
            "valu_issue_frac": round(v / (ms * 1e-3) / PEAK, 4) if ms else 0.0,
            "salu_per_valu": round(c.get("SQ_INSTS_SALU", 0.0) / v, 4) if v else 0.0,
        }
    tot_ms = sum(ms for _, ms in stats.values())
    tot_v = sum(c.get("SQ_INSTS_VALU", 0.0) for c in cnt.values())
    out = {
        "kernel": "gic::bc6h (k_bc6h_quant + k_bc6h_shake + k_bc6h_final)",
        "size": a.size, "rows": a.size, "steps": a.steps,
        "valu_insts_per_step": tot_v / a.steps,
        "kernel_ms_per_step": round(tot_ms / a.steps, 4),
        "valu_frac": round(tot_v / (tot_ms * 1e-3) / PEAK, 4),
        "valu_peak": PEAK,
        "kernels": kernels,
        "method": "rocprofv3 --pmc (counters only) and, in its own run, --kernel-trace --stats over "
                  "tools/time_bc6h.py (warm-up call + 2 timed calls); peak = 256 CU x 4 SIMD x 2.4 GHz / 2",
    }
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(f"{a.out}: {tot_v / a.steps:.4g} VALU/step, {tot_ms / a.steps:.2f} ms/step, "
          f"issue {100 * out['valu_frac']:.1f}%")


if __name__ == "__main__":
    main()
