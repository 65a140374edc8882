"""Per-launch VALU issue figures of a kernel from a rocprofv3 --pmc csv directory.

    python tools/valu_json.py <pmc dir> <kernel substring> <bench json> <out json> [--size S --rows R]
                              [--skip N --take M --leg KEY]

--skip/--take pick a window of the matching dispatches (two bench legs that
launch the same kernel template, e.g. bc7enc16 uber 4 then uber 0); --leg takes
the launch duration from that leg's kernel_ms.

Writes the per-launch SQ_INSTS_VALU (wave instructions, summed over the chip),
waves, and the VALU issue rate against the gfx950 peak (256 CUs x 4 SIMDs, one
wave-instruction per SIMD every 2 cycles at 2.4 GHz = 1.2288e12 /s; same figure
as the 157.3 TFLOP/s f32 vector peak, MI355X_MICROARCH.md).  The launch duration
is the kernel's own average from the --kernel-trace run when a kernel_stats csv
is given with --stats, else the bench line's kernel_ms.
"""
import argparse
import collections
import csv
import glob
import json

PEAK = 256 * 4 * 2.4e9 / 2


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("pmc_dir")
    ap.add_argument("kernel")
    ap.add_argument("bench_json")
    ap.add_argument("out")
    ap.add_argument("--stats", default="")
    ap.add_argument("--size", type=int, default=8192)
    ap.add_argument("--rows", type=int, default=8192)
    ap.add_argument("--skip", type=int, default=0, help="drop the first N matching dispatches")
    ap.add_argument("--take", type=int, default=0, help="keep at most N matching dispatches (0 = all)")
    ap.add_argument("--leg", default="", help="take kernel_ms from this sub-object of the bench line")
    a = ap.parse_args()
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    names = {}
    for f in glob.glob(a.pmc_dir + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if a.kernel not in r["Kernel_Name"]:
                continue
            d = int(r.get("Dispatch_Id") or r.get("Correlation_Id") or 0)
            per[d][r["Counter_Name"]] += float(r["Counter_Value"])
            names[d] = r["Kernel_Name"]
    if not per:
        raise SystemExit(f"no dispatch of {a.kernel} in {a.pmc_dir}")
    disp = sorted(per)[a.skip:]
    if a.take:
        disp = disp[:a.take]
    keys = sorted({k for d in disp for k in per[d]})
    avg = {k: sum(per[d][k] for d in disp) / len(disp) for k in keys}
    bench = json.loads(open(a.bench_json).read().strip().splitlines()[-1])
    if a.leg:
        bench = bench[a.leg]
    dur_ms = bench["kernel_ms"]
    src = "bench kernel_ms (HIP events, launch stream)" + (f", leg {a.leg}" if a.leg else "")
    if a.stats and not a.leg:
        for r in csv.DictReader(open(a.stats)):
            if a.kernel in r["Name"]:
                dur_ms = float(r["AverageNs"]) / 1e6
                src = f"rocprofv3 --kernel-trace --stats average ({a.stats})"
                break
    insts = avg["SQ_INSTS_VALU"]
    out = {
        "kernel": names[disp[0]],
        "size": a.size,
        "rows": a.rows,
        "dispatches": len(disp),
        "counters_per_launch": {k: avg[k] for k in keys},
        "valu_insts_per_launch": insts,
        "valu_insts_per_wave": insts / max(avg.get("SQ_WAVES", 1), 1),
        "launch_ms": dur_ms,
        "launch_ms_source": src,
        "valu_issue_rate": insts / (dur_ms * 1e-3),
        "valu_peak": PEAK,
        "valu_frac": insts / (dur_ms * 1e-3) / PEAK,
        "method": "rocprofv3 --pmc (counters only) over bench.py; SQ_INSTS_VALU summed over the chip per "
                  "dispatch, averaged over dispatches; peak = 256 CU x 4 SIMD x 2.4 GHz / 2 cycles per "
                  "wave64 VALU instruction",
    }
    if "SQ_ACTIVE_INST_VALU" in avg and "SQ_BUSY_CYCLES" in avg and avg["SQ_BUSY_CYCLES"]:
        out["active_inst_valu_per_busy_cycle"] = avg["SQ_ACTIVE_INST_VALU"] / avg["SQ_BUSY_CYCLES"]
    if "GRBM_GUI_ACTIVE" in avg:
        out["effective_clock_ghz"] = avg["GRBM_GUI_ACTIVE"] / 8 / (dur_ms * 1e-3) / 1e9
    json.dump(out, open(a.out, "w"), indent=1)
    print(json.dumps({k: out[k] for k in ("kernel", "valu_insts_per_launch", "valu_frac", "launch_ms")}))


if __name__ == "__main__":
    main()
