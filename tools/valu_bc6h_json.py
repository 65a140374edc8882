"""Per-step VALU issue figures of the BC6H encoder (all its kernels) from a
tools/prof_bc6h_r04.sh directory (trace/ = --kernel-trace, pmc/ = the SQ
counters of the same workload, run separately).

    python tools/valu_bc6h_json.py <dir> <out json> [--size 1024]

tools/time_bc6h.py makes a small warm-up call (64 texel rows) and then full
calls; only the dispatches of the full calls are used (per kernel, the ones of
the largest grid), averaged per call.  valu_insts_per_step = SQ_INSTS_VALU
summed over the chip and over every gic::bc6h kernel of one call; bench.py's
bc6h legs divide it by their own measured step duration.  The per-kernel rows
keep the time split and the issue fraction against the gfx950 peak (256 CUs x
4 SIMDs, one wave64 VALU instruction per SIMD every 2 cycles at 2.4 GHz).
"""
import argparse
import collections
import csv
import glob
import json

PEAK = 256 * 4 * 2.4e9 / 2


def _grid(r):
    if "Grid_Size" in r:
        return int(r["Grid_Size"])
    return int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])


def _full_dispatches(rows, key):
    """{dispatch id: row} of the largest-grid dispatches of each bc6h kernel"""
    by = collections.defaultdict(list)
    for r in rows:
        if "bc6h" in r["Kernel_Name"]:
            by[r["Kernel_Name"]].append(r)
    out = {}
    for name, rs in by.items():
        g = max(_grid(r) for r in rs)
        for r in rs:
            if _grid(r) == g:
                out[int(r[key])] = r
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("out")
    ap.add_argument("--size", type=int, default=1024)
    a = ap.parse_args()
    trace = []
    for f in glob.glob(a.dir + "/trace/**/*kernel_trace.csv", recursive=True):
        trace += list(csv.DictReader(open(f)))
    full = _full_dispatches(trace, "Dispatch_Id")
    dur = collections.defaultdict(list)
    for r in full.values():
        dur[r["Kernel_Name"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    pmc_rows = []
    for f in glob.glob(a.dir + "/pmc/**/*counter_collection.csv", recursive=True):
        pmc_rows += list(csv.DictReader(open(f)))
    gmax = collections.defaultdict(int)
    for r in pmc_rows:
        if "bc6h" in r["Kernel_Name"]:
            gmax[r["Kernel_Name"]] = max(gmax[r["Kernel_Name"]], _grid(r))
    cnt = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in pmc_rows:
        if "bc6h" in r["Kernel_Name"] and _grid(r) == gmax[r["Kernel_Name"]]:
            cnt[r["Kernel_Name"]][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[r["Kernel_Name"]].add(int(r["Dispatch_Id"]))
    if not dur or not cnt:
        raise SystemExit(f"no gic::bc6h kernels in {a.dir}")
    kernels = {}
    tot_ms = tot_v = 0.0
    for name in sorted(dur, key=lambda k: -sum(dur[k])):
        ms = sum(dur[name]) / len(dur[name])
        nd = max(1, len(disp[name]))
        c = {k: v / nd for k, v in cnt[name].items()}
        v = c.get("SQ_INSTS_VALU", 0.0)
        tot_ms += ms
        tot_v += v
        kernels[name.split("(")[0]] = {
            "ms_per_call": round(ms, 4), "counters_per_call": {k: c[k] for k in sorted(c)},
            "valu_issue_frac": round(v / (ms * 1e-3) / PEAK, 4) if ms else 0.0,
            "salu_per_valu": round(c.get("SQ_INSTS_SALU", 0.0) / v, 4) if v else 0.0,
        }
    out = {
        "kernel": "gic::bc6h (k_bc6h_prep + quant + shake + final + encode)",
        "size": a.size, "rows": a.size,
        "valu_insts_per_step": tot_v,
        "kernel_ms_per_step": round(tot_ms, 4),
        "valu_frac": round(tot_v / (tot_ms * 1e-3) / PEAK, 4),
        "valu_peak": PEAK,
        "kernels": kernels,
        "method": "rocprofv3 --pmc (counters only) and, in its own run, --kernel-trace over tools/time_bc6h.py "
                  "(a 64-row warm-up call, then full calls: only the full calls' dispatches); per-call averages; "
                  "peak = 256 CU x 4 SIMD x 2.4 GHz / 2",
    }
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(f"{a.out}: {tot_v:.4g} VALU/step, {tot_ms:.2f} ms/step, issue {100 * out['valu_frac']:.1f}%")
    for k, v in kernels.items():
        print(f"  {k[-28:]:28s} {v['ms_per_call']:9.3f} ms  issue {100 * v['valu_issue_frac']:5.1f}%  "
              f"SALU/VALU {v['salu_per_valu']:.2f}")


if __name__ == "__main__":
    main()
