"""VALU wave-instructions of one whole BC7 pass from a rocprofv3 --pmc csv directory.

    python tools/valu_pass.py <pmc dir> <out json> --match gic::bc7:: [--size 8192 --rows 2048]
                              [--passes 1] [--label ...]

Sums every counter over all dispatches whose kernel name contains --match
(the whole phase pipeline of one pass: prep, quantisers, shakers, select),
divides by --passes, and lists the per-kernel shares.  bench.py divides
`valu_insts_per_pass` by the pass time it measures live (HIP events) to get
the pass's VALU issue fraction against the gfx950 peak (256 CUs x 4 SIMDs x
2.4 GHz / 2 cycles per wave64 VALU instruction = 1.2288e12 /s).
"""
import argparse
import collections
import csv
import glob
import json


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("pmc_dir")
    ap.add_argument("out")
    ap.add_argument("--match", default="gic::bc7::")
    ap.add_argument("--size", type=int, default=8192)
    ap.add_argument("--rows", type=int, default=2048, help="block rows of the pass")
    ap.add_argument("--passes", type=int, default=1)
    ap.add_argument("--label", default="")
    ap.add_argument("--command", default="")
    a = ap.parse_args()
    tot = collections.defaultdict(float)
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = set()
    for f in glob.glob(a.pmc_dir + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            if a.match not in name:
                continue
            k = name[name.find("k_"):name.find("(")] if "k_" in name else name[:60]
            v = float(r["Counter_Value"])
            tot[r["Counter_Name"]] += v
            per[k][r["Counter_Name"]] += v
            disp.add(r.get("Dispatch_Id") or r.get("Correlation_Id"))
    if not tot:
        raise SystemExit(f"no dispatch matching {a.match} in {a.pmc_dir}")
    valu = tot["SQ_INSTS_VALU"] / a.passes
    kernels = sorted(per, key=lambda k: -per[k]["SQ_INSTS_VALU"])
    out = {
        "label": a.label,
        "size": a.size,
        "rows": a.rows,
        "passes": a.passes,
        "dispatches": len(disp),
        "valu_insts_per_pass": valu,
        "counters_per_pass": {k: v / a.passes for k, v in sorted(tot.items())},
        "kernels": {k: {"valu_insts_per_pass": per[k]["SQ_INSTS_VALU"] / a.passes,
                        "share_of_valu": round(per[k]["SQ_INSTS_VALU"] / tot["SQ_INSTS_VALU"], 4)}
                    for k in kernels},
        "command": a.command,
        "method": "rocprofv3 --pmc (counters only, kernels serialised) over one pass; SQ_INSTS_VALU summed over "
                  "the chip and over every dispatch of the pass; bench.py divides by its own live pass time",
    }
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(f"{a.out}: {valu:.4g} VALU wave-instructions per pass over {len(disp)} dispatches")


if __name__ == "__main__":
    main()
