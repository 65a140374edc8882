# VALU/SALU issue counters of the BC7 kernels, one --pmc pass (counters only).
#   bash tools/pmc_bc7_valu.sh <tag> [rows]  -> gpurun_out/pmc7_<tag>/
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/pmc7_$1
ROWS=${2:-64}
mkdir -p $O
C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv -d $O -o run -- \
  python3 $R/bench.py --format bc7 --rows $ROWS --no-cpu --steps 1 --warmup 1 > $O/bc7.json 2> $O/bc7.err || exit 1
python3 - $O <<'PY'
import csv, glob, sys, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0][-28:]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in sorted(agg.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
    if v.get("SQ_WAVE_CYCLES", 0) < 1e6: continue
    print(k, " ".join(f"{c[3:]}={v[c]:.3g}" for c in sorted(v)))
PY
