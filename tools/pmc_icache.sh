set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/ic
mkdir -p $O
timeout -k 10 120 rocprofv3 -L > $O/counters.txt 2>&1 || true
C=""
for c in SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_IFETCH_LEVEL SQ_INSTS_SMEM SQ_INST_LEVEL_SMEM; do
  grep -q "\b$c\b" $O/counters.txt && C="$C $c"
done
echo "counters: $C"
timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv -d $O/p -o run -- python3 $R/bench.py --format bc7 --rows 64 --no-cpu --steps 1 --warmup 1 > $O/bc7.json 2> $O/bc7.err || exit 1
python3 - $O/p <<'PY'
import csv, glob, sys, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0][-28:]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in agg.items():
    if "shake_wave<8>" in k or "quant_reg<3>" in k or "shake_wave<4>" in k:
        print(k, " ".join(f"{c}={v[c]:.3g}" for c in sorted(v)))
PY
