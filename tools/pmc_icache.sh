set -o pipefail
# Instruction-cache and LDS-wait counters of the BC7 exact-search kernels, 64 block rows
# of 8K G1, one counter pass per run (2 SQC counters a pass).
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/ic
mkdir -p $O
timeout -k 10 120 rocprofv3 -L > $O/counters.txt 2>&1 || true
pass() {
  local name=$1; shift
  local C=""
  for c in "$@"; do grep -q "\b$c\b" $O/counters.txt && C="$C $c"; done
  [ -z "$C" ] && { echo "$name: none of $* listed"; return 0; }
  echo "$name: $C"
  timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $O/$name -o run -- \
    python3 $R/bench.py --format bc7 --rows 64 --no-cpu --steps 1 --warmup 1 > $O/$name.json 2> $O/$name.err
}
pass ic1 SQC_ICACHE_REQ SQC_ICACHE_MISSES SQ_WAVES SQ_IFETCH || exit 1
pass ic2 SQC_ICACHE_HITS SQC_ICACHE_MISSES_DUPLICATE SQ_WAVE_CYCLES SQ_IFETCH_LEVEL || exit 1
pass lds SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INST_LEVEL_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_INSTS_VALU || exit 1
python3 - $O <<'PY'
import csv, glob, sys, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(sys.argv[1] + "/*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("gic::bc7::", "")
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in sorted(agg.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
    if "bc7" in k or "shake" in k or "quant" in k or "dual" in k:
        print(k, " ".join(f"{c}={v[c]:.4g}" for c in sorted(v)))
PY
