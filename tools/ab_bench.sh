# A/B of whole-library variants over the bench legs (BC1, BC4/BC5, bc7enc16, BC6H,
# BC7 exact on --bc7-rows block rows), twice in alternation: in-tree library first,
# then gpurun_var/<variant>/lib.so.   bash tools/ab_bench.sh <tag> <bc7 rows> <variant>...
set -o pipefail
TAG=$1; ROWS=$2; shift 2
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/abb_$TAG
mkdir -p $O
cd $R
for rep in 1 2; do
  for v in default "$@"; do
    if [ "$v" = default ]; then L=""; else L=$R/gpurun_var/$v/lib.so; fi
    GIC_LIBRARY=$L timeout -k 10 400 python3 bench.py --steps 10 --warmup 2 --no-cpu --no-batch --bc7-rows $ROWS \
        --bc7-shake-ranks 0 --bc7-mse-bound 0 > $O/${v}_$rep.json 2> $O/${v}_$rep.err || { tail -20 $O/${v}_$rep.err; exit 1; }
    python3 - $O/${v}_$rep.json $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
out = [f"bc1 {d['ms_per_step']:.3f}"]
for k in ("bc4", "bc5", "bc7enc16", "bc7enc16_fast", "bc6h", "bc6h_signed", "bc7"):
    if k in d:
        x = d[k]
        out.append(f"{k} {x.get('ms_per_step', x.get('ms_per_pass', 0)):.3f}")
print(sys.argv[2], " ".join(out), flush=True)
PY
  done
done
echo done
