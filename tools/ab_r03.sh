# A/B timing of library variants on the GPU box (round 3):
#   bash tools/ab_r03.sh <tag> <variant>...   -> gpurun_out/ab_<tag>/
# BC7 exact on 256 block rows and the BC4/BC5 legs, the in-tree library first,
# each variant from gpurun_dbg/<variant>/lib.so, twice in alternation; then the
# GPU test suite on the in-tree library.
set -o pipefail
TAG=$1; shift
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/ab_$TAG
mkdir -p $O
cd $R
for rep in 1 2; do
  for v in default "$@"; do
    if [ "$v" = default ]; then L=""; else L=$R/gpurun_dbg/$v/lib.so; fi
    echo "== $v" >> $O/bc7.txt
    GIC_LIBRARY=$L timeout -k 10 300 python3 tools/time_bc7_bounded.py --rows 256 --bound 0 >> $O/bc7.txt 2>&1 || exit 1
    GIC_LIBRARY=$L timeout -k 10 300 python3 bench.py --no-cpu --bc7-rows 0 --no-bc7enc --bc6h-size 0 --steps 10 > $O/bcx_$v.json 2>>$O/bcx.err || exit 1
    python3 -c "import json,sys; d=json.load(open('$O/bcx_$v.json')); print('$v', 'bc1', d['kernel_ms'], 'bc4', d['bc4']['kernel_ms'], 'bc5', d['bc5']['kernel_ms'])" >> $O/bcx.txt
  done
done
cat $O/bc7.txt | grep -v amdgpu.ids
cat $O/bcx.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
echo done
