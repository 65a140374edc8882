# A/B timing of BC1 library variants on the 8K G1 texture (tools/time_bc1.py),
# in-tree library first, then gpurun_var/<variant>/lib.so, twice in
# alternation; then the GPU tests matching a pytest -k expression.
#   bash tools/ab_bc1.sh <tag> "<pytest -k>" <variant>...   -> gpurun_out/ab_<tag>/
set -o pipefail
TAG=$1; K=$2; shift 2
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/ab_$TAG
mkdir -p $O
cd $R
for rep in 1 2; do
  for v in default "$@"; do
    if [ "$v" = default ]; then L=""; else L=$R/gpurun_var/$v/lib.so; fi
    GIC_LIBRARY=$L timeout -k 10 200 python3 tools/time_bc1.py 20 >> $O/bc1.txt 2>&1 || exit 1
  done
done
grep -v amdgpu.ids $O/bc1.txt
if [ -n "$K" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$K" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
  tail -2 $O/tests.log
fi
echo done
