# A/B timing of BC7 library variants (exact search on 256 block rows of the 8K
# G1 texture, and the bounded exit over the whole 8K), in-tree library first,
# each variant from gpurun_var/<variant>/lib.so, twice in alternation; then the
# BC7 GPU tests (pytest -k expression, default "bc7") on the in-tree library.
#   bash tools/ab_bc7x.sh <tag> "<pytest -k>" <variant>...   -> gpurun_out/ab_<tag>/
set -o pipefail
TAG=$1; K=${2:-bc7}; shift 2
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/ab_$TAG
mkdir -p $O
cd $R
for rep in 1 2; do
  for v in default "$@"; do
    if [ "$v" = default ]; then L=""; else L=$R/gpurun_var/$v/lib.so; fi
    echo "== $v" >> $O/bc7.txt
    GIC_LIBRARY=$L timeout -k 10 300 python3 tools/time_bc7_bounded.py --rows 256 --bound 0 >> $O/bc7.txt 2>&1 || exit 1
    GIC_LIBRARY=$L timeout -k 10 300 python3 tools/time_bc7_bounded.py --rows 2048 --bound 0.5 >> $O/bc7.txt 2>&1 || exit 1
  done
done
grep -v amdgpu.ids $O/bc7.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$K" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
echo done
