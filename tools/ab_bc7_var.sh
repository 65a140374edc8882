# BC7 variant check + A/B: the exact-BC7 GPU tests with gpurun_var/<first variant>/lib.so, then
# tools/ab_kstats.sh over the in-tree library and the variants.
#   bash tools/ab_bc7_var.sh <tag> <variant>...
set -o pipefail
TAG=$1; shift
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/abv_$TAG
cd $R
GIC_LIBRARY=$R/gpurun_var/$1/lib.so timeout -k 10 600 python -u -m pytest tests/test_gpu_bc7.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/abv_$TAG/tests.log 2>&1 || { tail -30 gpurun_out/abv_$TAG/tests.log; exit 1; }
tail -2 gpurun_out/abv_$TAG/tests.log
bash tools/ab_kstats.sh $TAG "$@"
