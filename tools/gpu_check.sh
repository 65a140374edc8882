# GPU check on the box: new/named tests first, then the whole -m gpu suite,
# then a short 2-rank gloo rehearsal of the batch64 path (ranks share the GPU).
#   bash tools/gpu_check.sh <tag> [pytest -k expr for the first pass]
set -o pipefail
TAG=${1:-r03}
K=${2:-batch}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/check_$TAG
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$K" > $O/first.log 2>&1 || { tail -30 $O/first.log; exit 1; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/all.log 2>&1 || { tail -30 $O/all.log; exit 1; }
tail -3 $O/all.log
timeout -k 10 300 python -u bench.py --gpus 2 --dist-backend gloo --workload batch64 --batch-slices 4 --batch-size 1024 --steps 1 --warmup 1 > $O/batch_2rank_gloo.json 2> $O/batch_2rank_gloo.err || { tail -30 $O/batch_2rank_gloo.err; exit 1; }
cat $O/batch_2rank_gloo.json
echo done
