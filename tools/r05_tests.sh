# -m gpu suite + smoke on the box (usage: bash tools/r05_tests.sh <tag> [pytest -k expr])
set -o pipefail
TAG=${1:-r05}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/tests_$TAG
mkdir -p $O
cd $R
K=${2:+-k "$2"}
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread $K > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" >> $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
