# rocprofv3 kernel stats of a short BC7 bench: bash tools/prof_kernels.sh ROWS OUTNAME
set -o pipefail
ROWS=${1:-64}; OUT=${2:-prof_k}
R=${GRAFT_REPO_ROOT:-$PWD}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/$OUT -o run -- python3 $R/bench.py --format bc7 --rows $ROWS --steps 1 --warmup 1 --no-cpu > $R/gpurun_out/$OUT.log 2>&1
rc=$?
python3 $R/tools/kstats.py $(find $R/gpurun_out/$OUT -name "*.db" | head -1)
exit $rc
