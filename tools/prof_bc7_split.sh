# Per-kernel BC7 time, exact vs pruned search (one internal stream so kernel
# times add up): rocprofv3 kernel trace + stats over bench.py --format bc7.
# Usage (GPU box): bash tools/prof_bc7_split.sh <tag> [rows]
set -o pipefail
TAG=${1:-bc7split}
ROWS=${2:-128}
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for K in 0 2; do
  GIC_BC7_SINGLE_STREAM=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d $R/gpurun_out/prof_${TAG}_k$K -o run -- python3 $R/bench.py --format bc7 --rows $ROWS --steps 1 \
    --warmup 1 --no-cpu --bc7-shake-ranks $K > $R/gpurun_out/prof_${TAG}_k$K.json 2> $R/gpurun_out/prof_${TAG}_k$K.err || exit 1
done
echo ok
