# Round-3 (e): per-kernel split of the bounded-exit BC7 path over the whole
# 8K G1 texture (one internal stream), rocprofv3 kernel trace + stats.
#   bash tools/prof_r03e.sh <tag>
set -o pipefail
TAG=$1
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/prof_$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
GIC_BC7_SINGLE_STREAM=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/bounded -o run -- \
  python3 $R/tools/time_bc7_bounded.py --rows 2048 --bound 0.5 > $O/bounded.txt 2>&1 || exit 1
grep -v amdgpu.ids $O/bounded.txt
echo done
