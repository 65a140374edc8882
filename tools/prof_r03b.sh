# Round-3 (b): section split of the exact BC7 shakers (GIC_PROFILE variant in
# gpurun_dbg/prof) and the default bench line.
#   bash tools/prof_r03b.sh <tag>   -> gpurun_out/prof_<tag>/
set -o pipefail
TAG=${1:-r03b}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/prof_$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
GIC_LIBRARY=$R/gpurun_dbg/prof/lib.so GIC_BC7_SINGLE_STREAM=1 timeout -k 10 300 python3 $R/tools/prof_sections.py 64 > $O/sections.txt 2>&1 || exit 1
cat $O/sections.txt
timeout -k 10 500 python3 $R/bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
echo done
