# Round-3 measurements on the GPU box:
#   bash tools/prof_r03.sh <tag>   -> gpurun_out/prof_<tag>/
#  1. BC7 bounded exit on the whole 8K G1 (exact and pruned survivors) and the exact search on 256 rows
#  2. BC6H throughput (1024^2 HDR)
#  3. the bounded leg under rocprofv3 --kernel-trace --stats, single stream
set -o pipefail
TAG=${1:-r03}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/prof_$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 $R/tools/time_bc7_bounded.py --rows 2048 --bound 0.5 > $O/bounded.txt 2>&1 || exit 1
timeout -k 10 300 python3 $R/tools/time_bc7_bounded.py --rows 2048 --bound 0.5 --shake-ranks 2 >> $O/bounded.txt 2>&1 || exit 1
cat $O/bounded.txt
timeout -k 10 300 python3 $R/tools/time_bc6h.py --size 1024 > $O/bc6h.txt 2>&1 || exit 1
cat $O/bc6h.txt
GIC_BC7_SINGLE_STREAM=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_bounded -o run -- python3 $R/tools/time_bc7_bounded.py --rows 2048 --bound 0.5 > $O/bounded_under_rocprof.txt 2>&1 || exit 1
echo done
