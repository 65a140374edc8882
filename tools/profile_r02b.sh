# Round-2 (second pass) profile set on the GPU box: the default bench line, the
# same command under rocprofv3 --kernel-trace --stats (BC1, BC7, bc7enc16,
# BC4/BC5 kernels), and one --pmc pass of VALU issue counters over the BC1 and
# bc7enc16 legs (counters only, no tracing domains).
#   bash tools/profile_r02b.sh <tag>   -> gpurun_out/prof_<tag>/
set -o pipefail
TAG=${1:-r02b}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/prof_$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 python3 $R/bench.py > $O/bench.json 2> $O/bench.err || exit 1
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/bench.py > $O/bench_under_rocprof.json 2> $O/rocprof.err || exit 1
C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv -d $O/valu -o run -- python3 $R/bench.py --no-cpu --bc7-rows 0 --no-bc45 --steps 3 --warmup 1 > $O/valu.json 2> $O/valu.err || exit 1
echo done
