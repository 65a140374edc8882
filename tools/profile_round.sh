# Round profile: default bench line, the same command under rocprofv3 kernel
# trace + stats, and separate PMC passes for HBM traffic of the BC1 kernel.
# Usage (on the GPU box): bash tools/profile_round.sh <tag>
set -o pipefail
TAG=${1:-r01}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/prof_$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 python3 $R/bench.py > $O/bench.json 2> $O/bench.err || exit 1
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/bench.py > $O/bench_under_rocprof.json 2> $O/rocprof.err || exit 1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python3 $R/bench.py --no-cpu --bc7-rows 0 --steps 3 --warmup 1 > /dev/null 2> $O/pmc_fetch.err || exit 1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python3 $R/bench.py --no-cpu --bc7-rows 0 --steps 3 --warmup 1 > /dev/null 2> $O/pmc_write.err || exit 1
echo done
