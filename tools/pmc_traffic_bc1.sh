# HBM traffic of the BC1 kernel: FETCH_SIZE and WRITE_SIZE in separate --pmc
# passes (counters only) over the default BC1 workload.
#   bash tools/pmc_traffic_bc1.sh <tag>   -> gpurun_out/prof_<tag>/pmc_{fetch,write}/
set -o pipefail
TAG=${1:-r02c}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/prof_$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python3 $R/bench.py --no-cpu --bc7-rows 0 --no-bc7enc --no-bc45 --bc6h-size 0 --no-batch --steps 3 --warmup 1 > /dev/null 2> $O/pmc_fetch.err || exit 1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python3 $R/bench.py --no-cpu --bc7-rows 0 --no-bc7enc --no-bc45 --bc6h-size 0 --no-batch --steps 3 --warmup 1 > /dev/null 2> $O/pmc_write.err || exit 1
echo done
