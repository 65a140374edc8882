set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_bc7 -o run -- python3 $R/bench.py --format bc7 --rows 16 --steps 2 --warmup 1 --no-cpu > $R/gpurun_out/bench_bc7.log 2>&1
rc=$?
find $R/gpurun_out/prof_bc7 -name "*kernel_stats.csv" | head -1 | xargs cat
tail -2 $R/gpurun_out/bench_bc7.log
exit $rc
