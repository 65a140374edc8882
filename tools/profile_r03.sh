# Round-3 profile set on the GPU box: the -m gpu suite + smoke, the default
# bench line, the same command under rocprofv3 --kernel-trace --stats, SQ issue
# counters over the BC1/BC4/BC5/bc7enc16 legs and the exact BC7 search (64 block
# rows, one stream) with a kernel trace of that same run for the launch times, and
# BC1 FETCH_SIZE / WRITE_SIZE, each --pmc pass its own run.
#   bash tools/profile_r03.sh <tag> [tests|prof|all]  -> gpurun_out/prof_<tag>/
set -o pipefail
TAG=${1:-r03}
WHAT=${2:-all}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/prof_$TAG
mkdir -p $O
if [ "$WHAT" != prof ]; then
  cd $R
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
  tail -3 $O/gpu_tests.log
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" >> $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
  tail -1 $O/gpu_tests.log
fi
[ "$WHAT" = tests ] && { echo done; exit 0; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 python3 $R/bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
tail -c 600 $O/bench.json
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/bench.py > $O/bench_under_rocprof.json 2> $O/rocprof.err || { tail -20 $O/rocprof.err; exit 1; }
C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv -d $O/valu -o run -- python3 $R/bench.py --no-cpu --bc7-rows 0 --bc7-mse-bound 0 --bc6h-size 0 --steps 3 --warmup 1 > $O/valu.json 2> $O/valu.err || { tail -20 $O/valu.err; exit 1; }
GIC_BC7_SINGLE_STREAM=1 timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv -d $O/valu_bc7 -o run -- python3 $R/tools/time_bc7_bounded.py --rows 64 --bound 0 > $O/valu_bc7.log 2>&1 || { tail -20 $O/valu_bc7.log; exit 1; }
GIC_BC7_SINGLE_STREAM=1 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_bc7 -o run -- python3 $R/tools/time_bc7_bounded.py --rows 64 --bound 0 > $O/trace_bc7.log 2>&1 || { tail -20 $O/trace_bc7.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python3 $R/bench.py --no-cpu --bc7-rows 0 --no-bc7enc --no-bc45 --bc7-mse-bound 0 --bc6h-size 0 --steps 3 --warmup 1 > /dev/null 2> $O/pmc_fetch.err || { tail -20 $O/pmc_fetch.err; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python3 $R/bench.py --no-cpu --bc7-rows 0 --no-bc7enc --no-bc45 --bc7-mse-bound 0 --bc6h-size 0 --steps 3 --warmup 1 > /dev/null 2> $O/pmc_write.err || { tail -20 $O/pmc_write.err; exit 1; }
echo done
