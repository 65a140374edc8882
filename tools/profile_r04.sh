# Round-4 profile set on the GPU box (see tools/profile_r03.sh for the layout):
#   bash tools/profile_r04.sh <tag> tests  -> the -m gpu suite + smoke
#   bash tools/profile_r04.sh <tag> prof   -> the default bench under rocprofv3 --kernel-trace --stats,
#       SQ issue counters over the bench legs (no CPU legs, no batch legs) and over the
#       exact BC7 search (64 block rows, one stream) with its own kernel trace
set -o pipefail
TAG=${1:-r04}
WHAT=${2:-tests}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/prof_$TAG
mkdir -p $O
if [ "$WHAT" = tests ]; then
  cd $R
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
  tail -3 $O/gpu_tests.log
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" >> $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
  tail -1 $O/gpu_tests.log
  echo done
  exit 0
fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/bench.py --steps 20 --warmup 5 > $O/bench_under_rocprof.json 2> $O/rocprof.err || { tail -20 $O/rocprof.err; exit 1; }
tail -c 300 $O/bench_under_rocprof.json
C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
timeout -s KILL 300 rocprofv3 --pmc $C --output-format csv -d $O/valu -o run -- python3 $R/bench.py --no-cpu --bc7-rows 0 --bc7-mse-bound 0 --bc6h-size 0 --no-batch --steps 3 --warmup 1 > $O/valu.json 2> $O/valu.err || { tail -20 $O/valu.err; exit 1; }
GIC_BC7_SINGLE_STREAM=1 timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv -d $O/valu_bc7 -o run -- python3 $R/tools/time_bc7_bounded.py --rows 64 --bound 0 > $O/valu_bc7.log 2>&1 || { tail -20 $O/valu_bc7.log; exit 1; }
GIC_BC7_SINGLE_STREAM=1 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_bc7 -o run -- python3 $R/tools/time_bc7_bounded.py --rows 64 --bound 0 > $O/trace_bc7.log 2>&1 || { tail -20 $O/trace_bc7.log; exit 1; }
echo done
