# Round-5 profile set on the GPU box (collected by tools/collect_r05.py):
#   bash tools/profile_r05.sh <tag> bench  -> the default bench line (the driver's command) and the same
#                                             command under rocprofv3 --kernel-trace --stats
#   bash tools/profile_r05.sh <tag> pmc    -> SQ issue counters of the bench legs and of the exact BC7 search
#       (64 block rows, one stream, with its kernel trace), BC1 FETCH_SIZE / WRITE_SIZE passes, the
#       one-pass VALU totals of the four BC7 8K legs, the BC6H per-kernel time and SQ counters
#       (tools/prof_bc6h_r04.sh -> gpurun_out/p6_<tag>/), and the block-call latencies
set -o pipefail
TAG=${1:-r05}
WHAT=${2:-bench}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/prof_$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
if [ "$WHAT" = bench ]; then
  timeout -k 10 540 python3 $R/bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
  tail -c 400 $O/bench.json
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/bench.py --steps 20 --warmup 5 > $O/bench_under_rocprof.json 2> $O/rocprof.err || { tail -20 $O/rocprof.err; exit 1; }
  echo done
  exit 0
fi
C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
timeout -s KILL 300 rocprofv3 --pmc $C --output-format csv -d $O/valu -o run -- python3 $R/bench.py --no-cpu --bc7-rows 0 --bc7-mse-bound 0 --bc6h-size 0 --no-batch --steps 3 --warmup 1 > $O/valu.json 2> $O/valu.err || { tail -20 $O/valu.err; exit 1; }
GIC_BC7_SINGLE_STREAM=1 timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv -d $O/valu_bc7 -o run -- python3 $R/tools/time_bc7_bounded.py --rows 64 --bound 0 > $O/valu_bc7.log 2>&1 || { tail -20 $O/valu_bc7.log; exit 1; }
GIC_BC7_SINGLE_STREAM=1 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_bc7 -o run -- python3 $R/tools/time_bc7_bounded.py --rows 64 --bound 0 > $O/trace_bc7.log 2>&1 || { tail -20 $O/trace_bc7.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python3 $R/bench.py --no-cpu --bc7-rows 0 --no-bc7enc --no-bc45 --bc6h-size 0 --no-batch --steps 3 --warmup 1 > $O/pmc_fetch.json 2> $O/pmc_fetch.err || { tail -20 $O/pmc_fetch.err; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python3 $R/bench.py --no-cpu --bc7-rows 0 --no-bc7enc --no-bc45 --bc6h-size 0 --no-batch --steps 3 --warmup 1 > $O/pmc_write.json 2> $O/pmc_write.err || { tail -20 $O/pmc_write.err; exit 1; }
for leg in "bc7 0 0" "bc7_pruned 2 0" "bc7_bounded 0 0.5" "bc7_bounded_pruned 2 0.5"; do
  set -- $leg
  timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $O/pass_$1 -o run -- python3 $R/tools/time_bc7_bounded.py --rows 2048 --shake-ranks $2 --bound $3 --no-warm > $O/pass_$1.log 2>&1 || { tail -20 $O/pass_$1.log; exit 1; }
done
bash $R/tools/prof_bc6h_r04.sh $TAG > $O/bc6h.txt 2>&1 || { tail -20 $O/bc6h.txt; exit 1; }
cd $R
if [ -x gpurun_var/block_latency ]; then timeout -k 10 120 ./gpurun_var/block_latency 2000 > $O/block_latency.txt 2>&1 || exit 1; cat $O/block_latency.txt; fi
echo done
