# VALU issue counters for the BC1 and BC7 kernels (one rocprofv3 --pmc pass per
# workload, counters only -- no tracing domains).  Usage on the GPU box:
#   bash tools/pmc_valu.sh <tag>      -> gpurun_out/valu_<tag>/{bc1,bc7}/...
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
TAG=${1:-r01}
O=$R/gpurun_out/valu_$TAG
mkdir -p $O
timeout -k 10 120 rocprofv3 -L > $O/counters.txt 2>&1 || true
C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
for c in SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY; do
  grep -q "\b$c\b" $O/counters.txt && C="$C $c"
done
grep -q "\bGRBM_GUI_ACTIVE\b" $O/counters.txt && C="$C GRBM_GUI_ACTIVE"
echo "counters: $C" > $O/pass.txt
timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv -d $O/bc1 -o run -- \
  python3 $R/bench.py --format bc1 --no-cpu --bc7-rows 0 --steps 3 --warmup 1 > $O/bc1.json 2> $O/bc1.err || exit 1
timeout -s KILL 300 rocprofv3 --pmc $C --output-format csv -d $O/bc7 -o run -- \
  python3 $R/bench.py --format bc7 --rows 128 --no-cpu --steps 1 --warmup 1 --bc7-shake-ranks 0 > $O/bc7.json 2> $O/bc7.err || exit 1
echo done
