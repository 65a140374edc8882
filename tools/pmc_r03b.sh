# Round-3 (b) SQ issue counters, each pass its own rocprofv3 run (counters only):
# the exact BC7 search (64 block rows, single stream) and the BC1/BC4/BC5 legs.
#   bash tools/pmc_r03b.sh <tag>  -> gpurun_out/pmc_<tag>/
set -o pipefail
TAG=${1:-r03b}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc_$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
SQ="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU"
GIC_BC7_SINGLE_STREAM=1 timeout -s KILL 240 rocprofv3 --pmc $SQ --output-format csv -d $O/bc7_sq -o run -- python3 $R/tools/time_bc7_bounded.py --rows 64 --bound 0 > $O/bc7_sq.log 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --pmc $SQ --output-format csv -d $O/bcx_sq -o run -- python3 $R/bench.py --no-cpu --bc7-rows 0 --no-bc7enc --bc6h-size 0 --steps 3 --warmup 1 > $O/bcx_sq.json 2>&1 || exit 1
for d in bc7_sq bcx_sq; do echo "== $d"; python3 $R/tools/pmc_summary.py $O/$d; done > $O/summary.txt 2>&1 || true
cat $O/summary.txt
echo done
