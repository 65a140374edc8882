# Exact BC7 search (64 block rows of 8K G1, one internal stream): per-kernel
# time (rocprofv3 --kernel-trace --stats) and, in a separate run, the SQ issue
# counters (--pmc, counters only).   bash tools/prof_bc7x.sh <tag> [rows]
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pbx_$1; ROWS=${2:-64}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export GIC_BC7_SINGLE_STREAM=1
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
  python3 $R/tools/time_bc7_bounded.py --rows $ROWS --bound 0 > $O/trace.txt 2>&1 || exit 1
C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
timeout -s KILL 300 rocprofv3 --pmc $C --output-format csv -d $O/pmc -o run -- \
  python3 $R/tools/time_bc7_bounded.py --rows $ROWS --bound 0 > $O/pmc.txt 2>&1 || exit 1
python3 $R/tools/kstats_pmc.py $O > $O/summary.txt && cat $O/summary.txt
