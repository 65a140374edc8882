# BC6H unsigned and signed (1024^2 synthetic HDR): per-kernel time
# (--kernel-trace --stats) and, in separate runs, the SQ issue counters (--pmc).
#   bash tools/prof_bc6h_r04.sh <tag>  -> gpurun_out/p6_<tag>/{u,s}/
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/p6_$1
cd /tmp && export TMPDIR=/tmp
C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
for k in unsigned signed; do
  mkdir -p $O/$k
  timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$k/trace -o run -- \
    python3 $R/tools/time_bc6h.py --size 1024 --reps 2 --only $k > $O/$k/trace.txt 2>&1 || exit 1
  timeout -s KILL 300 rocprofv3 --pmc $C --output-format csv -d $O/$k/pmc -o run -- \
    python3 $R/tools/time_bc6h.py --size 1024 --reps 2 --only $k > $O/$k/pmc.txt 2>&1 || exit 1
  python3 $R/tools/kstats_pmc.py $O/$k > $O/$k/summary.txt && cat $O/$k/summary.txt
done
