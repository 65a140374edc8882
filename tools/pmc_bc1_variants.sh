set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/bc1v
mkdir -p $O
cd $R
timeout -k 10 120 python3 tools/time_bc1.py > $O/time.log 2>&1 || exit 1
for v in "$@"; do GIC_LIBRARY=$R/gpurun_dbg/$v/lib.so timeout -k 10 120 python3 tools/time_bc1.py >> $O/time.log 2>&1 || exit 1; done
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_IFETCH SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_WAVES --output-format csv -d $O/pmc -o run -- python3 $R/tools/time_bc1.py 2 > $O/pmc.log 2>&1 || exit 1
cat $O/time.log
