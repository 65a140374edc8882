# PMC pass over bench.py (counters only): instruction mix and stall cycles.  $1 = format, $2.. = extra bench args
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
F=$1; shift
mkdir -p $R/gpurun_out
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_SMEM -d $R/gpurun_out/pmc_$F -o run --output-format csv -- python3 $R/bench.py --format $F --steps 1 --warmup 1 --no-cpu "$@" > $R/gpurun_out/pmc_$F.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VMEM SQ_INSTS_LDS SQ_INSTS_FLAT GRBM_GUI_ACTIVE -d $R/gpurun_out/pmc2_$F -o run --output-format csv -- python3 $R/bench.py --format $F --steps 1 --warmup 1 --no-cpu "$@" >> $R/gpurun_out/pmc_$F.log 2>&1
