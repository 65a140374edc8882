# PMC pass over the BC7 bench (counters only, kernel trace off): instruction mix and stall cycles
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 120 rocprofv3 -L > $R/gpurun_out/counters.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_SMEM -d $R/gpurun_out/pmc_bc7 -o run --output-format csv -- python3 $R/bench.py --format bc7 --rows 8 --steps 1 --warmup 1 --no-cpu > $R/gpurun_out/pmc_bc7.log 2>&1
