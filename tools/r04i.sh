set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/prof_r04i; mkdir -p $O
bash tools/ab_bc1.sh r04i "" bc1old || exit 1
bash tools/ab_quick.sh r04i 2 qs2 qhead || exit 1
cd $R && timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_quant_equiv.py tests/test_gpu_parity.py tests/test_gpu_bc7.py tests/test_gpu_bc7_sample.py tests/test_capi.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash tools/pmc_traffic_bc1.sh r04i || exit 1
cd /tmp && export TMPDIR=/tmp
C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
timeout -k 10 240 python3 $R/bench.py --no-cpu --bc7-rows 0 --no-bc7enc --no-bc45 --bc6h-size 0 --no-batch --steps 3 --warmup 1 > $O/bench_bc1.json 2> $O/bench_bc1.err || exit 1
timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv -d $O/pmc_valu -o run -- python3 $R/bench.py --no-cpu --bc7-rows 0 --no-bc7enc --no-bc45 --bc6h-size 0 --no-batch --steps 3 --warmup 1 > /dev/null 2> $O/pmc_valu.err || exit 1
cd $R && bash tools/prof_bc7x.sh r04i 256 || exit 1
echo ok
