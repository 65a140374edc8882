# fast/slow shake kernels: BC7 GPU tests (exact parity), then A/B timing
set -o pipefail
O=gpurun_out/r04b; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_gpu_bc7.py tests/test_gpu_bc7_sample.py -k "not performance_levels" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash tools/ab_quick.sh r04b 2 occ6
