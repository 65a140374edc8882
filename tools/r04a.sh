set -o pipefail
O=gpurun_out/r04a; mkdir -p $O
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt -fno-gpu-flush-denormals-to-zero -fno-fast-math tools/rcp_check.hip -o /tmp/rcp_check 2>/dev/null || exit 1
timeout -k 10 120 /tmp/rcp_check > $O/rcp_check.txt 2>&1; echo "rcp rc=$?" >> $O/rcp_check.txt
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "non_finite" tests/test_gpu_bc7.py::test_iteration_cap_hits_are_counted -s > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --batch-slices 4 --batch-size 512 --bc7-rows 8 --bc6h-size 130 --cpu-seconds 2 > $O/bench_small.json 2> $O/bench_small.err || { tail -30 $O/bench_small.err; exit 1; }
tail -3 $O/tests.log; cat $O/rcp_check.txt
