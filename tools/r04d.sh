set -o pipefail
O=gpurun_out/r04d; mkdir -p $O
bash tools/ab_quick.sh r04d 2 spcall || exit 1
bash tools/ab_bc1.sh r04d "" bc1old bc1w2 || exit 1
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --bc7-rows 0 --no-bc7enc --bc6h-size 0 --no-batch --no-cpu > $O/bench_bcx.json 2> $O/bench_bcx.err || { tail -20 $O/bench_bcx.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench_bcx.json').read().strip().splitlines()[-1])
print('bc1', d['kernel_ms'], 'bc4', d['bc4']['kernel_ms'], 'bc5', d['bc5']['kernel_ms'])"
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_bc7.py tests/test_gpu_bc7_sample.py -k "not performance_levels" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
GIC_LIBRARY=$GRAFT_REPO_ROOT/gpurun_dbg/prof/lib.so timeout -k 10 300 python3 tools/prof_sections.py 64 > $O/sections.txt 2>&1 || { tail -5 $O/sections.txt; exit 1; }
cat $O/sections.txt
