# The new block-status test, then configs[4] on one GPU at the bench defaults
# (bounded exit 0.5 with exact survivors, 16-row chunks), one timed step.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/b64
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "block_api" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 600 python3 -u bench.py --workload batch64 --steps 1 --warmup 1 > $O/batch64.json 2> $O/batch64.err || { tail -20 $O/batch64.err; exit 1; }
tail -c 1500 $O/batch64.json
echo done
