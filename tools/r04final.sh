set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04final; mkdir -p $O
cd $R
timeout -k 10 1000 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/ > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
