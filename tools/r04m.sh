set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04m; mkdir -p $O
cd $R
echo "== new (in-tree)" >> $O/lat.txt
timeout -k 10 120 ./gpurun_dbg/block_latency 2000 >> $O/lat.txt 2>&1 || exit 1
echo "== old (pageable copies)" >> $O/lat.txt
LD_LIBRARY_PATH=$R/gpurun_dbg/apiold timeout -k 10 120 ./gpurun_dbg/block_latency 2000 >> $O/lat.txt 2>&1 || exit 1
cat $O/lat.txt
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_capi.py tests/test_gpu_parity.py -k "block" > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -2 $O/tests.log
