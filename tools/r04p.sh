set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04p; mkdir -p $O
bash tools/ab_bc1.sh r04p "" bc1w4 || exit 1
for rep in 1 2; do
  for v in "" $R/gpurun_dbg/bc6w6/lib.so; do
    GIC_LIBRARY=$v timeout -k 10 200 python3 tools/time_bc6h.py >> $O/bc6h.txt 2>&1 || exit 1
  done
done
grep -v amdgpu.ids $O/bc6h.txt
cd $R && timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_capi.py tests/test_gpu_parity.py -k "block" > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 120 ./gpurun_dbg/block_latency 2000 > $O/lat.txt 2>&1 || exit 1
cat $O/lat.txt
