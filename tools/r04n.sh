set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04n; mkdir -p $O
for rep in 1 2; do
  for v in "" $R/gpurun_dbg/b45/lib.so; do
    GIC_LIBRARY=$v timeout -k 10 200 python3 tools/time_bc45.py 20 >> $O/bc45.txt 2>&1 || exit 1
  done
done
grep -v amdgpu.ids $O/bc45.txt
for rep in 1 2; do
  for v in "" $R/gpurun_dbg/bc6old/lib.so; do
    GIC_LIBRARY=$v timeout -k 10 200 python3 tools/time_bc6h.py >> $O/bc6h.txt 2>&1 || exit 1
  done
done
grep -v amdgpu.ids $O/bc6h.txt
cd $R && timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_gpu_bc6h.py tests/test_capi.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash tools/ab_quick.sh r04n 2 qB qC || exit 1
