set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04k; mkdir -p $O
for rep in 1 2; do
  for v in "" $R/gpurun_dbg/encL2/lib.so $R/gpurun_dbg/encL3/lib.so; do
    GIC_LIBRARY=$v timeout -k 10 200 python3 tools/time_bc7enc.py >> $O/enc.txt 2>&1 || exit 1
  done
done
grep -v amdgpu.ids $O/enc.txt
