set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04n; mkdir -p $O
for rep in 1 2; do
  for v in "" $R/gpurun_dbg/b45/lib.so; do
    GIC_LIBRARY=$v timeout -k 10 200 python3 tools/time_bc45.py 20 >> $O/bc45.txt 2>&1 || exit 1
  done
done
grep -v amdgpu.ids $O/bc45.txt
