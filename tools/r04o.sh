set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04o; mkdir -p $O
bash tools/ab_quick.sh r04o 2 side || exit 1
for rep in 1 2; do
  for v in "" $R/gpurun_dbg/side/lib.so; do
    echo "== $v" >> $O/bounded.txt
    GIC_LIBRARY=$v timeout -k 10 300 python3 tools/time_bc7_bounded.py --rows 2048 --bound 0.5 >> $O/bounded.txt 2>&1 || exit 1
  done
done
grep -v amdgpu.ids $O/bounded.txt
