set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04s; mkdir -p $O
for rep in 1 2; do
  for v in "" $R/gpurun_dbg/bc23old/lib.so; do
    GIC_LIBRARY=$v timeout -k 10 200 python3 tools/time_bc23.py >> $O/bc23.txt 2>&1 || exit 1
  done
done
grep -v amdgpu.ids $O/bc23.txt
set -o pipefail
R=$GRAFT_REPO_ROOT
bash tools/profile_r04.sh r04e tests || exit 1
mkdir -p $R/gpurun_out/b05 && cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 python3 $R/bench.py --steps 20 --warmup 5 > $R/gpurun_out/b05/bench.json 2> $R/gpurun_out/b05/bench.err || { tail -5 $R/gpurun_out/b05/bench.err; exit 1; }
tail -c 400 $R/gpurun_out/b05/bench.json
