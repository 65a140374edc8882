# BC6H per-kernel times (rocprofv3 kernel stats) for the in-tree library and
# each gpurun_dbg/<variant>/lib.so:  bash tools/prof_bc6h.sh <tag> <variant>...
set -o pipefail
TAG=$1; shift
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/prof6_$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in default "$@"; do
  if [ "$v" = default ]; then L=""; else L=$R/gpurun_dbg/$v/lib.so; fi
  GIC_LIBRARY=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o run -- \
    python3 $R/tools/time_bc6h.py --size 512 --reps 1 > $O/$v.txt 2>&1 || exit 1
  grep -v amdgpu.ids $O/$v.txt | tail -2
done
echo done
