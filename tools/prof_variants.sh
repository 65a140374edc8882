# Per-kernel times (rocprofv3 kernel stats, one internal stream) of the exact
# BC7 search on 64 block rows of the 8K G1 texture, for the in-tree library and
# each gpurun_dbg/<variant>/lib.so.   bash tools/prof_variants.sh <tag> <variant>...
set -o pipefail
TAG=$1; shift
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/profv_$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in default "$@"; do
  if [ "$v" = default ]; then L=""; else L=$R/gpurun_dbg/$v/lib.so; fi
  GIC_LIBRARY=$L GIC_BC7_SINGLE_STREAM=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o run -- \
    python3 $R/tools/time_bc7_bounded.py --rows 64 --bound 0 > $O/$v.txt 2>&1 || exit 1
done
echo done
