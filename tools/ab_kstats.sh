# Per-kernel A/B of BC7 library variants: rocprofv3 --kernel-trace --stats over
# the exact search on 64 block rows (one stream), in-tree library first, then
# each variant from gpurun_var/<variant>/lib.so.
#   bash tools/ab_kstats.sh <tag> <variant>...   -> gpurun_out/abk_<tag>/
set -o pipefail
TAG=$1; shift
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/abk_$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in default "$@"; do
  if [ "$v" = default ]; then L=""; else L=$R/gpurun_var/$v/lib.so; fi
  GIC_LIBRARY=$L GIC_BC7_SINGLE_STREAM=1 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o run -- python3 $R/tools/time_bc7_bounded.py --rows 64 --bound 0 > $O/$v.log 2>&1 || { tail -20 $O/$v.log; exit 1; }
  grep "block rows" $O/$v.log
  python3 $R/tools/kstats_csv.py $O/$v 10 || exit 1
done
echo done
