# A/B of BC1 library variants on the 8K G1 texture: timing (tools/time_bc1.py,
# twice in alternation) and, per variant, one --pmc FETCH_SIZE pass (counters
# only), so scratch spill traffic shows next to the time.
#   bash tools/ab_bc1_traffic.sh <tag> <variant>...   -> gpurun_out/ab_<tag>/
set -o pipefail
TAG=$1; shift
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/ab_$TAG
mkdir -p $O
cd $R
for rep in 1 2; do
  for v in default "$@"; do
    if [ "$v" = default ]; then L=""; else L=$R/gpurun_dbg/$v/lib.so; fi
    GIC_LIBRARY=$L timeout -k 10 200 python3 tools/time_bc1.py 20 >> $O/bc1.txt 2>&1 || exit 1
  done
done
grep -v amdgpu.ids $O/bc1.txt
cd /tmp && export TMPDIR=/tmp
for v in default "$@"; do
  if [ "$v" = default ]; then L=""; else L=$R/gpurun_dbg/$v/lib.so; fi
  GIC_LIBRARY=$L timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch_$v -o run -- python3 $R/tools/time_bc1.py 2 > $O/fetch_$v.log 2>&1 || exit 1
  python3 -c "import sys; sys.path.insert(0, '$R/tools'); from refresh_profiles import per_launch; f, n = per_launch('$O/fetch_$v/run_counter_collection.csv', 'bc1_image_kernel', 'FETCH_SIZE'); print('$v FETCH_SIZE', round(f), 'KB per launch,', n, 'launches')" || exit 1
done
echo done
