# Round-3 (d): per-kernel split of the exact BC7 search (one internal stream),
# rocprofv3 kernel trace + stats over tools/time_bc7_bounded.py; then an A/B of
# the given variants.   bash tools/prof_r03d.sh <tag> <variant>...
set -o pipefail
TAG=$1; shift
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/prof_$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
GIC_BC7_SINGLE_STREAM=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/exact -o run -- \
  python3 $R/tools/time_bc7_bounded.py --rows 64 --bound 0 > $O/exact.txt 2>&1 || exit 1
cd $R
for v in default "$@"; do
  if [ "$v" = default ]; then L=""; else L=$R/gpurun_dbg/$v/lib.so; fi
  echo "== $v" >> $O/ab.txt
  GIC_LIBRARY=$L timeout -k 10 300 python3 tools/time_bc7_bounded.py --rows 256 --bound 0 >> $O/ab.txt 2>&1 || exit 1
done
grep -v amdgpu.ids $O/ab.txt
echo done
