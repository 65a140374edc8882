# A/B timing of BC7 library variants on the exact search (256 block rows of
# the 8K G1 texture), in-tree library first, each variant from
# gpurun_dbg/<variant>/lib.so, alternating REPS times.
#   bash tools/ab_quick.sh <tag> <reps> <variant>...   -> gpurun_out/abq_<tag>/bc7.txt
set -o pipefail
TAG=$1; REPS=$2; shift 2
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/abq_$TAG
mkdir -p $O
cd $R
for rep in $(seq $REPS); do
  for v in default "$@"; do
    if [ "$v" = default ]; then L=""; else L=$R/gpurun_dbg/$v/lib.so; fi
    echo "== $v" >> $O/bc7.txt
    GIC_LIBRARY=$L timeout -k 10 300 python3 tools/time_bc7_bounded.py --rows 256 --bound 0 >> $O/bc7.txt 2>&1 || exit 1
  done
done
grep -v amdgpu.ids $O/bc7.txt
