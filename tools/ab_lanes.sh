# BC7 internal stream count A/B: the exact search and the bounded exit over the
# whole 8K G1 texture with GIC_BC7_LANES = 1..4, twice in alternation.
#   bash tools/ab_lanes.sh <tag>   -> gpurun_out/ab_<tag>/lanes.txt
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/ab_$1
mkdir -p $O
cd $R
for rep in 1 2; do
  for n in 2 3 4; do
    echo "== lanes $n" >> $O/lanes.txt
    GIC_BC7_LANES=$n timeout -k 10 200 python3 tools/time_bc7_bounded.py --rows 2048 --bound 0 >> $O/lanes.txt 2>&1 || exit 1
    GIC_BC7_LANES=$n timeout -k 10 200 python3 tools/time_bc7_bounded.py --rows 2048 --bound 0.5 >> $O/lanes.txt 2>&1 || exit 1
  done
done
grep -v amdgpu.ids $O/lanes.txt
