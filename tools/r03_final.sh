# Round-3 closing GPU call: BC7 exact A/B against gpurun_dbg/<variant>, the shaker
# section profile (gpurun_dbg/prof), then the whole profile set
# (tools/profile_r03.sh <tag> all: -m gpu suite, smoke, bench, rocprof, PMC).
#   bash tools/r03_final.sh <tag> <variant>
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/ab_$1
mkdir -p $O
cd $R
for rep in 1 2; do
  for v in default $2; do
    if [ "$v" = default ]; then L=""; else L=$R/gpurun_dbg/$v/lib.so; fi
    echo "== $v" >> $O/bc7.txt
    GIC_LIBRARY=$L timeout -k 10 300 python3 tools/time_bc7_bounded.py --rows 256 --bound 0 >> $O/bc7.txt 2>&1 || exit 1
  done
done
grep -v amdgpu.ids $O/bc7.txt
GIC_LIBRARY=$R/gpurun_dbg/prof/lib.so timeout -k 10 300 python3 tools/prof_sections.py 64 > $O/sections.txt 2>&1 || { tail $O/sections.txt; exit 1; }
grep -v amdgpu.ids $O/sections.txt
bash $R/tools/profile_r03.sh $1 all
