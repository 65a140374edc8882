# A/B of the in-tree BC7 library against gpurun_dbg/<variant>, BC7 GPU tests,
# then the shaker section profile of gpurun_dbg/prof (a -DGIC_PROFILE build).
#   bash tools/r03_batch2.sh <tag> <variant>
set -o pipefail
R=$GRAFT_REPO_ROOT
bash $R/tools/ab_bc7x.sh $1 "bc7 and not enc and not batch" $2 || exit 1
cd $R
GIC_LIBRARY=$R/gpurun_dbg/prof/lib.so timeout -k 10 300 python3 tools/prof_sections.py 64 > $R/gpurun_out/ab_$1/sections.txt 2>&1 || { tail $R/gpurun_out/ab_$1/sections.txt; exit 1; }
grep -v amdgpu.ids $R/gpurun_out/ab_$1/sections.txt
echo done
