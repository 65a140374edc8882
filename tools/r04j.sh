set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04j; mkdir -p $O
GIC_LIBRARY=$R/gpurun_dbg/prof/lib.so timeout -k 10 300 python3 tools/prof_sections.py 64 > $O/sections.txt 2>&1 || { tail -5 $O/sections.txt; exit 1; }
grep -v amdgpu.ids $O/sections.txt
bash tools/ab_quick.sh r04j 2 dq3 || exit 1
echo ok
