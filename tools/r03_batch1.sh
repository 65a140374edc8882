# Round-3 measurement batch: BC1 variant A/B with traffic, BC7 shaker section
# profile (GIC_PROFILE variant), single-stream kernel trace of the exact search.
set -o pipefail
R=$GRAFT_REPO_ROOT
bash $R/tools/ab_bc1_traffic.sh bc1lds head3 lds2 || exit 1
O=$R/gpurun_out/r03_batch1
mkdir -p $O
cd $R
GIC_LIBRARY=$R/gpurun_dbg/prof/lib.so timeout -k 10 300 python3 tools/prof_sections.py 64 > $O/sections.txt 2>&1 || { tail $O/sections.txt; exit 1; }
grep -v amdgpu.ids $O/sections.txt
cd /tmp && export TMPDIR=/tmp
GIC_BC7_SINGLE_STREAM=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/exact -o run -- python3 $R/tools/time_bc7_bounded.py --rows 256 --bound 0 > $O/exact.txt 2>&1 || exit 1
grep -v amdgpu.ids $O/exact.txt
echo done
