set -o pipefail
O=gpurun_out/r04e; mkdir -p $O
bash tools/ab_quick.sh r04e 2 occ7 || exit 1
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_gpu_bc7.py tests/test_gpu_bc7_sample.py -k "not performance_levels" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
GIC_LIBRARY=$GRAFT_REPO_ROOT/gpurun_dbg/prof/lib.so timeout -k 10 300 python3 tools/prof_sections.py 64 > $O/sections.txt 2>&1 || { tail -5 $O/sections.txt; exit 1; }
cat $O/sections.txt
timeout -k 10 200 python3 tools/time_bc45.py 20 > $O/bc45.txt 2>&1 || { tail -5 $O/bc45.txt; exit 1; }
grep -v amdgpu.ids $O/bc45.txt
bash tools/prof_bc6h_r04.sh r04e || exit 1
