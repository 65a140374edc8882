# BC1 A/B with traffic (in-tree vs gpurun_dbg/bc1h), BC7 exact A/B (in-tree vs
# gpurun_dbg/noquad), then the BC1/BC2/BC3/BC4/BC5 GPU parity tests.
set -o pipefail
R=$GRAFT_REPO_ROOT
bash $R/tools/ab_bc1_traffic.sh bc1b bc1h || exit 1
O=$R/gpurun_out/ab_q1
mkdir -p $O
cd $R
for rep in 1 2; do
  for v in default noquad; do
    if [ "$v" = default ]; then L=""; else L=$R/gpurun_dbg/$v/lib.so; fi
    echo "== $v" >> $O/bc7.txt
    GIC_LIBRARY=$L timeout -k 10 300 python3 tools/time_bc7_bounded.py --rows 256 --bound 0 >> $O/bc7.txt 2>&1 || exit 1
  done
done
grep -v amdgpu.ids $O/bc7.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
echo done
