# Exhaustive GPU check of the BC1 fast divisions (tools/rcp_check), BC1 A/B with
# traffic (in-tree vs gpurun_dbg/bc1h), then the BC1-BC5 GPU parity tests.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/ab_d1
mkdir -p $O
cd $R
timeout -k 10 120 ./tools/rcp_check > $O/rcp_check.txt 2>&1; rc=$?
cat $O/rcp_check.txt
[ $rc -le 1 ] || exit 1
bash $R/tools/ab_bc1_traffic.sh d1 bc1h || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_decode.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
echo done
