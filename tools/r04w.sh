set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04w; mkdir -p $O
cd $R
export LD_LIBRARY_PATH=$R/gfx_imagecompress_amd/lib
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "bc4_block_batch or block_api" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -6 $O/tests.log
timeout -k 10 120 ./gpurun_dbg/launch_probe > $O/probe.txt 2>&1 || exit 1
timeout -k 10 120 ./gpurun_dbg/block_latency 2000 > $O/lat.txt 2>&1 || exit 1
cat $O/probe.txt $O/lat.txt
