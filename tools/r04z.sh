set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04z; mkdir -p $O
cd $R
export LD_LIBRARY_PATH=$R/gfx_imagecompress_amd/lib
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_bc7enc.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 120 ./gpurun_dbg/block_latency 2000 > $O/lat.txt 2>&1 || exit 1
cat $O/lat.txt
