set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04v; mkdir -p $O
cd $R
export LD_LIBRARY_PATH=$R/gfx_imagecompress_amd/lib
echo "== default scheduling" > $O/probe.txt
timeout -k 10 120 ./gpurun_dbg/launch_probe >> $O/probe.txt 2>&1 || exit 1
echo "== hipDeviceScheduleSpin" >> $O/probe.txt
timeout -k 10 120 ./gpurun_dbg/launch_probe spin >> $O/probe.txt 2>&1 || exit 1
cat $O/probe.txt
