set -o pipefail
R=$GRAFT_REPO_ROOT
bash $R/tools/pmc_valu.sh r01c || exit 1
cd /tmp && export TMPDIR=/tmp
GIC_BC7_SINGLE_STREAM=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_r01c_bc7 -o run -- python3 $R/bench.py --format bc7 --rows 512 --steps 1 --warmup 1 --no-cpu > $R/gpurun_out/prof_r01c_bc7.json 2>$R/gpurun_out/prof_r01c_bc7.err || exit 1
echo ok
