set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04q; mkdir -p $O
bash tools/ab_bc1.sh r04q "" bc1u || exit 1
