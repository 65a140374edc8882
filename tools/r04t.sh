set -o pipefail
R=$GRAFT_REPO_ROOT
bash tools/profile_r04.sh r04e prof || exit 1
bash tools/pmc_traffic_bc1.sh r04e || exit 1
