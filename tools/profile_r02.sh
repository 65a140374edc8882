# Round-2 profile set (GPU box): default bench + the same under rocprofv3
# kernel trace/stats + FETCH_SIZE / WRITE_SIZE passes (tools/profile_round.sh),
# VALU PMC passes (tools/pmc_valu.sh, exact BC7 search), a single-stream BC7
# kernel trace of the exact and of the pruned search, and a small batch64
# (configs[4]) run.  Then on the host: python tools/refresh_profiles.py r02 r02 prof_r02_bc7_k0 r02
set -o pipefail
R=$GRAFT_REPO_ROOT
bash $R/tools/profile_round.sh r02 || exit 1
bash $R/tools/pmc_valu.sh r02 || exit 1
bash $R/tools/prof_bc7_split.sh r02_bc7 128 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 $R/bench.py --workload batch64 --batch-slices 8 --batch-size 1024 --steps 1 --warmup 1 \
  > $R/gpurun_out/batch64_small.json 2> $R/gpurun_out/batch64_small.err || exit 1
echo done
