set -o pipefail
R=$GRAFT_REPO_ROOT
bash tools/profile_r04.sh r04e tests || exit 1
mkdir -p $R/gpurun_out/b05 && cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 python3 $R/bench.py --steps 20 --warmup 5 > $R/gpurun_out/b05/bench.json 2> $R/gpurun_out/b05/bench.err || { tail -5 $R/gpurun_out/b05/bench.err; exit 1; }
tail -c 400 $R/gpurun_out/b05/bench.json
