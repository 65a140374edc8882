set -o pipefail
O=gpurun_out/sweep; mkdir -p $O
for f in bc4 bc5; do timeout -k 10 200 python3 bench.py --format $f --no-cpu --bc7-rows 0 > $O/$f.json 2>$O/$f.err || exit 1; done
for q in 0.05 0.1 0.2 0.3 0.5 0.7 0.9; do timeout -k 10 300 python3 bench.py --format bc7 --rows 512 --steps 2 --warmup 1 --no-cpu --bc7-quality $q > $O/bc7_q$q.json 2>$O/bc7_q$q.err || exit 1; echo q$q done; done
