# Round-5 first box call: the default bench (new split/ordering), a 2-rank gloo
# rehearsal of the 8K split on one GPU, and one-pass VALU counters of the BC7 8K legs.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05a
mkdir -p $O
cd $R
timeout -k 10 600 python3 bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
tail -c 600 $O/bench.json
timeout -k 10 300 python3 bench.py --gpus 2 --dist-backend gloo --bc7-rows 16 --no-batch --bc6h-size 256 --steps 3 --warmup 1 --cpu-seconds 4 > $O/gloo2.json 2> $O/gloo2.err || { tail -30 $O/gloo2.err; exit 1; }
tail -c 300 $O/gloo2.json
cd /tmp && export TMPDIR=/tmp
C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
for leg in "bc7 0 0" "bc7_pruned 2 0" "bc7_bounded 0 0.5" "bc7_bounded_pruned 2 0.5"; do
  set -- $leg
  timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $O/pmc_$1 -o run -- python3 $R/tools/time_bc7_bounded.py --rows 2048 --shake-ranks $2 --bound $3 --no-warm > $O/pmc_$1.log 2>&1 || { tail -20 $O/pmc_$1.log; exit 1; }
  python3 $R/tools/valu_pass.py $O/pmc_$1 $O/valu_$1_pass.json --label "$1: 8K G1 one pass, shake ranks $2, bound $3" --command "tools/time_bc7_bounded.py --rows 2048 --shake-ranks $2 --bound $3 --no-warm" || exit 1
done
echo done
