# A/B timing of BC7 library variants in one box session: bash tools/ab_bc7.sh ROWS name1 name2 ...
# (variant "main" = the in-tree build, others = gpurun_dbg/<name>/lib.so); each run twice, interleaved
ROWS=$1; shift
for rep in 1 2; do
  for v in "$@"; do
    if [ "$v" = main ]; then L=""; else L=$PWD/gpurun_dbg/$v/lib.so; fi
    GIC_LIBRARY=$L timeout -k 10 200 python3 bench.py --format bc7 --rows $ROWS --steps 1 --warmup 1 --no-cpu 2>/dev/null \
      | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['kernel_ms'], d['blocks_per_s'])" || exit 1
  done
done
