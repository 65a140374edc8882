# BC1 2-wave vs 3-wave build (time + FETCH_SIZE), BC4 static channel select (time).
set -o pipefail
R=$GRAFT_REPO_ROOT
bash $R/tools/ab_bc1_traffic.sh w2 w2 || exit 1
O=$R/gpurun_out/ab_b4
mkdir -p $O
cd $R
for rep in 1 2; do
  for v in default b4; do
    if [ "$v" = default ]; then L=""; else L=$R/gpurun_dbg/$v/lib.so; fi
    GIC_LIBRARY=$L timeout -k 10 200 python3 bench.py --format bc4 --no-cpu --steps 50 --warmup 5 > $O/$v.$rep.json 2>&1 || exit 1
    python3 -c "import json; d=json.loads(open('$O/$v.$rep.json').read().strip().splitlines()[-1]); print('$v', d['ms_per_step'], d['value'], d.get('gpu_parity'))"
  done
done
echo done
