# BC4/BC5 parity tests + the 8K BC4/BC5 legs + their VALU counters (usage: bash tools/r05_bc45.sh <tag>)
set -o pipefail
TAG=${1:-r05}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/bc45_$TAG
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "bc4 or bc5 or BC4 or BC5 or bc45 or snorm or smoke" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu --no-bc7enc --no-batch --bc7-rows 0 --bc6h-size 0 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));print('bc1',d['ms_per_step'],'bc4',d['bc4']['ms_per_step'],'bc5',d['bc5']['ms_per_step'])"
cd /tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/kt -o kt -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu --no-bc7enc --no-batch --bc7-rows 0 --bc6h-size 0 > $O/kt.log 2>&1 || { tail -20 $O/kt.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES -d $O/pmc -o pmc -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu --no-bc7enc --no-batch --bc7-rows 0 --bc6h-size 0 > $O/pmc.log 2>&1 || { tail -20 $O/pmc.log; exit 1; }
echo done
