# The one gpurun recipe (round 6; replaces the per-round tools/r0*.sh scripts).
# On the box:  bash tools/box.sh <step> <tag> [args...]   (steps chain with &&)
#   tests  <tag> [pytest -k expr]   the -m gpu suite, then smoke()
#   bench  <tag> [bench.py args]    bench.py -> gpurun_out/<tag>/bench.json
#   kstats <tag> <cmd...>           rocprofv3 --kernel-trace --stats of a python command
#   pmc    <tag> <counters> <cmd...> one rocprofv3 --pmc pass (<counters> quoted, space-separated)
#   run    <tag> <cmd...>           a plain command, output in gpurun_out/<tag>/run.log
# Every GPU step runs under its own time limit; a failure ends the call.
set -o pipefail
STEP=$1
TAG=$2
shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R" || exit 1
case "$STEP" in
tests)
  K=()
  [ -n "$1" ] && K=(-k "$1")
  timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${K[@]}" \
    > "$O/gpu_tests.log" 2>&1 || { tail -40 "$O/gpu_tests.log"; exit 1; }
  tail -3 "$O/gpu_tests.log"
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" >> "$O/gpu_tests.log" 2>&1 \
    || { tail -30 "$O/gpu_tests.log"; exit 1; }
  tail -1 "$O/gpu_tests.log"
  ;;
bench)
  timeout -k 10 900 python3 -u bench.py "$@" > "$O/bench.json" 2> "$O/bench.err" || { tail -30 "$O/bench.err"; exit 1; }
  tail -c 1500 "$O/bench.json"
  ;;
kstats)
  export TMPDIR=/tmp
  timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kstats" -o run -- "$@" \
    > "$O/kstats.log" 2>&1 || { tail -30 "$O/kstats.log"; exit 1; }
  python3 tools/kstats_csv.py "$O/kstats" > "$O/kernel_stats.txt" 2>/dev/null || true
  head -30 "$O/kernel_stats.txt"
  ;;
pmc)
  C=$1
  shift
  export TMPDIR=/tmp
  timeout -s KILL 300 rocprofv3 --pmc $C --output-format csv -d "$O/pmc" -o run -- "$@" > "$O/pmc.log" 2>&1 \
    || { tail -20 "$O/pmc.log"; exit 1; }
  echo "pmc done: $C"
  ;;
run)
  timeout -k 10 900 "$@" > "$O/run.log" 2>&1 || { tail -40 "$O/run.log"; exit 1; }
  tail -20 "$O/run.log"
  ;;
*)
  echo "unknown step $STEP"
  exit 2
  ;;
esac
