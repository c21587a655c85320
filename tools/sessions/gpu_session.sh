#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, kernel-trace profile and
# PMC passes.  Every GPU step has its own time limit; the first failure ends
# the script (no retries).  Usage: tools/gpu_session.sh TAG [steps...]
#   steps: test smoke bench benchall prof pmc   (default: all but benchall)
set -u
TAG=${1:-r01}; shift || true
STEPS=${*:-test smoke bench prof pmc}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
run() {  # run <seconds> <log> cmd...
  local t=$1 log=$2; shift 2
  echo "[$(date +%T)] $* (limit ${t}s)" | tee -a "$O/session.log"
  timeout -k 10 "$t" "$@" > "$O/$log" 2>&1
  local rc=$?
  echo "[$(date +%T)] rc=$rc" | tee -a "$O/session.log"
  if [ $rc -ne 0 ]; then tail -40 "$O/$log"; exit $rc; fi
}
for s in $STEPS; do
  case $s in
    test)  run 900 pytest_gpu.log python -u -m pytest tests -m gpu -x -v -rA --durations=15 --timeout 300 --timeout-method thread ;;
    smoke) run 300 smoke.log python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run 400 bench_c2.log python bench.py ;;
    benchall)
      for c in c3 c4 c5; do run 400 bench_$c.log python bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline; done ;;
    prof)  run 400 prof.log rocprofv3 --kernel-trace --stats -d "$O/prof" -o c2 --output-format csv -- \
             python3 "$R/bench.py" --steps 5 --warmup 1 --no-cpu-baseline ;;
    pmc)
      run 400 pmc_fetch.log rocprofv3 --pmc FETCH_SIZE -d "$O/pmc_fetch" -o c2 --output-format csv -- \
             python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline
      run 400 pmc_write.log rocprofv3 --pmc WRITE_SIZE -d "$O/pmc_write" -o c2 --output-format csv -- \
             python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "session done" | tee -a "$O/session.log"
