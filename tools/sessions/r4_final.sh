#!/bin/bash
# Round-4 evidence on the committed tree: the whole GPU suite, smoke(), the
# default bench line, C3/C5 lines, rocprofv3 kernel statistics for C2 and C3,
# PMC passes for k_wave @ C2 and k_long @ C3, HTML / vector-mode rates.
# Every GPU step has its own limit; the first failure ends the script.
set -u
TAG=${TAG:-r4z}
R=$PWD
O=$R/gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
step() { local t=$1 log=$2; shift 2; echo "[$(date +%T)] $log" | tee -a $O/session.log
  timeout -k 10 $t "$@" > $O/$log 2>&1; local rc=$?; echo "[$(date +%T)] rc=$rc" | tee -a $O/session.log
  if [ $rc -ne 0 ]; then tail -30 $O/$log; exit $rc; fi; }
for s in ${STEPS:-suite smoke bench lines prof pmc rates}; do
  case $s in
    suite) step 1000 pytest_gpu.txt python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread; tail -1 $O/pytest_gpu.txt ;;
    smoke) step 300 smoke.txt python -u -c "import __graft_entry__ as g; g.smoke()"; tail -2 $O/smoke.txt ;;
    bench) step 400 bench.json python bench.py ;;
    lines) for c in c3 c4 c5; do step 400 bench_$c.json python bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-host --no-sub; done ;;
    prof)
      (cd /tmp && step 300 prof_c2.log rocprofv3 --kernel-trace --stats -d $O/prof_c2 -o c2 --output-format csv -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-host --no-sub) || exit 1
      (cd /tmp && step 300 prof_c3.log rocprofv3 --kernel-trace --stats -d $O/prof_c3 -o c3 --output-format csv -- python3 $R/bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline --no-host --no-sub) || exit 1 ;;
    pmc)
      step 400 pmc_c2.log bash tools/pmc_session.sh ${TAG}_pmc_c2 c2 k_wave
      step 400 pmc_c3.log bash tools/pmc_session.sh ${TAG}_pmc_c3 c3 k_long ;;
    rates)
      step 300 html_rate.json python3 tools/html_rate.py
      step 400 vec_rate.jsonl python3 tools/vec_rate.py ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "session done" | tee -a $O/session.log
