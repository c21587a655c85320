# Round 3 step check: GPU suite, smoke, C3/C5 lines, host path + service rate.
set -u
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r3s2}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1; rc=$?
tail -3 $O/pytest_gpu.txt
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/pytest_gpu.txt | head -20; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { cat $O/smoke.txt; exit 1; }
cat $O/smoke.txt
TAG=${TAG:-r3s2}/ab VARIANTS="${AB:-build}" CONFIGS="${CONFIGS:-c3 c5}" bash tools/sessions/ab.sh > $O/ab.txt 2>&1 || { cat $O/ab.txt; exit 1; }
cat $O/ab.txt
[ -n "${NOBENCH:-}" ] && exit 0
timeout -k 10 400 python bench.py --cpu-seconds 5 > $O/bench.json 2> $O/bench.err || exit 1
tail -c 600 $O/bench.json
timeout -k 10 300 python tools/service_rate.py --docs 200000 --seconds 8 > $O/service_rate.json 2> $O/service_rate.err || { tail -5 $O/service_rate.err; exit 1; }
cat $O/service_rate.json
