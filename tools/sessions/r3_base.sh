# Round 3 GPU check: GPU suite, smoke, then bench lines for C2 (with the C3
# sub-object) and C5, plus a C3 kernel trace.
set -u
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r3base}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1; rc=$?
tail -3 $O/pytest_gpu.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit 1
cat $O/smoke.txt
[ -n "${NOBENCH:-}" ] && exit 0
timeout -k 10 400 python bench.py --cpu-seconds 5 > $O/bench.json 2> $O/bench.err || exit 1
timeout -k 10 400 python bench.py --config c5 --no-cpu-baseline > $O/bench_c5.json 2> $O/bench_c5.err || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace_c3 -o c3 --output-format csv -- python3 bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline --no-sub --no-host > $O/trace_c3.json 2> $O/trace_c3.err || exit 1

CLD_PROFILE_STAGES=1 timeout -k 10 300 python tools/wave_prof.py c2:1000000 c3:20000 c5:200000 > $O/stages.txt 2>&1 || exit 1
echo stages done
[ -n "${AB:-}" ] || exit 0
TAG=${TAG:-r3base}/ab VARIANTS="$AB" CONFIGS="c3 c5" bash tools/sessions/ab.sh > $O/ab.txt 2>&1 || { cat $O/ab.txt; exit 1; }
cat $O/ab.txt
