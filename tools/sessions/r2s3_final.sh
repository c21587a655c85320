# Session-3 evidence, part 2: GPU suite, smoke, a kernel trace of the default
# bench (C2 headline with the C3 sub-object), C3 kernel trace, bench lines per config.
set -u
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r2s3}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1; rc=$?
tail -3 $O/pytest_gpu.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit 1
cat $O/smoke.txt
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o bench --output-format csv -- python3 bench.py --no-cpu-baseline > $O/trace_bench.json 2> $O/trace_bench.err || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace_c2 -o c2 --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-sub --no-host > $O/trace_c2.json 2> $O/trace_c2.err || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace_c3 -o c3 --output-format csv -- python3 bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline --no-sub --no-host > $O/trace_c3.json 2> $O/trace_c3.err || exit 1
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || exit 1
for c in c3 c4 c5; do
  timeout -k 10 400 python bench.py --config $c > $O/bench_$c.json 2> $O/bench_$c.err || exit 1
done
echo final done
