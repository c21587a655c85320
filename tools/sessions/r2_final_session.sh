# Round-2 evidence on the current tree: GPU suite, smoke, PMC passes of the
# dominant kernels (k_wave at C2, k_long at C3 -- the sizes bench.py runs),
# a kernel-trace of the default bench, then bench lines for every config.
set -u
export TMPDIR=/tmp
O=gpurun_out/r2final; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1; rc=$?
tail -3 $O/pytest_gpu.txt
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit 1
cat $O/smoke.txt
bash tools/pmc_session.sh r2final_pmc_c2 c2 'k_wave' 1000000 || exit 1
bash tools/pmc_session.sh r2final_pmc_c3 c3 'k_long' 100000 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o bench --output-format csv -- python3 bench.py --no-cpu-baseline > $O/trace_bench.json 2> $O/trace_bench.err || exit 1
for c in c3 c4 c5; do
  timeout -k 10 400 python bench.py --config $c > $O/bench_$c.json 2> $O/bench_$c.err || exit 1
done
echo final done
