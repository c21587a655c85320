# Round-2 profile of the current tree: stage cycles of k_long (C3), kernel
# trace stats of the default bench, PMC passes for c3 k_long (100K pages).
set -u
export TMPDIR=/tmp
O=gpurun_out/r2l; mkdir -p $O
timeout -k 10 300 python tools/wave_prof.py c3:30000 > $O/wave_prof.log 2>&1 || exit 1
cat $O/wave_prof.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o bench --output-format csv -- python3 bench.py --no-cpu-baseline > $O/trace_bench.json 2> $O/trace_bench.err || exit 1
tail -c 400 $O/trace_bench.json
bash tools/pmc_session.sh r2l_pmc_c3 c3 'k_long' 100000 || exit 1
python tools/pmc_summary.py gpurun_out/r2l_pmc_c3 > $O/pmc_c3_summary.json
cat $O/pmc_c3_summary.json | head -60
