# Round-3 evidence on the current tree: PMC passes of the dominant kernels
# (k_wave at C2, k_long at C3), kernel traces (C2, C3), bench lines per config.
set -u
export TMPDIR=/tmp
T=${TAG:-r3e}
O=gpurun_out/$T; mkdir -p $O
bash tools/pmc_session.sh ${T}_pmc_c2 c2 'k_wave' 1000000 || exit 1
bash tools/pmc_session.sh ${T}_pmc_c3 c3 'k_long' 100000 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace_c2 -o c2 --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-sub --no-host > $O/trace_c2.json 2> $O/trace_c2.err || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace_c3 -o c3 --output-format csv -- python3 bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline --no-sub --no-host > $O/trace_c3.json 2> $O/trace_c3.err || exit 1
echo traces done
[ -n "${NOBENCH:-}" ] && exit 0
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || exit 1
for c in ${CONFIGS:-c4 c5}; do
  timeout -k 10 400 python bench.py --config $c --no-cpu-baseline > $O/bench_$c.json 2> $O/bench_$c.err || exit 1
done
echo bench done
