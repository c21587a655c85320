# PMC of k_wave on the C2 bench alone (no C3 sub-run, no host path), and
# kernel traces of the C2 and C3 bench lines alone, so every per-launch figure
# is one configuration's.
set -u
export TMPDIR=/tmp
O=gpurun_out/r2final2; mkdir -p $O
bash tools/pmc_session.sh r2final2_pmc_c2 c2 'k_wave' 1000000 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_c2 -o c2 --output-format csv -- python3 bench.py --no-cpu-baseline --no-sub --no-host > $O/trace_c2.json 2> $O/trace_c2.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_c3 -o c3 --output-format csv -- python3 bench.py --config c3 --no-cpu-baseline > $O/trace_c3.json 2> $O/trace_c3.err || exit 1
echo final2 done
