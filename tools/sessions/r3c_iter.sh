# Iteration check: GPU suite, C2 bench line, one k_wave PMC pass at C2,
# then (CONFIGS) kernel lines for other configs.
set -u
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r3c_iter}; mkdir -p $O
if [ -z "${NOTEST:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${K:+-k "$K"} > $O/pytest_gpu.txt 2>&1; rc=$?
  tail -3 $O/pytest_gpu.txt
  [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/pytest_gpu.txt | head -30; exit $rc; }
fi
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-sub --no-host > $O/bench_c2.json 2> $O/bench_c2.err || { tail $O/bench_c2.err; exit 1; }
python -c "import json; d=json.loads(open('$O/bench_c2.json').read().strip().splitlines()[-1]); print('c2', d['value'], d['kernels']['wave_ms'])"
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD \
    --kernel-include-regex k_wave -d $O/wave/pmc1 -o c2 --output-format csv -- \
    python3 bench.py --config c2 --steps 2 --warmup 1 --no-cpu-baseline --no-sub --no-host > $O/pmc_wave.log 2>&1 || { tail -20 $O/pmc_wave.log; exit 1; }
python3 tools/pmc_summary.py $O/wave | python3 -c "import json,sys; d=json.load(sys.stdin); c=d['counters_per_launch']; print('k_wave per doc', {k: round(v/1e6,1) for k,v in c.items()})"
for c in ${CONFIGS:-}; do
  timeout -k 10 300 python bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-sub --no-host > $O/$c.log 2>&1 || { tail -20 $O/$c.log; exit 1; }
  tail -1 $O/$c.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']; print('$c', d['value'], k['wave_ms'], k['long_ms'], k['general_ms'], d['passes_hist'])"
done
