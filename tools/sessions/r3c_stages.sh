# k_wave stage pricing: one PMC pass per WAVE_STOP variant (the document ends
# after stage k) plus the full build, C2.
set -u
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r3c_stages}; mkdir -p $O
for v in ${VARIANTS:-build_v_stop0 build_v_stop1 build_v_stop2 build_v_stop3 build_v_stop4 build_v_stop5 build}; do
  CLD_MI355X_LIB=$PWD/language-detector_amd/$v/libcld_mi355x.so timeout -s KILL 150 rocprofv3 \
    --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD \
    --kernel-include-regex k_wave -d $O/$v/pmc1 -o c2 --output-format csv -- \
    python3 bench.py --config c2 --steps 2 --warmup 1 --no-cpu-baseline --no-sub --no-host > $O/$v.log 2>&1 || { tail -20 $O/$v.log; exit 1; }
  python3 tools/pmc_summary.py $O/$v | python3 -c "import json,sys; d=json.load(sys.stdin); c=d['counters_per_launch']; print('$v', {k: round(v/1e6,2) for k,v in c.items()})"
done
# C5 with and without the one-language C3 pages (does the C5 k_long time follow the data?)
for m in 0 0.25; do
  CLD_C3_MONO_FRAC=$m timeout -k 10 300 python bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline --no-sub --no-host > $O/c5_mono$m.log 2>&1 || { tail -20 $O/c5_mono$m.log; exit 1; }
  echo c5 mono $m; tail -1 $O/c5_mono$m.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']; print(d['value'], k['wave_ms'], k['long_ms'], d['passes_hist'])"
done
