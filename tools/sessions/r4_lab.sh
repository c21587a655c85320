# k_long lab variants (never shipped): C3 time and HBM traffic per launch
set -u
export TMPDIR=/tmp
O=gpurun_out/r4_lab; mkdir -p $O
for v in ${VARIANTS:-build build_v_nocache build_v_noadds}; do
  L=$PWD/language-detector_amd/$v/libcld_mi355x.so
  CLD_MI355X_LIB=$L timeout -k 10 300 python3 bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline --no-sub --no-host > $O/$v.json 2>$O/$v.err || { tail $O/$v.err; exit 1; }
  CLD_MI355X_LIB=$L timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_long -d $O/$v/pmc1 -o c3 --output-format csv -- python3 bench.py --config c3 --steps 2 --warmup 1 --no-cpu-baseline --no-sub --no-host > $O/$v.pmc.log 2>&1 || { tail $O/$v.pmc.log; exit 1; }
  CLD_MI355X_LIB=$L timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_long -d $O/$v/pmc2 -o c3 --output-format csv -- python3 bench.py --config c3 --steps 2 --warmup 1 --no-cpu-baseline --no-sub --no-host > $O/$v.pmc2.log 2>&1 || { tail $O/$v.pmc2.log; exit 1; }
  python3 -c "
import json,sys; sys.path.insert(0,'tools'); import pmc_summary
a=json.loads(open('$O/$v.json').read().strip().splitlines()[-1])
s=pmc_summary.summarise('$O/$v')
print('$v: c3', round(a['value']/1e6,3), 'M docs/s, k_long', round(a['kernels']['long_ms'],2), 'ms, passes', a['passes_hist'], 'write GB', round(s.get('hbm_write_bytes',0)/1e9,2), 'fetch GB', round(s.get('hbm_fetch_bytes',0)/1e9,2))"
done
