# k_long variants: C3 / C5 kernel lines and a C3 WRITE_SIZE pass each
set -u
export TMPDIR=/tmp
O=gpurun_out/r3d_lab; mkdir -p $O
for v in ${VARIANTS:-build_v_prev build}; do
  L=$PWD/language-detector_amd/$v/libcld_mi355x.so
  for c in c3 c5; do
    CLD_MI355X_LIB=$L timeout -k 10 300 python bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-sub --no-host > $O/$v.$c.json 2>&1 || { tail $O/$v.$c.json; exit 1; }
  done
  CLD_MI355X_LIB=$L timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_long -d $O/$v/pmc1 -o c3 --output-format csv -- python3 bench.py --config c3 --steps 2 --warmup 1 --no-cpu-baseline --no-sub --no-host > $O/$v.pmc.log 2>&1 || { tail $O/$v.pmc.log; exit 1; }
  python3 -c "
import json,sys; sys.path.insert(0,'tools'); import pmc_summary
a=json.loads(open('$O/$v.c3.json').read().strip().splitlines()[-1]); b=json.loads(open('$O/$v.c5.json').read().strip().splitlines()[-1])
s=pmc_summary.summarise('$O/$v')
print('$v c3', round(a['value']/1e6,3), 'M', round(a['kernels']['long_ms'],2), 'ms | c5', round(b['value']/1e6,2), 'M', round(b['kernels']['long_ms'],2), 'ms | c3 write GB', round(s.get('hbm_write_bytes',0)/1e9,2))"
done
