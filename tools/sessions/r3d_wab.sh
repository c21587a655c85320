# k_wave variants: C2 kernel lines and a WRITE_SIZE pass each
set -u
export TMPDIR=/tmp
O=gpurun_out/r3d_wab; mkdir -p $O
for v in ${VARIANTS:-build_v_prev build}; do
  L=$PWD/language-detector_amd/$v/libcld_mi355x.so
  CLD_MI355X_LIB=$L timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-sub --no-host > $O/$v.json 2>&1 || { tail $O/$v.json; exit 1; }
  CLD_MI355X_LIB=$L timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_wave -d $O/$v/pmc1 -o c2 --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-sub --no-host > $O/$v.pmc.log 2>&1 || { tail $O/$v.pmc.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/$v.json').read().strip().splitlines()[-1])
import sys; sys.path.insert(0,'tools'); import pmc_summary; s=pmc_summary.summarise('$O/$v')
print('$v', round(d['value']/1e6,2), 'M', round(d['kernels']['wave_ms'],3), 'ms  write GB', round(s.get('hbm_write_bytes',0)/1e9,2))"
done
