# k_long at C3 with fewer resident waves per CU: time and HBM writes
set -u
export TMPDIR=/tmp
O=gpurun_out/r4_waves; mkdir -p $O
for w in ${WAVES_LIST:-16 12 8}; do
  CLD_LONG_WAVES=$w timeout -k 10 300 python3 bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline --no-sub --no-host > $O/w$w.json 2>$O/w$w.err || { tail $O/w$w.err; exit 1; }
  CLD_LONG_WAVES=$w timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_long -d $O/w$w/pmc1 -o c3 --output-format csv -- python3 bench.py --config c3 --steps 2 --warmup 1 --no-cpu-baseline --no-sub --no-host > $O/w$w.pmc.log 2>&1 || { tail $O/w$w.pmc.log; exit 1; }
  CLD_LONG_WAVES=$w timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_long -d $O/w$w/pmc2 -o c3 --output-format csv -- python3 bench.py --config c3 --steps 2 --warmup 1 --no-cpu-baseline --no-sub --no-host > $O/w$w.pmc2.log 2>&1 || { tail $O/w$w.pmc2.log; exit 1; }
  python3 -c "
import json,sys; sys.path.insert(0,'tools'); import pmc_summary
a=json.loads(open('$O/w$w.json').read().strip().splitlines()[-1])
s=pmc_summary.summarise('$O/w$w')
print('waves/CU $w: c3', round(a['value']/1e6,3), 'M docs/s, k_long', round(a['kernels']['long_ms'],2), 'ms, write GB', round(s.get('hbm_write_bytes',0)/1e9,2), 'fetch GB', round(s.get('hbm_fetch_bytes',0)/1e9,2))"
done
