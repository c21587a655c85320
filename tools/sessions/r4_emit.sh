# k_long with 32-bit emission indices: parity, C3/C5 lines, C3 HBM traffic
set -u
export TMPDIR=/tmp
O=$PWD/gpurun_out/r4_emit; mkdir -p $O
R=$PWD
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_reference.py tests/test_gpu_parity.py tests/test_gpu_vector.py tests/test_gpu_repeats.py > $O/pt.txt 2>&1 || { tail -30 $O/pt.txt; exit 1; }
tail -n 1 $O/pt.txt
for c in c3 c5; do
  timeout -k 10 300 python3 bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-sub --no-host > $O/$c.json 2>$O/$c.err || { tail $O/$c.err; exit 1; }
done
(cd /tmp && timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_long -d $O/pmc1 -o c3 --output-format csv -- python3 $R/bench.py --config c3 --steps 2 --warmup 1 --no-cpu-baseline --no-sub --no-host > $O/pmc1.log 2>&1) || { tail $O/pmc1.log; exit 1; }
(cd /tmp && timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_long -d $O/pmc2 -o c3 --output-format csv -- python3 $R/bench.py --config c3 --steps 2 --warmup 1 --no-cpu-baseline --no-sub --no-host > $O/pmc2.log 2>&1) || { tail $O/pmc2.log; exit 1; }
python3 -c "
import json,sys; sys.path.insert(0,'tools'); import pmc_summary
a=json.loads(open('$O/c3.json').read().strip().splitlines()[-1]); b=json.loads(open('$O/c5.json').read().strip().splitlines()[-1])
s=pmc_summary.summarise('$O')
print('c3 %.3f M docs/s k_long %.2f ms | c5 %.2f M k_long %.2f ms | c3 write %.2f GB fetch %.2f GB' % (a['value']/1e6, a['kernels']['long_ms'], b['value']/1e6, b['kernels']['long_ms'], s['hbm_write_bytes']/1e9, s['hbm_fetch_bytes']/1e9))"
