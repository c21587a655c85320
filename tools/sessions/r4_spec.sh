# k_long speculation: parity on small and full batches, request-sized rates with it on / off
set -u
O=$PWD/gpurun_out/r4_spec; mkdir -p $O
make -s -C tools > /dev/null
timeout -k 10 700 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_reference.py tests/test_gpu_parity.py tests/test_gpu_streams.py tests/test_gpu_repeats.py tests/test_gpu_vector.py > $O/pt.txt 2>&1 || { tail -30 $O/pt.txt; exit 1; }
tail -n 1 $O/pt.txt
for sp in 1 0; do
  CLD_LONG_SPEC=$sp REQ_RATE_CALLERS=${CALLERS:-1,8,32,64} timeout -k 10 400 python3 tools/req_rate.py > $O/spec$sp.jsonl 2> $O/spec$sp.err || { tail $O/spec$sp.err; exit 1; }
  python3 -c "
import json
for l in open('$O/spec$sp.jsonl'):
    d=json.loads(l)
    if 'callers' in d: print('spec $sp callers', d['callers'], 'docs/s %.0f'%d['docs_per_s'], 'p50 %.1f ms p99 %.1f ms'%(d['latency_ms_p50'], d['latency_ms_p99']))
    else: print(d['workload'][:40], '%.0f'%d['docs_per_s'])"
done
for c in c3 c5; do
  timeout -k 10 300 python3 bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-sub --no-host > $O/$c.json 2>$O/$c.err || { tail $O/$c.err; exit 1; }
  python3 -c "
import json; a=json.loads(open('$O/$c.json').read().strip().splitlines()[-1]); print('$c %.3f M docs/s k_long %.2f ms' % (a['value']/1e6, a['kernels']['long_ms']))"
done
