# request-sized rates and HTML end to end after tail-bound chunking
set -u
O=$PWD/gpurun_out/r4_spec2; mkdir -p $O
make -s -C tools > /dev/null
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_streams.py tests/test_gpu_reference.py > $O/pt.txt 2>&1 || { tail -30 $O/pt.txt; exit 1; }
tail -n 1 $O/pt.txt
REQ_RATE_CALLERS=${CALLERS:-1,8,32,64,128} timeout -k 10 400 python3 tools/req_rate.py > $O/req.jsonl 2> $O/req.err || { tail $O/req.err; exit 1; }
python3 -c "
import json
for l in open('$O/req.jsonl'):
    d=json.loads(l)
    if 'callers' in d: print('callers', d['callers'], 'docs/s %.0f'%d['docs_per_s'], 'p50 %.1f ms p99 %.1f ms'%(d['latency_ms_p50'], d['latency_ms_p99']))
    else: print(d['workload'][:40], '%.0f'%d['docs_per_s'])"
CLD_NO_CPU=1 timeout -k 10 300 python3 tools/html_rate.py > $O/html.json 2> $O/html.err || { tail $O/html.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/html.json')); print('html e2e %.3f M kernel %.3f M' % (d['docs_per_s_end_to_end']/1e6, d['docs_per_s_kernel']/1e6))"
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-sub > $O/c2.json 2> $O/c2.err || { tail $O/c2.err; exit 1; }
python3 -c "
import json; a=json.loads(open('$O/c2.json').read().strip().splitlines()[-1]); print('c2 %.2f M' % (a['value']/1e6), json.dumps(a['host_path']))"
