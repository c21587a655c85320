# request-sized C-harness rates on this tree: contexts per GPU x concurrent callers
set -u
O=$PWD/gpurun_out/r4_req; mkdir -p $O
make -s -C tools > /dev/null
for ctx in 1 2 4; do
  CLD_MI355X_CONTEXTS=$ctx REQ_RATE_CALLERS=${CALLERS:-1,8,32,64,128} timeout -k 10 400 python3 tools/req_rate.py > $O/ctx$ctx.jsonl 2> $O/ctx$ctx.err || { tail $O/ctx$ctx.err; exit 1; }
  python3 -c "
import json
for l in open('$O/ctx$ctx.jsonl'):
    d=json.loads(l)
    if 'callers' in d: print('contexts $ctx callers', d['callers'], 'docs/s %.0f'%d['docs_per_s'], 'p50 %.1f ms p99 %.1f ms'%(d['latency_ms_p50'], d['latency_ms_p99']))
    else: print(d['workload'][:40], '%.0f'%d['docs_per_s'])"
done
