# A/B of the library at each round-3 commit (trees under _ab/<sha>, each with
# its own bench.py and corpus) against HEAD, C5 and C3 kernel lines.
set -u
O=gpurun_out/${TAG:-r3c_regress}; mkdir -p $O
for t in ${TREES:-53c3cbe 1a9d1dc 92ce54f a38c0ca 66578f6 HEAD}; do
  d=_ab/$t; [ $t = HEAD ] && d=.
  for c in ${CONFIGS:-c5 c3}; do
    (cd $d && timeout -k 10 300 python bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-sub --no-host) > $O/$t.$c.log 2>&1 || { tail -20 $O/$t.$c.log; exit 1; }
    echo $t $c; tail -1 $O/$t.$c.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']; print(d['value'], k['wave_ms'], k['long_ms'], k['general_ms'], d['passes_hist'])"
  done
done
