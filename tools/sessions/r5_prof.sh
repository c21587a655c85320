# rocprofv3 kernel statistics of bench lines: PROFCFG configs, PROFENV extra env
set -u
TAG=${TAG:-r5f}; R=$PWD; O=$R/gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
for c in ${PROFCFG:-c3 c5}; do
  (cd /tmp && timeout -k 10 300 env ${PROFENV:-X=1} rocprofv3 --kernel-trace --stats -d $O/prof_$c -o $c --output-format csv -- python3 $R/bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-host --no-sub > $O/prof_$c.log 2>&1) || { tail -20 $O/prof_$c.log; exit 1; }
done
find $O -name "*kernel_stats.csv" | while read f; do echo "== $f"; cut -d, -f1-8 "$f" | head -12; done
