# k_long read-ahead variants (LNG_PF) after the emission-index change: C3 / C5 k_long time
set -u
O=$PWD/gpurun_out/r4_pf; mkdir -p $O
for v in build build_v_pf0 build_v_pf6 build_v_pf7; do
  for c in c3 c5; do
    CLD_MI355X_LIB=$PWD/language-detector_amd/$v/libcld_mi355x.so timeout -k 10 300 python3 bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-sub --no-host > $O/$v.$c.json 2>$O/$v.$c.err || { tail $O/$v.$c.err; exit 1; }
    python3 -c "
import json; a=json.loads(open('$O/$v.$c.json').read().strip().splitlines()[-1]); print('$v $c %.3f M docs/s k_long %.2f ms' % (a['value']/1e6, a['kernels']['long_ms']))"
  done
done
