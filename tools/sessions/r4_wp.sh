# persistent k_wave lab variants: C2 kernel time, SALU per tweet; parity of the first
set -u
export TMPDIR=/tmp
O=$PWD/gpurun_out/r4_wp; mkdir -p $O
R=$PWD
for v in build build_v_wpinf build_v_wp1 build_v_wp2 build_v_wp4; do
  L=$R/language-detector_amd/$v/libcld_mi355x.so
  CLD_MI355X_LIB=$L timeout -k 10 200 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-sub --no-host > $O/$v.json 2>$O/$v.err || { tail $O/$v.err; exit 1; }
  CLD_MI355X_LIB=$L timeout -k 10 200 python3 bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline --no-sub --no-host > $O/$v.c5.json 2>$O/$v.c5.err || { tail $O/$v.c5.err; exit 1; }
  python3 -c "
import json
a=json.loads(open('$O/$v.json').read().strip().splitlines()[-1]); b=json.loads(open('$O/$v.c5.json').read().strip().splitlines()[-1])
print('$v', 'c2 %.2f M wave_ms %.3f | c5 %.2f M wave_ms %.3f' % (a['value']/1e6, a['kernels']['wave_ms'], b['value']/1e6, b['kernels']['wave_ms']))"
done
CLD_MI355X_LIB=$R/language-detector_amd/build_v_wp2/libcld_mi355x.so timeout -k 10 500 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_reference.py > $O/pt_wp2.txt 2>&1; tail -n 2 $O/pt_wp2.txt
