set -u
O=gpurun_out/ab7; mkdir -p $O
CLD_MI355X_LIB=$PWD/language-detector_amd/build_wv7/libcld_mi355x.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_wv7.log 2>&1 || { tail -20 $O/pytest_wv7.log; exit 1; }
tail -1 $O/pytest_wv7.log
for v in build build_wv7; do
  for c in c2 c4; do
    CLD_MI355X_LIB=$PWD/language-detector_amd/$v/libcld_mi355x.so timeout -k 10 200 python bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline > $O/$v.$c.log 2>&1 || exit 1
    echo $v $c; tail -1 $O/$v.$c.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['kernels']['wave_ms'])"
  done
done
