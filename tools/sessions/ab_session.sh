set -u
O=gpurun_out/ab1; mkdir -p $O
for v in build build_wv5 build_wv4; do
  for c in c2 c4; do
    CLD_MI355X_LIB=$PWD/language-detector_amd/$v/libcld_mi355x.so timeout -k 10 200 python bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline > $O/$v.$c.log 2>&1 || exit 1
    echo $v $c; tail -1 $O/$v.$c.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['kernels']['wave_ms'])"
  done
done
timeout -k 10 300 python tools/wave_prof.py c2:1000000 c4:200000 c5:200000 c3:20000 > $O/wave_prof.log 2>&1; cat $O/wave_prof.log
