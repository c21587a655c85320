#!/bin/bash
# A/B of k_long occupancy variants on C3 and C5 (bench lines under gpurun_out/ablong)
set -u
O=gpurun_out/ablong; mkdir -p $O
for v in ${VARIANTS:-build build_lw8 build_lw9}; do
  for c in ${CONFIGS:-c3 c5}; do
    CLD_MI355X_LIB=$PWD/language-detector_amd/$v/libcld_mi355x.so timeout -k 10 300 python bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > $O/$v.$c.log 2>&1 || exit 1
    echo $v $c; tail -1 $O/$v.$c.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['kernels']['long_plus_general_ms'])"
  done
done
