#!/bin/bash
# A/B of k_wave occupancy builds: GPU parity suite on each variant, then C2/C4 bench lines.
# Usage: VARIANTS="build build_wv8" bash tools/ab_wave7.sh   (libraries built beforehand, in-tree)
set -u
O=gpurun_out/abwave; mkdir -p $O
for v in ${VARIANTS:-build build_wv8}; do
  CLD_MI355X_LIB=$PWD/language-detector_amd/$v/libcld_mi355x.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_$v.log 2>&1 || { tail -20 $O/pytest_$v.log; exit 1; }
  echo $v; tail -1 $O/pytest_$v.log
done
for v in ${VARIANTS:-build build_wv8}; do
  for c in c2 c4; do
    CLD_MI355X_LIB=$PWD/language-detector_amd/$v/libcld_mi355x.so timeout -k 10 200 python bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline > $O/$v.$c.log 2>&1 || exit 1
    echo $v $c; tail -1 $O/$v.$c.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['kernels']['wave_ms'])"
  done
done
