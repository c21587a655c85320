#!/bin/bash
# A/B of library variants: VARIANTS (dirs under language-detector_amd/) x CONFIGS.
# One bench line per (variant, config) under gpurun_out/$TAG/.  Stops at the first failure.
set -u
TAG=${TAG:-ab}; O=gpurun_out/$TAG; mkdir -p $O
for v in ${VARIANTS:-build}; do
  for c in ${CONFIGS:-c3}; do
    CLD_MI355X_LIB=$PWD/language-detector_amd/$v/libcld_mi355x.so timeout -k 10 300 \
      python bench.py --config $c --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline --no-sub --no-host ${EXTRA:-} > $O/$v.$c.log 2>&1 || { tail -20 $O/$v.$c.log; exit 1; }
    echo $v $c; tail -1 $O/$v.$c.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']; print(d['value'], k['wave_ms'], k['long_ms'], k['general_ms'], k['last_batch']['general_docs'], d['passes_hist'], k['last_batch']['long_requeue_reasons'])"
  done
done
