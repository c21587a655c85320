#!/bin/bash
# Session-3 A/B: bench lines per variant/config, then the k_long stage profile per variant.
set -u
TAG=${TAG:-s3}; O=gpurun_out/$TAG; mkdir -p $O
TAG=$TAG VARIANTS="${VARIANTS:-build}" CONFIGS="${CONFIGS:-c3 c5}" bash tools/ab.sh || exit 1
for v in ${PVARIANTS:-}; do
  CLD_MI355X_LIB=$PWD/language-detector_amd/$v/libcld_mi355x.so timeout -k 10 300 \
    python tools/wave_prof.py ${PCFG:-c3:20000} > $O/prof_$v.log 2>&1 || { tail -20 $O/prof_$v.log; exit 1; }
  echo "prof $v"; cat $O/prof_$v.log
done
