#!/bin/bash
# Stage-cycle profile (CLD_PROFILE_STAGES) of each library variant, one line block per variant.
set -u
TAG=${TAG:-s3p}; O=gpurun_out/$TAG; mkdir -p $O
for v in ${PVARIANTS:-build}; do
  CLD_MI355X_LIB=$PWD/language-detector_amd/$v/libcld_mi355x.so timeout -k 10 300 \
    python tools/wave_prof.py ${PCFG:-c3:20000} > $O/prof_$v.log 2>&1 || { tail -20 $O/prof_$v.log; exit 1; }
  echo "prof $v"; grep "long cycles" $O/prof_$v.log
done
