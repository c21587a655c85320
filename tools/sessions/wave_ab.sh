#!/bin/bash
# k_wave A/B (round 6): per library variant (dirs under language-detector_amd/),
# the C2 bench line (k_wave ms) and one counter pass on k_wave (instructions
# and cycles per wave).  VARIANTS (default "build"), TAG.
set -u
TAG=${TAG:-wave_ab}; R=$PWD; O=$R/gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
for v in ${VARIANTS:-build}; do
  L=$R/language-detector_amd/$v/libcld_mi355x.so
  CLD_MI355X_LIB=$L timeout -k 10 300 python bench.py --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline --no-sub --no-host \
      > $O/$v.bench.log 2>&1 || { tail -20 $O/$v.bench.log; exit 1; }
  (cd /tmp && CLD_MI355X_LIB=$L timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY \
      SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU --kernel-include-regex k_wave -d $O/$v.pmc -o c2 \
      --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-sub --no-host > $O/$v.pmc.log 2>&1) \
      || { tail -20 $O/$v.pmc.log; exit 1; }
  echo "$v $(tail -1 $O/$v.bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['kernels']['wave_ms'])")"
done
echo "wave_ab done"
