#!/bin/bash
# Parity suite + bench on the default build, then A/B variants (bench + parity each),
# then the stage profile of the default build.  First failure ends it.
set -u
TAG=${TAG:-s3x}; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
TAG=$TAG bash tools/s3_session.sh || exit 1
for v in ${AB:-}; do
  TAG=$TAG TESTS=0 VARIANTS="$v" CONFIGS="c3 c5" bash tools/s3_session.sh || exit 1
  CLD_MI355X_LIB=$PWD/language-detector_amd/$v/libcld_mi355x.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_$v.log 2>&1
  rc=$?; echo "pytest $v: $(tail -1 $O/pytest_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
TAG=$TAG PCFG="${PCFG:-c3:20000 c5:200000}" bash tools/s3_prof.sh
