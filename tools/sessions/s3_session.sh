#!/bin/bash
# Session-3 GPU check: parity suite, then bench lines (C2/C3/C5 by default).
# Every GPU step has its own limit; the first failure ends the script.
set -u
TAG=${TAG:-s3}; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -rA --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
  rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest_gpu.log | head -30; exit $rc; }
fi
TAG=$TAG VARIANTS="${VARIANTS:-build}" CONFIGS="${CONFIGS:-c2 c3 c5}" bash tools/ab.sh
