# GPU suite on the in-tree build (unless NOTEST), then A/B C2 (or CONFIGS)
# kernel lines of library variants, REPS times each, interleaved.
set -u
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r3c_ab}; mkdir -p $O
if [ -z "${NOTEST:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${K:+-k "$K"} > $O/pytest_gpu.txt 2>&1; rc=$?
  tail -2 $O/pytest_gpu.txt
  [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/pytest_gpu.txt | head -30; exit $rc; }
fi
for rep in $(seq ${REPS:-2}); do
for v in ${VARIANTS:-build}; do
  for c in ${CONFIGS:-c2}; do
    CLD_MI355X_LIB=$PWD/language-detector_amd/$v/libcld_mi355x.so timeout -k 10 300 \
      python bench.py --config $c --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline --no-sub --no-host > $O/$v.$c.$rep.log 2>&1 || { tail -20 $O/$v.$c.$rep.log; exit 1; }
    tail -1 $O/$v.$c.$rep.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']; print('$v $c', round(d['value']/1e6,3), 'M', round(k['wave_ms'],3), round(k['long_ms'],3), d['passes_hist'])"
  done
done
done
