set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r2c
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r2c/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/r2c/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
TAG=r2c VARIANTS="build" CONFIGS="c3 c5" bash tools/ab.sh && \
timeout -k 10 200 python bench.py --steps 10 > gpurun_out/r2c/bench_default.log 2>&1; tail -1 gpurun_out/r2c/bench_default.log
