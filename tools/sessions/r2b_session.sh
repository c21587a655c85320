set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r2b
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r2b/pytest_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/r2b/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
TAG=r2b VARIANTS="build build_w4" CONFIGS="c3" bash tools/ab.sh && TAG=r2b VARIANTS="build" CONFIGS="c2 c5" bash tools/ab.sh
