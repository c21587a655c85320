# A library variant through the GPU suite (LIB=dir under language-detector_amd/), then A/B lines.
set -u
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r3inc}; mkdir -p $O
L=$PWD/language-detector_amd/${LIB:-build}/libcld_mi355x.so
CLD_MI355X_LIB=$L timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${K:+-k "$K"} > $O/pytest_gpu.txt 2>&1; rc=$?
tail -3 $O/pytest_gpu.txt
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/pytest_gpu.txt | head -30; exit $rc; }
TAG=${TAG:-r3inc}/ab VARIANTS="${AB:-build}" CONFIGS="${CONFIGS:-c3 c5}" bash tools/sessions/ab.sh > $O/ab.txt 2>&1 || { cat $O/ab.txt; exit 1; }
cat $O/ab.txt
