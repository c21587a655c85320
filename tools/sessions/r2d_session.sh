set -u
export TMPDIR=/tmp
O=gpurun_out/r2d; mkdir -p $O
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -5 $O/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/wave_prof.py c3:30000 c5:200000 > $O/wave_prof.log 2>&1 || exit 1
cat $O/wave_prof.log
bash tools/pmc_session.sh r2d_pmc_c3 c3 'k_long' 30000
