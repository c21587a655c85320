# Quick GPU check of a change: the GPU suite (optionally -k FILTER), smoke.
set -u
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r3q}; mkdir -p $O
K=${K:-}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${K:+-k "$K"} > $O/pytest_gpu.txt 2>&1; rc=$?
tail -5 $O/pytest_gpu.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit 1
cat $O/smoke.txt
