#!/bin/bash
# vector-mode parity tests and throughput after the MapBack resume cursor
O=gpurun_out/r3h; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_vector.py tests/test_gpu_reference.py -x -v --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
echo "tests ok"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/vec -o vec -- python3 tools/vec_rate.py > $O/vec_rate.jsonl 2> $O/vec.err || { tail $O/vec.err; exit 1; }
echo "vec ok"
cat $O/vec_rate.jsonl
