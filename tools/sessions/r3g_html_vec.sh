#!/bin/bash
# HTML rewrite tests + rate, vector-mode tests, vector-mode rate (A/B of the
# longest-first order, rocprofv3 kernel stats of the default)
O=gpurun_out/r3g; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_html_hints.py tests/test_gpu_vector.py -x -v --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
echo "tests ok"
timeout -k 10 200 python -u tools/html_rate.py > $O/html_rate.json 2> $O/html_rate.err || { tail $O/html_rate.err; exit 1; }
echo "html ok"
CLD_VEC_ORDER=0 timeout -k 10 200 python -u tools/vec_rate.py > $O/vec_rate_noorder.jsonl 2> $O/vec_noorder.err || { tail $O/vec_noorder.err; exit 1; }
echo "vec A ok"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/vec -o vec -- python3 tools/vec_rate.py > $O/vec_rate.jsonl 2> $O/vec.err || { tail $O/vec.err; exit 1; }
echo "vec B ok"
cat $O/html_rate.json $O/vec_rate_noorder.jsonl $O/vec_rate.jsonl
