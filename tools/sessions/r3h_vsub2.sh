#!/bin/bash
# vector mode with 256 MB sub-batches: default occupancy vs 4 waves/SIMD; then the vector tests
O=gpurun_out/r3h2; mkdir -p $O
for v in build build_gv4; do
  CLD_MI355X_LIB=language-detector_amd/$v/libcld_mi355x.so timeout -k 10 200 python -u tools/vec_rate.py > $O/vocc_$v.jsonl 2> $O/vocc_$v.err || { tail $O/vocc_$v.err; exit 1; }
  echo "lib $v"; cat $O/vocc_$v.jsonl
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_vector.py -x -v --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
