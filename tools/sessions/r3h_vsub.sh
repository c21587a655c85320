#!/bin/bash
# vector mode A/B: sequential-kernel occupancy (compiler's 2 waves/SIMD vs 4 vs 7)
# and sub-batch size (32 MB default vs 128 MB of text per launch)
O=gpurun_out/r3h; mkdir -p $O
for v in build build_gv4 build_gv8; do
  CLD_MI355X_LIB=language-detector_amd/$v/libcld_mi355x.so timeout -k 10 200 python -u tools/vec_rate.py > $O/vocc_$v.jsonl 2> $O/vocc_$v.err || { tail $O/vocc_$v.err; exit 1; }
  echo "lib $v"; cat $O/vocc_$v.jsonl
done
CLD_VEC_SUB_MB=128 timeout -k 10 200 python -u tools/vec_rate.py > $O/vsub_128.jsonl 2> $O/vsub_128.err || { tail $O/vsub_128.err; exit 1; }
echo "sub 128 MB"; cat $O/vsub_128.jsonl
