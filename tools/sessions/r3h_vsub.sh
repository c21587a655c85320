#!/bin/bash
# vector mode: sub-batch size A/B (32 MB default vs 128 MB vs 512 MB of text per launch)
O=gpurun_out/r3h; mkdir -p $O
for mb in 32 128 512; do
  CLD_VEC_SUB_MB=$mb timeout -k 10 200 python -u tools/vec_rate.py > $O/vsub_$mb.jsonl 2> $O/vsub_$mb.err || { tail $O/vsub_$mb.err; exit 1; }
  echo "sub $mb MB"; cat $O/vsub_$mb.jsonl
done
