#!/bin/bash
# Round-6 GPU sessions on the committed tree.  STEPS picks what runs, in order:
#   suite  the whole GPU suite          tests  PYTESTS=<files/ids> only
#   diag   one mixed batch (tools/diag_batch.py) against the oracle
#   smoke  __graft_entry__.smoke()      bench  the default bench line
#   lines  C3/C4/C5 bench lines         prof   rocprofv3 kernel statistics, C2 and C3
#   pmc    PMC passes (k_wave @ C2, k_long @ C3)
#   dl     detect_language per-call rates (tools/dl_rate.py)
#   dlc5   the same on C5 documents only, DLVARS runtime variants (A/B)
#   req    request-sized batch rates (tools/req_rate.py)
#   rates  HTML and vector-mode rates
#   gpus2  bench.py --gpus 2 on this 1-GPU box: must refuse (exit 3), print no line
#   tabsize  C2 / C3 lines and L2 hit counters with Q1 and its larger-table variants
#            (tools/synth_quad.py SYNQ_BUCKETS; language-detector_amd/data/variants/)
# Every GPU step has its own limit; the first failure ends the script.
set -u
TAG=${TAG:-r6a}
R=$PWD
O=$R/gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
step() { local t=$1 log=$2; shift 2; echo "[$(date +%T)] $log" | tee -a $O/session.log
  timeout -k 10 $t "$@" > $O/$log 2>&1; local rc=$?
  if [ $rc -eq 0 ] && grep -q "HSA_STATUS_ERROR" $O/$log; then rc=99; fi   # a GPU fault even on exit 0
  echo "[$(date +%T)] rc=$rc" | tee -a $O/session.log
  if [ $rc -ne 0 ]; then tail -30 $O/$log; exit $rc; fi; }
for s in ${STEPS:-suite smoke bench}; do
  case $s in
    suite) step 1000 pytest_gpu.txt python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread; tail -1 $O/pytest_gpu.txt ;;
    diag) step 150 diag.txt python -u tools/diag_batch.py ;;
    tests) step 600 pytest_sel.txt python -u -m pytest ${PYTESTS} -m gpu -x -v --timeout 200 --timeout-method thread; tail -1 $O/pytest_sel.txt ;;
    smoke) step 300 smoke.txt python -u -c "import __graft_entry__ as g; g.smoke()"; tail -2 $O/smoke.txt ;;
    bench) step 400 bench.json python bench.py ;;
    lines) for c in c3 c4 c5; do step 400 bench_$c.json python bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-host --no-sub; done ;;
    prof)
      (cd /tmp && step 300 prof_c2.log rocprofv3 --kernel-trace --stats -d $O/prof_c2 -o c2 --output-format csv -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-host --no-sub) || exit 1
      (cd /tmp && step 300 prof_c3.log rocprofv3 --kernel-trace --stats -d $O/prof_c3 -o c3 --output-format csv -- python3 $R/bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline --no-host --no-sub) || exit 1 ;;
    pmc)
      step 400 pmc_c2.log bash tools/pmc_session.sh ${TAG}_pmc_c2 c2 k_wave
      step 400 pmc_c3.log bash tools/pmc_session.sh ${TAG}_pmc_c3 c3 "k_l(span|score|group|finish|rep|ong)" ;;
    dl) step 400 dl_rate.jsonl python3 tools/dl_rate.py ;;
    dlc5) step 600 dl_c5_ab.jsonl env DL_RATE_CFG=c5 DL_RATE_CALLERS=${DLCALLERS:-1,8,64} DL_RATE_VARIANTS="${DLVARS:--}" python3 tools/dl_rate.py ;;
    ab)  # staged vs fused long-document path (A/B), C3 and C5 lines
      for c in ${ABCFG:-c3 c5}; do
        step 400 ab_${c}_staged.json python bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-host --no-sub
        step 400 ab_${c}_fused.json env CLD_LONG_STAGED=0 python bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-host --no-sub
      done ;;
    dlab) step 600 dl_ab.jsonl env DL_RATE_VARIANTS="${DLVARS:--;CLD_TINY_ZC=1;CLD_TINY=0}" DL_RATE_CFG=c2 python3 tools/dl_rate.py ;;
    req) step 400 req_rate.jsonl env REQ_RATE_CALLERS=${REQCALLERS:-1,8,32,128} python3 tools/req_rate.py ;;
    reqab) step 400 req_staged.jsonl env CLD_LONG_SMALL=0 REQ_RATE_CALLERS=${REQCALLERS:-1,8,32} python3 tools/req_rate.py
           step 400 req_fused.jsonl env REQ_RATE_CALLERS=${REQCALLERS:-1,8,32} python3 tools/req_rate.py ;;
    rates)
      step 300 html_rate.json python3 tools/html_rate.py
      step 400 vec_rate.jsonl python3 tools/vec_rate.py ;;
    gpus2) timeout -k 10 120 python bench.py --gpus 2 --docs 1000 --steps 1 > $O/gpus2.txt 2>&1; rc=$?
           echo "rc=$rc" >> $O/gpus2.txt; cat $O/gpus2.txt; [ $rc -eq 3 ] || exit 1 ;;
    tabsize)
      for t in ${TABS:-language-detector_amd/data/cld2_synth_q1.cldt language-detector_amd/data/variants/cld2_synth_q1_b65536.cldt language-detector_amd/data/variants/cld2_synth_q1_b262144.cldt language-detector_amd/data/variants/cld2_synth_q1_b1048576.cldt}; do
        b=$(basename $t .cldt)
        for c in ${TABCFG:-c2 c3}; do
          if [ $c = c3 ]; then a="--steps 3 --warmup 1 --no-cpu-baseline"; k="k_l(span|score|group|finish|rep|ong)"; else a="--cpu-seconds 3"; k=k_wave; fi
          step 300 tab_${b}_$c.json env CLD_MI355X_TABLES=$R/$t python bench.py --config $c $a --no-host --no-sub
          (cd /tmp && step 120 tab_${b}_pmc_$c.log env CLD_MI355X_TABLES=$R/$t rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-include-regex "$k" -d $O/tab_${b}_pmc_$c -o $c --output-format csv -- python3 $R/bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline --no-host --no-sub) || exit 1
        done
      done ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "session done" | tee -a $O/session.log
