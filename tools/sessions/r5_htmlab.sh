# HTML rates (no CPU baseline) under several library builds: VARIANTS="base h1 ..."
set -u
O=gpurun_out/${TAG:-r5h}; mkdir -p $O
for v in ${VARIANTS:-base}; do
  if [ "$v" = base ]; then lib=""; else lib="$PWD/language-detector_amd/build_v_$v/libcld_mi355x.so"; fi
  echo "[$(date +%T)] $v" | tee -a $O/session.log
  CLD_MI355X_LIB=$lib CLD_NO_CPU=1 HTML_RATE_SETS=${SETS:-mixed,16k,64k} timeout -k 10 400 python3 tools/html_rate.py > $O/html_$v.jsonl 2> $O/html_$v.err || { tail -5 $O/html_$v.err; exit 1; }
done
