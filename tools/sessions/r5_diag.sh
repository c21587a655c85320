# detect_language under 64 / 256 callers with each HIP wait mode, and the
# box's CPU quota use (cgroup cpu.stat) per run
set -u
O=gpurun_out/r5d; mkdir -p $O
{ nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null; } > $O/cpu.txt
python3 - <<'PY' > /dev/null
import sys,os
sys.path.insert(0,'language-detector_amd')
import corpus, numpy as np
b,o=corpus.c2(20000,seed=17); b.tofile('/tmp/c2.bin'); o.astype(np.uint64).tofile('/tmp/c2.off')
PY
st() { awk '/^usage_usec|^nr_throttled|^throttled_usec/{printf "%s ", $2}' /sys/fs/cgroup/cpu.stat; }
for v in ${VARS:-"-" "CLD_SYNC=block" "CLD_SYNC=yield" "CLD_COALESCE_SPIN_US=0"}; do
  for c in 64 256; do
    a=$(st); t0=$(date +%s.%N)
    env ${v/#-/X=1} CLD_MI355X_TABLES=language-detector_amd/data/cld2_synth_q1.cldt timeout -k 10 120 tools/build/dl_bench gpu /tmp/c2.bin /tmp/c2.off $c $((20000/c+100)) > $O/one.json 2>> $O/err.txt || exit 1
    b=$(st); t1=$(date +%s.%N)
    python3 -c "
import json,sys
d=json.load(open('$O/one.json')); a='$a'.split(); b='$b'.split()
d['variant']='$v'; d['cpu_cores_used']=(int(b[0])-int(a[0]))/1e6/($t1-$t0); d['throttled_periods']=int(b[1])-int(a[1]); d['throttled_ms']=(int(b[2])-int(a[2]))/1e3
print(json.dumps(d))" >> $O/diag.jsonl
  done
done
