# k_wave stage pricing on C2 (lab builds that stop after stage k; never shipped)
set -u
export TMPDIR=/tmp
O=$PWD/gpurun_out/r4_stops; mkdir -p $O
R=$PWD
for v in build_v_stop1 build_v_stop2 build_v_stop3 build_v_stop4 build_v_stop5 build_v_stop6 build; do
  L=$R/language-detector_amd/$v/libcld_mi355x.so
  CLD_MI355X_LIB=$L timeout -k 10 200 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-sub --no-host > $O/$v.json 2>$O/$v.err || { tail $O/$v.err; exit 1; }
  (cd /tmp && CLD_MI355X_LIB=$L timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-include-regex k_wave -d $O/$v -o c2 --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-sub --no-host > $O/$v.pmc.log 2>&1) || { tail $O/$v.pmc.log; exit 1; }
  python3 -c "
import csv, collections, json
a=json.loads(open('$O/$v.json').read().strip().splitlines()[-1])
rows=list(csv.DictReader(open('$O/$v/c2_counter_collection.csv')))
acc=collections.defaultdict(float); disp=set()
for r in rows: acc[r['Counter_Name']]+=float(r['Counter_Value']); disp.add(r['Dispatch_Id'])
n=len(disp)*1e6
print('$v', 'wave_ms %.3f'%a['kernels']['wave_ms'], ' '.join('%s %.0f'%(k.replace('SQ_',''),v/n) for k,v in sorted(acc.items())))"
done
