# compiler-flag variants (lab builds): C2 k_wave time and SALU, C3 k_long time; parity of the faster
set -u
export TMPDIR=/tmp
O=$PWD/gpurun_out/r4_flags; mkdir -p $O
R=$PWD
for v in build build_v_ifcvt build_v_unroll; do
  L=$R/language-detector_amd/$v/libcld_mi355x.so
  CLD_MI355X_LIB=$L timeout -k 10 200 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-sub --no-host > $O/$v.c2.json 2>$O/$v.err || { tail $O/$v.err; exit 1; }
  CLD_MI355X_LIB=$L timeout -k 10 300 python3 bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline --no-sub --no-host > $O/$v.c3.json 2>>$O/$v.err || { tail $O/$v.err; exit 1; }
  (cd /tmp && CLD_MI355X_LIB=$L timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VALU --kernel-include-regex k_wave -d $O/$v -o c2 --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-sub --no-host > $O/$v.pmc.log 2>&1) || { tail $O/$v.pmc.log; exit 1; }
  python3 -c "
import csv, collections, json
a=json.loads(open('$O/$v.c2.json').read().strip().splitlines()[-1]); b=json.loads(open('$O/$v.c3.json').read().strip().splitlines()[-1])
rows=list(csv.DictReader(open('$O/$v/c2_counter_collection.csv')))
acc=collections.defaultdict(float); disp=set()
for r in rows: acc[r['Counter_Name']]+=float(r['Counter_Value']); disp.add(r['Dispatch_Id'])
n=len(disp)*1e6
print('$v c2 %.2f M (k_wave %.3f ms, SALU %.0f VALU %.0f) c3 %.3f M (k_long %.2f ms)' % (a['value']/1e6, a['kernels']['wave_ms'], acc['SQ_INSTS_SALU']/n, acc['SQ_INSTS_VALU']/n, b['value']/1e6, b['kernels']['long_ms']))"
done
