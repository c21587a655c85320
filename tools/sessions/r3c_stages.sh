# k_wave stage pricing: one PMC pass per WAVE_STOP variant (the wave ends at
# stop point k) plus the full build, C2; first the SALU-counter probe.
set -u
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r3c_stages}; mkdir -p $O
timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_SMEM SQ_WAVES \
  -d $O/probe -o probe --output-format csv -- ./tools/probe/salu_probe > $O/probe.log 2>&1 || tail -3 $O/probe.log
python3 - <<PY
import csv, glob, collections
d = collections.defaultdict(dict)
for f in glob.glob("$O/probe/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        d[r["Kernel_Name"].split("(")[0]][r["Counter_Name"]] = float(r["Counter_Value"])
for k, v in d.items(): print("probe", k, v)
PY
for v in ${VARIANTS:-0 1 2 31 32 33 3 4 51 52 53 54 5 61 62 63 full}; do
  lib=build_v_stop$v; [ $v = full ] && lib=build
  CLD_MI355X_LIB=$PWD/language-detector_amd/$lib/libcld_mi355x.so timeout -s KILL 150 rocprofv3 \
    --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD \
    --kernel-include-regex k_wave -d $O/$v/pmc1 -o c2 --output-format csv -- \
    python3 bench.py --config c2 --steps 2 --warmup 1 --no-cpu-baseline --no-sub --no-host > $O/$v.log 2>&1 || { tail -20 $O/$v.log; exit 1; }
  python3 tools/pmc_summary.py $O/$v | python3 -c "import json,sys; d=json.load(sys.stdin); c=d['counters_per_launch']; print('stop $v', ' '.join('%s=%.0f' % (k[8:] if k.startswith('SQ_INSTS') else k, v/1e6) for k,v in sorted(c.items())))"
done
