# k_long stage cycles (CLD_PROFILE_STAGES=1): C3, and C5 with and without the one-language pages.
set -u
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r3c_lprof}; mkdir -p $O
CLD_PROFILE_STAGES=1 timeout -k 10 300 python tools/wave_prof.py c3:20000 c5:200000 > $O/stages.txt 2>&1 || { tail $O/stages.txt; exit 1; }
CLD_C3_MONO_FRAC=0 CLD_PROFILE_STAGES=1 timeout -k 10 300 python tools/wave_prof.py c5:200000 > $O/stages_mono0.txt 2>&1 || { tail $O/stages_mono0.txt; exit 1; }
cat $O/stages.txt $O/stages_mono0.txt
