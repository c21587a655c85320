# rocprofv3 kernel statistics of a config under several library builds:
# VARIANTS="base st8 ..." (base = build/, else language-detector_amd/build_v_<name>/), PROFCFG configs
set -u
for v in ${VARIANTS:-base}; do
  if [ "$v" = base ]; then env_=X=1; else env_="CLD_MI355X_LIB=$PWD/language-detector_amd/build_v_$v/libcld_mi355x.so"; fi
  TAG=${TAG:-r5ab}_$v PROFCFG="${PROFCFG:-c3}" PROFENV="$env_" bash tools/sessions/r5_prof.sh > /dev/null || exit 1
done
