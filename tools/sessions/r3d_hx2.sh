set -u
for v in build build_v_hx1 build_v_hx2; do
  echo "== $v"; CLD_MI355X_LIB=$PWD/language-detector_amd/$v/libcld_mi355x.so timeout -k 10 300 python tools/html_probe.py 2>&1 | head -2
done
