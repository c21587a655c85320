# HTML rewrite timing experiments (HTML_EXP variants; results of the variants are wrong by design)
set -u
O=gpurun_out/r3d_hx; mkdir -p $O
for v in build build_v_hx1 build_v_hx2 build_v_hx4 build_v_hx8; do
  CLD_MI355X_LIB=$PWD/language-detector_amd/$v/libcld_mi355x.so timeout -k 10 300 python tools/html_rate.py > $O/$v.json 2>&1 || { tail $O/$v.json; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$v.json').read().strip().splitlines()[-1]); print('$v', round(d['rewrite_route_wave_ms'],1), round(d['long_ms'],1), d['general_docs'])"
done
