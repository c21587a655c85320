"""Per-kernel average ms per step from rocprofv3 kernel statistics of
tools/sessions/r5_libab.sh runs: ab_summary.py TAG variant... [config]."""
import csv
import glob
import sys

tag, cfg = sys.argv[1], "c3"
vs = sys.argv[2:]
if vs and vs[-1].startswith("c") and vs[-1][1:].isdigit():
    cfg, vs = vs[-1], vs[:-1]
for v in vs:
    f = glob.glob("gpurun_out/%s_%s/prof_%s/*kernel_stats.csv" % (tag, v, cfg))
    if not f:
        print(v, "missing")
        continue
    rows = list(csv.DictReader(open(f[0])))
    steps = max(int(r["Calls"]) for r in rows if "k_route" in r["Name"])
    tot = sum(float(r["TotalDurationNs"]) for r in rows if "rocclr" not in r["Name"]) / steps / 1e6
    d = {r["Name"].split("(")[0].replace("void ", "").replace("cld::", ""): float(r["AverageNs"]) / 1e6 for r in rows}
    print("%-6s %s total/step %.2f ms  %s" % (v, cfg, tot, {k: round(x, 2) for k, x in d.items() if x > 0.3}))
