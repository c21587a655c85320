"""Summarise a tabsize session (tools/sessions/r6.sh STEPS=tabsize) into one
JSON line per (table, config): docs/s, the dominant kernel's time, the CPU
baseline's bit-exactness on its sample, and the L2 hit rate of the dominant
kernel(s) from the TCC_HIT/TCC_MISS pass.

    python tools/tabsize_summary.py gpurun_out/<tag> > profiles/<name>.jsonl
"""
import csv
import glob
import json
import os
import re
import sys


def line(path):
    for l in open(path):
        if l.startswith("{"):
            return json.loads(l)
    return None


def l2_hit(d):
    h = m = 0.0
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            v = float(r["Counter_Value"])
            if r["Counter_Name"] == "TCC_HIT_sum":
                h += v
            elif r["Counter_Name"] == "TCC_MISS_sum":
                m += v
    return h / (h + m) if h + m else None


def main(o):
    for f in sorted(glob.glob(os.path.join(o, "tab_*.json"))):
        m = re.match(r"tab_(.+)_(c\w+)\.json$", os.path.basename(f))
        table, cfg = m.group(1), m.group(2)
        d = line(f)
        if d is None:
            continue
        k = d["kernels"]
        cpu = d.get("cpu_baseline") or {}
        print(json.dumps({"table": table, "config": cfg, "docs_per_s": d["value"],
                          "wave_ms": k["wave_ms"], "long_ms": k["long_ms"],
                          "l2_hit": l2_hit(os.path.join(o, "tab_%s_pmc_%s" % (table, cfg))),
                          "gpu_bit_exact_on_cpu_sample": cpu.get("gpu_bit_exact_on_sample"),
                          "tables": d.get("tables", "")[:200], "source": o}))


if __name__ == "__main__":
    main(sys.argv[1])
