"""Summarise a tools/pmc_session.sh run: per-launch averages of every counter
for the profiled kernel (first, cold launch excluded when there are more)."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def summarise(d):
    """Per-launch counters: per kernel name the average over its dispatches
    (the first, cold one excluded when there are more), summed over the
    kernels the regex matched -- a pipeline of kernels (the staged long path)
    is reported per launch of the whole pipeline."""
    per = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))   # counter -> kernel -> dispatch -> value
    kinfo = {}
    for f in sorted(glob.glob(os.path.join(d, "pmc*", "**", "*counter_collection.csv"), recursive=True)):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0]
            per[r["Counter_Name"]][k][int(r["Dispatch_Id"])] += float(r["Counter_Value"])
            kinfo[k] = {"grid": int(r["Grid_Size"]), "vgpr": int(r["VGPR_Count"]), "sgpr": int(r["SGPR_Count"]),
                        "scratch": int(r["Scratch_Size"]), "lds": int(r["LDS_Block_Size"])}
    vals = defaultdict(float)
    for c, byk in per.items():
        for k, byd in byk.items():
            v = [byd[x] for x in sorted(byd)]
            if len(v) > 1:
                v = v[1:]
            vals[c] += sum(v) / len(v)
    info = {"kernel": " + ".join(sorted(kinfo)), "kernels": kinfo}
    if len(kinfo) == 1:
        info.update(next(iter(kinfo.values())))
    out = dict(info)
    out["counters_per_launch"] = dict(vals)
    v = vals
    if "SQ_WAVE_CYCLES" in v:
        w = v["SQ_WAVE_CYCLES"]
        out["frac_active_inst"] = v.get("SQ_ACTIVE_INST_ANY", 0) / w
        out["frac_wait_any"] = v.get("SQ_WAIT_ANY", 0) / w
        out["frac_wait_inst_any"] = v.get("SQ_WAIT_INST_ANY", 0) / w
    if "TCC_HIT_sum" in v:
        out["l2_hit_rate"] = v["TCC_HIT_sum"] / max(1.0, v["TCC_HIT_sum"] + v["TCC_MISS_sum"])
    if "FETCH_SIZE" in v:
        out["hbm_fetch_bytes"] = 2 * 1024 * v["FETCH_SIZE"]   # gfx950: FETCH_SIZE reports half (MI355X_MICROARCH.md)
    if "WRITE_SIZE" in v:
        out["hbm_write_bytes"] = 1024 * v["WRITE_SIZE"]
    return out


if __name__ == "__main__":
    # pmc_summary.py DIR [CONFIG DOCS]: with CONFIG, also record the summary as
    # profiles/pmc_current.json[CONFIG] (what bench.py reads for traffic / issue)
    s = summarise(sys.argv[1])
    print(json.dumps(s, indent=1))
    if len(sys.argv) > 3:
        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        path = os.path.join(root, "profiles", "pmc_current.json")
        cur = json.load(open(path)) if os.path.exists(path) else {}
        s["docs"] = int(sys.argv[3])
        s["source"] = os.path.relpath(sys.argv[1], root)
        if "hbm_fetch_bytes" in s and "hbm_write_bytes" in s:
            s["hbm_bytes_per_launch"] = s["hbm_fetch_bytes"] + s["hbm_write_bytes"]
        cur[sys.argv[2]] = s
        with open(path, "w") as f:
            json.dump(cur, f, indent=1, sort_keys=True)
