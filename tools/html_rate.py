"""HTML-mode throughput (is_plain_text = false) on synthetic HTML pages (sets:
mixed 200-6000 B, 16k and 64k pages, and the same with 4-byte characters on
every page: emoji, emoji16k, emoji64k; HTML_RATE_SETS),
inputs resident on the host (cld_detect_batch_ex): docs/s from the device
timers (every kernel of the batch: the HTML rewrite, k_wave, k_long) and end to end, beside the reference CLD2 (oracle/_ref/librefcld2.so,
ExtDetectLanguageSummary with is_plain_text = false) on the box's cores over a
bounded sample of the same pages; every page is checked against it."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "language-detector_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
os.environ.setdefault("CLD_MI355X_TABLES", os.path.join(ROOT, "language-detector_amd", "data", "cld2_synth_q1.cldt"))
import cld_amd  # noqa: E402
import corpus  # noqa: E402

cld_amd.init_device(0)
# sets: name -> (pages, lo, hi, distinct); HTML_RATE_SETS picks them (comma
# list).  Long-page sets repeat `distinct` generated pages (the generator is
# Python; the rates do not depend on pages being distinct).
SETS = {"mixed": (100_000, 200, 6000, 100_000), "16k": (100_000, 14_000, 18_000, 2000),
        "64k": (25_000, 56_000, 72_000, 500)}
SETS.update({"emoji": SETS["mixed"], "emoji16k": SETS["16k"], "emoji64k": SETS["64k"]})


def pages(npages, lo, hi, distinct, emoji=0.0):
    b, o = corpus.html(distinct, seed=77, lo=lo, hi=hi, emoji=emoji)
    if distinct == npages:
        return b, o
    idx = np.arange(npages) % distinct
    lens = np.diff(o)[idx]
    offs = np.zeros(npages + 1, np.uint64)
    np.cumsum(lens, out=offs[1:])
    buf = np.concatenate([b[o[i]:o[i + 1]] for i in range(distinct)] * (npages // distinct) +
                         [b[o[i]:o[i + 1]] for i in range(npages % distinct)])
    return buf, offs
FIELDS = ("lang3", "summary_lang", "percent3", "is_reliable", "text_bytes", "normalized3")
try:
    import refcld
    refcld.verify_build()
    rc = refcld.instance(cld_amd.SYNTH_TABLES)
except Exception as e:  # (the reference checker build is optional here)
    rc, rc_err = None, repr(e)
threads = int(os.environ.get("CLD_CPU_THREADS", "16"))
for name in os.environ.get("HTML_RATE_SETS", "mixed").split(","):
    npages, lo, hi, distinct = SETS[name]
    emoji = 1.0 if name.startswith("emoji") else 0.0
    buf, offs = pages(npages, lo, hi, distinct, emoji)
    print("set %s: %d pages, %d bytes" % (name, npages, int(offs[-1])), file=sys.stderr, flush=True)
    cld_amd.detect_batch_ex(buf=buf, offsets=offs, html=True)        # warm
    best = None
    for _ in range(3):
        t0 = time.time()
        got = cld_amd.detect_batch_ex(buf=buf, offsets=offs, html=True)
        wall = time.time() - t0
        st = cld_amd.last_stats(0)
        kms = st.short_ms + st.long_ms + st.general_ms
        if best is None or kms < best[0]:
            best = (kms, wall, st.short_ms, st.long_ms, st.general_ms, int(st.general_docs), int(st.long_docs))
    n = len(offs) - 1
    kms, wall, wms, lms, gms, gdocs, ldocs = best
    line = {"workload": "%dK synthetic HTML pages, %d-%d B (corpus.html seed 77, %d distinct%s)"
                        % (n // 1000, lo, hi, distinct, ", 4-byte characters on every page" if emoji else ""),
            "set": name,
            "docs": n, "bytes": int(offs[-1]), "kernel_ms": kms, "rewrite_route_wave_ms": wms, "long_ms": lms,
            "general_ms": gms, "long_docs": ldocs, "general_docs": gdocs, "docs_per_s_kernel": n / (kms / 1e3),
            "docs_per_s_end_to_end": n / wall}
    if rc is None or os.environ.get("CLD_NO_CPU"):
        line["cpu_baseline"] = {"error": "skipped" if rc is not None else rc_err}
    else:
        # every page against the reference (16 threads), then its rate on a bounded sample
        t0 = time.time()
        want = rc.detect_batch(buf, offs, plain=np.zeros(n, np.uint8), threads=threads)
        full_s = time.time() - t0
        bad = np.zeros(n, bool)
        for f in FIELDS:
            bad |= (np.asarray(got[f], np.float64) != np.asarray(want[f], np.float64)).reshape(n, -1).any(axis=1)
        line["mismatches_vs_reference"] = int(bad.sum())
        m = min(n, 20000)
        sb, so = buf[:int(offs[m])], offs[:m + 1]
        t0, reps = time.time(), 0
        while time.time() - t0 < 10.0:
            rc.detect_batch(sb, so, plain=np.zeros(m, np.uint8), threads=threads)
            reps += 1
        cpu = m * reps / (time.time() - t0)
        line["cpu_baseline"] = {"value": cpu, "unit": "docs/s", "cores": threads, "kind": "reference",
                                "sample": "%d pages x %d passes, reference CLD2 (is_plain_text=false)" % (m, reps),
                                "full_set_seconds": round(full_s, 2)}
    print(json.dumps(line), flush=True)
