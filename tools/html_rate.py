"""HTML-mode throughput (is_plain_text = false) on 100K synthetic HTML pages,
inputs resident on the host (cld_detect_batch_ex): docs/s from the device
timers (every kernel of the batch: the HTML rewrite, k_wave, k_long,
k_general) and end to end, beside the reference CLD2 (oracle/_ref/librefcld2.so,
ExtDetectLanguageSummary with is_plain_text = false) on the box's cores over a
bounded sample of the same pages, checked equal to the GPU on that sample."""
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
buf, offs = corpus.html(100_000, seed=77)
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
line = {"workload": "100K synthetic HTML pages, 200-6000 B (corpus.html seed 77)", "docs": n, "bytes": int(offs[-1]),
        "kernel_ms": kms, "rewrite_route_wave_ms": wms, "long_ms": lms, "general_ms": gms,
        "long_docs": ldocs, "general_docs": gdocs, "docs_per_s_kernel": n / (kms / 1e3), "docs_per_s_end_to_end": n / wall}
try:
    import refcld
    refcld.verify_build()
    rc = refcld.instance(cld_amd.SYNTH_TABLES)
    if os.environ.get("CLD_NO_CPU"): raise RuntimeError("skipped")
    threads = int(os.environ.get("CLD_CPU_THREADS", "16"))
    m = 20000
    sb, so = buf[:int(offs[m])], offs[:m + 1]
    want = rc.detect_batch(sb, so, plain=np.zeros(m, np.uint8), threads=threads)
    t0, reps = time.time(), 0
    while time.time() - t0 < 10.0:
        rc.detect_batch(sb, so, plain=np.zeros(m, np.uint8), threads=threads)
        reps += 1
    cpu = m * reps / (time.time() - t0)
    same = all(np.array_equal(got[f][:m].astype(np.float64), want[f].astype(np.float64))
               for f in ("lang3", "summary_lang", "percent3", "is_reliable", "text_bytes", "normalized3"))
    line["cpu_baseline"] = {"value": cpu, "unit": "docs/s", "cores": threads, "kind": "reference",
                            "sample": "%d pages x %d passes, reference CLD2 (is_plain_text=false)" % (m, reps),
                            "gpu_bit_exact_on_sample": bool(same)}
except Exception as e:  # (the reference checker build is optional here)
    line["cpu_baseline"] = {"error": repr(e)}
print(json.dumps(line))
