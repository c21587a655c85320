"""Single-document latency of the long-document path: the longest C5
documents and 16/64 KB C3 pages, each run alone (a batch of one) on GPU 0;
kernel ms from the library's HIP events, spans from the oracle's scanner
(test infrastructure).  A launch lasts as long as its longest document, so
this is the floor of every batch that holds such a document.  JSON lines."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("language-detector_amd", "oracle", "tests"):
    sys.path.insert(0, os.path.join(ROOT, p))
os.environ.setdefault("CLD_MI355X_TABLES", os.path.join(ROOT, "language-detector_amd", "data", "cld2_synth_q1.cldt"))
import cld_amd  # noqa: E402
import corpus  # noqa: E402
from oracle import Oracle  # noqa: E402
from test_html_hints import oracle_spans  # noqa: E402

# LAT_PROFILE=1: the fused kernel's per-stage cycles per document too
# (CLD_PROFILE_STAGES: k_long's diagnostic instantiation)
PROF = os.environ.get("LAT_PROFILE") == "1"
if PROF:
    os.environ["CLD_PROFILE_STAGES"] = "1"
LSTAGES = ["classify", "span+lower", "squeeze", "repeats", "words+chain", "quad", "octa/uni/bi", "score"]
cld_amd.init()
o = Oracle()
docs = []
b5, o5 = corpus.c5(int(os.environ.get("LAT_C5_DOCS", "1000000")))
lens = np.diff(o5)
for i in np.argsort(-lens)[:12]:
    docs.append(("c5 #%d" % i, bytes(b5[o5[i]:o5[i + 1]])))
for page in (16384, 65536):
    b3, o3 = corpus.c3(3, page=page, seed=5)
    for i in range(3):
        docs.append(("c3 page %d #%d" % (page, i), bytes(b3[o3[i]:o3[i + 1]])))
for name, d in docs:
    buf, offs = cld_amd.pack([d])
    for _ in range(2):
        cld_amd.detect_batch(buf=buf, offsets=offs)
    cld_amd.kernel_times(0)
    if PROF:
        cld_amd.stage_cycles(0)
    reps = 3
    for _ in range(reps):
        r = cld_amd.detect_batch(buf=buf, offsets=offs)
    ms, launches = cld_amd.kernel_times(0)
    st = cld_amd.last_stats(0)
    spans = oracle_spans(o, d, True)
    extra = {}
    if PROF:
        c = cld_amd.stage_cycles(0).astype(np.float64)[8:16] / reps
        extra = {"stage_kcycles": {LSTAGES[k]: round(c[k] / 1e3, 1) for k in range(8)}}
    print(json.dumps({"doc": name, "bytes": len(d), "spans": len(spans), **extra,
                      "span_bytes_max": max((len(t) for _, t in spans), default=0),
                      "passes": [int(x) for x in st.passes[:3]], "long_ms": round(ms[1] / max(1, launches), 3),
                      "general_ms": round(ms[2] / max(1, launches), 3)}), flush=True)
