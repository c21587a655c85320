"""ResultChunkVector throughput (cld_detect_batch_vec) on 100K C5 documents and
50K HTML pages, host buffers, end to end, with the reference CLD2 in vector
mode (oracle/_ref/librefcld2.so, ExtDetectLanguageSummary with a
ResultChunkVector) on 16 host threads timed beside it and compared result for
result, chunk for chunk.  Plain documents run the parallel kernels
(k_long<VEC>); HTML pages and hand-ons its sequential span source (cld_seq.hip).
One JSON line per workload."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("language-detector_amd", "oracle"):
    sys.path.insert(0, os.path.join(ROOT, p))
os.environ.setdefault("CLD_MI355X_TABLES", os.path.join(ROOT, "language-detector_amd", "data", "cld2_synth_q1.cldt"))
import cld_amd  # noqa: E402
import corpus  # noqa: E402
import refcld  # noqa: E402

FIELDS = ("lang3", "summary_lang", "percent3", "is_reliable", "text_bytes", "normalized3")
refcld.verify_build()
ref = refcld.instance(os.environ["CLD_MI355X_TABLES"])
cld_amd.init_device(0)
n_c5 = int(os.environ.get("VEC_RATE_DOCS", "100000"))
for name, (buf, offs), html in (("c5 plain text", corpus.c5(n_c5, seed=5), False),
                                ("html", corpus.html(n_c5 // 2, seed=78), True)):
    n = len(offs) - 1
    cld_amd.detect_batch_vec(buf=buf, offsets=offs, html=html)       # warm (allocates the arena)
    t0 = time.time()
    res, chunks, coffs = cld_amd.detect_batch_vec(buf=buf, offsets=offs, html=html)
    wall = time.time() - t0
    st = cld_amd.last_stats(0)
    t0 = time.time()
    rres, rch, rco = ref.detect_batch_vec(buf, offs, plain=np.zeros(n, np.uint8) if html else None, threads=16)
    rwall = time.time() - t0
    bad = np.zeros(n, bool)
    for f in FIELDS:
        bad |= (res[f].astype(np.float64) != rres[f].astype(np.float64)).reshape(n, -1).any(axis=1)
    cnt_bad = np.diff(coffs.astype(np.int64)) != np.diff(rco.astype(np.int64))
    bad |= cnt_bad
    if not cnt_bad.any():
        neq = np.zeros(len(chunks), bool)
        for f in ("offset", "bytes", "lang1"):
            neq |= chunks[f] != rch[f]
        bad[np.searchsorted(coffs, np.nonzero(neq)[0], side="right") - 1] = True
    same_chunks = not bad.any()
    print(json.dumps({"workload": "%d %s documents with ResultChunkVector" % (n, name), "bytes": int(offs[-1]),
                      "chunks": int(coffs[-1]), "docs_per_s_end_to_end": n / wall, "seconds": wall,
                      "parallel_kernel_docs": int(st.long_docs), "sequential_kernel_docs": int(st.general_docs),
                      "reference_cpu": {"docs_per_s": n / rwall, "threads": 16, "kind": "reference"},
                      "documents_differing": int(bad.sum()), "first_differing": [int(i) for i in np.nonzero(bad)[0][:8]],
                      "all_equal_to_reference": same_chunks}), flush=True)
