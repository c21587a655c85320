"""Rate on messy input (GPU box): the corrupted corpora of
tests/test_gpu_corrupt.docs_for (malformed UTF-8 spliced into C2/C3/C4/C5
documents, plus random bytes) against the same documents uncorrupted, end to
end through cld_detect_batch from host buffers; and the share of documents
that take the sequential span source (last_stats general_docs).  One JSON
line per corpus."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("language-detector_amd", "oracle", "tests"):
    sys.path.insert(0, os.path.join(ROOT, p))
import cld_amd  # noqa: E402
import corpus  # noqa: E402
import test_gpu_corrupt as tc  # noqa: E402

cld_amd.init_device(0, tables=cld_amd.SYNTH_TABLES)
seed, n_each = 101, 12000
clean = []
for cfg, n in (("c2", n_each), ("c3", max(8, n_each // 40)), ("c4", n_each // 2), ("c5", n_each)):
    b, o = corpus.GENERATORS[cfg](n, seed=seed)
    clean += [bytes(b[o[i]:o[i + 1]]) for i in range(n)]
rng = np.random.default_rng(seed)
messy = [tc.corrupt(rng, d) for d in clean]
for name, docs in (("clean", clean), ("corrupted", messy)):
    buf, offs = cld_amd.pack(docs)
    out = None
    for _ in range(2):
        cld_amd.detect_batch(buf=buf, offsets=offs)
    t = time.perf_counter()
    reps = 5
    for _ in range(reps):
        cld_amd.detect_batch(buf=buf, offsets=offs)
    dt = (time.perf_counter() - t) / reps
    st = cld_amd.last_stats(0)
    print(json.dumps({"corpus": name, "docs": len(docs), "bytes": len(buf), "ms": round(dt * 1e3, 2),
                      "docs_per_s": round(len(docs) / dt), "seq_docs": int(st.general_docs),
                      "long_docs": int(st.long_docs), "short_docs": int(st.short_docs)}), flush=True)
