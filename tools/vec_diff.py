"""Debug aid: documents where cld_detect_batch_vec differs from the reference in
vector mode -- both results and vectors, plus the text, as JSON lines."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("language-detector_amd", "oracle"):
    sys.path.insert(0, os.path.join(ROOT, p))
os.environ.setdefault("CLD_MI355X_TABLES", os.path.join(ROOT, "language-detector_amd", "data", "cld2_synth_q1.cldt"))
import cld_amd  # noqa: E402
import corpus  # noqa: E402
import refcld  # noqa: E402

FIELDS = ("lang3", "summary_lang", "percent3", "is_reliable", "text_bytes", "normalized3")
ref = refcld.instance(os.environ["CLD_MI355X_TABLES"])
cld_amd.init_device(0)
cfg = sys.argv[1] if len(sys.argv) > 1 else "c5"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 20000
html = cfg == "html"
buf, offs = corpus.html(n, seed=78) if html else corpus.GENERATORS[cfg](n)
res, chunks, coffs = cld_amd.detect_batch_vec(buf=buf, offsets=offs, html=html)
shown = 0
kinds = {}
for i in range(n):
    doc = bytes(buf[offs[i]:offs[i + 1]])
    rb, cb = ref.detect_vec(doc, plain=not html)
    g = [(int(c["offset"]), int(c["bytes"]), int(c["lang1"])) for c in chunks[coffs[i]:coffs[i + 1]]]
    w = [(int(c["offset"]), int(c["bytes"]), int(c["lang1"])) for c in cb]
    fd = [f for f in FIELDS if not np.array_equal(np.asarray(res[i][f], np.float64), np.asarray(rb[f], np.float64))]
    if g == w and not fd:
        continue
    k = ("vec" if g != w else "") + ("+" + ",".join(fd) if fd else "")
    kinds[k] = kinds.get(k, 0) + 1
    if shown < 12:
        shown += 1
        print(json.dumps({"doc": i, "len": len(doc), "fields": fd,
                          "gpu": {f: np.asarray(res[i][f]).tolist() for f in FIELDS},
                          "ref": {f: np.asarray(rb[f]).tolist() for f in FIELDS},
                          "gpu_vec": g[:40], "ref_vec": w[:40], "text": doc[:3000].decode("utf-8", "replace")},
                         ensure_ascii=False), flush=True)
print(json.dumps({"differing_kinds": kinds}))
