"""Spans of one document on cuda:0 (k_long's debug dump, CLD_DEBUG_DOC=0:
its S records) beside the oracle's trace.  Usage: span_diff.py DOC.bin"""
import os
import sys

import numpy as np

os.environ["CLD_DEBUG_DOC"] = "0"
os.environ.setdefault("CLD_DEBUG_OUT", "/tmp/cld_dbg.bin")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("language-detector_amd", "oracle"):
    sys.path.insert(0, os.path.join(ROOT, p))
import cld_amd  # noqa: E402
from oracle import Oracle  # noqa: E402

doc = open(sys.argv[1], "rb").read()
cld_amd.init_device(0, tables=cld_amd.SYNTH_TABLES)
got = cld_amd.detect_batch(docs=[doc])
st = cld_amd.last_stats(0)
print("gpu", got[0], "long", st.long_docs, "seq", st.general_docs, "passes", list(st.passes), flush=True)
w = np.fromfile(os.environ["CLD_DEBUG_OUT"], dtype=np.uint32)
n, w, i = int(w[0]), w[1:], 0
spans, texts = [], []
while i < n:
    t = int(w[i])
    if t == ord('S'):
        spans.append(tuple(int(x) for x in w[i + 1:i + 4])); i += 4
    elif t == ord('T'):
        tb = int(np.int32(np.uint32(w[i + 1]))); nw = (max(tb, 0) + 3) // 4
        texts.append(w[i + 2:i + 2 + nw].astype("<u4").tobytes()[:max(tb, 0)]); i += 2 + nw
    elif t == ord('R'):
        nb, nd, nx = (int(x) for x in w[i + 3:i + 6]); i += 6 + 2 * (nb + nd + nx)
    elif t == ord('C'):
        i += 18
    else:
        raise ValueError("bad record %d at %d" % (t, i))
_, r, lines = Oracle().detect(doc, trace=True)
ospans = [ln for ln in lines if ln.startswith("span")]
print("oracle text_bytes", r.text_bytes, "spans", len(ospans), "gpu S records", len(spans), flush=True)
for k in range(max(len(spans), len(ospans))):
    a = spans[k] if k < len(spans) else None
    b = ospans[k] if k < len(ospans) else None
    print(k, a, b)
out = os.environ.get("SPAN_TEXT_OUT")
if out:                                           # the GPU's scored span texts, for replay on the CPU
    with open(out, "wb") as f:
        for x in texts:
            f.write(len(x).to_bytes(4, "little") + x)
