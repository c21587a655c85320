"""Debug dump of one document through k_long (CLD_DEBUG_DOC): per-span
(script, text_bytes, pass) records, next to the oracle's span trace.
Usage: dbg_doc.py CONFIG N SEED INDEX [boiler_frac]"""
import os
import sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "language-detector_amd")); sys.path.insert(0, os.path.join(ROOT, "oracle"))
os.environ.setdefault("CLD_MI355X_TABLES", os.path.join(ROOT, "language-detector_amd", "data", "cld2_synth_q1.cldt"))
os.environ["CLD_DEBUG_DOC"] = "0"
out = os.path.join(ROOT, "gpurun_out", "dbg_doc.bin")
os.environ["CLD_DEBUG_OUT"] = out
import cld_amd, corpus
from oracle import Oracle

cfg, n, seed, idx = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
kw = {"boiler_frac": float(sys.argv[5])} if len(sys.argv) > 5 else {}
b, o = corpus.GENERATORS[cfg](n, seed=seed, **kw)
d = bytes(b[o[idx]:o[idx + 1]])
cld_amd.init_device(0)
g = cld_amd.detect_batch(docs=[d])
w = np.fromfile(out, dtype=np.uint32)
cnt, w = int(w[0]), w[1:]
i = 0
while i < cnt:
    t = chr(w[i])
    if t == "S":
        print("gpu span ul=%d tb=%d pass=%d" % (w[i + 1], w[i + 2], w[i + 3])); i += 4
    elif t == "R":
        nb, nd, nx = w[i + 3], w[i + 4], w[i + 5]; i += 6 + 2 * (nb + nd + nx)
    elif t == "C":
        i += 18
    else:
        print("?", w[i]); break
lang, r, tr = Oracle().detect(d, trace=True)
print("gpu", g[0])
print("ref passes", r.passes, "text_bytes", r.text_bytes)
for l in tr:
    if l.startswith("span ") or "restart" in l or l.startswith("recurse"):
        print("ref", l)
