"""Shrinks a document on which cuda:0 and the oracle disagree: the shortest
failing prefix, then the shortest failing suffix of that, then single-byte
deletions until none still fails (each round one GPU batch of all candidates).
Usage: [BISECT_MODE=vec] corrupt_bisect.py DOC.bin [OUT.bin]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("language-detector_amd", "oracle"):
    sys.path.insert(0, os.path.join(ROOT, p))
import cld_amd  # noqa: E402
from oracle import Oracle  # noqa: E402

FIELDS = ("lang3", "summary_lang", "percent3", "is_reliable", "text_bytes", "normalized3")
cld_amd.init_device(0, tables=cld_amd.SYNTH_TABLES)
o = Oracle()


VEC = os.environ.get("BISECT_MODE", "plain") == "vec"    # cld_detect_batch_vec: result fields and the vector


def failing(docs):
    buf, offs = cld_amd.pack(docs)
    if VEC:
        got, chunks, coffs = cld_amd.detect_batch_vec(buf=buf, offsets=offs)
        bad = np.zeros(len(docs), bool)
        ref = []
        for i, d in enumerate(docs):
            r, ch = o.detect_vec(d)
            ref.append((r.summary_lang, list(r.lang3), list(r.percent3), r.text_bytes, list(r.normalized3),
                        [(int(c["offset"]), int(c["bytes"]), int(c["lang1"])) for c in ch]))
            g = got[i]
            mine = (int(g["summary_lang"]), [int(x) for x in g["lang3"]], [int(x) for x in g["percent3"]],
                    int(g["text_bytes"]), [float(x) for x in g["normalized3"]],
                    [(int(c["offset"]), int(c["bytes"]), int(c["lang1"])) for c in chunks[coffs[i]:coffs[i + 1]]])
            bad[i] = mine != ref[-1]
        return bad, got, ref
    got = cld_amd.detect_batch(buf=buf, offsets=offs)
    ref = o.detect_batch(buf, offs, threads=8)
    bad = np.zeros(len(docs), bool)
    for f in FIELDS:
        bad |= (got[f] != ref[f]).reshape(len(docs), -1).any(axis=1)
    return bad, got, ref


d = open(sys.argv[1], "rb").read()
assert failing([d])[0][0], "the document does not fail"
# long documents: binary search for a failing prefix, then suffix, first (one document per step)
while len(d) > 4096:
    n0 = len(d)
    lo, hi = 0, len(d)                         # d[:hi] fails
    while hi - lo > 64:
        mid = (lo + hi) // 2
        if failing([d[:mid]])[0][0]:
            hi = mid
        else:
            lo = mid
    d = d[:hi]
    lo, hi = 0, len(d)                         # d[lo:] fails
    while hi - lo > 64:
        mid = (lo + hi) // 2
        if failing([d[mid:]])[0][0]:
            lo = mid
        else:
            hi = mid
    d = d[lo:]
    # then blocks of 1/16 of it at a time
    bs = max(64, len(d) // 16)
    cands = [d[:k] + d[k + bs:] for k in range(0, len(d), bs)]
    ks = np.nonzero(failing(cands)[0])[0]
    if len(ks):
        d = cands[ks[0]]
    print("long: %d bytes" % len(d), flush=True)
    if len(d) >= n0:
        break
# shortest failing prefix, then suffix
for side in ("prefix", "suffix"):
    cands = [d[:k] for k in range(1, len(d) + 1)] if side == "prefix" else [d[k:] for k in range(len(d))]
    bad = failing(cands)[0]
    ks = np.nonzero(bad)[0]
    d = cands[ks[0]] if side == "prefix" else cands[ks[-1]]
    print("%s: %d bytes" % (side, len(d)), flush=True)
# single-byte deletions, greedily
changed = True
while changed and len(d) > 1:
    changed = False
    cands = [d[:k] + d[k + 1:] for k in range(len(d))]
    bad = failing(cands)[0]
    ks = np.nonzero(bad)[0]
    if len(ks):
        d = cands[ks[0]]
        changed = True
print("minimal: %d bytes: %r" % (len(d), d), flush=True)
bad, got, ref = failing([d])
print("gpu", got[0], flush=True)
print("oracle", ref[0], flush=True)
if len(sys.argv) > 2:
    open(sys.argv[2], "wb").write(d)
