"""Vector-mode counterpart of tools/corrupt_diag.py: cld_detect_batch_vec on
the corrupted corpora against the oracle, mismatches counted per kind of
document (corrupted text / random bytes) and the first few printed and saved
under gpurun_out/corrupt_diag/ for replay."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("language-detector_amd", "oracle", "tests"):
    sys.path.insert(0, os.path.join(ROOT, p))
import cld_amd  # noqa: E402
from oracle import Oracle  # noqa: E402
import test_gpu_corrupt as tc  # noqa: E402
from test_gpu_vector import vecs, oracle_vecs  # noqa: E402

out_dir = os.path.join(ROOT, "gpurun_out", "corrupt_diag")
os.makedirs(out_dir, exist_ok=True)
cld_amd.init_device(0, tables=cld_amd.SYNTH_TABLES)
o = Oracle()
UB = (0xC0, 0xC1, 0xF5, 0xF6, 0xF7)
for seed, n in ((14, 800), (15, 800), (16, 800)):
    docs = tc.docs_for(seed, n, random_docs=os.environ.get("DIAG_RANDOM", "1") != "0")
    buf, offs = cld_amd.pack(docs)
    got, chunks, coffs = cld_amd.detect_batch_vec(buf=buf, offsets=offs)
    gv = vecs(chunks, coffs)
    rr, ov = oracle_vecs(o, cld_amd, buf, offs)
    def fields(g):
        return (int(g["summary_lang"]), list(g["lang3"]), list(g["percent3"]), int(g["text_bytes"]),
                list(g["normalized3"]))

    def ofields(r):
        return (r.summary_lang, list(r.lang3), list(r.percent3), r.text_bytes, list(r.normalized3))

    bad = [i for i in range(len(docs)) if gv[i] != ov[i] or fields(got[i]) != ofields(rr[i])]
    kinds = {}
    for i in bad:
        d = docs[i]
        k = ("ub" if any(b in UB for b in d) else "") + ("hi" if any(b >= 0xF8 for b in d) else "")
        kinds[k or "plain-malformed"] = kinds.get(k or "plain-malformed", 0) + 1
    print("seed %d: %d docs, %d vector mismatches, by kind %s" % (seed, len(docs), len(bad), kinds), flush=True)
    for i in bad[:4]:
        with open(os.path.join(out_dir, "vec_s%d_d%d.bin" % (seed, i)), "wb") as f:
            f.write(docs[i])
        j = next((j for j in range(min(len(gv[i]), len(ov[i]))) if gv[i][j] != ov[i][j]), None)
        print(" doc %d len %d first diff at chunk %s: gpu %s oracle %s; fields gpu %s oracle %s" % (
            i, len(docs[i]), j, gv[i][j:j + 3] if j is not None else gv[i][:3],
            ov[i][j:j + 3] if j is not None else ov[i][:3], fields(got[i]), ofields(rr[i])), flush=True)
