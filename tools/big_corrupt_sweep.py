"""Long corrupted documents for the GPU box: C3 pages and C5 documents run
together into 20 KB-1.5 MB documents with malformed UTF-8 spliced in
(tests/test_gpu_corrupt.corrupt), plain and vector mode against the oracle,
with the synthetic Q1 tables and then the shipped Q0 tables (BIG_TABLES=q0)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("language-detector_amd", "oracle", "tests"):
    sys.path.insert(0, os.path.join(ROOT, p))
import cld_amd  # noqa: E402
import corpus  # noqa: E402
from oracle import Oracle  # noqa: E402
import test_gpu_corrupt as tc  # noqa: E402
from test_gpu_vector import vecs, oracle_vecs  # noqa: E402

FIELDS = ("lang3", "summary_lang", "percent3", "is_reliable", "text_bytes", "normalized3")
tables = cld_amd.Q0_TABLES if os.environ.get("BIG_TABLES") == "q0" else cld_amd.SYNTH_TABLES
cld_amd.init_device(0, tables=tables)
o = Oracle(tables=tables)
out_dir = os.path.join(ROOT, "gpurun_out", "corrupt_diag")
os.makedirs(out_dir, exist_ok=True)
total = 0
for seed in (int(x) for x in os.environ.get("BIG_SEEDS", "60,61").split(",")):
    rng = np.random.default_rng(seed)
    b3, o3 = corpus.c3(200, seed=seed)
    b5, o5 = corpus.c5(4000, seed=seed)
    pieces = [bytes(b3[o3[i]:o3[i + 1]]) for i in range(200)] + [bytes(b5[o5[i]:o5[i + 1]]) for i in range(4000)]
    docs = []
    for _ in range(120):
        target = int(rng.choice([20000, 70000, 200000, 1500000]))
        d = bytearray()
        while len(d) < target:
            d += pieces[int(rng.integers(len(pieces)))] + b" "
        docs.append(tc.corrupt(rng, bytes(d)) if rng.random() < 0.8 else bytes(d))
    buf, offs = cld_amd.pack(docs)
    got = cld_amd.detect_batch(buf=buf, offsets=offs)
    st = cld_amd.last_stats(0)
    ref = o.detect_batch(buf, offs, threads=16)
    n = len(docs)
    bad = np.zeros(n, bool)
    for f in FIELDS:
        bad |= (got[f] != ref[f]).reshape(n, -1).any(axis=1)
    idx = np.nonzero(bad)[0]
    total += len(idx)
    print("%s seed %d: %d docs, %d bytes, %d mismatches %s; long %d seq %d" % (
        os.path.basename(tables), seed, n, len(buf), len(idx), idx[:5], st.long_docs, st.general_docs), flush=True)
    for i in idx[:2]:
        with open(os.path.join(out_dir, "big_s%d_d%d.bin" % (seed, i)), "wb") as f:
            f.write(docs[i])
    vd = [d for d in docs if len(d) < 300000][:40]
    vb, vo = cld_amd.pack(vd)
    g, chunks, coffs = cld_amd.detect_batch_vec(buf=vb, offsets=vo)
    gv = vecs(chunks, coffs)
    rr, ov = oracle_vecs(o, cld_amd, vb, vo)
    vidx = [i for i in range(len(vd)) if gv[i] != ov[i] or (int(g[i]["summary_lang"]), list(g[i]["percent3"]),
            int(g[i]["text_bytes"])) != (rr[i].summary_lang, list(rr[i].percent3), rr[i].text_bytes)]
    total += len(vidx)
    print("%s seed %d vec: %d docs, %d mismatches %s" % (os.path.basename(tables), seed, len(vd), len(vidx), vidx[:5]),
          flush=True)
print("total mismatches", total, flush=True)
