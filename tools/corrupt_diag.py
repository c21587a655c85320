"""Diagnostic for tests/test_gpu_corrupt.py: the corrupted corpora on cuda:0
against the oracle; every mismatching document is rerun alone and in two
variants (ill-formed leads C0/C1/F5-F7 replaced by 0xFF, or removed), and
saved under gpurun_out/corrupt_diag/ for replay on the CPU oracle."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("language-detector_amd", "oracle", "tests"):
    sys.path.insert(0, os.path.join(ROOT, p))
import cld_amd  # noqa: E402
from oracle import Oracle  # noqa: E402
from test_gpu_corrupt import docs_for  # noqa: E402

FIELDS = ("lang3", "summary_lang", "percent3", "is_reliable", "text_bytes", "normalized3")
UB = (0xC0, 0xC1, 0xF5, 0xF6, 0xF7)
out_dir = os.path.join(ROOT, "gpurun_out", "corrupt_diag")
os.makedirs(out_dir, exist_ok=True)
cld_amd.init_device(0, tables=cld_amd.SYNTH_TABLES)
o = Oracle()


def run(docs):
    buf, offs = cld_amd.pack(docs)
    got = cld_amd.detect_batch(buf=buf, offsets=offs)
    st = cld_amd.last_stats(0)
    ref = o.detect_batch(buf, offs, threads=8)
    bad = np.zeros(len(docs), bool)
    for f in FIELDS:
        bad |= (got[f] != ref[f]).reshape(len(docs), -1).any(axis=1)
    return got, ref, bad, st


def show(tag, g, r):
    print("  %-10s gpu lang %s pct %s tb %d ns %s | oracle lang %s pct %s tb %d ns %s passes %d" % (
        tag, list(g["lang3"]), list(g["percent3"]), g["text_bytes"], list(g["normalized3"]),
        list(r["lang3"]), list(r["percent3"]), r["text_bytes"], list(r["normalized3"]), r["passes"]), flush=True)


for seed in (int(s) for s in os.environ.get("DIAG_SEEDS", "11,12").split(",")):
    docs = docs_for(seed, 3000)
    got, ref, bad, st = run(docs)
    idx = np.nonzero(bad)[0]
    print("seed %d: %d docs, %d mismatches %s; stats short %d long %d seq %d" % (
        seed, len(docs), len(idx), idx[:10], st.short_docs, st.long_docs, st.general_docs), flush=True)
    for i in idx[:8]:
        d = docs[i]
        with open(os.path.join(out_dir, "s%d_d%d.bin" % (seed, i)), "wb") as f:
            f.write(d)
        print(" doc %d: %d bytes, %d ill-formed leads" % (i, len(d), sum(b in UB for b in d)), flush=True)
        show("batch", got[i], ref[i])
        for tag, v in (("alone", d), ("ub->ff", bytes(0xFF if b in UB else b for b in d)),
                       ("ub-gone", bytes(b for b in d if b not in UB))):
            g1, r1, b1, st1 = run([v])
            show(tag + ("*" if b1[0] else ""), g1[0], r1[0])
    # random bytes without the ill-formed leads
    rng = np.random.default_rng(seed)
    rdocs = []
    for _ in range(3000):
        a = rng.integers(0, 256, int(rng.integers(0, 3000)), dtype=np.uint8)
        a[np.isin(a, np.array(UB, np.uint8))] = 0xFF
        rdocs.append(a.tobytes())
    _, _, b2, st2 = run(rdocs)
    print("seed %d: random bytes without ill-formed leads: %d mismatches of %d (long %d seq %d)" % (
        seed, int(b2.sum()), len(rdocs), st2.long_docs, st2.general_docs), flush=True)
