"""Wider corruption sweep than tests/test_gpu_corrupt.py, for the GPU box:
many seeds of the corrupted corpora (tests/test_gpu_corrupt.docs_for) in
plain mode with each CLD2 flag set, with random CLDHints, HTML mode, and
vector mode, against the
oracle; prints the mismatch count per leg and saves the first mismatching
documents under gpurun_out/corrupt_diag/ (tools/corrupt_bisect.py shrinks
them).  SWEEP_SEEDS (default 20-27)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("language-detector_amd", "oracle", "tests"):
    sys.path.insert(0, os.path.join(ROOT, p))
import cld_amd  # noqa: E402
from oracle import Oracle  # noqa: E402
import test_gpu_corrupt as tc  # noqa: E402
from test_gpu_html_hints import priors_for, random_hints  # noqa: E402
from test_gpu_vector import vecs, oracle_vecs  # noqa: E402

FIELDS = ("lang3", "summary_lang", "percent3", "is_reliable", "text_bytes", "normalized3")
out_dir = os.path.join(ROOT, "gpurun_out", "corrupt_diag")
os.makedirs(out_dir, exist_ok=True)
# SWEEP_TABLES=q0: the shipped Q0 tables on both sides; SWEEP_MAX_BAD: splices per document (7)
tables = cld_amd.Q0_TABLES if os.environ.get("SWEEP_TABLES") == "q0" else cld_amd.SYNTH_TABLES
max_bad = int(os.environ.get("SWEEP_MAX_BAD", "7"))
cld_amd.init_device(0, tables=tables)
o = Oracle(tables=tables)


def diff(got, ref, n):
    bad = np.zeros(n, bool)
    for f in FIELDS:
        bad |= (got[f] != ref[f]).reshape(n, -1).any(axis=1)
    return np.nonzero(bad)[0]


def save(tag, docs, idx):
    for i in idx[:3]:
        with open(os.path.join(out_dir, "%s_d%d.bin" % (tag, i)), "wb") as f:
            f.write(docs[i])


total = 0
seeds = [int(s) for s in os.environ.get("SWEEP_SEEDS", "20,21,22,23,24,25,26,27").split(",")]
for seed in seeds:
    docs = tc.docs_for(seed, 3000, max_bad=max_bad)
    buf, offs = cld_amd.pack(docs)
    n = len(docs)
    for flags in (0, 0x100, 0x4000, 0x4100):
        got = cld_amd.detect_batch(buf=buf, offsets=offs, flags=flags)
        ref = o.detect_batch_ex(buf, offs, flags=flags, threads=16)
        idx = diff(got, ref, n)
        total += len(idx)
        save("sw_s%d_f%x" % (seed, flags), docs, idx)
        print("seed %d flags %#x: %d docs, %d mismatches %s" % (seed, flags, n, len(idx), idx[:5]), flush=True)
    hints = random_hints(cld_amd, n, seed=seed)         # CLDHints (tld, content-language, encoding, language)
    got = cld_amd.detect_batch_ex(buf=buf, offsets=offs, hints=hints)
    pr = priors_for(cld_amd, buf, offs, False, hints)
    ref = o.detect_batch_ex(buf, offs, priors=pr, threads=16)
    idx = diff(got, ref, n)
    total += len(idx)
    save("sw_s%d_hints" % seed, docs, idx)
    print("seed %d hints: %d docs (%d hinted), %d mismatches %s" % (seed, n, int((pr != 0).any(axis=1).sum()),
                                                                   len(idx), idx[:5]), flush=True)
    pages = [b"<p>" + d.replace(b" ", b" <b>x</b> ", 2) + b" &amp;&#233;</p>" for d in docs[:2500]]
    pb, po = cld_amd.pack(pages)
    got = cld_amd.detect_batch_ex(buf=pb, offsets=po, html=True)
    pr = priors_for(cld_amd, pb, po, True, None)
    ref = o.detect_batch_ex(pb, po, plain=np.zeros(len(pages), np.uint8), priors=pr, threads=16)
    idx = diff(got, ref, len(pages))
    total += len(idx)
    save("sw_s%d_html" % seed, pages, idx)
    print("seed %d html: %d pages, %d mismatches %s" % (seed, len(pages), len(idx), idx[:5]), flush=True)
    vd = docs[:1500]
    vb, vo = cld_amd.pack(vd)
    g, chunks, coffs = cld_amd.detect_batch_vec(buf=vb, offsets=vo)
    gv = vecs(chunks, coffs)
    rr, ov = oracle_vecs(o, cld_amd, vb, vo)
    idx = [i for i in range(len(vd)) if gv[i] != ov[i] or (int(g[i]["summary_lang"]), list(g[i]["percent3"]),
           int(g[i]["text_bytes"])) != (rr[i].summary_lang, list(rr[i].percent3), rr[i].text_bytes)]
    total += len(idx)
    save("sw_s%d_vec" % seed, vd, idx)
    print("seed %d vec: %d docs, %d mismatches %s" % (seed, len(vd), len(idx), idx[:5]), flush=True)
print("total mismatches", total, flush=True)
