"""cld_detect_batch_vec (ResultChunkVector) on the GPU vs the oracle, chunk for
chunk, and vs the reference CLD2 itself (oracle/_ref/librefcld2.so travels
with the tree; a missing or stale build fails the test, refcld.verify_build)."""
import os

import numpy as np
import pytest

import corpus
from test_gpu_html_hints import random_hints, soft_limit_pages

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def vecs(chunks, coffs):
    return [[(int(c["offset"]), int(c["bytes"]), int(c["lang1"])) for c in chunks[coffs[i]:coffs[i + 1]]]
            for i in range(len(coffs) - 1)]


def oracle_vecs(oracle, gpu, buf, offs, html=False, hints=None):
    res, out = [], []
    for i in range(len(offs) - 1):
        doc = bytes(buf[offs[i]:offs[i + 1]])
        pri = None
        if html or hints is not None:
            _, pri = gpu.hint_priors(doc, html=html, hints=hints[i] if hints is not None else None)
        r, ch = oracle.detect_vec(doc, plain=not html, priors=pri)
        res.append(r)
        out.append([(int(c["offset"]), int(c["bytes"]), int(c["lang1"])) for c in ch])
    return res, out


def check(gpu, oracle, buf, offs, what, html=False, hints=None):
    got, chunks, coffs = gpu.detect_batch_vec(buf=buf, offsets=offs, html=html, hints=hints)
    gv = vecs(chunks, coffs)
    rr, ov = oracle_vecs(oracle, gpu, buf, offs, html, hints)
    for i, (g, o) in enumerate(zip(gv, ov)):
        assert g == o, "%s doc %d: gpu %s oracle %s" % (what, i, g[:6], o[:6])
        r = rr[i]
        assert (int(got[i]["summary_lang"]), list(got[i]["lang3"]), list(got[i]["percent3"]),
                int(got[i]["text_bytes"]), list(got[i]["normalized3"])) == \
            (r.summary_lang, list(r.lang3), list(r.percent3), r.text_bytes, list(r.normalized3)), (what, i)
    return gv


@pytest.mark.parametrize("cfg,n", [("c2", 3000), ("c3", 60), ("c4", 2000), ("c5", 2000)])
def test_vector_corpora(gpu, oracle, cfg, n):
    buf, offs = corpus.GENERATORS[cfg](n)
    gv = check(gpu, oracle, buf, offs, cfg)
    assert sum(len(v) for v in gv) >= n


def test_vector_squeeze_html_hints(gpu, oracle):
    buf, offs = corpus.c3(30, boiler_frac=0.5)
    gv = check(gpu, oracle, buf, offs, "squeeze")
    assert max(len(v) for v in gv) > 5
    # the Squeeze restart's CheapSqueezeInplaceOverwrite runs in k_long<VEC>
    assert gpu.last_stats().general_docs == 0
    buf, offs = corpus.html(300, seed=12)
    check(gpu, oracle, buf, offs, "html", html=True)
    buf, offs = corpus.c2(1500, seed=13)
    check(gpu, oracle, buf, offs, "hints", hints=random_hints(gpu, 1500, 14))
    from test_gpu_parity import EDGE
    b, o = gpu.pack(EDGE)
    check(gpu, oracle, b, o, "edge")


def test_vector_html_soft_limit_pages(gpu, oracle):
    """Rewritten pages of kMaxScriptBytes and more in vec mode: page offsets
    serve both MapBack and the span soft limit."""
    docs = soft_limit_pages(n=12, seed=0xC1D20071, big=0)
    buf, offs = gpu.pack(docs)
    check(gpu, oracle, buf, offs, "html soft limit", html=True)


def test_vector_matches_reference_directly(gpu):
    """GPU vs the reference's own ExtDetectLanguageSummary vector (the
    checker library built from oracle/refcld; it must be present and current).
    Also with the reference's flags (kCLDFlagScoreAsQuads / kCLDFlagBestEffort)."""
    import refcld
    refcld.verify_build()
    r = refcld.instance(os.environ["CLD_MI355X_TABLES"])
    buf, offs = corpus.c5(1500, seed=15)
    for flags in (0, 0x0100, 0x4000):
        got, chunks, coffs = gpu.detect_batch_vec(buf=buf, offsets=offs, flags=flags)
        gv = vecs(chunks, coffs)
        for i in range(len(offs) - 1):
            doc = bytes(buf[offs[i]:offs[i + 1]])
            rb, cb = r.detect_vec(doc, flags=flags)
            assert gv[i] == [(int(c["offset"]), int(c["bytes"]), int(c["lang1"])) for c in cb], (flags, i)
            # every result field: vector mode scores differently (the Overwrite
            # forms of Squeeze / CheapRepWords), so the results are checked too
            for f in ("lang3", "summary_lang", "percent3", "is_reliable", "text_bytes", "normalized3"):
                assert np.array_equal(np.asarray(got[i][f], np.float64), np.asarray(rb[f], np.float64)), (flags, i, f)


def test_vector_capacity_contract(gpu):
    buf, offs = corpus.c2(200, seed=16)
    _, chunks, coffs = gpu.detect_batch_vec(buf=buf, offsets=offs)
    import ctypes
    n = len(offs) - 1
    out = np.zeros(n, dtype=gpu.RESULT_DTYPE)
    co = np.zeros(n + 1, dtype=np.uint64)
    small = np.zeros(3, dtype=gpu.CHUNK_DTYPE)
    rc = gpu.lib().cld_detect_batch_vec(buf.ctypes.data, offs.ctypes.data, n, None, 0, out.ctypes.data,
                                        small.ctypes.data, 3, co.ctypes.data)
    assert rc == -28 and int(co[-1]) == len(chunks)       # CLD_ENOSPC with the needed size
    assert np.array_equal(co, coffs)


def test_vector_overflow_retry_keeps_the_batch():
    """A document whose chunk vector outgrows its pool region is redone alone
    with a larger one; the batch is not failed (CLD_VEC_POOL_SMALL shrinks the
    first-pass regions to one chunk, so every multi-chunk document takes the
    retry).  Child
    process: the variable is read once per process."""
    import subprocess
    import sys
    code = r'''
import cld_amd, corpus
from oracle import Oracle
cld_amd.init()
o = Oracle()
b, off = corpus.c5(800, seed=17)
res, chunks, coffs = cld_amd.detect_batch_vec(buf=b, offsets=off)
for i in range(len(off) - 1):
    r, ch = o.detect_vec(bytes(b[off[i]:off[i + 1]]))
    assert [(int(c["offset"]), int(c["bytes"]), int(c["lang1"])) for c in chunks[coffs[i]:coffs[i + 1]]] == \
        [(int(c["offset"]), int(c["bytes"]), int(c["lang1"])) for c in ch], i
    assert int(res[i]["summary_lang"]) == r.summary_lang, i
assert sum(int(coffs[i + 1] - coffs[i]) > 1 for i in range(len(off) - 1)) > 50   # these took the retry
print("retry ok")
'''
    env = dict(os.environ, CLD_VEC_POOL_SMALL="1",
               PYTHONPATH=os.pathsep.join(os.path.join(ROOT, p) for p in ("language-detector_amd", "oracle", "tests")))
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0 and "retry ok" in r.stdout, r.stdout[-2000:] + r.stderr[-3000:]


def test_failed_document_is_redone_alone_and_the_batch_stands():
    """One document the kernels cannot score (fault injection: CLD_FAULT_DOC=k
    makes batch document k fail in k_long) costs neither the
    batch nor the process: it comes back marked CLD_LANG_FAILED, is redone
    alone (as document 0 of a one-document batch, which succeeds), and every
    result equals the reference.  With CLD_FAULT_DOC=0 the retry fails too:
    cld_detect_batch returns CLD_EIO with that document marked and all others
    equal to the reference, and detect_language answers "en" instead of
    aborting.  Child process: the variable is read once per process."""
    import subprocess
    import sys
    code = r'''
import sys, numpy as np, cld_amd, corpus, refcld, os
cld_amd.init()
ref = refcld.instance(os.environ["CLD_MI355X_TABLES"])
fault = int(os.environ["CLD_FAULT_DOC"])
b, off = corpus.c3(40, seed=21)                      # long documents: k_wave -> k_long
want = ref.detect_batch(b, off, threads=8)
F = ("lang3", "summary_lang", "percent3", "is_reliable", "text_bytes", "normalized3")
try:
    got = cld_amd.detect_batch(buf=b, offsets=off)
    failed = np.zeros(len(off) - 1, bool)
except cld_amd.PartialBatchError as e:
    got, failed = e.value, e.failed
for f in F:
    d = (np.asarray(got[f], np.float64) != np.asarray(want[f], np.float64)).reshape(len(got), -1).any(axis=1)
    assert not (d & ~failed).any(), (f, np.nonzero(d & ~failed)[0][:5])
if fault == 0:
    assert list(np.nonzero(failed)[0]) == [0] and int(got[0]["summary_lang"]) == cld_amd.LANG_FAILED
    assert cld_amd.detect_language(bytes(b[off[0]:off[1]])) == "en"
else:
    assert not failed.any()
print("isolation ok", fault, int(failed.sum()))
'''
    for fault in ("5", "0"):
        env = dict(os.environ, CLD_FAULT_DOC=fault,
                   PYTHONPATH=os.pathsep.join(os.path.join(ROOT, p) for p in ("language-detector_amd", "oracle", "tests")))
        r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=110)
        assert r.returncode == 0 and "isolation ok" in r.stdout, r.stdout[-2000:] + r.stderr[-3000:]
