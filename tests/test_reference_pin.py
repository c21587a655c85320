"""The oracle pinned END TO END to the reference CLD2 itself (CPU).

oracle/refcld builds the reference's own sources in its dynamic-data mode
(-DCLD2_DYNAMIC_MODE, the configuration cld2/internal/compile_dynamic.sh
documents): no scoring table is compiled in, the reference's loader reads the
tables at run time from a cld2_data_file00 that tools/cld2_data_file.py writes
from the same CLDT blob the oracle and the GPU path read (the writer itself is
pinned to that loader by tests/test_dynamic_data.py).  So the reference's
DetectLanguageSummaryV2 / ExtDetectLanguageSummary run here, on identical
tables and documents, and every result field must agree with the oracle:
every config, both quad tables (Q0 = the empty placeholder, Q1 = synthetic),
HTML mode, hints, the reference's own test documents and the edge cases.

What stays unpinned: answers of the REAL quadgram table, which the reference
checkout lacks (.MISSING_LARGE_BLOBS); both sides run the tables given.  And
documents with the ill-formed lead bytes C0, C1, F5, F6, F7: for them the
reference's UTF8GenericPropertyTwoByte (utf8statetable.cc:378-403) indexes
its state table with an exit code and reads past the table -- undefined
behaviour (AddressSanitizer stops it with a SEGV; the result depends on what
lies behind the table in memory).  The oracle and the GPU path bound every
table read and give such characters script 0 (non-letter).
"""
import os

import numpy as np
import pytest

import corpus

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DATA = os.path.join(ROOT, "language-detector_amd", "data")
SYNTH = os.path.join(DATA, "cld2_synth_q1.cldt")
Q0 = os.path.join(DATA, "cld2_q0.cldt")
FIELDS = ("lang3", "percent3", "normalized3", "text_bytes", "summary_lang", "is_reliable")
UB_LEADS = (0xC0, 0xC1, 0xF5, 0xF6, 0xF7)


def defined(doc):
    """False for documents that drive the reference into its out-of-bounds read."""
    return not any(b in UB_LEADS for b in doc)


def _have_ref():
    import refcld
    return os.path.exists(refcld.LIB) or os.path.isdir("/root/reference/cld2/internal")


needs_ref = pytest.mark.skipif(not _have_ref(), reason="reference library not built and sources absent")


def ref(tables):
    import refcld
    return refcld.instance(tables)


def same(a, b, what):
    n = len(a)
    bad = np.zeros(n, bool)
    for f in FIELDS:
        bad |= (a[f].astype(np.float64) != b[f].astype(np.float64)).reshape(n, -1).any(axis=1)
    assert not bad.any(), "%s: %d of %d documents differ, first %s" % (what, bad.sum(), n, np.nonzero(bad)[0][:5])


@pytest.fixture(scope="module")
def oracles():
    from oracle import Oracle
    return {SYNTH: Oracle(SYNTH), Q0: Oracle(Q0)}


def _oracle(oracles, tables):
    o = oracles[tables]
    o.lib.cldo_load(tables.encode())          # the oracle's tables are global too: select them
    return o


@needs_ref
@pytest.mark.parametrize("tables", [SYNTH, Q0], ids=["Q1", "Q0"])
@pytest.mark.parametrize("cfg,n", [("c2", 30000), ("c3", 400), ("c4", 8000), ("c5", 8000)])
def test_oracle_equals_reference(oracles, tables, cfg, n):
    buf, offs = corpus.GENERATORS[cfg](n)
    o = _oracle(oracles, tables)
    same(o.detect_batch(buf, offs, threads=8), ref(tables).detect_batch(buf, offs, threads=8), cfg)


@needs_ref
def test_oracle_equals_reference_on_fixtures_and_edges(oracles, golden, kats):
    from test_gpu_parity import EDGE
    docs = [bytes.fromhex(t["text_hex"]) for t in golden["test_pairs"]]
    docs += [bytes.fromhex(d["text_hex"]) for d in golden["html_docs"]]
    docs += [k["text"].encode() for k in kats] + list(EDGE)
    dropped = [d for d in docs if not defined(d)]
    assert len(dropped) == 2                  # the two C0 A9 test strings
    docs = [d for d in docs if defined(d)]
    import cld_amd
    buf, offs = cld_amd.pack(docs)
    for tables in (SYNTH, Q0):
        o = _oracle(oracles, tables)
        same(o.detect_batch(buf, offs, threads=4), ref(tables).detect_batch(buf, offs, threads=4), "fixtures")


@needs_ref
def test_oracle_equals_reference_html_and_hints(oracles):
    """HTML mode (tags, entities, lang= priors) and CLDHints: the oracle is fed
    the product's host hint code output (cld_hint_priors); the reference
    applies its own ApplyHints.  Equal results pin both."""
    import cld_amd
    from test_gpu_html_hints import priors_for, random_hints
    o = _oracle(oracles, SYNTH)
    r = ref(SYNTH)
    buf, offs = corpus.html(1200, seed=23)
    n = len(offs) - 1
    pr = priors_for(cld_amd, buf, offs, True, None)
    same(o.detect_batch_ex(buf, offs, plain=np.zeros(n, np.uint8), priors=pr, threads=8),
         r.detect_batch(buf, offs, plain=np.zeros(n, np.uint8), threads=8), "html")
    buf, offs = corpus.html(600, seed=24, emoji=1.0)               # 4-byte characters, raw and as entities
    n = len(offs) - 1
    pr = priors_for(cld_amd, buf, offs, True, None)
    same(o.detect_batch_ex(buf, offs, plain=np.zeros(n, np.uint8), priors=pr, threads=8),
         r.detect_batch(buf, offs, plain=np.zeros(n, np.uint8), threads=8), "html with 4-byte characters")
    for cfg, n, seed in (("c2", 15000, 41), ("c3", 200, 42), ("c4", 4000, 43)):
        buf, offs = corpus.GENERATORS[cfg](n)
        hints = random_hints(cld_amd, n, seed)
        pr = priors_for(cld_amd, buf, offs, False, hints)
        same(o.detect_batch_ex(buf, offs, priors=pr, threads=8), r.detect_batch(buf, offs, hints=hints, threads=8),
             cfg + " hints")


def _vec(ch):
    return [(int(x["offset"]), int(x["bytes"]), int(x["lang1"])) for x in ch]


@needs_ref
def test_result_chunk_vector_equals_reference(oracles):
    """ExtDetectLanguageSummary with a ResultChunkVector: the oracle's offset
    maps (OffsetMap in the scanner and the lowercaser), SharpenBoundaries /
    BetterBoundary, SummaryBufferToVector, the Overwrite variants of
    Squeeze/RepWords, MoveLang1ToLang2's vector merge and FinishResultVector
    must give the reference's vector, chunk for chunk, and the same summary
    fields (which SharpenBoundaries changes through the chunk byte counts)."""
    import cld_amd
    from test_gpu_html_hints import random_hints
    o = _oracle(oracles, SYNTH)
    r = ref(SYNTH)
    cases = []
    for cfg, n in (("c2", 1500), ("c3", 60), ("c4", 1000), ("c5", 1500)):
        buf, offs = corpus.GENERATORS[cfg](n)
        cases += [(bytes(buf[offs[i]:offs[i + 1]]), True, None) for i in range(n)]
    buf, offs = corpus.c3(40, boiler_frac=0.5)                     # squeeze restarts: Overwrite variant
    cases += [(bytes(buf[offs[i]:offs[i + 1]]), True, None) for i in range(40)]
    buf, offs = corpus.html(300, seed=9)                            # HTML: tags and entities in the maps
    cases += [(bytes(buf[offs[i]:offs[i + 1]]), False, None) for i in range(300)]
    buf, offs = corpus.c2(800, seed=77)
    hints = random_hints(cld_amd, 800, 78)
    cases += [(bytes(buf[offs[i]:offs[i + 1]]), True, hints[i]) for i in range(800)]
    multi = 0
    for doc, plain, h in cases:
        pri = None
        if h is not None or not plain:
            _, pri = cld_amd.hint_priors(doc, html=not plain, hints=h)
        ra, ca = o.detect_vec(doc, plain=plain, priors=pri)
        rb, cb = r.detect_vec(doc, plain=plain, hints=h)
        assert _vec(ca) == _vec(cb), doc[:120]
        assert (ra.summary_lang, list(ra.lang3), list(ra.percent3), ra.text_bytes, list(ra.normalized3)) == \
            (rb["summary_lang"], list(rb["lang3"]), list(rb["percent3"]), rb["text_bytes"], list(rb["normalized3"]))
        multi += len(ca) > 1
    assert multi > 200


FLAG_SETS = (0x0100, 0x4000, 0x4100)     # kCLDFlagScoreAsQuads, kCLDFlagBestEffort, both (compact_lang_det.h:343-349)


def flag_docs(golden):
    """Documents where the two flags matter: the reference's unit-test strings
    (20 script-only languages: ScoreAsQuads sends them to the quadgram path)
    and short mixed tweets (BestEffort keeps languages under 41% reliability
    and small top percents)."""
    docs = [bytes.fromhex(t["text_hex"]) for t in golden["test_pairs"]]
    docs = [d for d in docs if defined(d)]
    b, o = corpus.c2(3000, seed=505)
    docs += [bytes(b[o[i]:o[i + 1]]) for i in range(3000)]
    b, o = corpus.c5(3000, seed=506)
    docs += [bytes(b[o[i]:o[i + 1]]) for i in range(3000)]
    b, o = corpus.c4(1500, seed=507)
    docs += [bytes(b[o[i]:o[i + 1]]) for i in range(1500)]
    # a few words each of several languages: small percents
    b, o = corpus.c2(400, seed=508)
    for i in range(0, 400, 4):
        docs.append(b" ".join(bytes(b[o[j]:o[j + 1]])[:24] for j in range(i, i + 4)))
    return docs


@needs_ref
@pytest.mark.parametrize("flags", FLAG_SETS, ids=["score_as_quads", "best_effort", "both"])
def test_oracle_equals_reference_with_flags(oracles, golden, flags):
    """ExtDetectLanguageSummary's result-affecting `flags`: the oracle with the
    flags = the reference called with them, on both quad tables; and the flag
    visibly changes results on these documents (else the test proves nothing)."""
    import cld_amd
    docs = flag_docs(golden)
    buf, offs = cld_amd.pack(docs)
    for tables in (SYNTH, Q0):
        o = _oracle(oracles, tables)
        got = o.detect_batch_ex(buf, offs, threads=8, flags=flags)
        same(got, ref(tables).detect_batch(buf, offs, threads=8, flags=flags), "flags %#x" % flags)
        base = o.detect_batch_ex(buf, offs, threads=8)
        changed = (got["summary_lang"] != base["summary_lang"]) | (got["lang3"] != base["lang3"]).any(axis=1) | \
            (got["is_reliable"] != base["is_reliable"])
        assert changed.sum() >= 10, "flags %#x changed only %d results" % (flags, changed.sum())


@needs_ref
def test_result_chunk_vector_with_flags_equals_reference(oracles, golden):
    o = _oracle(oracles, SYNTH)
    r = ref(SYNTH)
    docs = flag_docs(golden)[:300]
    for flags in FLAG_SETS:
        for doc in docs:
            ra, ca = o.detect_vec(doc, flags=flags)
            rb, cb = r.detect_vec(doc, flags=flags)
            assert _vec(ca) == _vec(cb), (flags, doc[:80])
            assert (ra.summary_lang, list(ra.lang3), list(ra.percent3)) == \
                (rb["summary_lang"], list(rb["lang3"]), list(rb["percent3"])), (flags, doc[:80])
