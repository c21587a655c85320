"""GPU path vs the reference CLD2 itself (no oracle in between), on the GPU
box, with the synthetic Q1 tables and again with the product's shipped Q0
(conftest.ref_tables): oracle/_ref/librefcld2.so is the reference's own sources built in its
dynamic-data mode (oracle/refcld), and it travels with the tree like the
product's library.  Tables: the same CLDT the GPU loads, written as a
cld2_data_file00 and read by the reference's loader.  A missing checker, or
one not built from this tree's oracle/refcld recipe, is a failure, not a skip
(refcld.verify_build)."""
import os

import numpy as np
import pytest

import corpus

pytestmark = pytest.mark.gpu
FIELDS = ("lang3", "summary_lang", "percent3", "is_reliable", "text_bytes", "normalized3")


@pytest.fixture(scope="module")
def ref(ref_tables):
    """The reference on the tables of this round of the module (Q1, then the shipped Q0)."""
    return ref_tables[1]


def same(got, want, what):
    n = len(got)
    bad = np.zeros(n, bool)
    for f in FIELDS:
        bad |= (got[f].astype(np.float64) != want[f].astype(np.float64)).reshape(n, -1).any(axis=1)
    assert not bad.any(), "%s: %d of %d differ, first %s" % (what, bad.sum(), n, np.nonzero(bad)[0][:5])


@pytest.mark.parametrize("cfg,n", [("c2", 100000), ("c3", 2000), ("c4", 50000), ("c5", 50000)])
def test_gpu_equals_reference(gpu, ref, cfg, n):
    buf, offs = corpus.GENERATORS[cfg](n)
    same(gpu.detect_batch(buf=buf, offsets=offs), ref.detect_batch(buf, offs, threads=16), cfg)


def test_gpu_equals_reference_html_hints(gpu, ref):
    from test_gpu_html_hints import random_hints
    buf, offs = corpus.html(2000, seed=31)
    n = len(offs) - 1
    same(gpu.detect_batch_ex(buf=buf, offsets=offs, html=True),
         ref.detect_batch(buf, offs, plain=np.zeros(n, np.uint8), threads=16), "html")
    buf, offs = corpus.c5(20000, seed=32)
    hints = random_hints(gpu, 20000, 33)
    same(gpu.detect_batch_ex(buf=buf, offsets=offs, hints=hints), ref.detect_batch(buf, offs, hints=hints, threads=16),
         "c5 hints")


def test_gpu_html_four_byte_characters_on_parallel_kernels(gpu, ref):
    """HTML pages with emoji and other 4-byte characters (raw and as numeric
    entities, corpus.html emoji=1): rewritten on the GPU like any other page
    (k_build_cpt4: no 4-byte character lowers differently in HTML mode) and
    scored by k_wave / k_long -- none on the sequential span source -- equal to the
    reference, with and without chunk vectors."""
    for lo, hi, n, seed in ((200, 6000, 3000, 41), (14000, 18000, 300, 42), (41000, 90000, 40, 43)):
        buf, offs = corpus.html(n, seed=seed, lo=lo, hi=hi, emoji=1.0)
        assert (np.asarray(buf) >= 0xF0).sum() >= n              # 4-byte lead bytes on the pages
        got = gpu.detect_batch_ex(buf=buf, offsets=offs, html=True)
        st = gpu.last_stats(0)
        assert st.general_docs == 0, (lo, hi, st.general_docs)
        same(got, ref.detect_batch(buf, offs, plain=np.zeros(n, np.uint8), threads=16), "html 4-byte %d-%d" % (lo, hi))
    buf, offs = corpus.html(1000, seed=44, emoji=1.0)
    n = len(offs) - 1
    res, chunks, coffs = gpu.detect_batch_vec(buf=buf, offsets=offs, html=True)
    st = gpu.last_stats(0)
    rres, rch, rco = ref.detect_batch_vec(buf, offs, plain=np.zeros(n, np.uint8), threads=16)
    same(res, rres, "html 4-byte vectors")
    assert np.array_equal(coffs.astype(np.int64), rco.astype(np.int64))
    for f in ("offset", "bytes", "lang1"):
        assert np.array_equal(chunks[f], rch[f])
    assert st.long_docs >= 0.99 * n, (st.long_docs, st.general_docs)


@pytest.mark.parametrize("flags", [0x0100, 0x4000, 0x4100], ids=["score_as_quads", "best_effort", "both"])
def test_gpu_equals_reference_with_flags(gpu, ref, ref_tables, golden, flags):
    """CLD2's result-affecting flags (compact_lang_det.h:343-349) through every
    batch entry point: the wave / long kernels (cld_detect_batch), the hinted
    and HTML paths (cld_detect_batch_ex), each equal to the reference called
    with the same flags; and the flags change results on these documents."""
    from test_reference_pin import flag_docs
    docs = flag_docs(golden)
    b3, o3 = corpus.c3(300, seed=509)
    docs += [bytes(b3[o3[i]:o3[i + 1]]) for i in range(300)]
    buf, offs = gpu.pack(docs)
    want = ref.detect_batch(buf, offs, threads=16, flags=flags)
    got = gpu.detect_batch(buf=buf, offsets=offs, flags=flags)
    same(got, want, "batch flags %#x" % flags)
    same(gpu.detect_batch_ex(buf=buf, offsets=offs, flags=flags), want, "batch_ex flags %#x" % flags)
    base = gpu.detect_batch(buf=buf, offsets=offs)
    if ref_tables[0] == "q1":                # (with Q0 most Latin documents have no language to move)
        assert ((got["summary_lang"] != base["summary_lang"]) | (got["is_reliable"] != base["is_reliable"]) |
                (got["lang3"] != base["lang3"]).any(axis=1)).sum() >= 10
    from test_gpu_html_hints import random_hints
    hb, ho = corpus.html(500, seed=510)
    n = len(ho) - 1
    same(gpu.detect_batch_ex(buf=hb, offsets=ho, html=True, flags=flags),
         ref.detect_batch(hb, ho, plain=np.zeros(n, np.uint8), threads=16, flags=flags), "html flags %#x" % flags)
    cb, co = corpus.c5(5000, seed=511)
    hints = random_hints(gpu, 5000, 512)
    same(gpu.detect_batch_ex(buf=cb, offsets=co, hints=hints, flags=flags),
         ref.detect_batch(cb, co, hints=hints, threads=16, flags=flags), "hints flags %#x" % flags)


def test_small_batches_speculate_and_equal_reference(gpu, ref):
    """Small batches of long documents: a long list of at most 64 documents
    goes to the fused k_long, which gives the longest of them a pass-1 wave and
    a pass-2 wave (speculation) and takes pass 2's result only where pass 1 was
    not good enough; larger ones (request-sized C5 batches: ~200 long
    documents) take the staged path.  Pages that need pass 2 (Repeats), ones
    that stop after pass 1, hinted and HTML pages, each equal to the reference."""
    for n, seed in ((64, 810), (600, 811)):
        b3, o3 = corpus.c3(n, seed=seed)
        got = gpu.detect_batch(buf=b3, offsets=o3)
        st = gpu.last_stats(0)
        assert st.long_docs == n and st.general_docs == 0
        assert st.passes[1] > n // 6 and st.passes[0] > 0    # both outcomes of the pass-1 wave occur (Q0: 44 / 556)
        same(got, ref.detect_batch(b3, o3, threads=16), "c3 %d" % n)
    for seed in (812, 813, 814):                         # ~1 MiB requests, each with ~180 long documents
        b5, o5 = corpus.c5(1000, seed=seed)
        same(gpu.detect_batch(buf=b5, offsets=o5), ref.detect_batch(b5, o5, threads=16), "c5 request %d" % seed)
    from test_gpu_html_hints import random_hints
    hb, ho = corpus.html(300, seed=815)
    n = len(ho) - 1
    same(gpu.detect_batch_ex(buf=hb, offsets=ho, html=True),
         ref.detect_batch(hb, ho, plain=np.zeros(n, np.uint8), threads=16), "html 300")
    cb, co = corpus.c3(200, seed=816)
    hints = random_hints(gpu, 200, 817)
    same(gpu.detect_batch_ex(buf=cb, offsets=co, hints=hints), ref.detect_batch(cb, co, hints=hints, threads=16),
         "c3 hints")
