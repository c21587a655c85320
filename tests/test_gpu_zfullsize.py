"""Full-size parity against the reference CLD2 itself, on the tree as built:
every document of BASELINE's C2 (1M tweets), C3 (100K 16 KB pages) and C4
(1.1M CJK-heavy documents), 200K documents of C5's stream, and 100K HTML pages
(is_plain_text = false, cld_detect_batch_ex; a quarter of them with emoji and
other 4-byte characters, raw and as entities), through the
product's batch entry point (cld_detect_batch: routing, k_wave, k_long) and through oracle/_ref/librefcld2.so (the reference's own sources
in dynamic-data mode, 16 host threads), every result field compared.  Twice:
with the synthetic Q1 quadgram table (the suite's default) and with the
product's shipped Q0 tables, loaded on both sides through the cld2 data-file
loaders (cld_load_data_from_file / the reference's loadDataFromFile).

Documents holding the ill-formed lead bytes C0, C1, F5-F7 (undefined
behaviour in the reference) are excluded and counted; the
generators produce none.  Corpora come from tests/fullsize.py (generated in
the background from session start).  Named to run last in the GPU suite."""
import os

import numpy as np
import pytest

import fullsize

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIELDS = ("lang3", "summary_lang", "percent3", "is_reliable", "text_bytes", "normalized3")


def ub_docs(buf, offs):
    pos = np.nonzero(np.isin(np.asarray(buf), np.array([0xC0, 0xC1, 0xF5, 0xF6, 0xF7], np.uint8)))[0]
    ub = np.zeros(len(offs) - 1, dtype=bool)
    ub[np.unique(np.searchsorted(offs, pos, side="right") - 1)] = True
    return ub


@pytest.mark.timeout(900)                     # (the first one may wait for its corpus generator)
@pytest.mark.parametrize("name", ["c2", "c3", "c4", "c5", "html"])
def test_full_size_equals_reference(gpu, ref_tables, name):
    label, ref = ref_tables
    buf, offs = fullsize.load(name)
    n = len(offs) - 1
    html = name == "html"                       # is_plain_text = false (cld_detect_batch_ex, CLD_FLAG_HTML)
    got = gpu.detect_batch_ex(buf=buf, offsets=offs, html=True) if html else gpu.detect_batch(buf=buf, offsets=offs)
    st = gpu.last_stats(0)
    want = ref.detect_batch(buf, offs, plain=np.zeros(n, np.uint8) if html else None, threads=16)
    bad = np.zeros(n, bool)
    for f in FIELDS:
        bad |= (got[f].astype(np.float64) != want[f].astype(np.float64)).reshape(n, -1).any(axis=1)
    ub = ub_docs(buf, offs)
    bad &= ~ub
    print("%s/%s: %d documents, %d bytes, %d mismatches, %d excluded (ill-formed lead bytes); "
          "k_wave %d, k_long %d, sequential spans %d; passes %s" % (name, label, n, int(offs[-1]), int(bad.sum()),
                                                              int(ub.sum()), st.short_docs, st.long_docs,
                                                              st.general_docs, list(st.passes)))
    assert not bad.any(), "%s/%s: %d of %d differ, first %s" % (name, label, bad.sum(), n, np.nonzero(bad)[0][:5])
    assert ub.sum() == 0
    assert st.passes[3] == 0
    assert st.general_docs == 0, "%s: %d documents on the sequential kernel" % (name, st.general_docs)


@pytest.mark.timeout(900)
@pytest.mark.parametrize("name", ["c2", "c3", "c4", "c5", "html"])
def test_full_size_vectors_equal_reference(gpu, ref_tables, name):
    """cld_detect_batch_vec on the same corpora: every result field and every
    ResultChunkVector equal to the reference's ExtDetectLanguageSummary with a
    vector; plain documents must run the parallel kernels (k_long<VEC>), only
    the few they hand on (Squeeze pages, length-changing lowercasing) the
    sequential one."""
    label, ref = ref_tables
    buf, offs = fullsize.load(name)
    n = len(offs) - 1
    html = name == "html"
    res, chunks, coffs = gpu.detect_batch_vec(buf=buf, offsets=offs, html=html)
    st = gpu.last_stats(0)
    rres, rch, rco = ref.detect_batch_vec(buf, offs, plain=np.zeros(n, np.uint8) if html else None, threads=16)
    bad = np.zeros(n, bool)
    for f in FIELDS:
        bad |= (res[f].astype(np.float64) != rres[f].astype(np.float64)).reshape(n, -1).any(axis=1)
    cnt_bad = np.diff(coffs.astype(np.int64)) != np.diff(rco.astype(np.int64))
    bad |= cnt_bad
    if not cnt_bad.any():
        neq = np.zeros(len(chunks), bool)
        for f in ("offset", "bytes", "lang1"):
            neq |= chunks[f] != rch[f]
        bad[np.searchsorted(coffs, np.nonzero(neq)[0], side="right") - 1] = True
    bad &= ~ub_docs(buf, offs)
    print("%s/%s vectors: %d documents, %d chunks, %d differ; parallel kernel %d, sequential %d"
          % (name, label, n, int(coffs[-1]), int(bad.sum()), st.long_docs, st.general_docs))
    assert not bad.any(), "%s/%s: %d of %d differ, first %s" % (name, label, bad.sum(), n, np.nonzero(bad)[0][:5])
    assert st.long_docs >= 0.99 * n, (st.long_docs, st.general_docs)
