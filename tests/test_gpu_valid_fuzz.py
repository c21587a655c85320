"""Valid-UTF-8 fuzz (tools/valid_fuzz.py: random code points of many scripts,
combining marks, digits, punctuation, symbols, 4-byte characters, exotic
spaces) on the GPU against the reference CLD2 itself, which is defined on such
text: every result field with and without ScoreAsQuads / BestEffort, and the
ResultChunkVector.  Needs an MI355X."""
import numpy as np
import pytest

import refcld
from valid_fuzz import FIELDS, gen

pytestmark = pytest.mark.gpu


def test_valid_fuzz_equals_reference(gpu):
    refcld.verify_build()
    ref = refcld.instance(gpu.SYNTH_TABLES)
    docs = gen(np.random.default_rng(74), 2000)
    buf, offs = gpu.pack(docs)
    n = len(docs)
    for flags in (0, 0x100, 0x4000):
        got = gpu.detect_batch(buf=buf, offsets=offs, flags=flags)
        want = ref.detect_batch(buf, offs, threads=16, flags=flags)
        for f in FIELDS:
            bad = np.nonzero((got[f].astype(np.float64) != want[f].astype(np.float64)).reshape(n, -1).any(axis=1))[0]
            assert len(bad) == 0, (flags, f, bad[:5])
    vd = docs[:600]
    vb, vo = gpu.pack(vd)
    g, chunks, coffs = gpu.detect_batch_vec(buf=vb, offsets=vo)
    for i in range(len(vd)):
        rb, cb = ref.detect_vec(vd[i])
        want_v = [(int(c["offset"]), int(c["bytes"]), int(c["lang1"])) for c in cb]
        have_v = [(int(c["offset"]), int(c["bytes"]), int(c["lang1"])) for c in chunks[coffs[i]:coffs[i + 1]]]
        assert have_v == want_v and int(g[i]["summary_lang"]) == int(rb["summary_lang"]), i
