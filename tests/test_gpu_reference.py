"""GPU path vs the reference CLD2 itself (no oracle in between), on the GPU
box: oracle/_ref/librefcld2.so is the reference's own sources built in its
dynamic-data mode (oracle/refcld), and it travels with the tree like the
product's library.  Tables: the same CLDT the GPU loads, written as a
cld2_data_file00 and read by the reference's loader."""
import os

import numpy as np
import pytest

import corpus

pytestmark = pytest.mark.gpu
FIELDS = ("lang3", "summary_lang", "percent3", "is_reliable", "text_bytes", "normalized3")


@pytest.fixture(scope="module")
def ref():
    import refcld
    if not os.path.exists(refcld.LIB):
        pytest.skip("oracle/_ref/librefcld2.so not built")
    return refcld.instance(os.environ["CLD_MI355X_TABLES"])


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
