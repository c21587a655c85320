"""Randomised corruption sweep: ordinary documents of every benchmark config
with malformed UTF-8 spliced in at random places -- lone continuation bytes,
truncated and overlong sequences, surrogates, 5- and 6-byte leads, embedded
NULs, and the ill-formed leads C0/C1/F5-F7 (undefined in the reference, script
0 in the oracle and on the GPU) -- plus documents of
random bytes, through the three entry points (cld_detect_batch, HTML mode of
cld_detect_batch_ex, cld_detect_batch_vec) against the oracle, bit for bit.
Every routing path sees them: k_wave, the staged span kernels, the fused
k_long and its sequential span source.  The reference itself is no judge here:
it reads past its tables on such bytes and segfaults on random ones.
Needs an MI355X."""
import os

import numpy as np
import pytest

import corpus
from test_gpu_html_hints import priors_for
from test_gpu_parity import assert_same
from test_gpu_vector import check as vec_check

pytestmark = pytest.mark.gpu

BAD = [b"\x80", b"\xbf", b"\x80\x80\x80", b"\xc3", b"\xe4\xb8", b"\xf0\x9f\x98", b"\xc0\xaf", b"\xc1\xbf",
       b"\xe0\x80\xaf", b"\xed\xa0\x80", b"\xed\xbf\xbf", b"\xf4\x90\x80\x80", b"\xf5\x80\x80\x80", b"\xf6", b"\xf7\xbf",
       b"\xf8\x88\x80\x80\x80", b"\xfc\x84\x80\x80\x80\x80", b"\xfe", b"\xff", b"\x00", b"\xf0\x9f\x98\x80",
       b"\xc2\xa0", b"\xe3\x80\x80"]


def corrupt(rng, d, max_bad=7):
    d = bytearray(d)
    for _ in range(int(rng.integers(0, max_bad))):
        p = int(rng.integers(0, len(d) + 1))
        k = int(rng.integers(3))
        if k == 0:                                        # splice a bad sequence in
            d[p:p] = BAD[int(rng.integers(len(BAD)))]
        elif k == 1 and p < len(d):                       # overwrite one byte
            d[p] = int(rng.integers(0x80, 0x100))
        elif p > 0:                                       # cut the document there (maybe inside a character)
            del d[p:]
    return bytes(d)


def docs_for(seed, n_each, random_docs=True, max_bad=7):
    rng = np.random.default_rng(seed)
    docs = []
    for cfg, n in (("c2", n_each), ("c3", max(8, n_each // 40)), ("c4", n_each // 2), ("c5", n_each)):
        b, o = corpus.GENERATORS[cfg](n, seed=seed)
        docs += [corrupt(rng, bytes(b[o[i]:o[i + 1]]), max_bad) for i in range(n)]
    for _ in range(n_each // 10 if random_docs else 0):   # random bytes, 0-3000 of them
        docs.append(rng.integers(0, 256, int(rng.integers(0, 3000)), dtype=np.uint8).tobytes())
    order = rng.permutation(len(docs))
    return [docs[i] for i in order]


@pytest.mark.parametrize("seed", [11, 12])
def test_corrupted_documents_plain(gpu, oracle, seed):
    docs = docs_for(seed, 3000)
    buf, offs = gpu.pack(docs)
    got = gpu.detect_batch(buf=buf, offsets=offs)
    assert_same(got, oracle.detect_batch(buf, offs, threads=16), "corrupted, plain (seed %d)" % seed)


@pytest.mark.parametrize("flags", [0x100, 0x4100])      # kCLDFlagScoreAsQuads, with kCLDFlagBestEffort
def test_corrupted_documents_flags(gpu, oracle, flags):
    docs = docs_for(20, 3000)                             # (seed 20 reached GetScore(-1): an empty chunk tote)
    buf, offs = gpu.pack(docs)
    got = gpu.detect_batch(buf=buf, offsets=offs, flags=flags)
    assert_same(got, oracle.detect_batch_ex(buf, offs, flags=flags, threads=16), "corrupted, flags %#x" % flags)


def test_corrupted_documents_html(gpu, oracle):
    docs = docs_for(13, 1200)
    pages = [b"<p>" + d.replace(b" ", b" <b>x</b> ", 2) + b" &eacute;t&eacute; &#x1F600;</p>" for d in docs]
    buf, offs = gpu.pack(pages)
    n = len(pages)
    got = gpu.detect_batch_ex(buf=buf, offsets=offs, html=True)
    pr = priors_for(gpu, buf, offs, True, None)
    ref = oracle.detect_batch_ex(buf, offs, plain=np.zeros(n, np.uint8), priors=pr, threads=16)
    assert_same(got, ref, "corrupted, html")


def test_corrupted_documents_vector(gpu, oracle):
    docs = docs_for(14, 1200)
    buf, offs = gpu.pack(docs)
    vec_check(gpu, oracle, buf, offs, "corrupted, vector")


GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "corrupt")


def test_shrunk_regressions(gpu, oracle):
    """The documents the sweeps shrank (tools/corrupt_bisect.py), one per fixed
    difference: an orphan continuation byte in a Repeats span; a span with
    text_bytes < 1 in vector mode; a character that ends in the first byte of
    a window with no character start (the carry was kept); an empty chunk tote
    under ScoreAsQuads.  Plain with both flags, and vector mode."""
    docs = [open(os.path.join(GOLDEN, f), "rb").read() for f in sorted(os.listdir(GOLDEN))]
    assert len(docs) == 4
    buf, offs = gpu.pack(docs)
    for flags in (0, 0x100):
        got = gpu.detect_batch(buf=buf, offsets=offs, flags=flags)
        assert_same(got, oracle.detect_batch_ex(buf, offs, flags=flags), "shrunk regressions, flags %#x" % flags)
    vec_check(gpu, oracle, buf, offs, "shrunk regressions, vector")
