"""k_long's sequential span source (cld_seq.hip, the SEQ instantiation): the
documents the parallel span builder hands on -- malformed UTF-8, a character
cut at the end (its Repeats carry), blocks of words wider than the LDS text
window (read in place from the slot, lng::WinG), a page past kDocCap, HTML
pages -- scored bit for bit like the oracle, in the three entry points
(cld_detect_batch, cld_detect_batch_ex HTML mode, cld_detect_batch_vec).
Needs an MI355X."""
import numpy as np
import pytest

import corpus
from test_gpu_html_hints import priors_for
from test_gpu_parity import assert_same
from test_gpu_vector import check as vec_check

pytestmark = pytest.mark.gpu
LETTERS = "abcdefghijklmnopqrstuvwxyz"


def long_words(rng, n_words, lo, hi, alphabet=LETTERS):
    return " ".join("".join(rng.choice(list(alphabet), int(rng.integers(lo, hi)))) for _ in range(n_words))


def seq_docs(rng, big=True, ordinary=400):
    """Documents that take the sequential span source, with ordinary ones mixed in."""
    b2, o2 = corpus.c2(4000, seed=31)
    tw = [bytes(b2[o2[i]:o2[i + 1]]) for i in range(4000)]
    docs = []
    # 64-word blocks wider than the window: words of 100-400 letters
    for k in range(6):
        docs.append(long_words(rng, 120 + 20 * k, 100, 400).encode())
    docs.append(long_words(rng, 90, 100, 300, "абвгдежзийклмнопрстуфхцчшщыэюя").encode())
    # one 20 KB word, and one between ordinary text
    docs.append("".join(rng.choice(list(LETTERS), 20000)).encode())
    docs.append(b" ".join(tw[:20]) + b" " + "".join(rng.choice(list(LETTERS), 9000)).encode() + b" " + b" ".join(tw[20:40]))
    # malformed UTF-8 inside letter runs, and a character cut at the end
    bad = [b"\x80", b"\xbf\xbf", b"\xc3", b"\xc3 ", b"\xe0\x80\x80", b"\xed\xa0\x80", b"\xf0\x9f", b"\xe4\xb8",
           b"\xf8\x88\x80\x80", b"\xff", b"\xc1\xbf"]
    for k in range(60):
        d = bytearray(b" ".join(tw[40 + 6 * k:46 + 6 * k + (k % 7) * 20]))
        for _ in range(1 + k % 4):
            p = int(rng.integers(1, max(2, len(d) - 4)))
            d[p:p] = bad[int(rng.integers(len(bad)))]
        if k % 3 == 0:
            d += bad[k % len(bad)]                      # cut (or stray) at the very end
        docs.append(bytes(d))
    # ordinary documents between them
    docs += tw[1000:1000 + ordinary]
    if big:                                             # past kDocCap (1 MB): the whole page on lane 0
        docs.append(b" ".join(tw[1400:4000]) * 4)
    order = rng.permutation(len(docs))
    return [docs[i] for i in order]


def test_sequential_spans_plain(gpu, oracle):
    rng = np.random.default_rng(5)
    docs = seq_docs(rng)
    assert max(len(d) for d in docs) > (1 << 20)
    buf, offs = gpu.pack(docs)
    got = gpu.detect_batch(buf=buf, offsets=offs)
    st = gpu.last_stats(0)
    assert_same(got, oracle.detect_batch(buf, offs, threads=16), "sequential spans, plain")
    assert st.general_docs >= 8, (st.general_docs, list(st.long_requeue))   # the wide-block pages at least


def test_sequential_spans_html(gpu, oracle):
    rng = np.random.default_rng(6)
    docs = seq_docs(rng, big=False)
    pages = [b"<p>" + d.replace(b" ", b" <b>x</b> ", 3) + b" &eacute;t&eacute;</p>" for d in docs]
    buf, offs = gpu.pack(pages)
    n = len(pages)
    got = gpu.detect_batch_ex(buf=buf, offsets=offs, html=True)
    pr = priors_for(gpu, buf, offs, True, None)
    ref = oracle.detect_batch_ex(buf, offs, plain=np.zeros(n, np.uint8), priors=pr, threads=16)
    assert_same(got, ref, "sequential spans, html")


def test_sequential_spans_vector(gpu, oracle):
    rng = np.random.default_rng(7)
    docs = seq_docs(rng, big=False, ordinary=100)
    buf, offs = gpu.pack(docs)
    vec_check(gpu, oracle, buf, offs, "sequential spans, vector")
    assert gpu.last_stats().general_docs >= 1
