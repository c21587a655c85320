"""HIP path vs the C oracle, bit-exact, through the C ABI (needs an MI355X)."""
import json
import os
import threading

import numpy as np
import pytest

import corpus

pytestmark = pytest.mark.gpu
FIELDS = ("lang3", "summary_lang", "percent3", "is_reliable", "text_bytes", "normalized3")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def assert_same(gpu_res, ref, what):
    for f in FIELDS:
        a, b = gpu_res[f], ref[f]
        if not np.array_equal(a, b):
            bad = np.nonzero((a != b).reshape(len(a), -1).any(axis=1))[0]
            raise AssertionError("%s: %s differs on %d docs, first %s: gpu=%s oracle=%s"
                                 % (what, f, len(bad), bad[:5], gpu_res[bad[0]], ref[bad[0]]))


def check(gpu, oracle, buf, offs, what, threads=8):
    got = gpu.detect_batch(buf=buf, offsets=offs)
    ref = oracle.detect_batch(buf, offs, threads=threads)
    assert_same(got, ref, what)
    return got


def test_golden_and_kat_documents(gpu, oracle, golden, kats):
    docs = [bytes.fromhex(t["text_hex"]) for t in golden["test_pairs"]]
    docs += [bytes.fromhex(d["text_hex"]) for d in golden["html_docs"]]
    docs += [k["text"].encode() for k in kats]
    buf, offs = gpu.pack(docs)
    check(gpu, oracle, buf, offs, "fixtures")


EDGE = [
    b"", b" ", b"\t\n", b"a", b"A", b"1234567890", b"!!!???", b"\x00", b"a\x00b c", b"\xc3", b"\xff\xfe\xfd",
    b"\xe0\xa0", b"\xf0\x9f\x98\x80 smile", b"\xc0\xa9bad", "Ünïcödé ÀÉÎ ÇŒ".encode(),
    "İstanbul'da KIŞ".encode(), "Ⱥ Ⱦ ȺȺȺ".encode(), b"x" * 255, b"x" * 256, b"x" * 257, b"ab " * 5000,
    ("العربية abc рус " * 50).encode(),
    ("ꙮ" * 100).encode(), ("á" * 200).encode(), b"http://x.y/z @user #tag",
]


def test_edge_cases(gpu, oracle):
    buf, offs = gpu.pack(EDGE)
    check(gpu, oracle, buf, offs, "edge")


def test_bucket_boundaries_and_requeue(gpu, oracle):
    """Documents around the short-kernel capacity and ones needing passes 2/3
    (Squeeze restart, Repeats) must agree whichever kernel finishes them."""
    rng = np.random.default_rng(5)
    b2, o2 = corpus.c2(4000, seed=11)
    docs = []
    for L in (200, 250, 255, 256, 257, 260, 300, 511, 512, 513, 1000, 4000):
        i = int(rng.integers(0, 3000))
        d = bytes(b2[o2[i]:o2[i + 40]])[:L]
        docs.append(d)
    docs.append(("aaaa bbbb cccc " * 400).encode())                 # repetitive, below the trigger
    docs.append(corpus.BOILERPLATE * 40 + bytes(b2[o2[0]:o2[30]]))  # squeeze trigger: predicted bytes
    docs.append(("a b c d e f g h " * 300).encode())                # squeeze trigger: spaces
    docs.append((" ".join(["w%d" % i for i in range(2000)])).encode())
    docs.append(bytes(b2[o2[0]:o2[300]]))                           # ~40 KB mixed-language: pass 3
    buf, offs = gpu.pack(docs)
    check(gpu, oracle, buf, offs, "boundaries")


@pytest.mark.parametrize("cfg,n", [("c2", 50000), ("c4", 20000), ("c5", 3000), ("c3", 48)])
def test_synthetic_corpora(gpu, oracle, cfg, n):
    buf, offs = corpus.GENERATORS[cfg](n)
    check(gpu, oracle, buf, offs, cfg, threads=16)


def test_long_documents(gpu, oracle):
    """Spans beyond the 40,928-byte script buffer, the len/2 soft split for
    40-80 KB remainders, and 1000-hit rounds."""
    b3, o3 = corpus.c3(8, page=65536 * 2)
    docs = [bytes(b3[o3[i]:o3[i + 1]]) for i in range(4)]
    b2, o2 = corpus.c2(6000, seed=3)
    docs.append(bytes(b2[o2[0]:o2[-1]]).replace(b" ", b" "))          # ~800 KB single document
    buf, offs = gpu.pack(docs)
    check(gpu, oracle, buf, offs, "long")
    st = gpu.last_stats(0)
    assert st.general_docs == 0, list(st.long_requeue)           # up to 1 MB: the wavefront path


def test_squeeze_documents_stay_on_the_wavefront_path(gpu, oracle):
    """CheapSqueezeTriggerTest restarts (compact_lang_det_impl.cc:1867-1900) and
    the Squeeze / Squeeze+Repeats passes run in k_long: bit-exact, and no
    document falls through to the sequential span source."""
    b3, o3 = corpus.c3(2000, seed=21, boiler_frac=0.05)
    b2, o2 = corpus.c2(3000, seed=22)
    docs = [bytes(b3[o3[i]:o3[i + 1]]) for i in range(2000)]
    docs += [corpus.BOILERPLATE * k + bytes(b2[o2[10 * k]:o2[10 * k + 25 + k]]) for k in range(8, 80, 3)]
    docs += [("a b c d e f g h " * (150 + 7 * k)).encode() + bytes(b2[o2[k]:o2[k + 5]]) for k in range(20)]
    buf, offs = gpu.pack(docs)
    got = check(gpu, oracle, buf, offs, "squeeze")
    st = gpu.last_stats(0)
    ref = oracle.detect_batch(buf, offs, threads=16)
    assert int((ref["passes"] == 3).sum()) >= 60          # the Squeeze restarts taken
    assert st.general_docs == 0, list(st.long_requeue)
    assert st.passes[2] == int((ref["passes"] == 3).sum())
    assert len(got) == len(docs)


def test_full_size_c3_c4_properties(gpu, oracle):
    """BASELINE sizes of C3 (100K x 16 KB pages) and C4 (1M x 150 B + 100K x
    4 KB CJK): an oracle-checked random sample and re-batching invariance."""
    rng = np.random.default_rng(7)
    for cfg, n, k in (("c3", 100_000, 1500), ("c4", 1_100_000, 20000)):
        buf, offs = corpus.GENERATORS[cfg](n)
        got = gpu.detect_batch(buf=buf, offsets=offs)
        st = gpu.last_stats(0)
        assert st.general_docs == 0, (cfg, list(st.long_requeue))
        idx = np.sort(rng.choice(n, size=k, replace=False))
        docs = [bytes(buf[offs[i]:offs[i + 1]]) for i in idx]
        sb, so = gpu.pack(docs)
        assert_same(got[idx], oracle.detect_batch(sb, so, threads=16), cfg + " sample")
        perm = rng.permutation(len(docs))
        pb, po = gpu.pack([docs[i] for i in perm])
        again = gpu.detect_batch(buf=pb, offsets=po)
        inv = np.empty_like(perm); inv[perm] = np.arange(len(perm))
        assert_same(again[inv], got[idx], cfg + " permuted")
        del buf, offs, got


def test_full_size_c2_properties(gpu, oracle):
    """At BASELINE size (1M tweets): a random 20K sample is bit-exact vs the
    oracle, and results are invariant under batch permutation / splitting."""
    buf, offs = corpus.c2(1_000_000)
    got = gpu.detect_batch(buf=buf, offsets=offs)
    rng = np.random.default_rng(1)
    idx = np.sort(rng.choice(1_000_000, size=20000, replace=False))
    docs = [bytes(buf[offs[i]:offs[i + 1]]) for i in idx]
    sb, so = gpu.pack(docs)
    assert_same(got[idx], oracle.detect_batch(sb, so, threads=16), "c2 sample")
    # permutation / re-batching invariance
    perm = rng.permutation(len(docs))
    pb, po = gpu.pack([docs[i] for i in perm])
    again = gpu.detect_batch(buf=pb, offsets=po)
    inv = np.empty_like(perm); inv[perm] = np.arange(len(perm))
    assert_same(again[inv], got[idx], "permuted")
    counts = np.bincount(got["summary_lang"], minlength=614)
    assert counts.sum() == 1_000_000 and (counts > 0).sum() >= 12


def test_detect_language_abi_concurrent(gpu, oracle, kats):
    """wrapper.h detect_language: equal to the oracle's wrapper semantics, also
    under concurrent callers (coalesced micro-batches)."""
    texts = [k["text"] for k in kats] * 8
    want = [oracle.detect_language(t) for t in texts]
    got = [None] * len(texts)

    def worker(lo):
        for i in range(lo, len(texts), 8):
            got[i] = gpu.detect_language(texts[i])

    th = [threading.Thread(target=worker, args=(k,)) for k in range(8)]
    [t.start() for t in th]
    [t.join() for t in th]
    assert got == want
    assert gpu.detect_language(" 私はガラスを食べられます。それは私を傷つけません。") == "ja"
    assert gpu.detect_language("") == "en"


CLOSE_GROUPS = [["da", "no"], ["es", "gl"], ["cs", "sk"], ["id", "ms"], ["hr", "sr", "bs"], ["pt", "gl"],
                ["en", "fr", "de", "it", "es"], ["ro", "it"], ["sw", "rw"], ["tl", "ceb"]]


def mixed_short_docs(n, seed=0xC1D2_00AA):
    """Short (<= 256 B) documents mixing words of 2-4 languages in random
    proportions, half of them from a close set: they exercise the document
    level -- close pairs (RefineScoredClosePairs), unreliable languages
    (RemoveUnreliableLanguages) and the top-3 sort -- inside the wave kernel."""
    with open(os.path.join(ROOT, "language-detector_amd", "data", "vocab.json"), encoding="utf-8") as f:
        vocab = json.load(f)
    latin = [l for l in vocab if l not in ("un",) and len(vocab[l]) >= 100]
    rng = np.random.default_rng(seed)
    docs = []
    for _ in range(n):
        if rng.random() < 0.5:
            langs = list(CLOSE_GROUPS[rng.integers(len(CLOSE_GROUPS))])
        else:
            langs = list(rng.choice(latin, size=rng.integers(2, 5), replace=False))
        w = rng.dirichlet(np.ones(len(langs)) * 0.7)
        out, size = [], 0
        target = int(rng.integers(20, 250))
        while True:
            lang = langs[rng.choice(len(langs), p=w)]
            word = vocab[lang][rng.integers(len(vocab[lang]))]
            b = len(word.encode("utf-8")) + 1
            if size + b > target:
                break
            out.append(word)
            size += b
        docs.append(" ".join(out))
    return docs


def test_mixed_language_short_documents(gpu, oracle):
    buf, offs = gpu.pack(mixed_short_docs(40000))
    got = check(gpu, oracle, buf, offs, "mixed-language short documents")
    # the mixture must reach the document-level passes the wave kernel gates
    assert (got["percent3"][:, 1] > 0).sum() > 5000
    assert (~got["is_reliable"].astype(bool)).sum() > 1000


STAGED = r'''
import numpy as np, cld_amd, corpus
from oracle import Oracle
from test_gpu_parity import assert_same
cld_amd.init()
o = Oracle()
b3, o3 = corpus.c3(20000, seed=171)
want = o.detect_batch(b3, o3, threads=16)
got = cld_amd.detect_batch(buf=b3, offsets=o3)
assert_same(got, want, "c3 staged")
st = cld_amd.last_stats(0)
assert st.general_docs == 0 and st.long_docs == 20000, (st.general_docs, st.long_docs)
print("staged ok", st.passes[0], st.passes[1])
'''


def test_staged_long_path_and_its_hand_ons(gpu, oracle):
    """The staged long-document path (cld_long.hip st_spans / st_score /
    st_rep in k_lspan / k_lscore / k_lrep, span-parallel documents in
    k_lgroup / k_lfinish) and the documents it hands to the fused k_long: a
    span block wider than its 2 KB LDS window (a 3 KB word), hundreds of
    spans (span-parallel, passes 1 and 2), more than 1,024 spans, the Squeeze
    restart, pass 2 with Repeats -- in one batch large enough to take the
    staged path (more than 4 documents per fused wave), all equal to the
    oracle and none on the sequential span source.
    Then the store exhausted (CLD_LONG_STORE_MB=1, child process): every
    document the store cannot hold goes to the fused kernel, same results."""
    import subprocess
    import sys
    b3, o3 = corpus.c3(17000, seed=172, page=2048)
    docs = [bytes(b3[o3[i]:o3[i + 1]]) for i in range(17000)]
    b2, o2 = corpus.c2(3000, seed=173)
    docs[5] = b"x" * 3000 + b" " + bytes(b2[o2[0]:o2[40]])                  # one 3 KB word
    docs[9] = " ".join(["ab", "где", "xy", "कि"] * 300).encode()             # ~1200 spans
    docs[11] = ("abc дом " * 500).encode()                                      # many two-script spans (span-parallel)
    docs[13] = corpus.BOILERPLATE * 20 + bytes(b2[o2[0]:o2[30]])             # the Squeeze restart
    # span-parallel documents (more than 48 spans, cld_long.hip "span-parallel
    # scoring"): the words of 16 KB four-script pages shuffled, so scripts
    # alternate every word or few -- hundreds of spans, pass 1 and pass 2
    rng = np.random.default_rng(174)
    bw, ow = corpus.c3(400, seed=175, page=8192)
    for k in range(400):
        w = bytes(bw[ow[k]:ow[k + 1]]).split()
        rng.shuffle(w)
        cut = int(rng.integers(len(w) // 4, len(w)))
        docs[20 + 7 * k] = b" ".join(w[:cut])
    buf, offs = gpu.pack(docs)
    got = check(gpu, oracle, buf, offs, "staged")
    st = gpu.last_stats(0)
    assert st.general_docs == 0, list(st.long_requeue)
    assert st.passes[1] > 1000                                                # pass 2 (Repeats) taken
    env = dict(os.environ, CLD_LONG_STORE_MB="1",
               PYTHONPATH=os.pathsep.join(os.path.join(ROOT, p) for p in ("language-detector_amd", "oracle", "tests")))
    r = subprocess.run([sys.executable, "-c", STAGED], env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0 and "staged ok" in r.stdout, r.stdout[-2000:] + r.stderr[-3000:]
    assert len(got) == len(docs)


def test_documents_over_one_megabyte(gpu, oracle):
    """Documents between 1 and 4 MB (over k_long's kDocCap): the staged path
    writes their spans straight into a worst-case region of its store with the
    letter-stop bitmap there too (cld_long.hip st_spans_big), in a small batch
    and in a large one -- equal to the oracle, none on the sequential span source."""
    rng = np.random.default_rng(181)
    b3, o3 = corpus.c3(260, seed=182)
    b2, o2 = corpus.c2(40000, seed=183)
    big = []
    for k in range(20):
        size = int(rng.integers(1_100_000, 4_000_000))
        if k % 2:
            d = bytes(b3[:size])                                  # four-script pages back to back
        else:
            d = bytes(b2[o2[0]:o2[-1]])[:size]                    # tweets run together
        big.append(d)
    buf, offs = gpu.pack(big)
    check(gpu, oracle, buf, offs, "over 1 MB", threads=16)
    st = gpu.last_stats(0)
    assert st.general_docs == 0, list(st.long_requeue)
    # in a batch large enough for the staged path proper
    docs = [bytes(b2[o2[i]:o2[i + 40]]) for i in range(0, 20000 * 40 // 40, 1)][:20000] + big[:4]
    buf, offs = gpu.pack(docs)
    check(gpu, oracle, buf, offs, "over 1 MB, large batch", threads=16)
    assert gpu.last_stats(0).general_docs == 0
