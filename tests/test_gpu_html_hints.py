"""cld_detect_batch_ex (HTML mode + CLDHints) on the GPU vs the oracle, bit-exact.

The per-document priors come from the product's host hint code
(cld_hint_priors, pinned to the reference's hint code by
tests/test_html_hints.py::test_hint_priors_match_reference); the oracle then
scores each document with the same priors and is_plain_text flag.  HTML
pages are rewritten into plain text on the GPU (cld_html.hip: tags -> one
space, entities decoded, lookahead marks) and scored by the wave / long
kernels; pages the rewrite cannot take are scanned by k_long's sequential
span source (cld_seq.hip).  Hinted plain documents stay on the wave / long kernels,
which add the prior boosts and apply the whacks in their chunk totes.
"""
import numpy as np
import pytest

import corpus
from test_gpu_parity import assert_same

pytestmark = pytest.mark.gpu


def priors_for(gpu, buf, offs, html, hints):
    n = len(offs) - 1
    pr = np.zeros((n, 16), dtype=np.uint32)
    for i in range(n):
        doc = bytes(buf[offs[i]:offs[i + 1]])
        _, pr[i] = gpu.hint_priors(doc, html=html, hints=hints[i] if hints is not None else None)
    return pr


def random_hints(gpu, n, seed):
    rng = np.random.default_rng(seed)
    tags = ["en", "fr", "de", "es", "it", "pt", "nl", "ru", "uk", "id", "ms", "hr", "sr", "bs", "zh", "zh-tw",
            "ja", "mi,en", "da,nb", "cs", "sk", "xx"]
    tlds = ["id", "fr", "de", "ru", "ua", "cn", "tw", "com", "br", "my", "hr", "es"]
    out = []
    for _ in range(n):
        r = rng.random()
        if r < 0.25:
            out.append(gpu.Hints.make())                                   # no hint at all
            continue
        cl = tags[int(rng.integers(0, len(tags)))] if rng.random() < 0.5 else None
        tld = tlds[int(rng.integers(0, len(tlds)))] if rng.random() < 0.4 else None
        enc = int(rng.integers(0, 75)) if rng.random() < 0.3 else gpu.UNKNOWN_ENCODING
        lang = int(rng.integers(0, 100)) if rng.random() < 0.3 else gpu.UNKNOWN_LANGUAGE
        out.append(gpu.Hints.make(cl, tld, enc, lang))
    return out


def test_html_documents(gpu, oracle):
    buf, offs = corpus.html(1500, seed=21)
    n = len(offs) - 1
    got = gpu.detect_batch_ex(buf=buf, offsets=offs, html=True)
    st = gpu.last_stats()
    assert st.general_docs < n // 10                 # the rewritten pages run on the parallel kernels
    pr = priors_for(gpu, buf, offs, True, None)
    assert (pr != 0).any(axis=1).sum() > n // 2      # lang= attributes became priors
    ref = oracle.detect_batch_ex(buf, offs, plain=np.zeros(n, np.uint8), priors=pr, threads=16)
    assert_same(got, ref, "html")
    # HTML mode matters: the plain-text answer differs on some pages
    plain = oracle.detect_batch(buf, offs, threads=16)
    assert (plain["text_bytes"] != ref["text_bytes"]).sum() > n // 2


def test_html_edge_documents(gpu, oracle):
    docs = [b"", b"<", b">", b"&", b"&amp;", b"<html lang='fr'>", b"<!-- unterminated", b"<script>x",
            b"<p>caf&eacute; cr&egrave;me br&ucirc;l&eacute;e</p>" * 20, b"&#x4e2d;&#25991;" * 40,
            b"<style>a{}</style >texto en espa&ntilde;ol " * 30, b"a < b > c & d" * 100,
            b"<meta http-equiv=content-language content=\"de\">Guten Tag " * 30,
            ("<b>" + "русский текст " * 300 + "</b>").encode(),
            b"<html lang=\"mi,en\">" + b"kia ora " * 400]
    buf, offs = gpu.pack(docs)
    n = len(docs)
    got = gpu.detect_batch_ex(buf=buf, offsets=offs, html=True)
    pr = priors_for(gpu, buf, offs, True, None)
    ref = oracle.detect_batch_ex(buf, offs, plain=np.zeros(n, np.uint8), priors=pr)
    assert_same(got, ref, "html edge")


def test_html_rewrite_lookahead_edges(gpu, oracle):
    """The rewrite's exactness edges: a script lookahead from a letter of
    another script onto an entity (decoded to a letter of either script, or
    undecodable and dropped), entities next to tags, runs broken by decoded
    non-letters, characters the HTML lowercaser treats differently, and a
    page past kMaxScriptBytes (its soft limit from page offsets)."""
    parts = ["abc\u03b1&eacute;def", "abc\u03b1&#945;def", "abc\u03b1&#1044;def", "abc\u03b1&bogus;def",
             "abc\u03b1&amp;def", "abc\u03b1&xyz def", "\u0434\u043e\u043c&#x434;\u043c", "\u03b1&&eacute;b",
             "x&lt;b&gt;y", "caf&eacute;<b>cr&egrave;me</b>", "na&iuml;ve&nbsp;text", "&#12354;&#12356;\u3042",
             "ABC&#65;&#x42;C", "\u00c9t\u00e9 &Eacute;t&eacute;", "word&#0;word", "&#55296;x",
             "<a <b>text</b> more", "<!-- c -->d&#101;f"]
    rare = ["\u0130stanbul &#304;zmir", "a&#x10000;b", "\U0001f600 ok"]   # 4-byte / HTML-lowering candidates
    rng = np.random.default_rng(7)
    docs = []
    for k in range(400):
        words = [parts[int(rng.integers(0, len(parts)))] for _ in range(int(rng.integers(1, 40)))]
        if k % 8 == 0:
            words.append(rare[(k // 8) % len(rare)])
        filler = ["le", "chat", "noir", "\u0434\u043e\u043c", "\u03b3\u03b1\u03c4\u03b1", "<i>", "</i>", "&amp;"]
        words += [filler[int(rng.integers(0, len(filler)))] for _ in range(int(rng.integers(0, 60)))]
        rng.shuffle(words)
        docs.append(" ".join(words).encode())
    docs.append(("<p>" + "caf&eacute; " * 4000 + "</p>").encode())        # 56 KB: the soft limit from page offsets
    buf, offs = gpu.pack(docs)
    n = len(docs)
    got = gpu.detect_batch_ex(buf=buf, offsets=offs, html=True)
    st = gpu.last_stats()
    assert st.general_docs < n // 4                # (the 4-byte pages are rewritten too since round 6)
    pr = priors_for(gpu, buf, offs, True, None)
    ref = oracle.detect_batch_ex(buf, offs, plain=np.zeros(n, np.uint8), priors=pr, threads=8)
    assert_same(got, ref, "html rewrite edges")


def test_html_rewrite_large_pages(gpu, oracle):
    """Pages past the LDS stage (kHtmlStage, 8 KB) are rewritten in place in
    HBM, with any number of '<' / '&' bytes (segments of kHtmlCands
    candidates, round 5); pages of kMaxScriptBytes (40,928) and more carry
    each rewritten byte's page offset, from which the span builders take the
    soft limit's raw bytes left -- none takes the sequential kernel."""
    parts = ["abcα&eacute;def", "дом&#x434;м", "x&lt;b&gt;y", "caf&eacute;<b>cr&egrave;me</b>",
             "na&iuml;ve&nbsp;text", "&#12354;&#12356;あ", "<a <b>text</b> more", "<!-- c -->d&#101;f",
             "le chat noir mange la souris grise"]
    docs = [("<p>" + "le chat noir mange la souris grise &amp; " * 500 + "</p>").encode(),         # 21 KB
            ("<p lang=ru>" + "русский текст " * 1200 + "</p>").encode(),  # 30 KB
            (" ".join(parts) + " ").encode() * 45,                                                  # 8.6 KB, 765 candidates
            ("<script>var x = '<p>';</script>" + "der Hund lief die Strasse entlang " * 400).encode(),  # 14 KB, a tag scan in HBM
            ("<div>" + "der Hund l&auml;uft &uuml;ber die Stra&szlig;e <br> " * 300 + "</div>").encode(),  # > kHtmlCands
            ("<p>" + "caf&eacute; " * 4000 + "</p>").encode()]                                       # 56 KB
    assert 8192 < min(len(d) for d in docs) and len(docs[1]) <= 32768
    buf, offs = gpu.pack(docs)
    n = len(docs)
    got = gpu.detect_batch_ex(buf=buf, offsets=offs, html=True)
    st = gpu.last_stats()
    assert st.general_docs == 0
    pr = priors_for(gpu, buf, offs, True, None)
    ref = oracle.detect_batch_ex(buf, offs, plain=np.zeros(n, np.uint8), priors=pr)
    assert_same(got, ref, "html large pages")
    # thousands of candidates: rewritten segment by segment, a tag or entity
    # reached in one segment running into the next
    many = [("<b>der</b> Hund <i>lief</i> &amp; die <span class='x'>Strasse</span> &lt;entlang&gt; " * k).encode()
            for k in (180, 230, 310)]
    many.append(("<p>" + ("<!-- " + "a<b>&amp;" * 300 + " --> le chat &eacute;tait noir ") * 3 + "</p>").encode())
    assert all(d.count(b"<") + d.count(b"&") > 1024 for d in many)
    mb, mo = gpu.pack(many)
    got = gpu.detect_batch_ex(buf=mb, offsets=mo, html=True)
    assert gpu.last_stats().general_docs == 0
    pr = priors_for(gpu, mb, mo, True, None)
    assert_same(got, oracle.detect_batch_ex(mb, mo, plain=np.zeros(len(many), np.uint8), priors=pr), "html candidates")


def soft_limit_pages(n=24, seed=0xC1D20061, big=2):
    """HTML pages past kMaxScriptBytes (41 to 200 KB, and `big` over 1 MB):
    long runs of one language's words (spans up to the soft limit) among tags
    with long attributes and entities, so the raw bytes left differ widely
    from the rewritten ones; some pages switch script partway."""
    rng = np.random.default_rng(seed)
    v = corpus.vocab()
    langs = ["en", "fr", "de", "es", "it", "pl", "cs", "ru", "bg", "el"]
    langs = [l for l in langs if l in v]
    marks = [b"<b>", b"</b>", b"<span class='note' style='color:#336699;font-weight:bold'>", b"</span>",
             b"<a href='http://www.example.com/articles/2013/index.html?id=12345'>", b"</a>", b"<br/>",
             b"<!-- navigation block -->", b"&amp;", b"&eacute;", b"&nbsp;", b"&bogus;", b"&", b"&#233;",
             "дом&&chat ".encode(), "word, &&дом ".encode(), b"x&&y "]
    docs = []
    sizes = list(np.linspace(41000, 200000, n).astype(int)) + [int(x) for x in rng.integers(1_100_000, 1_400_000, big)]
    for target in sizes:
        out, size = [b"<html><body><p>"], 15
        lang = langs[int(rng.integers(0, len(langs)))]
        switch = target * float(rng.uniform(0.3, 0.9)) if rng.random() < 0.4 else None
        markup = float(rng.uniform(0.1, 0.6))          # share of items that are markup
        while size < target:
            if switch is not None and size > switch:
                lang, switch = langs[int(rng.integers(0, len(langs)))], None
            if rng.random() < markup:
                t = marks[int(rng.integers(0, len(marks)))]
            else:
                w = v[lang]
                t = b" ".join(w[int(i)] for i in rng.integers(0, len(w), size=int(rng.integers(1, 6)))) + b" "
            out.append(t)
            size += len(t)
        out.append(b"</p></body></html>")
        docs.append(b"".join(out))
    return docs


def test_html_soft_limit_pages(gpu, oracle):
    """Pages of kMaxScriptBytes (40,928) and more: the span soft limit
    (getonescriptspan.cc:814-819) reads the page's raw bytes left, in both
    regimes (under 2 x kMaxScriptBytes left: half of them; more: the
    constant); the rewrite hands the span builders each byte's page offset
    (cld_html.hip hpos / hgap).  Pages over 1 MB take the staged path's
    worst-case regions.  Equal to the oracle; most pages stay on the parallel
    kernels (a page holding a character whose HTML lowering differs, or a
    4-byte one, is not rewritten)."""
    docs = soft_limit_pages()
    buf, offs = gpu.pack(docs)
    n = len(docs)
    got = gpu.detect_batch_ex(buf=buf, offsets=offs, html=True)
    st = gpu.last_stats()
    pr = priors_for(gpu, buf, offs, True, None)
    ref = oracle.detect_batch_ex(buf, offs, plain=np.zeros(n, np.uint8), priors=pr, threads=8)
    assert_same(got, ref, "html soft limit")
    assert st.general_docs < n // 2, st.general_docs


@pytest.mark.parametrize("cfg,n,seed", [("c2", 20000, 31), ("c3", 300, 32), ("c4", 11000, 33), ("c5", 20000, 34)])
def test_plain_documents_with_hints(gpu, oracle, cfg, n, seed):
    buf, offs = corpus.GENERATORS[cfg](n)
    hints = random_hints(gpu, n, seed=seed)
    got = gpu.detect_batch_ex(buf=buf, offsets=offs, hints=hints)
    st = gpu.last_stats()
    pr = priors_for(gpu, buf, offs, False, hints)
    hinted = int((pr != 0).any(axis=1).sum())
    assert hinted > n // 3
    assert st.general_docs == 0                      # hinted plain documents stay on the parallel kernels
    ref = oracle.detect_batch_ex(buf, offs, priors=pr, threads=16)
    assert_same(got, ref, cfg + " hints")
    # hints change answers (boosts / whacks reach the chunk totes)
    base = oracle.detect_batch(buf, offs, threads=16)
    assert (base["lang3"] != ref["lang3"]).any()


def test_ex_without_hints_is_detect_batch(gpu):
    buf, offs = corpus.c4(5000)
    a = gpu.detect_batch(buf=buf, offsets=offs)
    ga = gpu.last_stats().general_docs
    b = gpu.detect_batch_ex(buf=buf, offsets=offs)
    assert_same(b, a, "ex == batch")
    assert gpu.last_stats().general_docs == ga
