"""HTML mode and hints, pinned to the reference itself.

oracle/refscan links the reference's own scanner, entity and hint-code
translation units (no scoring table is needed for these stages, so they run
here without any stand-in).  The oracle's restatement must reproduce, on
seeded HTML-like input:
  * every span ScriptScanner::GetOneScriptSpanLower emits (script + lowered
    text), in HTML mode and in plain-text mode;
  * ScanToPossibleLetter's advance for tag-like fragments;
  * ReadEntity's value and length for entity-like fragments;
and the product's host hint code (cld_hint_priors, C ABI) must build the
same CLDLangPriors as the reference's hint code.  Detection results with HTML
and hints are then checked GPU vs oracle by the -m gpu tests.
"""
import ctypes
import os
import struct
import subprocess

import numpy as np
import pytest

import corpus

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REFSCAN = os.path.join(ROOT, "oracle", "_ref", "refscan")
HAVE_REF = os.path.isdir("/root/reference/cld2/internal")
needs_ref = pytest.mark.skipif(not HAVE_REF, reason="reference sources absent")


def refscan(mode, records, *args):
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle", "refscan")], check=True)
    inp = b"".join(struct.pack("<I", len(r)) + r for r in records)
    r = subprocess.run([REFSCAN, mode, *map(str, args)], input=inp, capture_output=True, check=True)
    return r.stdout


def parse_spans(out, n):
    res, p = [], 0
    for _ in range(n):
        (k,) = struct.unpack_from("<I", out, p); p += 4
        spans = []
        for _ in range(k):
            sc, tb = struct.unpack_from("<II", out, p); p += 8
            spans.append((sc, out[p:p + tb])); p += tb
        res.append(spans)
    return res


TRACE = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_char_p)


def oracle_spans(oracle, doc, plain):
    lines = []
    cb = TRACE(lambda _a, s: lines.append(s.decode()))
    oracle.lib.cldo_scan_spans.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, TRACE, ctypes.c_void_p]
    oracle.lib.cldo_scan_spans(doc, len(doc), int(plain), cb, None)
    out = []
    for l in lines:
        sc, _, hx = l.partition(" ")
        out.append((int(sc), bytes.fromhex(hx)))
    return out


def fragments(rng, n):
    """Tag- and entity-like byte strings: mutations of HTML constructs."""
    pieces = [b"<", b">", b"!", b"-", b'"', b"'", b"/", b"script", b"SCRIPT", b"style", b"Style", b"\n", b"\r",
              b" ", b"a", b"x=1", b"<!--", b"-->", b"</script>", b"</style>", b"</ script>", b"</scr", b"&", b";",
              b"#", b"x", b"12", b"0000", b"amp", b"eacute", b"lang", b"\xc3\xa9", b"\xe4\xb8\xad", b"\x00", b"="]
    out = []
    for _ in range(n):
        k = int(rng.integers(1, 14))
        out.append(b"".join(pieces[int(i)] for i in rng.integers(0, len(pieces), size=k)))
    return out


@needs_ref
@pytest.mark.parametrize("plain", [0, 1])
def test_html_spans_match_reference(oracle, plain):
    buf, offs = corpus.html(400, seed=99)
    docs = [bytes(buf[offs[i]:offs[i + 1]]) for i in range(400)]
    rng = np.random.default_rng(5)
    docs += [b" ".join(fragments(rng, 30)) for _ in range(200)]
    ref = parse_spans(refscan("spans", docs, plain), len(docs))
    n = 0
    for d, want in zip(docs, ref):
        got = oracle_spans(oracle, d, plain)
        assert got == want, d[:200]
        n += len(want)
    assert n > 1000


@needs_ref
def test_tag_parser_matches_reference(oracle):
    rng = np.random.default_rng(6)
    frs = [b"<" + f for f in fragments(rng, 20000)]
    out = np.frombuffer(refscan("tags", frs), dtype=np.int32)
    oracle.lib.cldo_scan_tag.argtypes = [ctypes.c_char_p, ctypes.c_int]
    got = [oracle.lib.cldo_scan_tag(f + b"\0" * 16, len(f)) for f in frs]
    assert got == out.tolist()
    assert len(set(got)) > 20


@needs_ref
def test_entity_reader_matches_reference(oracle):
    rng = np.random.default_rng(7)
    frs = [b"&" + f for f in fragments(rng, 20000)] + [e for e in corpus.HTML_ENTITIES]
    out = np.frombuffer(refscan("entities", frs), dtype=np.int32).reshape(-1, 2)
    oracle.lib.cldo_read_entity.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
    c = ctypes.c_int()
    got = []
    for f in frs:
        v = oracle.lib.cldo_read_entity(f + b"\0" * 16, len(f), ctypes.byref(c))
        got.append((v, c.value))
    assert got == [tuple(x) for x in out.tolist()]
    assert sum(1 for v, _ in got if v > 0) > 500


LANG_TAGS = ["en", "en-us", "EN-GB", "fr", "fr-ca", "de", "de-ch", "zh", "zh-tw", "zh-hant", "zh-cn", "pt-br",
             "es-419", "sr-latn", "nb", "no", "mi", "ja", "ko", "ru", "uk", "be", "id", "ms", "hr", "bs", "sr",
             "xx", "x-klingon", "tl", "fil", "iw", "he", "ar", "fa", "hi"]
TLDS = ["id", "fr", "de", "ru", "cn", "tw", "com", "uk", "xx", "jp", "br", "ch", "be", "ua", "by", "my", "hr",
        "ba", "rs", "org", "ID", "Fr"]


def hint_cases(seed, n):
    """(html body or b'', content-language, tld, encoding, language) tuples."""
    rng = np.random.default_rng(seed)
    pick = lambda xs: xs[int(rng.integers(0, len(xs)))]
    cases = []
    for _ in range(n):
        html = b""
        if rng.random() < 0.5:
            parts = [b"<html"]
            if rng.random() < 0.7:
                parts.append(b' lang="%s"' % pick(LANG_TAGS).encode())
            parts.append(b"><head>")
            if rng.random() < 0.4:
                parts.append(b'<meta http-equiv="Content-Language" content="%s">' % pick(LANG_TAGS).encode())
            if rng.random() < 0.3:
                parts.append(b"<meta name=language content='%s'>" % pick(LANG_TAGS).encode())
            if rng.random() < 0.3:
                parts.append(b"<p xml:lang='%s,%s'>x</p>" % (pick(LANG_TAGS).encode(), pick(LANG_TAGS).encode()))
            if rng.random() < 0.2:
                parts.append(b'<a lang="%s" href=x>' % pick(LANG_TAGS).encode())   # skipped tag kind
            parts.append(b"</head><body>texte du document</body></html>")
            html = b"".join(parts)
        cl = b""
        if rng.random() < 0.4:
            k = int(rng.integers(1, 4))
            cl = ",".join(pick(LANG_TAGS) for _ in range(k)).encode()
        tld = pick(TLDS).encode() if rng.random() < 0.4 else b""
        enc = int(rng.integers(0, 75)) if rng.random() < 0.4 else 23
        lang = int(rng.integers(0, 165)) if rng.random() < 0.3 else 26
        cases.append((html, cl, tld, enc, lang))
    return cases


@needs_ref
def test_hint_priors_match_reference():
    """cld_hint_priors (the product's host hint code) builds the same
    CLDLangPriors as the reference's compact_lang_det_hint_code.cc."""
    import cld_amd
    cases = hint_cases(8, 3000)
    recs = []
    for html, cl, tld, enc, lang in cases:
        recs += [html, cl, tld, str(enc).encode(), str(lang).encode()]
    out = refscan("hints", recs)
    p, nonzero = 0, 0
    for html, cl, tld, enc, lang in cases:
        (k,) = struct.unpack_from("<I", out, p); p += 4
        want = list(struct.unpack_from("<%dh" % k, out, p)); p += 2 * k
        h = cld_amd.Hints.make(cl or None, tld or None, enc, lang)
        got, boosts = cld_amd.hint_priors(html, html=bool(html), hints=h)
        assert got.tolist() == want, (html, cl, tld, enc, lang)
        nonzero += bool(want)
        if not want:
            assert not boosts.any()
    assert nonzero > 1500


def test_hint_boosts_shape():
    """ApplyHints' boost/whack split: a language hint boosts its language in the
    Latin ring with weight 8 (kLgProbV2TblBackmap[8] = 28); a close-set member
    (Indonesian / Malay) whacks the others of its set."""
    import cld_amd
    en = 0                                           # ENGLISH
    pri, b = cld_amd.hint_priors(hints=cld_amd.Hints.make(language=en))
    assert pri.tolist() == [(8 << 10) + en]
    assert (b[0] & 0xFF) == 28 and b[1:].sum() == 0
    # .id boosts Indonesian and carries a negative Malay prior: two members of
    # one close set, so no whack (close_set_count == 2)
    pri, b = cld_amd.hint_priors(hints=cld_amd.Hints.make(tld="id"))
    assert len(pri) == 2 and not b[8:].any()
    indonesian = [i for i in range(200) if cld_amd.language_code(i) == "id"][0]
    pri, b = cld_amd.hint_priors(hints=cld_amd.Hints.make(language=indonesian))
    assert b[8:12].any() and not b[12:].any()        # Malay whacked in the Latin ring
