"""Deterministic synthetic corpora for the BASELINE.json configurations.

Word vocabularies (data/vocab.json) are the whole-word training tokens of the
reference's octagram tables (see tools/synth_quad.py); CJK character pools
(data/cjk_charsets.json) are the characters of the reference unit-test CJK
documents (unittest_data.h kTeststr_{zh_Hans,zh_Hant,ja_Hani,ko_Hani}).

  c2  n x U[100,180] B tweets, >= 10 Latin-script languages, 10% capitalised
      words, 5% digit/punctuation tokens                       
  c3  n x 16384 B pages: four ~4 KB paragraphs in Latin / Cyrillic / Arabic /
      Devanagari languages in random order; a stated fraction (mono_frac,
      default 1/4) of pages is four paragraphs of ONE language instead, which
      finishes in pass 1 -- the rest need the Repeats pass      
  c4  zh-Hans/zh-Hant/ja/ko documents: 10 of every 11 ~150 B, 1 in 11 ~4 KB
      (1.1M docs = 1M x 150 B + 100K x 4 KB)                     
  c5  lognormal lengths (median 140 B, cap 64 KB) mixing c2..c4

All generators are vectorised numpy and return (buf uint8[], offsets uint64[n+1]).
"""
import json
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
SEEDS = {"c2": 0xC1D20002, "c3": 0xC1D20003, "c4": 0xC1D20004, "c5": 0xC1D20005, "c2n": 0xC1D20012}

C2_LANGS = ["en", "fr", "de", "es", "it", "pt", "nl", "sv", "da", "no", "fi", "pl", "cs", "ro", "hu", "tr"]
C3_SCRIPTS = {
    "Latn": ["en", "fr", "de", "es", "it", "pt", "nl", "pl", "cs", "sv"],
    "Cyrl": ["ru", "uk", "bg", "sr", "mk", "kk"],
    "Arab": ["ar", "fa", "ur"],
    "Deva": ["hi", "mr", "ne"],
}
PUNCT_TOKENS = ["2013", "12", "3.5", "(c)", "--", "1998", "#1", "100%", "...", "!", "?", "&", ":)", "9:30", "2,000"]

_vocab = None


def vocab():
    global _vocab
    if _vocab is None:
        with open(os.path.join(HERE, "data", "vocab.json"), encoding="utf-8") as f:
            _vocab = {k: [w.encode("utf-8") for w in v] for k, v in json.load(f).items()}
    return _vocab


class WordTable:
    """Concatenated 'word ' entries of several languages for vectorised assembly."""

    def __init__(self, lang_words):
        self.langs = list(lang_words)
        entries, self.lo, self.cnt = [], [], []
        for lang in self.langs:
            ws = lang_words[lang]
            self.lo.append(len(entries))
            self.cnt.append(len(ws))
            entries += [w + b" " for w in ws]
        self.punct_lo = len(entries)
        entries += [p.encode() + b" " for p in PUNCT_TOKENS]
        self.punct_cnt = len(PUNCT_TOKENS)
        self.lens = np.array([len(e) for e in entries], dtype=np.int64)
        self.starts = np.zeros(len(entries), dtype=np.int64)
        np.cumsum(self.lens[:-1], out=self.starts[1:])
        self.bytes = np.frombuffer(b"".join(entries), dtype=np.uint8)
        self.lo = np.array(self.lo, dtype=np.int64)
        self.cnt = np.array(self.cnt, dtype=np.int64)
        first = self.bytes[self.starts]
        self.capitalisable = (first >= ord("a")) & (first <= ord("z"))


def _assemble(rng, table, lang_idx, targets, kmax, cap_frac=0.10, punct_frac=0.05, pad_to=None):
    """Per document: words of its language until the next word would pass
    target bytes (at least one word).  Returns per-document byte arrays packed."""
    n = len(lang_idx)
    u = rng.random((n, kmax), dtype=np.float32)
    widx = table.lo[lang_idx][:, None] + np.minimum((u * table.cnt[lang_idx][:, None]).astype(np.int64),
                                                    table.cnt[lang_idx][:, None] - 1)
    if punct_frac:
        p = rng.random((n, kmax), dtype=np.float32) < punct_frac
        pi = rng.integers(0, table.punct_cnt, size=(n, kmax))
        widx = np.where(p, table.punct_lo + pi, widx)
    wl = table.lens[widx]
    cum = np.cumsum(wl, axis=1)
    m = np.maximum(1, (cum <= targets[:, None]).sum(axis=1))
    keep = np.arange(kmax)[None, :] < m[:, None]
    sel = widx[keep]                                   # row-major: doc order, word order
    seg = table.lens[sel]
    doc_bytes = cum[np.arange(n), m - 1]
    total = int(seg.sum())
    seg_start = np.zeros(len(sel), dtype=np.int64)
    np.cumsum(seg[:-1], out=seg_start[1:])
    src = np.repeat(table.starts[sel] - seg_start, seg) + np.arange(total, dtype=np.int64)
    out = table.bytes[src].copy()
    if cap_frac:
        c = (rng.random(len(sel), dtype=np.float32) < cap_frac) & table.capitalisable[sel]
        out[seg_start[c]] -= 32
    offs = np.zeros(n + 1, dtype=np.uint64)
    np.cumsum(doc_bytes, out=offs[1:])
    if pad_to is not None:                             # pad every document with spaces to pad_to bytes
        padded = np.full(n * pad_to, ord(" "), dtype=np.uint8)
        dst = np.repeat(np.arange(n, dtype=np.int64) * pad_to - offs[:-1].astype(np.int64), doc_bytes) + \
            np.arange(total, dtype=np.int64)
        padded[dst] = out
        return padded, np.arange(n + 1, dtype=np.uint64) * pad_to
    return out, offs


def c2(n, seed=SEEDS["c2"]):
    rng = np.random.default_rng(seed)
    v = vocab()
    table = WordTable({l: v[l] for l in C2_LANGS if l in v})
    lang_idx = rng.integers(0, len(table.langs), size=n)
    targets = rng.integers(100, 181, size=n)
    return _assemble(rng, table, lang_idx, targets, kmax=48)


BOILERPLATE = b"home | news | contact | login | "


C3_MONO_FRAC = float(os.environ.get("CLD_C3_MONO_FRAC", "0.25"))   # (override: experiments only)


def c3(n, seed=SEEDS["c3"], page=16384, boiler_frac=0.0, mono_frac=C3_MONO_FRAC):
    """Four paragraphs per page, one per script (random order, random language
    of that script), each ~page/4 bytes; pages padded with spaces to `page`.
    mono_frac: in that fraction of pages (seeded, drawn after everything else,
    so the other pages do not change with it) all four paragraphs are one
    language of one script: those pages are reliable and >= 70% one language
    after pass 1 and finish there (compact_lang_det_impl.cc:1978-1991), the
    four-script pages never are and take pass 2 (Repeats).
    boiler_frac: in that fraction of pages (seeded) the Latin paragraph opens
    with ~1 KB of repeated navigation boilerplate, which trips
    CheapSqueezeTriggerTest (compact_lang_det_impl.cc:952-971) and makes the
    document take the Squeeze passes."""
    rng = np.random.default_rng(seed)
    v = vocab()
    scripts = list(C3_SCRIPTS)
    tables = {s: WordTable({l: v[l] for l in C3_SCRIPTS[s] if l in v}) for s in scripts}
    para = page // 4 - 8
    order = np.argsort(rng.random((n, 4)), axis=1)     # script order per page
    parts = []
    for k in range(4):
        bufs = []
        for si, s in enumerate(scripts):
            rows = np.nonzero(order[:, k] == si)[0]
            t = tables[s]
            li = rng.integers(0, len(t.langs), size=len(rows))
            tg = rng.integers(para - 256, para + 1, size=len(rows))
            b, o = _assemble(rng, t, li, tg, kmax=para // 3, punct_frac=0.02)
            bufs.append((rows, b, o))
        parts.append(bufs)
    # stitch: page = para0 + para1 + para2 + para3, then pad
    lens = np.zeros((n, 4), dtype=np.int64)
    pieces = [[None] * 4 for _ in range(n)]
    for k in range(4):
        for rows, b, o in parts[k]:
            ol = o.astype(np.int64)
            lens[rows, k] = ol[1:] - ol[:-1]
            for j, r in enumerate(rows):
                pieces[r][k] = b[ol[j]:ol[j + 1]]
    out = np.full(n * page, ord(" "), dtype=np.uint8)
    boiler = np.zeros(n, dtype=bool)
    if boiler_frac:
        boiler[rng.random(n) < boiler_frac] = True
        bp = np.frombuffer(BOILERPLATE * (1024 // len(BOILERPLATE) + 1), dtype=np.uint8)[:1024]
    if mono_frac:
        mrng = np.random.default_rng(seed ^ 0x6D6F6E6F)
        mono = np.nonzero(mrng.random(n) < mono_frac)[0]
        ms = mrng.integers(0, len(scripts), size=len(mono))
        for si, sname in enumerate(scripts):
            rows = mono[ms == si]
            if not len(rows):
                continue
            t = tables[sname]
            li = mrng.integers(0, len(t.langs), size=len(rows))
            for k in range(4):
                tg = mrng.integers(para - 256, para + 1, size=len(rows))
                b, o = _assemble(mrng, t, li, tg, kmax=para // 3, punct_frac=0.02)
                ol = o.astype(np.int64)
                for j, r in enumerate(rows):
                    pieces[r][k] = b[ol[j]:ol[j + 1]]
            order[rows] = np.where(si == 0, 0, 1)          # (the boilerplate goes first on a Latin page)
    latin = np.argmax(order == 0, axis=1)              # slot of the Latin paragraph
    for r in range(n):
        ps = list(pieces[r])
        if boiler[r]:
            ps.insert(int(latin[r]), bp)
        doc = np.concatenate(ps)[:page]
        out[r * page:r * page + len(doc)] = doc
    return out, np.arange(n + 1, dtype=np.uint64) * page


_cjk = None


def cjk_pools():
    global _cjk
    if _cjk is None:
        with open(os.path.join(HERE, "data", "cjk_charsets.json"), encoding="utf-8") as f:
            _cjk = {k: [c.encode("utf-8") for c in v] for k, v in json.load(f).items()}
    return _cjk


def _interleave(mask, a, b):
    """Packed set a (rows where mask is False) and b (rows where True), in row order."""
    (ba, oa), (bb, ob) = a, b
    n = len(mask)
    lens = np.zeros(n, dtype=np.int64)
    lens[~mask] = np.diff(oa.astype(np.int64))
    lens[mask] = np.diff(ob.astype(np.int64))
    offs = np.zeros(n + 1, dtype=np.uint64)
    np.cumsum(lens, out=offs[1:])
    out = np.empty(int(offs[-1]), dtype=np.uint8)
    for m, (buf, o) in ((~mask, a), (mask, b)):
        rows = np.nonzero(m)[0]
        src_start = o[:-1].astype(np.int64)
        l = lens[rows]
        total = int(l.sum())
        if total == 0:
            continue
        seg = np.zeros(len(rows), dtype=np.int64)
        np.cumsum(l[:-1], out=seg[1:])
        rel = np.arange(total, dtype=np.int64) - np.repeat(seg, l)
        out[np.repeat(offs[rows].astype(np.int64), l) + rel] = buf[np.repeat(src_start, l) + rel]
    return out, offs


def c4(n, seed=SEEDS["c4"], lo=120, hi=180, long_every=11, long_lo=3800, long_hi=4300):
    """CJK 'words' are runs of 2-6 characters from the language's pool; one
    document in `long_every` (at seeded random positions) is ~4 KB, which
    takes the long-document kernel's CJK rounds (SURVEY 8d C4's 100K x 4 KB)."""
    rng = np.random.default_rng(seed)
    pools = cjk_pools()
    words = {}
    for lang, chars in pools.items():
        r = np.random.default_rng(seed ^ sum(lang.encode()))
        ws = set()
        while len(ws) < 400:
            k = int(r.integers(2, 7))
            ws.add(b"".join(chars[int(i)] for i in r.integers(0, len(chars), size=k)))
        words[lang] = sorted(ws)
    table = WordTable(words)
    lang_idx = rng.integers(0, len(table.langs), size=n)
    targets = rng.integers(lo, hi + 1, size=n)
    nl = n // long_every if long_every else 0
    long_mask = np.zeros(n, dtype=bool)
    if nl:
        long_mask[rng.choice(n, size=nl, replace=False)] = True
    short = _assemble(rng, table, lang_idx[~long_mask], targets[~long_mask], kmax=40, cap_frac=0.0, punct_frac=0.03)
    if not nl:
        return short
    lt = rng.integers(long_lo, long_hi + 1, size=nl)
    longs = _assemble(rng, table, lang_idx[long_mask], lt, kmax=long_hi // 7 + 8, cap_frac=0.0, punct_frac=0.03)
    return _interleave(long_mask, short, longs)


def c5(n, seed=SEEDS["c5"], cap=65536):
    """Lognormal lengths (median 140 B, p99 ~16 KB): tweets from c2/c4 pools,
    long documents from c3-style pages truncated to length."""
    rng = np.random.default_rng(seed)
    sigma = np.log(16384 / 140) / 2.326
    lens = np.minimum(cap, np.maximum(8, np.exp(np.log(140) + sigma * rng.standard_normal(n)))).astype(np.int64)
    short = lens <= 1024
    docs = [None] * n
    si = np.nonzero(short)[0]
    li = np.nonzero(~short)[0]
    b2, o2 = c2(len(si), seed=seed + 1)
    o2 = o2.astype(np.int64)
    for j, r in enumerate(si):
        docs[r] = b2[o2[j]:o2[j + 1]][:lens[r]]
    if len(li):
        pages = max(1, int(np.ceil(lens[li].max() / 16384)))
        b3, o3 = c3(len(li), seed=seed + 2, page=16384 * pages)
        o3 = o3.astype(np.int64)
        for j, r in enumerate(li):
            docs[r] = b3[o3[j]:o3[j] + lens[r]]
    offs = np.zeros(n + 1, dtype=np.uint64)
    np.cumsum([len(d) for d in docs], out=offs[1:])
    return np.concatenate(docs) if n else np.zeros(0, np.uint8), offs


HTML_TAGS = [b"p", b"div", b"span", b"b", b"i", b"em", b"td", b"tr", b"li", b"h1", b"h2", b"a", b"font", b"br"]
HTML_ENTITIES = [b"&amp;", b"&lt;", b"&gt;", b"&quot;", b"&nbsp;", b"&eacute;", b"&Eacute;", b"&uuml;", b"&ntilde;",
                 b"&copy;", b"&#233;", b"&#xE9;", b"&#1044;", b"&#x4e2d;", b"&#20013;", b"&mdash;", b"&hellip;",
                 b"&rsquo;", b"&bogus;", b"&", b"&#;", b"&#x;", b"&#65;", b"&#0000000065;", b"&#123456789;",
                 b"&lang", b"&lang;", b"&amp", b"&auml", b"&#150;", b"&#xFFFE;", b"&#55296;"]


# 4-byte characters for HTML pages (emoji, CJK extension B letters, Gothic and
# mathematical alphanumeric letters), raw and as numeric entities
FOUR_BYTE = ["\U0001F600", "\U0001F389", "\U0001F44D", "\u2764\uFE0F", "\U0001F1EB\U0001F1F7", "\U00020000",
             "\U00020B9F\U0002A6A5", "\U00010330\U00010331\U00010332", "\U0001D400\U0001D401", "\U0001F4AF!"]
FOUR_BYTE_ENT = [b"&#x1F600;", b"&#128512;", b"&#x20000;", b"&#x1D41A;", b"&#X1F389", b"&#x10330;"]


def html(n, seed=0xC1D20006, lo=200, hi=6000, emoji=0.0):
    """HTML pages for the is_plain_text=false path (no BASELINE config names
    it): words of one c2/c3 language wrapped in tags, with
    <script>/<style>/<!-- --> blocks, quoted attributes (some with CR/LF),
    lang= / meta content-language attributes, named and numeric entities, and
    stray '<' / '>' -- every construct the reference's tag parser and entity
    reader distinguish (getonescriptspan.cc:150-541).  emoji: the fraction of
    pages that also carry 4-byte characters (FOUR_BYTE, raw and as entities)
    between their words."""
    rng = np.random.default_rng(seed)
    v = vocab()
    langs = [l for l in C2_LANGS + sum(C3_SCRIPTS.values(), []) if l in v]
    docs = []
    for _ in range(n):
        lang = langs[int(rng.integers(0, len(langs)))]
        words = v[lang]
        target = int(rng.integers(lo, hi))
        out = [b"<html lang=\"" + lang.encode() + b"\"><head><title>"]
        if rng.random() < 0.3:
            out.append(b'<meta http-equiv="content-language" content="' + lang.encode() + b'">')
        four = emoji > 0 and rng.random() < emoji
        while sum(map(len, out)) < target:
            r = rng.random()
            if four and rng.random() < 0.08:
                if rng.random() < 0.75:
                    t = FOUR_BYTE[int(rng.integers(0, len(FOUR_BYTE)))].encode("utf-8")
                    out.append(t + (b" " if rng.random() < 0.6 else b""))
                else:
                    out.append(FOUR_BYTE_ENT[int(rng.integers(0, len(FOUR_BYTE_ENT)))])
            elif r < 0.55:
                k = int(rng.integers(1, 9))
                ws = [words[int(i)] for i in rng.integers(0, len(words), size=k)]
                if rng.random() < 0.2:
                    ws[0] = ws[0][:1].upper() + ws[0][1:]
                out.append(b" ".join(ws) + b" ")
            elif r < 0.70:
                t = HTML_TAGS[int(rng.integers(0, len(HTML_TAGS)))]
                if rng.random() < 0.3:
                    t = t.upper()
                attr = b""
                if rng.random() < 0.3:
                    q = b'"' if rng.random() < 0.7 else b"'"
                    val = b"x > y" if rng.random() < 0.3 else (b"a\nb" if rng.random() < 0.2 else b"cls")
                    attr = b" class=" + q + val + q
                out.append(b"<" + t + attr + b">" if rng.random() < 0.6 else b"</" + t + b">")
            elif r < 0.80:
                out.append(HTML_ENTITIES[int(rng.integers(0, len(HTML_ENTITIES)))])
            elif r < 0.85:
                body = b" ".join(words[int(i)] for i in rng.integers(0, len(words), size=3))
                kind = int(rng.integers(0, 4))
                if kind == 0:
                    out.append(b"<script type=\"text/javascript\">var s = '<b>" + body + b"</b>';</script>")
                elif kind == 1:
                    out.append(b"<STYLE>p { color: red } " + body + b"</STYLE >")
                elif kind == 2:
                    out.append(b"<!-- " + body + b" <b> -- -->")
                else:
                    out.append(b"<script>" + body + b"</scrip t>" + body + b"</script>")
            elif r < 0.90:
                out.append([b" < ", b" > ", b"<<", b"a<b", b"<!", b"<!-", b"<x '", b"\r\n", b"1 < 2 > 0", b"<>"][int(rng.integers(0, 10))])
            else:
                out.append(b"<span lang='" + lang.encode() + b"'>")
        if rng.random() < 0.8:
            out.append(b"</body></html>")
        docs.append(b"".join(out))
    offs = np.zeros(n + 1, dtype=np.uint64)
    np.cumsum([len(d) for d in docs], out=offs[1:])
    return (np.frombuffer(b"".join(docs), dtype=np.uint8).copy() if n else np.zeros(0, np.uint8)), offs


def c2n(n, seed=SEEDS["c2n"]):
    """C2's tweets with every ASCII letter of a document shifted by the same
    random non-zero amount (a Caesar shift per document): the same lengths,
    scripts and word shapes, but words the tables never saw -- nearly every
    quadgram probe misses and lands on a uniformly random bucket, so the probe
    gathers see the whole quad table (table-size sensitivity, DESIGN.md
    section 7; not a BASELINE config)."""
    buf, offs = c2(n, seed=seed)
    rng = np.random.default_rng(seed + 1)
    k = rng.integers(1, 26, size=n).astype(np.int16)
    per = np.repeat(k, np.diff(offs).astype(np.int64))
    b = buf.astype(np.int16)
    lo = (b >= 97) & (b <= 122)
    up = (b >= 65) & (b <= 90)
    b[lo] = (b[lo] - 97 + per[lo]) % 26 + 97
    b[up] = (b[up] - 65 + per[up]) % 26 + 65
    return b.astype(np.uint8), offs


GENERATORS = {"c2": c2, "c3": c3, "c4": c4, "c5": c5, "c2n": c2n}
