"""HTML-mode fuzz for the GPU box: pages assembled at random from text of the
benchmark corpora and HTML fragments -- tags, unterminated tags, comments,
script/style blocks, entities (named, numeric, broken), lang attributes and
content-language metas, stray '<' '>' '&', malformed UTF-8 -- through
cld_detect_batch_ex (HTML mode) and cld_detect_batch_vec (html=True) against
the oracle with the product's hint priors, or (HTML_REF=1, valid UTF-8 only)
against the reference CLD2 itself.  FUZZ_SEEDS (default 40-45)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("language-detector_amd", "oracle", "tests"):
    sys.path.insert(0, os.path.join(ROOT, p))
import cld_amd  # noqa: E402
import corpus  # noqa: E402
from oracle import Oracle  # noqa: E402
from test_gpu_html_hints import priors_for  # noqa: E402
from test_gpu_vector import vecs, oracle_vecs  # noqa: E402

FIELDS = ("lang3", "summary_lang", "percent3", "is_reliable", "text_bytes", "normalized3")
FRAG = [b"<p>", b"</p>", b"<b>", b"</b>", b"<br/>", b"<!-- c -->", b"<!--", b"-->", b"<script>var x=1;</script>",
        b"<script>", b"</script>", b"<style>p{a:b}</style>", b"<style>", b"&amp;", b"&lt;", b"&gt;", b"&nbsp;",
        b"&eacute;", b"&Eacute;", b"&#233;", b"&#x1F600;", b"&#128512;", b"&#xD800;", b"&#0;", b"&bogus;", b"&#",
        b"&#x", b"&", b"<", b">", b"<a href='x.html'>", b"</a>", b"<html lang=\"de\">", b"<html lang=fr>",
        b"<meta http-equiv=\"content-language\" content=\"es\">", b"<title>t</title>", b"<img alt=\"x\">",
        b"<div lang=ja>", b"</div>", b"<unclosed", b"\"", b"'", b"\xc3", b"\x80", b"\xf0\x9f\x98\x80", b"\xe2\x80\x8b",
        b"\xff", b"\n", b"\t", b" "]
# HTML_REF=1: valid UTF-8 only, and the reference CLD2 itself (its own HTML
# scanner and hint code) is the judge instead of the oracle
REF = os.environ.get("HTML_REF") == "1"
if REF:
    import refcld  # noqa: E402
    FRAG = [f for f in FRAG if f not in (b"\xc3", b"\x80", b"\xff")]
    ref_cld = refcld.instance(cld_amd.SYNTH_TABLES)
out_dir = os.path.join(ROOT, "gpurun_out", "corrupt_diag")
os.makedirs(out_dir, exist_ok=True)
cld_amd.init_device(0, tables=cld_amd.SYNTH_TABLES)
o = Oracle()
total = 0
for seed in (int(s) for s in os.environ.get("FUZZ_SEEDS", "40,41,42,43,44,45").split(",")):
    rng = np.random.default_rng(seed)
    words = []
    for cfg, n in (("c2", 3000), ("c4", 800), ("c5", 800)):
        b, o_ = corpus.GENERATORS[cfg](n, seed=seed)
        for i in range(n):
            words += bytes(b[o_[i]:o_[i + 1]]).split(b" ")[:20]
    pages = []
    for _ in range(3000):
        k = int(rng.choice([1, 5, 20, 80, 300, 1500]))
        parts = []
        for _ in range(k):
            parts.append(FRAG[int(rng.integers(len(FRAG)))] if rng.random() < 0.3 else words[int(rng.integers(len(words)))])
            parts.append(b" " if rng.random() < 0.7 else b"")
        pages.append(b"".join(parts))
    buf, offs = cld_amd.pack(pages)
    n = len(pages)
    got = cld_amd.detect_batch_ex(buf=buf, offsets=offs, html=True)
    st = cld_amd.last_stats(0)
    if REF:
        ref = ref_cld.detect_batch(buf, offs, plain=np.zeros(n, np.uint8), threads=16)
    else:
        pr = priors_for(cld_amd, buf, offs, True, None)
        ref = o.detect_batch_ex(buf, offs, plain=np.zeros(n, np.uint8), priors=pr, threads=16)
    bad = np.zeros(n, bool)
    for f in FIELDS:
        bad |= (got[f].astype(np.float64) != ref[f].astype(np.float64)).reshape(n, -1).any(axis=1)
    idx = np.nonzero(bad)[0]
    total += len(idx)
    for i in idx[:3]:
        with open(os.path.join(out_dir, "html_s%d_d%d.bin" % (seed, i)), "wb") as f:
            f.write(pages[i])
    print("seed %d html: %d pages (max %d B), %d mismatches %s; seq %d" % (seed, n, max(map(len, pages)), len(idx),
                                                                       idx[:5], st.general_docs), flush=True)
    vp = pages[:1200]
    vb, vo = cld_amd.pack(vp)
    g, chunks, coffs = cld_amd.detect_batch_vec(buf=vb, offsets=vo, html=True)
    gv = vecs(chunks, coffs)
    if REF:
        vidx = []
        for i in range(len(vp)):
            rb, cb = ref_cld.detect_vec(vp[i], plain=False)
            if gv[i] != [(int(c["offset"]), int(c["bytes"]), int(c["lang1"])) for c in cb] or \
                    int(g[i]["summary_lang"]) != int(rb["summary_lang"]) or int(g[i]["text_bytes"]) != int(rb["text_bytes"]):
                vidx.append(i)
    else:
        rr, ov = oracle_vecs(o, cld_amd, vb, vo, html=True)
        vidx = [i for i in range(len(vp)) if gv[i] != ov[i] or (int(g[i]["summary_lang"]), list(g[i]["percent3"]),
                int(g[i]["text_bytes"])) != (rr[i].summary_lang, list(rr[i].percent3), rr[i].text_bytes)]
    total += len(vidx)
    for i in vidx[:3]:
        with open(os.path.join(out_dir, "htmlvec_s%d_d%d.bin" % (seed, i)), "wb") as f:
            f.write(vp[i])
    print("seed %d html vec: %d pages, %d mismatches %s" % (seed, len(vp), len(vidx), vidx[:5]), flush=True)
print("total mismatches", total, flush=True)
