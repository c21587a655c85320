"""Step-by-step GPU check of the long-document path with progress prints and a
Python stack dump if a step stalls (faulthandler)."""
import faulthandler, json, os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "language-detector_amd")); sys.path.insert(0, os.path.join(ROOT, "oracle"))
import cld_amd, corpus
from oracle import Oracle

faulthandler.dump_traceback_later(40, repeat=True)
FIELDS = ("lang3", "summary_lang", "percent3", "is_reliable", "text_bytes", "normalized3")


def run(name, docs, ob):
    buf, offs = cld_amd.pack(docs)
    print("[%s] gpu start n=%d bytes=%d" % (name, len(docs), len(buf)), flush=True)
    t = time.time()
    g = cld_amd.detect_batch(buf=buf, offsets=offs)
    st = cld_amd.last_stats(0)
    print("[%s] gpu done %.2fs short=%d long=%d general=%d passes=%s ms=%.2f/%.2f/%.2f why=%s" % (
        name, time.time() - t, st.short_docs, st.long_docs, st.general_docs, list(st.passes), st.short_ms,
        st.long_ms, st.general_ms, list(st.long_requeue)), flush=True)
    t = time.time()
    r = ob.detect_batch(buf, offs, threads=16)
    print("[%s] oracle done %.2fs" % (name, time.time() - t), flush=True)
    bad = set()
    for f in FIELDS:
        m = (g[f] != r[f]).reshape(len(g), -1).any(axis=1)
        bad |= set(np.nonzero(m)[0].tolist())
    print("[%s] mismatches %d" % (name, len(bad)), flush=True)
    for i in sorted(bad)[:6]:
        print("   doc", i, "len", len(docs[i]), docs[i][:60], "\n    gpu", g[i], "\n    ref", r[i], flush=True)
    return len(bad)


def main():
    cld_amd.init()
    ob = Oracle()
    sel = sys.argv[1:] or ["single", "fixtures", "long", "c5", "c3"]
    nbad = 0
    if "single" in sel:
        for d in [b"x" * 300, ("hello world this is english text " * 12).encode()]:
            nbad += run("single", [d], ob)
    if "fixtures" in sel:
        g = json.load(open(os.path.join(ROOT, "tests/golden/cld2_unittest.json")))
        docs = [bytes.fromhex(t["text_hex"]) for t in g["test_pairs"]]
        kats = json.load(open(os.path.join(ROOT, "tests/golden/main_test.json")))["kats"]
        docs += [k["text"].encode() for k in kats]
        docs += [b"", b" ", b"a", b"\xc3", b"\xff\xfe", b"Hello, World!", "Ünïcödé ÀÉÎ".encode(), b"x" * 300,
                 b"ab " * 2000]
        nbad += run("fixtures", docs, ob)
    if "long" in sel:
        b2, o2 = corpus.c2(4000, seed=11)
        docs = [("aaaa bbbb cccc " * 400).encode(), (" ".join(["w%d" % i for i in range(2000)])).encode(),
                bytes(b2[o2[0]:o2[300]]), bytes(b2[o2[0]:o2[500]])]
        b3, o3 = corpus.c3(4, page=65536)
        docs += [bytes(b3[o3[i]:o3[i + 1]]) for i in range(4)]
        b4, o4 = corpus.c4(400)
        docs.append(bytes(b4[o4[0]:o4[-1]]))
        nbad += run("long", docs, ob)
    for name, n in (("c5", 20000), ("c3", 2000)):
        if name in sel:
            b, o = corpus.GENERATORS[name](n, seed=corpus.SEEDS[name] + 1)
            nbad += run(name, [bytes(b[o[i]:o[i + 1]]) for i in range(n)], ob)
    print("TOTAL MISMATCHES", nbad, flush=True)


main()
