"""First-contact GPU check: HIP path vs oracle on fixtures + synthetic corpora."""
import json, os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "language-detector_amd")); sys.path.insert(0, os.path.join(ROOT, "oracle"))
import cld_amd, corpus
from oracle import Oracle

def compare(name, buf, offs, ob, threads=16):
    t = time.time(); g = cld_amd.detect_batch(buf=buf, offsets=offs); tg = time.time() - t
    st = cld_amd.last_stats(0)
    t = time.time(); r = ob.detect_batch(buf, offs, threads=threads); tc = time.time() - t
    bad = []
    for f in ("lang3", "summary_lang", "percent3", "is_reliable", "text_bytes", "normalized3"):
        a = g[f].astype(np.float64); b = r[f].astype(np.float64)
        m = (a != b).reshape(len(a), -1).any(axis=1)
        bad += list(np.nonzero(m)[0])
    bad = sorted(set(bad))
    print("%-10s n=%-8d mismatches=%-5d gpu_wall=%.3fs cpu=%.3fs short=%d long=%d general=%d passes=%s "
          "kern short/long/general=%.3f/%.3f/%.3f ms"
          % (name, len(offs) - 1, len(bad), tg, tc, st.short_docs, st.long_docs, st.general_docs, list(st.passes),
             st.short_ms, st.long_ms, st.general_ms), flush=True)
    for i in bad[:5]:
        print("   doc", i, bytes(buf[offs[i]:offs[i+1]])[:80], "\n    gpu", g[i], "\n    cpu", r[i])
    return len(bad)

def main():
    cld_amd.init()
    print(cld_amd.lib().cld_version().decode())
    ob = Oracle()
    g = json.load(open(os.path.join(ROOT, "tests/golden/cld2_unittest.json")))
    docs = [bytes.fromhex(t["text_hex"]) for t in g["test_pairs"]]
    kats = json.load(open(os.path.join(ROOT, "tests/golden/main_test.json")))["kats"]
    docs += [k["text"].encode() for k in kats]
    docs += [b"", b" ", b"a", b"\xc3", b"\xff\xfe", b"Hello, World!", "Ünïcödé ÀÉÎ".encode(), b"x" * 300, b"ab " * 2000]
    buf, offs = cld_amd.pack(docs)
    nbad = compare("fixtures", buf, offs, ob)
    for name, n in (("c2", 20000), ("c4", 5000), ("c5", 2000), ("c3", 64)):
        b, o = corpus.GENERATORS[name](n)
        nbad += compare(name, b, o, ob)
    # re-queue paths: squeeze trigger, repeats, 1000-hit rounds, span limits
    b2, o2 = corpus.c2(4000, seed=11)
    long_docs = [("aaaa bbbb cccc " * 400).encode(), (" ".join(["w%d" % i for i in range(2000)])).encode(),
                 bytes(b2[o2[0]:o2[300]]), bytes(b2[o2[0]:o2[500]])]
    b3, o3 = corpus.c3(4, page=65536)
    long_docs += [bytes(b3[o3[i]:o3[i + 1]]) for i in range(4)]
    b4, o4 = corpus.c4(400)
    long_docs.append(bytes(b4[o4[0]:o4[-1]]))
    buf, offs = cld_amd.pack(long_docs)
    nbad += compare("longdocs", buf, offs, ob)
    for name, n in (("c5", 20000), ("c3", 2000)):
        b, o = corpus.GENERATORS[name](n, seed=corpus.SEEDS[name] + 1)
        nbad += compare(name + "b", b, o, ob)
    print("detect_language KATs:", [(k["expected"], cld_amd.detect_language(k["text"])) for k in kats[:6]])
    b, o = corpus.c2(1000000)
    for rep in range(2):
        t = time.time(); cld_amd.detect_batch(buf=b, offsets=o); dt = time.time() - t
        st = cld_amd.last_stats(0)
        print("c2 1M host-path wall %.3fs  %.2f Mdocs/s  kernels short %.3f ms general %.3f ms -> %.2f Mdocs/s kernel-only"
              % (dt, 1e6 / dt / 1e6, st.short_ms, st.general_ms, 1e6 / ((st.short_ms + st.general_ms) / 1e3) / 1e6), flush=True)
    print("TOTAL MISMATCHES", nbad)
    sys.exit(1 if nbad else 0)

main()
