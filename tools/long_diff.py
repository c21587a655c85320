"""Round-by-round diff of k_long against the oracle for single documents.

Runs each document alone with CLD_DEBUG_DOC=0 (the runtime dumps k_long's hit
buffers and chunk summaries), parses the oracle's trace of the same document
and prints the first differing round / chunk.  Usage on a GPU box:
    python tools/long_diff.py c5:1:73 c3:1:3 ...   (config:seed_offset:index)
"""
import os, re, sys
import numpy as np
os.environ["CLD_DEBUG_DOC"] = "0"
os.environ.setdefault("CLD_DEBUG_OUT", "/tmp/cld_dbg.bin")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "language-detector_amd")); sys.path.insert(0, os.path.join(ROOT, "oracle"))
import cld_amd, corpus
from oracle import Oracle


def gpu_dump(doc):
    cld_amd.detect_batch(docs=[doc])
    w = np.fromfile(os.environ["CLD_DEBUG_OUT"], dtype=np.uint32)
    n, w, i, recs = int(w[0]), w[1:], 0, []
    while i < n:
        t = int(w[i])
        if t == ord('S'):
            recs.append(("S", tuple(int(x) for x in w[i + 1:i + 4]))); i += 4
        elif t == ord('R'):
            off, nxt, nb, nd, nx = (int(x) for x in w[i + 1:i + 6]); i += 6
            pairs = w[i:i + 2 * (nb + nd + nx)].astype(np.int64).reshape(-1, 2); i += 2 * (nb + nd + nx)
            q = [(int(a), int(np.int32(np.uint32(b)))) for a, b in pairs[:nb]]
            d = [tuple(map(int, p)) for p in pairs[nb:nb + nd]]
            x = [tuple(map(int, p)) for p in pairs[nb + nd:]]
            recs.append(("R", (off, nxt, q, d, x)))
        elif t == ord('C'):
            v = [int(x) for x in w[i + 1:i + 18]]; i += 18
            recs.append(("C", v))
        elif t == ord('T'):
            tb = int(np.int32(np.uint32(w[i + 1]))); i += 2 + (max(tb, 0) + 3) // 4
        else:
            raise ValueError("bad record %d at %d" % (t, i))
    return recs


def oracle_rounds(ob, doc):
    _, _, lines = ob.detect(doc, trace=True)
    out, cur = [], None
    for ln in lines:
        if ln.startswith("hitbuffer"):
            cur = {"Q": [], "DL": [], "D": [], "C": []}
            out.append(cur)
        elif cur is not None:
            m = re.match(r"(Q|DL|D)\[(\d+)\](-?\d+),(-?\d+)$", ln)
            if m:
                cur[m.group(1)].append((int(m.group(3)), int(m.group(4))))
                continue
            m = re.match(r"\[(\d+)\] (\d+) lin\[(\d+)\] (\S+)\.(\d+) (\S+)\.(\d+) (\d+)B (\d+)# (\S+) (\d+)Rd (\d+)Rs", ln)
            if m:
                cur["C"].append(m.groups())
        if ln.startswith("recurse"):
            out.append("PASS2")
    return out


def main():
    cld_amd.init()
    ob = Oracle()
    for spec in sys.argv[1:]:
        cfg, so, idx = spec.split(":")
        n = int(idx) + 1
        b, o = corpus.GENERATORS[cfg](max(n, 8), seed=corpus.SEEDS[cfg] + int(so))
        doc = bytes(b[o[int(idx)]:o[int(idx) + 1]])
        recs = gpu_dump(doc)
        orr = [r for r in oracle_rounds(ob, doc) if r != "PASS2"]
        grounds = [r[1] for r in recs if r[0] == "R"]
        gchunks = []
        for r in recs:
            if r[0] == "R": gchunks.append([])
            elif r[0] == "C" and gchunks: gchunks[-1].append(r[1])
        print("== %s len=%d gpu rounds=%d oracle rounds=%d" % (spec, len(doc), len(grounds), len(orr)), flush=True)
        for k, (g, r) in enumerate(zip(grounds, orr)):
            off, nxt, q, d, x = g
            for name, gl, rl in (("Q", q, r["Q"]), ("DL", d, r["DL"]), ("D", x, r["D"])):
                if gl != rl:
                    j = next((j for j in range(min(len(gl), len(rl))) if gl[j] != rl[j]), min(len(gl), len(rl)))
                    print("  round %d (off %d next %d) %s differs: gpu n=%d oracle n=%d first at %d: gpu %s oracle %s"
                          % (k, off, nxt, name, len(gl), len(rl), j, gl[j:j + 3], rl[j:j + 3]))
            gc, rc = gchunks[k], r["C"]
            for j, (a, c) in enumerate(zip(gc, rc)):
                lo, hi, l1, l2, s1, s2, grams, rd, rs = a[:9]
                want = (int(c[1]), int(c[7]), int(c[4]), int(c[6]), int(c[8]), int(c[10]), int(c[11]))
                got = (lo, hi - lo, s1, s2, grams, rd, rs)
                if want != got:
                    print("  round %d chunk %d: gpu (lo,bytes,s1,s2,grams,rd,rs)=%s oracle=%s" % (k, j, got, want))
                    print("     ranges b[%d,%d) d[%d,%d) x[%d,%d) theta=%d eb=%d K=%d; round nb/nd/nx=%d/%d/%d"
                          % tuple(a[9:16] + [a[16] >> 16, a[16] & 0xFFFF, len(g[2]), len(g[3]), len(g[4])]))
                    for jj in range(min(4, len(gc))):
                        print("     chunk", jj, "ranges", gc[jj][9:16])
                    break
            if len(gc) != len(rc):
                print("  round %d: chunk count gpu %d oracle %d" % (k, len(gc), len(rc)))
        sys.stdout.flush()


main()
