"""Valid-UTF-8 fuzz against the reference CLD2 itself (oracle/_ref/librefcld2.so,
which travels with the tree): documents of random code points drawn from many
scripts -- letters, combining marks, digits, punctuation, symbols, emoji and
other 4-byte characters, exotic spaces -- where the reference is defined, so
it is the judge.  VALID_MODE=cpu compares the oracle with it here; on the GPU
box cld_detect_batch (plain, each flag set) and cld_detect_batch_vec are
compared with it.  VALID_SEEDS (default 70-73)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("language-detector_amd", "oracle", "tests"):
    sys.path.insert(0, os.path.join(ROOT, p))
import cld_amd  # noqa: E402
import refcld  # noqa: E402

RANGES = [(0x41, 0x5A), (0x61, 0x7A), (0xC0, 0x24F), (0x300, 0x36F), (0x370, 0x3FF), (0x400, 0x4FF), (0x531, 0x58F),
          (0x5D0, 0x5EA), (0x620, 0x64A), (0x660, 0x669), (0x900, 0x97F), (0x980, 0x9FF), (0xB80, 0xBFF),
          (0xE00, 0xE5B), (0x10A0, 0x10FF), (0x1100, 0x11FF), (0x1E00, 0x1EFF), (0x2000, 0x206F), (0x20A0, 0x20BF),
          (0x2100, 0x214F), (0x3040, 0x30FF), (0x4E00, 0x9FFF), (0xAC00, 0xD7A3), (0xFF01, 0xFF5E),
          (0x1F300, 0x1F6FF), (0x20000, 0x2A6DF), (0x21, 0x2F), (0x30, 0x39)]
WORDS = [0.55, 0.25, 0.2]           # word of one range / mixed / punctuation-space run


def gen(rng, n):
    docs = []
    for _ in range(n):
        L = int(rng.choice([0, 3, 30, 150, 600, 3000, 12000]))
        out = []
        size = 0
        while size < L:
            r = rng.random()
            if r < WORDS[0]:
                a, b = RANGES[int(rng.integers(len(RANGES)))]
                w = "".join(chr(int(rng.integers(a, b + 1))) for _ in range(int(rng.integers(1, 10))))
            elif r < WORDS[0] + WORDS[1]:
                w = "".join(chr(int(rng.integers(*RANGES[int(rng.integers(len(RANGES)))]))) for _ in range(int(rng.integers(1, 8))))
            else:
                w = rng.choice([" ", "  ", ", ", ". ", "\n", " ", "​", "　", "'", "\"", "-", "@x ", "#t "])
            out.append(w + (" " if rng.random() < 0.8 else ""))
            size += len(out[-1].encode("utf-8"))
        docs.append("".join(out).encode("utf-8"))
    return docs


FIELDS = ("lang3", "summary_lang", "percent3", "is_reliable", "text_bytes", "normalized3")


def main():
    mode = os.environ.get("VALID_MODE", "gpu")
    ref = refcld.instance(cld_amd.SYNTH_TABLES)
    if mode == "gpu":
        cld_amd.init_device(0, tables=cld_amd.SYNTH_TABLES)
    else:
        from oracle import Oracle
        o = Oracle()
    total = 0
    for seed in (int(s) for s in os.environ.get("VALID_SEEDS", "70,71,72,73").split(",")):
        rng = np.random.default_rng(seed)
        docs = gen(rng, 3000)
        buf, offs = cld_amd.pack(docs)
        n = len(docs)
        for flags in (0, 0x100, 0x4000):
            got = cld_amd.detect_batch(buf=buf, offsets=offs, flags=flags) if mode == "gpu" else \
                o.detect_batch_ex(buf, offs, flags=flags, threads=8)
            want = ref.detect_batch(buf, offs, threads=16, flags=flags)
            bad = np.zeros(n, bool)
            for f in FIELDS:
                bad |= (got[f].astype(np.float64) != want[f].astype(np.float64)).reshape(n, -1).any(axis=1)
            idx = np.nonzero(bad)[0]
            total += len(idx)
            print("%s seed %d flags %#x: %d docs, %d bytes, %d mismatches %s" % (mode, seed, flags, n, len(buf), len(idx),
                                                                               idx[:5]), flush=True)
        if mode == "gpu":
            vd = docs[:1000]
            vb, vo = cld_amd.pack(vd)
            g, chunks, coffs = cld_amd.detect_batch_vec(buf=vb, offsets=vo)
            vbad = 0
            for i in range(len(vd)):
                rb, cb = ref.detect_vec(vd[i])
                want_v = [(int(c["offset"]), int(c["bytes"]), int(c["lang1"])) for c in cb]
                have_v = [(int(c["offset"]), int(c["bytes"]), int(c["lang1"])) for c in chunks[coffs[i]:coffs[i + 1]]]
                if want_v != have_v or int(g[i]["summary_lang"]) != int(rb["summary_lang"]):
                    vbad += 1
            total += vbad
            print("gpu seed %d vec: %d docs, %d mismatches" % (seed, len(vd), vbad), flush=True)
    print("total mismatches", total, flush=True)


if __name__ == "__main__":
    main()
