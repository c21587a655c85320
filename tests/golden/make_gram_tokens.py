"""Generate tests/golden/gram_tokens.json from the reference's generated tables.

Run in the build container only (reads /root/reference as text).  Every
bucket line of the reference's generated octagram / CJK-bigram tables carries,
in a comment, the training token of each of its four slots, e.g.

    {{0x1682b002,0x53576003,...}},  // [000] _उमराव_, _þremur_, ...
    (cld2_generated_deltaoctachrome.cc:170+, cld2_generated_distinctoctachrome.cc:96+,
     cld_generated_cjk_delta_bi_4.cc:75+)

A fixture row is (CLDT section id, bucket index, token, slot keyvalue): data,
not source.  tests/test_hash_pins.py hashes each token the way GetOctaHits /
GetBiHits would see it in span text and checks that the probe of that table
lands in this bucket and returns this keyvalue.
"""
import json
import os
import re

REF = "/root/reference/cld2/internal"
HERE = os.path.dirname(os.path.abspath(__file__))
TABLES = [  # (file, CLDT section id, array name)
    ("cld2_generated_deltaoctachrome.cc", 15, "kDeltaOctaChrome1015"),
    ("cld2_generated_distinctoctachrome.cc", 16, "kDistinctOctaChrome1015"),
    ("cld_generated_cjk_delta_bi_4.cc", 11, "kCjkDeltaBi"),
]
LINE = re.compile(r"\s*\{\{(0x[0-9a-f]+),(0x[0-9a-f]+),(0x[0-9a-f]+),(0x[0-9a-f]+)\}\},\s*//\s*(?:\[[0-9a-f]+\])?\s*(.*)$")


def rows(fname, sid, array):
    txt = open(os.path.join(REF, fname), encoding="utf-8").read()
    start = txt.index("static const IndirectProbBucket4 %s[" % array)
    out, bucket = [], 0
    for line in txt[start:].splitlines()[1:]:
        if line.strip().startswith("};"):
            break
        m = LINE.match(line)
        if not m:
            continue
        kvs = [int(m.group(i), 16) for i in range(1, 5)]
        toks = [t.strip() for t in m.group(5).rstrip().rstrip(",").split(", ")]
        for kv, tok in zip(kvs, toks):
            if kv and tok and tok != "--":
                out.append([sid, bucket, tok, kv])
        bucket += 1
    return out, bucket


def main():
    fx = {"source": "token comments of %s" % ", ".join(f for f, _, _ in TABLES), "buckets": {}, "rows": []}
    for f, sid, arr in TABLES:
        r, nb = rows(f, sid, arr)
        fx["rows"] += r
        fx["buckets"][str(sid)] = nb
    with open(os.path.join(HERE, "gram_tokens.json"), "w", encoding="utf-8") as f:
        json.dump(fx, f, ensure_ascii=False, separators=(",", ":"))
    print(len(fx["rows"]), fx["buckets"])


if __name__ == "__main__":
    main()
