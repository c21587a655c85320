"""Pin the gram hashes and bucket probes to the reference (no GPU).

1. The reference's own hash functions: oracle/hashcheck links
   /root/reference/cld2/internal/cldutil_shared.cc (compiled where it lies) and
   compares QuadHashV2 / BiHashV2 / OctaHash40 / PairHash with the oracle on
   1M seeded spans of every length class, both space bits each way.
2. The reference's own table data: every slot of the generated octagram and
   CJK delta-bigram tables names its training token in a comment
   (tests/golden/gram_tokens.json, made by make_gram_tokens.py).  Hashing the
   token as GetOctaHits (cldutil.cc:416-533: whole word "_w_", first 8 chars
   "_w", word pair "_a__b_" -> PairHash) or GetBiHits (cldutil.cc:248-310)
   would, then probing (cldutil_shared.h:380-454), must land in that token's
   bucket and return that slot's keyvalue.
The GPU kernels' hashes are checked against this oracle bit-for-bit by the
-m gpu parity tests, so these pins carry over to the HIP path.
"""
import ctypes
import json
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HASHCHECK = os.path.join(ROOT, "oracle", "_ref", "hashcheck")


@pytest.fixture(scope="module")
def hooks(oracle):
    lib = oracle.lib
    lib.cldo_gram_hash.restype = ctypes.c_uint64
    lib.cldo_gram_hash.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int]
    lib.cldo_pair_hash.restype = ctypes.c_uint64
    lib.cldo_pair_hash.argtypes = [ctypes.c_uint64, ctypes.c_uint64]
    lib.cldo_probe.restype = ctypes.c_uint32
    lib.cldo_probe.argtypes = [ctypes.c_int, ctypes.c_uint64]
    return lib


@pytest.fixture(scope="module")
def tokens():
    with open(os.path.join(ROOT, "tests", "golden", "gram_tokens.json"), encoding="utf-8") as f:
        return json.load(f)


@pytest.mark.skipif(not os.path.isdir("/root/reference/cld2/internal"), reason="reference sources absent")
def test_reference_hash_functions_equal_oracle():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle", "hashcheck")], check=True)
    r = subprocess.run([HASHCHECK, "1000000"], capture_output=True, text=True)
    res = json.loads(r.stdout)
    assert r.returncode == 0, res
    assert res["spans"] == 1000000
    assert res["quad_mismatch"] == res["bi_mismatch"] == res["octa_mismatch"] == res["pair_mismatch"] == 0


def split_words(tok):
    """'_a__b_' -> [('a', True), ('b', True)]; '_navegaci_ferramen' -> two
    8-char prefixes; the bool says whether the word ended (a space follows)."""
    words, i = [], 0
    while i < len(tok):
        assert tok[i] == "_", tok
        j = tok.find("_", i + 1)
        if j < 0:
            words.append((tok[i + 1:], False))
            break
        if j + 1 == len(tok) or tok[j + 1] == "_":
            words.append((tok[i + 1:j], True))
            i = j + 1
        else:
            words.append((tok[i + 1:j], False))
            i = j
    return words


def gram_hash(lib, kind, before, gram, after):
    """Hash `gram` inside span text `before + gram + after` (the hashes read
    one byte before and one after the gram, and over-read up to 3 bytes)."""
    buf = ctypes.create_string_buffer(before + gram + after + b"\0" * 8)
    return lib.cldo_gram_hash(kind, ctypes.addressof(buf) + len(before), len(gram))


def octa_word_hash(lib, word, ended):
    # a whole word is followed by its space; an 8-char prefix by the 9th char
    return gram_hash(lib, 2, b" ", word.encode("utf-8"), b" " if ended else b"x")


def test_split_words():
    assert split_words("_secara__terus_") == [("secara", True), ("terus", True)]
    assert split_words("_se__registri") == [("se", True), ("registri", False)]
    assert split_words("_navegaci_ferramen") == [("navegaci", False), ("ferramen", False)]
    assert split_words("_zastosow") == [("zastosow", False)]


def test_octa_tokens_probe_their_slot(hooks, tokens):
    ok = bad = pairs = 0
    misses = []
    for sid, bucket, tok, kv in tokens["rows"]:
        if sid not in (15, 16):
            continue
        words = split_words(tok)
        if any(not e and len(w) != 8 for w, e in words):
            continue          # not a form GetOctaHits produces (never seen: see count below)
        hs = [octa_word_hash(hooks, w, e) for w, e in words]
        h = hs[0] if len(hs) == 1 else hooks.cldo_pair_hash(hs[0], hs[1])
        pairs += len(hs) == 2
        nb = tokens["buckets"][str(sid)]
        if (h + (h >> 12)) % nb == bucket and hooks.cldo_probe(sid, h) == kv:
            ok += 1
        else:
            bad += 1
            misses.append(tok)
    # all 19,536 listed slots (1,563 of them word pairs) probe exactly
    assert bad == 0, (ok, bad, misses[:20])
    assert ok >= 19_500 and pairs >= 1_500, (ok, pairs)


def test_cjk_bigram_tokens_match_reference_behaviour(hooks, tokens, verbose_golden, oracle):
    """The CJK delta-bigram slots' comment tokens are NOT what BiHashV2 sees at
    run time: the reference's own verbose run (CLD2UnitTestOutputVerbose.html)
    records zero delta-bigram hits on all four CJK documents although they
    contain dozens of the listed bigrams.  The oracle must agree: no listed
    token probes its slot, and the dumped CJK rounds have no delta hits in the
    oracle either (their base/distinct hits are pinned exactly by
    test_oracle_golden)."""
    listed = {t for s, _, t, _ in tokens["rows"] if s == 11}
    assert len(listed) >= 2_400
    landed = 0
    for sid, bucket, tok, kv in tokens["rows"]:
        if sid == 11:
            h = gram_hash(hooks, 1, b" ", tok.encode("utf-8"), b" ")
            landed += hooks.cldo_probe(11, h) == kv
    assert landed == 0
    seen = 0
    for sp in verbose_golden["spans"]:
        if sp["script"] != "Hani":
            continue
        text = sp["span_text"]
        seen += sum(text[i:i + 2] in listed for i in range(len(text) - 1))
        assert sp["rounds"][0]["delta"] == []                      # the reference's run
        _, _, tr = oracle.detect(text.encode("utf-8"), trace=True)
        assert not [l for l in tr if l.startswith("DL[")], sp["doc"]  # the oracle's run
    assert seen >= 30
