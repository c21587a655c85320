"""StripExtras / C-string preparation (cld_detect_batch flags 1-3, handlers.go
:198-210 and wrapper.cc's strlen) on the corrupted corpora
(tests/test_gpu_corrupt.docs_for), with '@user', URLs and NULs mixed in, on
the GPU box: prepared text and results against the oracle's prepare_batch +
detect_batch.  PREP_SEEDS (default 80-83)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("language-detector_amd", "oracle", "tests"):
    sys.path.insert(0, os.path.join(ROOT, p))
import cld_amd  # noqa: E402
from oracle import Oracle  # noqa: E402
import test_gpu_corrupt as tc  # noqa: E402

FIELDS = ("lang3", "summary_lang", "percent3", "is_reliable", "text_bytes", "normalized3")
cld_amd.init_device(0, tables=cld_amd.SYNTH_TABLES)
o = Oracle()
total = 0
for seed in (int(s) for s in os.environ.get("PREP_SEEDS", "80,81,82,83").split(",")):
    rng = np.random.default_rng(seed)
    docs = []
    for d in tc.docs_for(seed, 2000):
        k = int(rng.integers(4))
        if k == 1:
            d = b"@user_" + str(int(rng.integers(1000))).encode() + b" " + d
        elif k == 2:
            d = d + b" https://t.co/" + bytes(rng.integers(97, 123, 8, dtype=np.uint8)) + b" http://x.y/z?q=1"
        elif k == 3 and len(d) > 10:
            p = int(rng.integers(len(d)))
            d = d[:p] + b"\x00" + d[p:]
        docs.append(d)
    buf, offs = cld_amd.pack(docs)
    n = len(docs)
    for flags in (1, 2, 3):
        gb, go = cld_amd.prepare_batch(buf=buf, offsets=offs, flags=flags)
        rb, ro = o.prepare_batch(buf, offs, flags)
        pbad = 0 if np.array_equal(go, ro) else -1
        if pbad == 0:
            pbad = sum(bytes(gb[go[i]:go[i + 1]]) != bytes(rb[ro[i]:ro[i + 1]]) for i in range(n))
        got = cld_amd.detect_batch(buf=buf, offsets=offs, flags=flags)
        ref = o.detect_batch(rb, ro, threads=16)
        bad = np.zeros(n, bool)
        for f in FIELDS:
            bad |= (got[f] != ref[f]).reshape(n, -1).any(axis=1)
        total += int(bad.sum()) + abs(pbad)
        print("seed %d flags %d: %d docs, prepared-text mismatches %d, result mismatches %d %s" % (
            seed, flags, n, pbad, int(bad.sum()), np.nonzero(bad)[0][:5]), flush=True)
print("total mismatches", total, flush=True)
