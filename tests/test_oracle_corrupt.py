"""The oracle on the shrunk corruption fixtures (tests/golden/corrupt/, made by
tools/corrupt_bisect.py from the GPU sweeps): every mode and flag set answers
without tripping an internal check -- the ScoreAsQuads one used to reach the
oracle's GetScore(-1) abort -- and deterministically.  CPU only."""
import os

import cld_amd
from oracle import Oracle

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "corrupt")


def test_oracle_on_corruption_fixtures():
    docs = [open(os.path.join(GOLDEN, f), "rb").read() for f in sorted(os.listdir(GOLDEN))]
    buf, offs = cld_amd.pack(docs)
    o = Oracle()
    for flags in (0, 0x100, 0x4000, 0x4100):
        a = o.detect_batch_ex(buf, offs, flags=flags)
        b = o.detect_batch_ex(buf, offs, flags=flags, threads=4)
        assert (a == b).all()
    for d in docs:
        r, ch = o.detect_vec(d)
        assert sum(int(c["bytes"]) for c in ch) >= 0
