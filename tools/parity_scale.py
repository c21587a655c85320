"""Full-size parity sweep (GPU box): every document of the BASELINE-sized C2/C3/C4/C5
corpora (and the C3 boilerplate variant) through the HIP path and through the C
oracle (16 host threads), compared field by field.  One JSON line per config on
stdout; the summary goes to profiles/ by hand.  Test infrastructure: the oracle is
the checker here, never the thing measured."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("language-detector_amd", "oracle"):
    sys.path.insert(0, os.path.join(ROOT, p))
os.environ.setdefault("CLD_MI355X_TABLES", os.path.join(ROOT, "language-detector_amd", "data", "cld2_synth_q1.cldt"))
import cld_amd  # noqa: E402
import corpus  # noqa: E402
from oracle import Oracle  # noqa: E402

FIELDS = ("lang3", "summary_lang", "percent3", "is_reliable", "text_bytes", "normalized3")


def main():
    cld_amd.init_device(0)
    orc = Oracle()
    cfgs = [("c2", lambda: corpus.c2(1_000_000)), ("c3", lambda: corpus.c3(100_000)),
            ("c3_boiler5", lambda: corpus.c3(20_000, boiler_frac=0.05)), ("c4", lambda: corpus.c4(1_100_000)),
            ("c5", lambda: corpus.c5(1_000_000))]
    only = set(sys.argv[1:])
    for name, gen in cfgs:
        if only and name not in only:
            continue
        t0 = time.time()
        print("# %s: generating" % name, flush=True)
        buf, offs = gen()
        print("# %s: %d docs generated in %.1f s" % (name, len(offs) - 1, time.time() - t0), flush=True)
        got = cld_amd.detect_batch(buf=buf, offsets=offs)
        st = cld_amd.last_stats(0)
        ref = orc.detect_batch(buf, offs, threads=16)
        bad = np.zeros(len(got), dtype=bool)
        for f in FIELDS:
            bad |= (got[f] != ref[f]).reshape(len(got), -1).any(axis=1)
        print(json.dumps({"config": name, "docs": int(len(got)), "bytes": int(offs[-1]), "mismatches": int(bad.sum()),
                          "first_bad": [int(i) for i in np.nonzero(bad)[0][:5]],
                          "kernels": {"wave_docs": int(st.short_docs), "long_docs": int(st.long_docs),
                                      "general_docs": int(st.general_docs)},
                          "passes": [int(x) for x in st.passes], "seconds": round(time.time() - t0, 1)}),
              flush=True)
        del buf, offs, got, ref


if __name__ == "__main__":
    main()
