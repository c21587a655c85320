"""Full-size parity sweep (GPU box): every document of the BASELINE-sized C2/C3/C4/C5
corpora (and the C3 boilerplate variant) through the HIP path and through the C
oracle (16 host threads), compared field by field; with --ref, against the
reference CLD2 itself (oracle/_ref/librefcld2.so) instead, skipping the
documents whose ill-formed lead bytes are undefined behaviour there.  One JSON line per config on
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
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    use_ref = "--ref" in sys.argv
    if use_ref:
        import refcld
        orc = refcld.instance(os.environ["CLD_MI355X_TABLES"])
    else:
        orc = Oracle()
    cfgs = [("c2", lambda: corpus.c2(1_000_000)), ("c3", lambda: corpus.c3(100_000)),
            ("c3_boiler5", lambda: corpus.c3(20_000, boiler_frac=0.05)), ("c4", lambda: corpus.c4(1_100_000)),
            ("c5", lambda: corpus.c5(1_000_000)), ("html", lambda: corpus.html(100_000, seed=77))]
    only = set(args)
    for name, gen in cfgs:
        if only and name not in only:
            continue
        t0 = time.time()
        print("# %s: generating" % name, flush=True)
        buf, offs = gen()
        print("# %s: %d docs generated in %.1f s" % (name, len(offs) - 1, time.time() - t0), flush=True)
        html = name == "html"                  # is_plain_text = false (ExtDetectLanguageSummary)
        got = cld_amd.detect_batch_ex(buf=buf, offsets=offs, html=True) if html else \
            cld_amd.detect_batch(buf=buf, offsets=offs)
        st = cld_amd.last_stats(0)
        if html:
            plain = np.zeros(len(offs) - 1, np.uint8)
            ref = orc.detect_batch(buf, offs, plain=plain, threads=16) if use_ref else \
                orc.detect_batch_ex(buf, offs, plain=plain, threads=16)
        else:
            ref = orc.detect_batch(buf, offs, threads=16)
        bad = np.zeros(len(got), dtype=bool)
        for f in FIELDS:
            bad |= (got[f].astype(np.float64) != ref[f].astype(np.float64)).reshape(len(got), -1).any(axis=1)
        skipped = 0
        if use_ref:                            # C0, C1, F5-F7 lead bytes: the reference reads past its table
            pos = np.nonzero(np.isin(np.asarray(buf), np.array([0xC0, 0xC1, 0xF5, 0xF6, 0xF7], np.uint8)))[0]
            ub = np.zeros(len(got), dtype=bool)
            ub[np.unique(np.searchsorted(offs, pos, side="right") - 1)] = True
            skipped = int(ub.sum())
            bad &= ~ub
        print(json.dumps({"config": name, "docs": int(len(got)), "bytes": int(offs[-1]), "mismatches": int(bad.sum()),
                          "checker": "reference CLD2 (librefcld2.so)" if use_ref else "oracle", "skipped_ub": skipped,
                          "first_bad": [int(i) for i in np.nonzero(bad)[0][:5]],
                          "kernels": {"wave_docs": int(st.short_docs), "long_docs": int(st.long_docs),
                                      "general_docs": int(st.general_docs)},
                          "passes": [int(x) for x in st.passes], "seconds": round(time.time() - t0, 1)}),
              flush=True)
        del buf, offs, got, ref


if __name__ == "__main__":
    main()
