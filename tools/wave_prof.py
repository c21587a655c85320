"""Per-stage cycle breakdown of the wavefront kernel (needs CLD_PROFILE_STAGES=1)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "language-detector_amd"))
import cld_amd  # noqa: E402
import corpus  # noqa: E402

STAGES = ["load", "span", "lower", "quad/uni", "octa/bi", "score", "doc"]


def main():
    os.environ.setdefault("CLD_PROFILE_STAGES", "1")
    cld_amd.init_device(0)
    for cfg, n in (("c2", 1_000_000), ("c4", 200_000), ("c5", 200_000)):
        buf, offs = corpus.GENERATORS[cfg](n)
        cld_amd.detect_batch(buf=buf, offsets=offs)          # warm
        cld_amd.stage_cycles(0)
        cld_amd.kernel_time(0)
        cld_amd.detect_batch(buf=buf, offsets=offs)
        st = cld_amd.last_stats(0)
        c = cld_amd.stage_cycles(0).astype(np.float64)
        nw = max(1, st.short_docs)
        print("%s: %d docs, wave kernel %.3f ms, general %.3f ms, requeued %d" %
              (cfg, n, st.short_ms, st.general_ms, st.general_docs))
        tot = c[:7].sum()
        print("   cycles/doc total %.0f  " % (tot / nw) +
              "  ".join("%s %.0f (%.0f%%)" % (STAGES[i], c[i] / nw, 100 * c[i] / max(tot, 1)) for i in range(7)),
              flush=True)


if __name__ == "__main__":
    main()
