"""Per-stage cycle breakdown of the wavefront kernel (needs CLD_PROFILE_STAGES=1)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "language-detector_amd"))
os.environ.setdefault("CLD_MI355X_TABLES", os.path.join(ROOT, "language-detector_amd", "data", "cld2_synth_q1.cldt"))
import cld_amd  # noqa: E402
import corpus  # noqa: E402

STAGES = ["load", "span", "lower", "quad/uni", "octa/bi", "score", "doc"]
LSTAGES = ["classify", "span+lower", "squeeze", "repeats", "words+chain", "quad", "octa/uni/bi", "score"]


def main():
    os.environ.setdefault("CLD_PROFILE_STAGES", "1")
    cld_amd.init_device(0)
    cfgs = [a.split(":") for a in sys.argv[1:]] or [("c2", 1_000_000), ("c4", 200_000), ("c5", 200_000), ("c3", 20000)]
    for cfg, n in cfgs:
        n = int(n)
        buf, offs = corpus.GENERATORS[cfg](n)
        cld_amd.detect_batch(buf=buf, offsets=offs)          # warm
        cld_amd.stage_cycles(0)
        cld_amd.kernel_time(0)
        cld_amd.detect_batch(buf=buf, offsets=offs)
        st = cld_amd.last_stats(0)
        c = cld_amd.stage_cycles(0).astype(np.float64)
        nw = max(1, st.short_docs // 64)          # k_wave samples one document in 64
        print("%s: %d docs, wave kernel %.3f ms, long %.3f ms (%d docs), general %.3f ms (%d docs)" %
              (cfg, n, st.short_ms, st.long_ms, st.long_docs, st.general_ms, st.general_docs))
        tot = c[:7].sum()
        print("   wave cycles/doc total %.0f  " % (tot / nw) +
              "  ".join("%s %.0f (%.0f%%)" % (STAGES[i], c[i] / nw, 100 * c[i] / max(tot, 1)) for i in range(7)),
              flush=True)
        nl = max(1, st.long_docs)
        lt = c[8:16].sum()
        print("   long cycles/doc total %.0f  " % (lt / nl) +
              "  ".join("%s %.0f (%.0f%%)" % (LSTAGES[i], c[8 + i] / nl, 100 * c[8 + i] / max(lt, 1)) for i in range(8)),
              flush=True)
        if os.environ.get("CLD_PROF_SUB"):
            sub = ["base emissions", "delta/distinct", "chunk plan", "tote loop", "summaries"]
            st = c[8:13]
            print("   score sub-stages/doc " + "  ".join("%s %.0f" % (sub[i], st[i] / nl) for i in range(5)) +
                  "  rounds/doc %.1f  chunks/doc %.1f" % ((int(c[13]) & 0xFFFFF) / nl, (int(c[13]) >> 20) / nl),
                  flush=True)


if __name__ == "__main__":
    main()
