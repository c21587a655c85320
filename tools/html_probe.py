"""Rewrite-kernel timing probe: 20K HTML pages as generated, with every '&'
replaced, and with every '<' replaced (short_ms = k_html_rewrite + k_route +
k_wave)."""
import os
import sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "language-detector_amd"))
import cld_amd  # noqa: E402
import corpus  # noqa: E402

cld_amd.init_device(0, tables=cld_amd.SYNTH_TABLES)
buf, offs = corpus.html(20000, seed=77)
for name, b in (("as generated", buf), ("no '&'", np.where(buf == ord('&'), ord('x'), buf).astype(np.uint8)),
                ("no '<'", np.where(buf == ord('<'), ord('x'), buf).astype(np.uint8)),
                ("no '&' or '<'", np.where((buf == ord('<')) | (buf == ord('&')), ord('x'), buf).astype(np.uint8))):
    cld_amd.detect_batch_ex(buf=b, offsets=offs, html=True)
    ms = []
    for _ in range(3):
        cld_amd.detect_batch_ex(buf=b, offsets=offs, html=True)
        st = cld_amd.last_stats(0)
        ms.append((st.short_ms, st.long_ms, st.general_ms))
    print(name, "rewrite+route+wave %.2f ms, long %.2f ms, general %.2f ms (general docs %d)" % (min(ms) + (int(st.general_docs),)), flush=True)
if os.environ.get("CLD_PROFILE_STAGES"):
    cld_amd.stage_cycles(0)
    cld_amd.detect_batch_ex(buf=buf, offsets=offs, html=True)
    c = cld_amd.stage_cycles(0)
    print("rewrite step 2: %.0f cycles per page (wave-summed)" % (c[7] / 20000.0))
