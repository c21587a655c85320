"""HTML-mode throughput (is_plain_text = false; the exact sequential kernel k_general)
on 100K synthetic HTML pages, inputs resident on the host (cld_detect_batch_ex):
prints docs/s from the device timers and end to end."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "language-detector_amd"))
os.environ.setdefault("CLD_MI355X_TABLES", os.path.join(ROOT, "language-detector_amd", "data", "cld2_synth_q1.cldt"))
import cld_amd  # noqa: E402
import corpus  # noqa: E402

cld_amd.init_device(0)
buf, offs = corpus.html(100_000, seed=77)
cld_amd.detect_batch_ex(buf=buf, offsets=offs, html=True)        # warm
t0 = time.time()
cld_amd.detect_batch_ex(buf=buf, offsets=offs, html=True)
wall = time.time() - t0
st = cld_amd.last_stats(0)
n = len(offs) - 1
print(json.dumps({"workload": "100K synthetic HTML pages, 200-6000 B", "docs": n, "bytes": int(offs[-1]),
                  "general_ms": st.general_ms, "docs_per_s_kernel": n / (st.general_ms / 1e3),
                  "docs_per_s_end_to_end": n / wall, "general_docs": int(st.general_docs)}))
