"""Diagnostic: one batch of the hot path on cuda:0 (tweets + C3 pages, or the
corpus named by DIAG_CFG), results against the oracle, the batch statistics.
Run under AMD_SERIALIZE_KERNEL=3 a faulting kernel is reported at the launch
that follows it (the runtime's error line names the launcher)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "language-detector_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import cld_amd  # noqa: E402
import corpus  # noqa: E402

cld_amd.init_device(0, tables=cld_amd.SYNTH_TABLES)
n2, n3 = int(os.environ.get("DIAG_N2", 2000)), int(os.environ.get("DIAG_N3", 40))
b2, o2 = corpus.c2(n2)
b3, o3 = corpus.c3(n3)
docs = [bytes(b2[o2[i]:o2[i + 1]]) for i in range(n2)] + [bytes(b3[o3[i]:o3[i + 1]]) for i in range(n3)]
buf, offs = cld_amd.pack(docs)
print("batch: %d docs, %d bytes" % (len(docs), len(buf)), flush=True)
got = cld_amd.detect_batch(buf=buf, offsets=offs)
st = cld_amd.last_stats(0)
print("stats: short %d long %d seq %d passes %s requeue %s" % (st.short_docs, st.long_docs, st.general_docs,
                                                               list(st.passes), list(st.long_requeue)), flush=True)
from oracle import Oracle  # noqa: E402
ref = Oracle().detect_batch(buf, offs, threads=8)
bad = np.zeros(len(docs), bool)
for f in ("lang3", "summary_lang", "percent3", "is_reliable", "text_bytes", "normalized3"):
    bad |= (got[f] != ref[f]).reshape(len(docs), -1).any(axis=1)
print("mismatches vs oracle: %d, first %s" % (bad.sum(), np.nonzero(bad)[0][:5]), flush=True)
