"""ResultChunkVector throughput (cld_detect_batch_vec; the exact sequential kernel
k_general_vec) on 100K C5 documents and 50K HTML pages, host buffers, end to end."""
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
for name, (buf, offs), html in (("c5 plain text", corpus.c5(100_000, seed=5), False),
                                ("html", corpus.html(50_000, seed=78), True)):
    cld_amd.detect_batch_vec(buf=buf, offsets=offs, html=html)       # warm (allocates the arena)
    t0 = time.time()
    res, chunks, coffs = cld_amd.detect_batch_vec(buf=buf, offsets=offs, html=html)
    wall = time.time() - t0
    n = len(offs) - 1
    print(json.dumps({"workload": "%d %s documents with ResultChunkVector" % (n, name), "bytes": int(offs[-1]),
                      "chunks": int(coffs[-1]), "docs_per_s_end_to_end": n / wall}), flush=True)
