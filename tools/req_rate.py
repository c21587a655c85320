"""Request-sized throughput of the batch C ABI (tools/req_bench.c, timed in C):
100K C5 documents cut into requests of <= 1 MiB of text (the reference
service's body limit, handlers.go:33-68), issued by 1 and by 8 concurrent
callers, plus the reference CLD2 on 16 host threads over the same documents
for comparison.  One JSON line per caller count; the last line the reference."""
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("language-detector_amd", "oracle"):
    sys.path.insert(0, os.path.join(ROOT, p))
os.environ.setdefault("CLD_MI355X_TABLES", os.path.join(ROOT, "language-detector_amd", "data", "cld2_synth_q1.cldt"))
import corpus  # noqa: E402

n = int(os.environ.get("REQ_RATE_DOCS", "100000"))
buf, offs = corpus.c5(n, seed=5)
d = tempfile.mkdtemp()
buf.tofile(os.path.join(d, "c.bin"))
offs.astype(np.uint64).tofile(os.path.join(d, "o.bin"))
exe = os.path.join(ROOT, "tools", "build", "req_bench")
if os.environ.get("REQ_RATE_PROF"):   # kernel statistics of the single-caller run (rocprofv3)
    out = os.environ["REQ_RATE_PROF"]
    subprocess.run(["rocprofv3", "--kernel-trace", "--stats", "-d", out, "-o", "req", "--output-format", "csv", "--", exe,
                    os.path.join(d, "c.bin"), os.path.join(d, "o.bin"), "1", str(1 << 20), "1"], check=True,
                   timeout=600)
for callers in [int(c) for c in os.environ.get("REQ_RATE_CALLERS", "1,8").split(",")]:
    r = subprocess.run([exe, os.path.join(d, "c.bin"), os.path.join(d, "o.bin"), str(callers)],
                       capture_output=True, text=True, timeout=600)
    if r.returncode != 0:
        print(r.stdout, r.stderr, file=sys.stderr)
        sys.exit(1)
    line = json.loads(r.stdout.strip().splitlines()[-1])
    line["workload"] = "%d C5 documents in requests of <= 1 MiB, %d concurrent callers (C harness)" % (n, callers)
    print(json.dumps(line), flush=True)
import refcld  # noqa: E402
ref = refcld.instance(os.environ["CLD_MI355X_TABLES"])
t0 = time.time()
ref.detect_batch(buf, offs, threads=16)
w = time.time() - t0
print(json.dumps({"workload": "reference CLD2, same %d documents, 16 host threads" % n, "docs_per_s": n / w}))
