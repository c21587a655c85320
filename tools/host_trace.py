"""Timeline of the streamed host path (cld_detect_batch on pinned C2 buffers),
for rocprofv3 --kernel-trace --memory-copy-trace: where the time between the
kernels goes.  Run under the profiler; prints the wall time per call."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "language-detector_amd"))
os.environ.setdefault("CLD_MI355X_TABLES", os.path.join(ROOT, "language-detector_amd", "data", "cld2_synth_q1.cldt"))
import cld_amd  # noqa: E402
import corpus  # noqa: E402

n = int(os.environ.get("HOST_TRACE_DOCS", "1000000"))
buf, offs = corpus.c2(n)
cld_amd.init_device(0)
pb = cld_amd.host_array(len(buf), np.uint8)
pb[:] = buf
po = cld_amd.host_array(len(offs), np.uint64)
po[:] = offs
pout = cld_amd.host_array(n, cld_amd.RESULT_DTYPE)
pageable = os.environ.get("HOST_TRACE_PAGEABLE") == "1"     # as bench.py's pageable leg: numpy buffers
out = np.zeros(n, dtype=cld_amd.RESULT_DTYPE)
fresh = os.environ.get("HOST_TRACE_FRESH_OUT") == "1"       # a new result array per call (its page faults)
for i in range(6):
    t0 = time.perf_counter()
    if pageable:
        cld_amd.detect_batch(buf=buf, offsets=offs, out=None if fresh else out)
    else:
        rc = cld_amd.lib().cld_detect_batch(pb.ctypes.data, po.ctypes.data, n, pout.ctypes.data, 0)
        assert rc == 0
    print("call %d: %.3f ms" % (i, (time.perf_counter() - t0) * 1e3), flush=True)
