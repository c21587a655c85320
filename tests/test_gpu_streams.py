"""Batches on different caller streams plus a host-memory batch at the same
time: the runtime's per-device scratch (counters, re-queue lists, k_long
slots, staging) is shared, so every enqueue waits on the previous batch's
`done` event (cld_runtime.cpp, Device::done).  All results must still equal
the oracle's.  Device buffers and streams come straight from the HIP runtime
(ctypes), the way a caller that owns its own streams would make them."""
import ctypes
import os
import threading

import numpy as np
import pytest

import corpus
from test_gpu_parity import assert_same

pytestmark = pytest.mark.gpu


def hip():
    h = ctypes.CDLL("libamdhip64.so")
    h.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
    h.hipFree.argtypes = [ctypes.c_void_p]
    h.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    h.hipStreamCreate.argtypes = [ctypes.POINTER(ctypes.c_void_p)]
    h.hipStreamDestroy.argtypes = [ctypes.c_void_p]
    h.hipDeviceSynchronize.argtypes = []
    return h


H2D, D2H = 1, 2


def test_two_streams_and_a_host_batch(gpu, oracle):
    h = hip()
    sets = [corpus.c5(20000, seed=101), corpus.c3(300, seed=102), corpus.c2(50000, seed=103)]
    refs = [oracle.detect_batch(b, o, threads=16) for b, o in sets]
    bufs = []
    for b, o in sets[:2]:
        n = len(o) - 1
        ptrs = []
        for size in (max(len(b), 1), 8 * (n + 1), gpu.RESULT_DTYPE.itemsize * n):
            p = ctypes.c_void_p()
            assert h.hipMalloc(ctypes.byref(p), size) == 0
            ptrs.append(p)
        assert h.hipMemcpy(ptrs[0], b.ctypes.data, len(b), H2D) == 0
        assert h.hipMemcpy(ptrs[1], o.ctypes.data, 8 * (n + 1), H2D) == 0
        bufs.append((ptrs, n))
    streams = []
    for _ in range(2):
        s = ctypes.c_void_p()
        assert h.hipStreamCreate(ctypes.byref(s)) == 0
        streams.append(s)
    host_out = {}

    def host_batch():
        b, o = sets[2]
        host_out["r"] = gpu.detect_batch(buf=b, offsets=o)

    th = threading.Thread(target=host_batch)
    for rep in range(3):                 # stream 0, stream 1, with a host batch running alongside
        for k in range(2):
            (pb, po, pout), n = bufs[k]
            gpu.detect_batch_device(0, pb.value, po.value, n, pout.value, streams[k].value)
        if rep == 0:
            th.start()
    th.join()
    assert h.hipDeviceSynchronize() == 0
    for k in range(2):
        (pb, po, pout), n = bufs[k]
        got = np.zeros(n, dtype=gpu.RESULT_DTYPE)
        assert h.hipMemcpy(got.ctypes.data, pout, got.nbytes, D2H) == 0
        assert_same(got, refs[k], "stream %d" % k)
    assert_same(host_out["r"], refs[2], "host batch")
    for (ptrs, _) in bufs:
        for p in ptrs:
            h.hipFree(p)
    for s in streams:
        h.hipStreamDestroy(s)


FAN_OUT = r'''
import sys
import numpy as np
import cld_amd, corpus
from oracle import Oracle
from test_gpu_html_hints import priors_for, random_hints
from test_gpu_parity import assert_same
cld_amd.init()
o = Oracle()
b, off = corpus.c5(30000, seed=121)
assert_same(cld_amd.detect_batch(buf=b, offsets=off), o.detect_batch(b, off, threads=16), "fan-out batch")
docs = [cld_amd.last_stats(k).docs for k in (0, 1)]
assert docs[0] > 0 and docs[1] > 0 and sum(docs) == 30000, docs
hb, ho = corpus.html(600, seed=122)
n = len(ho) - 1
assert_same(cld_amd.detect_batch_ex(buf=hb, offsets=ho, html=True),
            o.detect_batch_ex(hb, ho, plain=np.zeros(n, np.uint8), priors=priors_for(cld_amd, hb, ho, True, None),
                              threads=16), "fan-out html")
hints = random_hints(cld_amd, 30000, 123)
assert_same(cld_amd.detect_batch_ex(buf=b, offsets=off, hints=hints),
            o.detect_batch_ex(b, off, priors=priors_for(cld_amd, b, off, False, hints), threads=16), "fan-out hints")
vb, vo = corpus.c5(800, seed=124)
res, chunks, coffs = cld_amd.detect_batch_vec(buf=vb, offsets=vo)
for i in range(len(vo) - 1):
    r, ch = o.detect_vec(bytes(vb[vo[i]:vo[i + 1]]))
    assert [(int(c["offset"]), int(c["bytes"]), int(c["lang1"])) for c in chunks[coffs[i]:coffs[i + 1]]] == \
        [(int(c["offset"]), int(c["bytes"]), int(c["lang1"])) for c in ch], i
    assert int(res[i]["summary_lang"]) == r.summary_lang, i
# request-sized batches from concurrent callers: each runs whole on the least
# busy context (cld_runtime.cpp pick_context), results as the oracle's
import threading
sb, so = corpus.c5(4000, seed=125)
want = o.detect_batch(sb, so, threads=16)
parts = np.array_split(np.arange(4000), 16)
got = [None] * 16
def work(k):
    lo, hi = int(parts[k][0]), int(parts[k][-1]) + 1
    got[k] = cld_amd.detect_batch(buf=sb, offsets=so[lo:hi + 1])
ths = [threading.Thread(target=work, args=(k,)) for k in range(16)]
for t in ths: t.start()
for t in ths: t.join()
assert_same(np.concatenate(got), want, "concurrent small batches")
print("fan-out ok", docs)
'''


def test_multi_context_fan_out():
    """The batch entry points' multi-device branch (one host thread per
    context writing out + cut[k]; cld_runtime.cpp cld_detect_batch /
    _ex / _vec) with GPU 0 registered twice (CLD_MI355X_DEVICE_MAP=0,0: two
    contexts with their own streams, tables and scratch), in a child process
    (the runtime's device set is fixed per process).  Both contexts must get
    documents, and every result must equal the oracle's; so must 16 concurrent
    request-sized calls, which each run whole on the least busy context."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, CLD_MI355X_DEVICE_MAP="0,0",
               PYTHONPATH=os.pathsep.join(os.path.join(root, p) for p in ("language-detector_amd", "oracle", "tests")))
    r = subprocess.run([sys.executable, "-c", FAN_OUT], env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    assert "fan-out ok" in r.stdout


def test_concurrent_request_sized_calls_coalesce(gpu, oracle):
    """Request-sized cld_detect_batch calls from 12 threads at once are run
    together (cld_runtime.cpp run_coalesced: one GPU batch per dispatch, the
    documents copied into pinned staging and the results handed back to each
    caller), with flags kept apart: every caller gets exactly its own results."""
    import threading
    from test_gpu_parity import assert_same
    b, o = corpus.c5(6000, seed=131)
    want = oracle.detect_batch(b, o, threads=16)
    want_be = oracle.detect_batch_ex(b, o, threads=16, flags=gpu.FLAG_BEST_EFFORT)
    parts = np.array_split(np.arange(6000), 24)
    got = [None] * 24

    def work(k):
        for rep in range(3):
            lo, hi = int(parts[k][0]), int(parts[k][-1]) + 1
            got[k] = gpu.detect_batch(buf=b, offsets=o[lo:hi + 1], flags=gpu.FLAG_BEST_EFFORT if k % 2 else 0)

    ths = [threading.Thread(target=work, args=(k,)) for k in range(24)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    for k in range(24):
        lo, hi = int(parts[k][0]), int(parts[k][-1]) + 1
        assert_same(got[k], (want_be if k % 2 else want)[lo:hi], "caller %d" % k)


CHUNKED = r'''
import numpy as np
import cld_amd, corpus
from oracle import Oracle
from test_gpu_parity import assert_same
cld_amd.init()
o = Oracle()
# 1 MB chunks: C2 streams through ~9 chunks in two alternating slots, C5
# (tail-bound: 4 MB chunks) through several; pageable and pinned result arrays
for name, (b, off) in (("c2", corpus.c2(60000, seed=141)), ("c5", corpus.c5(20000, seed=142))):
    want = o.detect_batch(b, off, threads=16)
    for rep in range(3):
        assert_same(cld_amd.detect_batch(buf=b, offsets=off), want, "%s chunked rep %d" % (name, rep))
print("chunked ok")
'''


def test_streamed_chunks_reuse_slots_safely():
    """The streamed host path alternates two chunk slots, so chunk c writes the
    device results of chunk c-2's slot while c-2's download may still be
    queued (cld_runtime.cpp run_host_stream: the kernels of chunk c wait for
    that download on the device).  With CLD_CHUNK_MB=1 every batch here is
    many chunks; every result must equal the oracle's, three times over."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, CLD_CHUNK_MB="1",
               PYTHONPATH=os.pathsep.join(os.path.join(root, p) for p in ("language-detector_amd", "oracle", "tests")))
    r = subprocess.run([sys.executable, "-c", CHUNKED], env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    assert "chunked ok" in r.stdout


def test_tiny_batches_equal_the_oracle(gpu, oracle):
    """Request-sized batches of short documents take run_tiny (one upload, one
    k_wave launch, one download; cld_runtime.cpp).  Batches of 1..1024
    documents -- tweets, CJK, and short documents k_wave hands on (several
    script spans), which the tiny path redoes on the streamed path -- must
    equal the oracle, alone and from 16 concurrent callers; a clean tweet batch
    must have run on the tiny path (no kernel events: short_ms == 0)."""
    import threading
    from test_gpu_parity import EDGE
    b2, o2 = corpus.c2(3000, seed=151)
    b4, o4 = corpus.c4(2000, seed=152)
    docs = [bytes(b2[o2[i]:o2[i + 1]]) for i in range(3000)] + [bytes(b4[o4[i]:o4[i + 1]]) for i in range(2000)]
    docs = [d for d in docs if len(d) <= 256]
    mixed = [("abc рус %d العربية ok " % k).encode() for k in range(40)] + [e for e in EDGE if len(e) <= 256]
    rng = np.random.default_rng(153)
    batches = []
    for size in (1, 2, 7, 64, 255, 1000, 1024):
        pick = [docs[int(i)] for i in rng.integers(0, len(docs), size)]
        if size in (7, 255):
            for j, m in zip(range(0, size, 3), mixed):
                pick[j] = m
        batches.append(pick)
    for pick in batches:
        pb, po = gpu.pack(pick)
        assert_same(gpu.detect_batch(buf=pb, offsets=po), oracle.detect_batch(pb, po, threads=8), "tiny %d" % len(pick))
    pb, po = gpu.pack(docs[:500])
    gpu.detect_batch(buf=pb, offsets=po)
    st = gpu.last_stats(0)
    assert st.short_docs == 500 and st.short_ms == 0, (st.short_docs, st.short_ms)
    got = [None] * 16
    packed = [gpu.pack(batches[k % len(batches)]) for k in range(16)]

    def work(k):
        for rep in range(4):
            got[k] = gpu.detect_batch(buf=packed[k][0], offsets=packed[k][1])
    ths = [threading.Thread(target=work, args=(k,)) for k in range(16)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    for k in range(16):
        assert_same(got[k], oracle.detect_batch(*packed[k], threads=8), "concurrent tiny %d" % k)


def test_detect_language_many_callers(gpu, oracle):
    """wrapper.h detect_language from 64 threads at once over tweets, CJK and
    long pages (coalesced micro-batches: tiny groups on run_tiny, the rest on
    the streamed path) equals the oracle's DetectLanguage answer per document."""
    import threading
    b2, o2 = corpus.c2(1500, seed=161)
    b5, o5 = corpus.c5(500, seed=162)
    texts = [bytes(b2[o2[i]:o2[i + 1]]) for i in range(1500)]
    texts += [bytes(b5[o5[i]:o5[i + 1]]) for i in range(500)]
    want = [oracle.detect_language(t) for t in texts]
    got = [None] * len(texts)

    def worker(lo):
        for i in range(lo, len(texts), 64):
            got[i] = gpu.detect_language(texts[i])
    th = [threading.Thread(target=worker, args=(k,)) for k in range(64)]
    [t.start() for t in th]
    [t.join() for t in th]
    bad = [i for i in range(len(texts)) if got[i] != want[i]]
    assert not bad, (len(bad), bad[:5], [got[i] for i in bad[:5]], [want[i] for i in bad[:5]])


DL_SHUTDOWN_SCRIPT = r"""
import sys, threading
sys.path[:0] = [sys.argv[1] + "/language-detector_amd", sys.argv[1] + "/oracle", sys.argv[1] + "/tests"]
import ctypes, corpus, cld_amd
from oracle import Oracle
b2, o2 = corpus.c2(2000, seed=171)
texts = [bytes(b2[o2[i]:o2[i + 1]]) for i in range(2000)]
want = [Oracle().detect_language(t) for t in texts]
for rnd in range(2):                       # the queue's dispatchers stop at cld_shutdown and restart after
    got = [None] * len(texts)
    def worker(lo):
        for i in range(lo, len(texts), 128):
            got[i] = cld_amd.detect_language(texts[i])
    th = [threading.Thread(target=worker, args=(k,)) for k in range(128)]
    [t.start() for t in th]
    [t.join() for t in th]
    bad = [i for i in range(len(texts)) if got[i] != want[i]]
    assert not bad, (rnd, len(bad), bad[:5])
    cld_amd.lib().cld_shutdown()
print("ok")
"""


def test_detect_language_queue_across_shutdown(tmp_path):
    """detect_language's per-call queue (cld_dlqueue.h) from 128 threads: every
    answer equals the oracle's, cld_shutdown stops the dispatcher threads
    before the contexts go, and the next call starts them again.  In its own
    process (it shuts the runtime down)."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    script = tmp_path / "dl_shutdown.py"
    script.write_text(DL_SHUTDOWN_SCRIPT)
    r = subprocess.run([sys.executable, str(script), root], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stdout[-2000:] + r.stderr[-3000:]
