"""Batches on different caller streams plus a host-memory batch at the same
time: the runtime's per-device scratch (counters, re-queue lists, k_long
slots, staging) is shared, so every enqueue waits on the previous batch's
`done` event (cld_runtime.cpp, Device::done).  All results must still equal
the oracle's.  Device buffers and streams come straight from the HIP runtime
(ctypes), the way a caller that owns its own streams would make them."""
import ctypes
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
