"""A stand-in for bench.py's HipBackend on the CPU (CLD_BENCH_MOCK): the
launcher, rank and line logic of bench.py run for real -- torch.distributed.run,
gloo, the barrier, max-over-ranks timing, the per-rank gather -- and only the
device work is the oracle on CPU tensors.  Test infrastructure
(tests/test_bench_ranks.py); CLD_BENCH_MOCK_GPUS sets how many GPUs it shows."""
import ctypes
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))


class _Stats:
    def __init__(self, n):
        self.passes = [n, 0, 0]
        self.short_docs, self.long_docs, self.general_docs = n, 0, 0
        self.long_requeue = [0] * 8


class Backend:
    dist_backend = "gloo"

    def __init__(self, local):
        from oracle import Oracle
        self.local, self.dev = local, torch.device("cpu")
        self.oracle = Oracle()
        self.ms, self.launches, self.n = 0.0, 0, 0

    @staticmethod
    def device_count():
        return int(os.environ.get("CLD_BENCH_MOCK_GPUS", "1"))

    def upload(self, arr):
        return torch.from_numpy(np.ascontiguousarray(arr).copy())

    def empty(self, nbytes):
        return torch.zeros(nbytes, dtype=torch.uint8)

    def detect(self, d_buf, d_offs, n, d_out):
        import cld_amd
        from oracle import RESULT_DTYPE as ORACLE_DTYPE
        t0 = time.perf_counter()
        tmp = np.zeros(n, dtype=ORACLE_DTYPE)
        rc = self.oracle.lib.cldo_detect_batch(ctypes.c_void_p(d_buf.data_ptr()), ctypes.c_void_p(d_offs.data_ptr()),
                                               n, tmp.ctypes.data, 1)
        assert rc == 0
        out = d_out.numpy().view(cld_amd.RESULT_DTYPE)
        for f in cld_amd.RESULT_DTYPE.names:
            out[f] = tmp[f]
        self.ms += (time.perf_counter() - t0) * 1e3
        self.launches += 1
        self.n = n

    def sync(self):
        pass

    def kernel_times(self):
        r = ([self.ms, 0.0, 0.0], self.launches)
        self.ms, self.launches = 0.0, 0
        return r

    def last_stats(self):
        return _Stats(self.n)

    def version(self):
        return "mock device (oracle on CPU)"
