"""Multi-rank document sharding (gloo, world_size 2, CPU).

The per-rank detector here is the oracle (CPU checker); on a GPU box the same
driver calls the HIP batch path.  What is tested is the host logic: the shard
plan covers every document exactly once, ranks agree on it, and the gathered
results equal a single-process run in corpus order."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, n, q):
    import sys
    for p in ("language-detector_amd", "oracle"):
        sys.path.insert(0, os.path.join(ROOT, p))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    import corpus
    import sharding
    from oracle import Oracle
    dist.init_process_group("gloo", rank=rank, world_size=world)
    buf, offs = corpus.c5(n)
    ob = Oracle()
    out = sharding.detect_sharded(buf, offs, dist, detect=lambda b, o: ob.detect_batch(b, o, threads=2))
    if rank == 0:
        ref = sharding.as_results(ob.detect_batch(buf, offs, threads=4))
        q.put(bool(np.array_equal(out.view(np.uint8), ref.view(np.uint8))))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_sharded_equals_single_process(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, 3000, q)) for r in range(world)]
    [p.start() for p in ps]
    [p.join(timeout=180) for p in ps]
    for p in ps:
        if p.is_alive():
            p.kill()
    assert all(p.exitcode == 0 for p in ps)
    assert q.get(timeout=5)


def test_plan_shards_cover_and_balance():
    import cld_amd
    import corpus
    import sharding
    buf, offs = corpus.c5(20000)
    for world in (1, 2, 3, 8, 64):
        cuts = cld_amd.plan_shards(offs, world)
        assert cuts[0] == 0 and cuts[-1] == len(offs) - 1 and np.all(np.diff(cuts) >= 0)
        # every shard carries 1/world of the estimated kernel cost, within one document
        c = np.concatenate([[0], np.cumsum(sharding.doc_costs(offs))])
        w = c[cuts[1:]] - c[cuts[:-1]]
        assert w.max() <= c[-1] / world + sharding.doc_costs(offs).max()
        assert w.min() >= c[-1] / world - sharding.doc_costs(offs).max() or world > len(offs) - 1
    # degenerate inputs
    z = np.zeros(1, np.uint64)
    assert list(cld_amd.plan_shards(z, 4)) == [0, 0, 0, 0, 0]


class _DeviceMock:
    """cld_amd's loaded library with only the device call replaced: the
    batch entry cld_detect_batch runs the oracle on the very pointers the
    product's marshalling (cld_amd.detect_batch) hands over."""

    def __init__(self, lib, oracle):
        self._lib, self._oracle, self.calls = lib, oracle, 0

    def __getattr__(self, name):
        return getattr(self._lib, name)

    def cld_detect_batch(self, bptr, offs_ptr, n, out_ptr, flags):
        import ctypes
        import cld_amd
        from oracle import RESULT_DTYPE as ORACLE_DTYPE
        assert flags == 0
        self.calls += 1
        n = int(n)
        tmp = np.zeros(n, dtype=ORACLE_DTYPE)               # the oracle's own record layout
        rc = self._oracle.lib.cldo_detect_batch(bptr, offs_ptr, n, tmp.ctypes.data, 2)
        out = np.frombuffer((ctypes.c_uint8 * (n * cld_amd.RESULT_DTYPE.itemsize)).from_address(out_ptr),
                            dtype=cld_amd.RESULT_DTYPE)
        for f in cld_amd.RESULT_DTYPE.names:                 # cld_result fields, as the device writes them
            out[f] = tmp[f]
        return rc


def _worker_mocked(rank, world, port, n, q):
    import sys
    for p in ("language-detector_amd", "oracle"):
        sys.path.insert(0, os.path.join(ROOT, p))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    import cld_amd
    import corpus
    import sharding
    from oracle import Oracle
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ob = Oracle()
    mock = _DeviceMock(cld_amd.lib(), ob)
    cld_amd._lib = mock
    buf, offs = corpus.c5(n)
    out = sharding.detect_sharded(buf, offs, dist)            # default detector: cld_amd.detect_batch
    if rank == 0:
        ref = sharding.as_results(ob.detect_batch(buf, offs, threads=4))
        q.put((mock.calls, bool(np.array_equal(out.view(np.uint8), ref.view(np.uint8)))))
    dist.destroy_process_group()


def test_gloo_sharded_through_product_binding():
    """detect_sharded over the real cld_amd ctypes path (packing, pointers,
    RESULT_DTYPE views, shard rebasing), mocked only at the device call."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    world = 2
    ps = [ctx.Process(target=_worker_mocked, args=(r, world, port, 2500, q)) for r in range(world)]
    [p.start() for p in ps]
    [p.join(timeout=180) for p in ps]
    for p in ps:
        if p.is_alive():
            p.kill()
    assert all(p.exitcode == 0 for p in ps)
    calls, same = q.get(timeout=5)
    assert calls == 1 and same
