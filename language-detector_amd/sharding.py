"""Document sharding across ranks (one process per GPU).

Documents are independent, so a corpus is split into
contiguous document ranges of equal estimated kernel cost (cld_plan_shards,
the same split cld_detect_batch uses across the GPUs of one process; the cost
model is doc_costs below).  Each rank scores its
own range on its own GPU; nothing is exchanged on the hot path.  Only the
40-byte result records travel back to the root rank, once, after scoring.
"""
import numpy as np

import cld_amd


def doc_costs(offsets):
    """Estimated kernel cost per document, cld_plan_shards' model (include/cld_mi355x.h):
    480 units for a document of <= 256 bytes (k_wave), 41/8 per byte + 2500 for a
    longer one (k_long); units of 10 ps of one MI355X."""
    ln = np.diff(np.asarray(offsets, dtype=np.uint64)).astype(np.int64)
    return np.where(ln <= 256, 480, (ln * 41) // 8 + 2500)


def shard_bounds(offsets, rank, world):
    """[lo, hi) document range of `rank` out of `world` (estimated-cost balanced)."""
    cuts = cld_amd.plan_shards(offsets, world)
    return int(cuts[rank]), int(cuts[rank + 1])


def local_shard(buf, offsets, rank, world):
    """(buf view, rebased offsets, lo, hi) of this rank's documents."""
    lo, hi = shard_bounds(offsets, rank, world)
    offsets = np.asarray(offsets, dtype=np.uint64)
    a, b = int(offsets[lo]), int(offsets[hi])
    return buf[a:b], offsets[lo:hi + 1] - np.uint64(a), lo, hi


def as_results(res):
    """Any record array with the cld_result field names -> RESULT_DTYPE."""
    if res.dtype == cld_amd.RESULT_DTYPE:
        return res
    out = np.zeros(len(res), dtype=cld_amd.RESULT_DTYPE)
    for f in cld_amd.RESULT_DTYPE.names:
        out[f] = res[f]
    return out


def detect_sharded(buf, offsets, dist, detect=None, root=0):
    """Score a corpus held (identically) by every rank; rank `root` returns all
    results in corpus order, other ranks return their own shard's results.

    detect(buf, offsets) -> RESULT_DTYPE array; defaults to the HIP batch path
    (cld_amd.detect_batch on this process's GPU)."""
    import torch
    detect = detect or (lambda b, o: cld_amd.detect_batch(buf=b, offsets=o))
    rank, world = dist.get_rank(), dist.get_world_size()
    sbuf, soffs, lo, hi = local_shard(buf, offsets, rank, world)
    res = as_results(detect(sbuf, soffs))
    if world == 1:
        return res
    n = len(offsets) - 1
    cuts = cld_amd.plan_shards(offsets, world)
    width = int(np.max(np.diff(cuts))) if n else 0
    # results move as raw bytes, padded to the widest shard (gather needs equal sizes)
    mine = torch.zeros(width * cld_amd.RESULT_DTYPE.itemsize, dtype=torch.uint8)
    mine[:res.nbytes] = torch.from_numpy(res.view(np.uint8).copy())
    bufs = [torch.zeros_like(mine) for _ in range(world)] if rank == root else None
    dist.gather(mine, bufs, dst=root)
    if rank != root:
        return res
    out = np.zeros(n, dtype=cld_amd.RESULT_DTYPE)
    for k in range(world):
        cnt = int(cuts[k + 1] - cuts[k])
        out[cuts[k]:cuts[k + 1]] = bufs[k].numpy()[:cnt * cld_amd.RESULT_DTYPE.itemsize].view(cld_amd.RESULT_DTYPE)
    return out
