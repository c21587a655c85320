#!/usr/bin/env python3
"""bench.py -- batched CLD2 DetectLanguage on MI355X (BASELINE.json metric).

A "step" is one pass of the hot path (DetectLanguageSummaryV2 per document,
compact_lang_det_impl.cc:1707-2106) over one batch of synthetic documents that
is already resident in HBM.  Default workload = BASELINE.json configs[1]
(1M ~140-byte tweets on one MI355X); --config c3/c4/c5 selects the others.

One process per GPU (torch.distributed, RCCL backend for the barrier and the
max-over-ranks timing only -- the path itself has no collective): each rank
scores its own shard of documents (weak scaling).  Rank 0 prints one JSON line.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c3|c4|c5]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "language-detector_amd"))

CONFIGS = {
    "c2": dict(docs=1_000_000, workload="C2: 1M synthetic tweets, U[100,180] B, 16 Latin-script languages "
                                        "(BASELINE.json configs[1])"),
    "c3": dict(docs=100_000, workload="C3: 100K synthetic 16 KB pages, Latin/Cyrillic/Arabic/Devanagari "
                                      "paragraphs (configs[2])"),
    "c4": dict(docs=1_000_000, workload="C4: 1M synthetic ~150 B zh/zh-Hant/ja/ko documents (configs[3])"),
    "c5": dict(docs=1_000_000, workload="C5 shard: lognormal lengths (median 140 B, p99 ~16 KB, cap 64 KB), "
                                        "mixed scripts (configs[4], one GPU's share)"),
}
HBM_PEAK_GBPS = 8000.0          # MI355X_MICROARCH.md chip table (spec)
ALG_BYTES_PER_DOC = 8 + 40      # + document bytes: offset + result record


def cpu_baseline(cfg, buf, offs, gpu_out, seconds):
    """Reference CPU restatement (oracle/) on the host cores, bounded sample.
    Also checks the GPU results of that sample bit-for-bit (checker role)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from oracle import Oracle
    ob = Oracle()
    threads = int(os.environ.get("CLD_CPU_THREADS", min(16, os.cpu_count() or 1)))
    n = len(offs) - 1
    sample = min(n, 200_000)
    o = offs[:sample + 1]
    b = buf[:int(o[-1])]
    ref = ob.detect_batch(b, o, threads=threads)            # warm + parity sample
    same = True
    for f in ("lang3", "summary_lang", "percent3", "is_reliable", "text_bytes", "normalized3"):
        same &= bool(np.array_equal(ref[f], gpu_out[f][:sample]))
    docs, t0 = 0, time.perf_counter()
    while True:
        ob.detect_batch(b, o, threads=threads)
        docs += sample
        dt = time.perf_counter() - t0
        if dt >= seconds:
            break
    return {"value": docs / dt, "unit": "docs/s", "cores": threads, "kind": "port",
            "sample": "%d %s documents (%.1f MB), %d passes in %.1f s, oracle/cld_oracle.c x%d pthreads"
                      % (sample, cfg, o[-1] / 1e6, docs // sample, dt, threads),
            "gpu_bit_exact_on_sample": same}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--docs", type=int, default=0, help="documents per GPU (default: config size)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))

    import torch
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group(backend="nccl")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    import cld_amd
    import corpus
    cld_amd.init_device(local)

    cfg = CONFIGS[args.config]
    n = args.docs or cfg["docs"]
    buf, offs = corpus.GENERATORS[args.config](n, seed=corpus.SEEDS[args.config] + 7919 * rank)
    d_buf = torch.from_numpy(buf).to(dev)
    d_offs = torch.from_numpy(offs.view(np.int64)).to(dev)
    d_out = torch.empty(n * 40, dtype=torch.uint8, device=dev)

    def step():
        cld_amd.detect_batch_device(0, d_buf.data_ptr(), d_offs.data_ptr(), n, d_out.data_ptr(), None)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    cld_amd.kernel_time(0)                      # reset the event accumulator

    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if dist:
        dist.barrier()
    elapsed = t1 - t0
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    short_ms, general_ms, launches = cld_amd.kernel_time(0)
    stats = cld_amd.last_stats(0)
    kernel_ms = (short_ms + general_ms) / max(1, launches)
    doc_bytes = int(offs[-1])
    alg_bytes = doc_bytes + ALG_BYTES_PER_DOC * n
    achieved = alg_bytes / (kernel_ms / 1e3) / 1e9

    traffic = None
    pmc = os.path.join(ROOT, "profiles", "pmc_%s.json" % args.config)
    if os.path.exists(pmc):
        with open(pmc) as f:
            p = json.load(f)
        if p.get("docs") == n:
            traffic = p.get("hbm_bytes_per_launch")

    if rank != 0:
        if dist:
            dist.destroy_process_group()
        return

    gpu_out = d_out.cpu().numpy().view(cld_amd.RESULT_DTYPE)
    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args.config, buf, offs, gpu_out, args.cpu_seconds)

    total_docs = n * world * args.steps
    line = {
        "metric": "docs/sec",
        "value": total_docs / elapsed,
        "unit": "docs/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (seeded corpus.py; vocabularies from the reference's octa tables; "
                "quadgram table synthetic -- the real one is a missing blob)",
        "config": {"workload": cfg["workload"], "docs_per_gpu": n, "bytes_per_gpu": doc_bytes,
                   "mean_doc_bytes": doc_bytes / n, "parallelism": "document shards, %d rank(s)" % world},
        "input_GBps": doc_bytes * world * args.steps / elapsed / 1e9,
        "passes_hist": [int(x) for x in stats.passes[:3]],
        "kernels": {"wave_ms": short_ms / max(1, launches), "long_plus_general_ms": general_ms / max(1, launches),
                    "last_batch": {"wave_ms": stats.short_ms, "long_ms": stats.long_ms, "general_ms": stats.general_ms,
                                   "wave_docs": int(stats.short_docs), "long_docs": int(stats.long_docs),
                                   "general_docs": int(stats.general_docs),
                                   "long_requeue_reasons": [int(x) for x in stats.long_requeue]}},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBPS, "traffic": traffic},
        "cpu_baseline": cpu,
    }
    print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
