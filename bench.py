#!/usr/bin/env python3
"""bench.py -- batched CLD2 DetectLanguage on MI355X (BASELINE.json metric:
"docs/sec + input GB/s at 1/2/4/8 MI355X, 140B tweets and 16KB pages").

A "step" is one pass of the hot path (DetectLanguageSummaryV2 per document,
compact_lang_det_impl.cc:1707-2106) over one batch of synthetic documents that
is already resident in HBM.  The headline is C2 (BASELINE.json configs[1]:
1M ~140-byte tweets on one MI355X); the same run measures the metric's second
half, C3 (configs[2]: 100K 16 KB pages), as the "c3" sub-object, and the
host-memory path (cld_detect_batch: pinned staging, chunked upload / kernels /
download on three streams) on C2 as "host_path".  --config c3/c4/c5 makes
another config the headline instead.

One process per GPU: `--gpus N` (N > 1) run without a torch.distributed
environment starts N ranks itself -- it counts the visible GPUs (without
initialising one), refuses N larger than that, and runs
`python -m torch.distributed.run --nproc-per-node N` on this same command line
as a child process, exiting with its code; under an existing launcher
(WORLD_SIZE set) `--gpus` must equal WORLD_SIZE.  RCCL carries only the
barrier, the max-over-ranks timing and the per-rank kernel times -- the path
itself has no collective: each rank scores its own shard of documents (weak
scaling).  Rank 0 prints one JSON line, with every rank's kernel time in
"per_rank".

Tables: the synthetic Q1 quadgram table, opted into explicitly
(CLD_MI355X_TABLES) so every quadgram branch does work; the library's own
default is the empty Q0 table (the real quadchrome table is a missing blob).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c3|c4|c5]
                    [--no-sub] [--no-host] [--no-cpu-baseline]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "language-detector_amd"))
os.environ.setdefault("CLD_MI355X_TABLES", os.path.join(ROOT, "language-detector_amd", "data", "cld2_synth_q1.cldt"))

# The long-document path between the library's second and third HIP events:
# the staged kernels (cld_long.hip "staged long-document path") and the fused
# k_long for the documents they hand on, plus the LPT ordering launches.
LONG_PATH = ("long-document path: k_lspan + k_lscore (x2) + k_lgroup (x2) + k_lfinish (x2) + k_lrep, "
             "k_long for hand-ons")
CONFIGS = {
    "c2": dict(docs=1_000_000, steps=20, kernel=0, name="k_wave",
               workload="C2: 1M synthetic tweets, U[100,180] B, 16 Latin-script languages (BASELINE.json configs[1])"),
    "c3": dict(docs=100_000, steps=3, kernel=1, name=LONG_PATH,
               workload="C3: 100K synthetic 16 KB pages, Latin/Cyrillic/Arabic/Devanagari paragraphs (configs[2])"),
    "c2n": dict(docs=1_000_000, steps=20, kernel=0, name="k_wave",
                workload="C2 with unseen words (a Caesar shift per tweet: nearly every quadgram probe misses; "
                         "table-size sensitivity, not a BASELINE config)"),
    "c4": dict(docs=1_100_000, steps=5, kernel=0, name="k_wave",
               workload="C4: 1M ~150 B + 100K ~4 KB synthetic zh/zh-Hant/ja/ko documents (configs[3])"),
    "c5": dict(docs=1_000_000, steps=5, kernel=1, name=LONG_PATH,
               workload="C5 shard: lognormal lengths (median 140 B, p99 ~16 KB, cap 64 KB), mixed scripts "
                        "(configs[4], one GPU's share)"),
}
HBM_PEAK_GBPS = 8000.0          # MI355X_MICROARCH.md chip table (spec)
ALG_BYTES_PER_DOC = 8 + 40      # + document bytes: offset + result record
# Issue ceilings (MI355X_MICROARCH.md: 256 CUs x 4 SIMD-32 at 2.4 GHz; a wave64
# VALU instruction issues over 2 cycles on its SIMD; one scalar unit per CU)
VALU_PEAK = 256 * 4 * 2.4e9 / 2      # wave-instructions / s
SALU_PEAK = 256 * 2.4e9              # wave-instructions / s
FIELDS = ("lang3", "summary_lang", "percent3", "is_reliable", "text_bytes", "normalized3")


def host_cores():
    """Cores this process may actually use: the affinity mask, capped by a
    cgroup CPU quota (the GPU box grants a share of a bigger machine)."""
    n = len(os.sched_getaffinity(0))
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            n = min(n, max(1, int(int(q) // int(p))))
    except (OSError, ValueError):
        pass
    model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return n, os.cpu_count(), model


def cpu_baseline(cfg, buf, offs, gpu_out, seconds, sample_docs):
    """The CPU path timed on the host cores over a bounded sample: the
    reference CLD2 itself when its checker build travels with the tree
    (oracle/_ref/librefcld2.so: the reference's own sources in its
    dynamic-data mode, tables loaded from a data file written from the same
    CLDT as the GPU's), else the oracle (oracle/cld_oracle.c, the C
    restatement).  Also checks the GPU results of that sample bit-for-bit
    (checker role)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    cores, nproc, model = host_cores()
    threads = int(os.environ.get("CLD_CPU_THREADS", cores))
    n = len(offs) - 1
    sample = min(n, sample_docs)
    o = offs[:sample + 1]
    b = buf[:int(o[-1])]
    import refcld
    if os.path.exists(refcld.LIB) and os.environ.get("CLD_CPU_BASELINE", "reference") == "reference":
        eng = refcld.instance(os.environ["CLD_MI355X_TABLES"])
        kind, what = "reference", "reference CLD2 (oracle/_ref/librefcld2.so, DetectLanguageSummaryV2)"
        fields = ("lang3", "summary_lang", "percent3", "is_reliable", "text_bytes", "normalized3")
    else:
        from oracle import Oracle
        eng = Oracle()
        kind, what = "port", "oracle/cld_oracle.c"
        fields = FIELDS
    ref = eng.detect_batch(b, o, threads=threads)            # warm + parity sample
    same = all(bool(np.array_equal(ref[f].astype(np.float64), gpu_out[f][:sample].astype(np.float64)))
               for f in fields)
    docs, t0 = 0, time.perf_counter()
    while True:
        eng.detect_batch(b, o, threads=threads)
        docs += sample
        dt = time.perf_counter() - t0
        if dt >= seconds:
            break
    return {"value": docs / dt, "unit": "docs/s", "cores": threads, "kind": kind,
            "input_GBps": docs / sample * float(o[-1]) / dt / 1e9,
            "sample": "%d %s documents (%.1f MB), %d passes in %.1f s, %s x %d threads"
                      % (sample, cfg, o[-1] / 1e6, docs // sample, dt, what, threads),
            "host": {"nproc": nproc, "usable_cores": cores, "cpu_model": model},
            "gpu_bit_exact_on_sample": same}


def pmc_summary(cfg):
    """Per-launch counters of the dominant kernel from the committed rocprofv3
    PMC summary of this tree (profiles/pmc_current.json, tools/pmc_session.sh)."""
    path = os.path.join(ROOT, "profiles", "pmc_current.json")
    if not os.path.exists(path):
        return None
    with open(path) as f:
        return json.load(f).get(cfg)


class HipBackend:
    """The product path on this rank's GPU: torch for HBM buffers and the
    stream sync, the library's C ABI (cld_detect_batch_device) for the work."""
    dist_backend = "nccl"

    def __init__(self, local):
        import torch
        import cld_amd
        self.torch, self.cld = torch, cld_amd
        torch.cuda.set_device(local)
        self.dev = torch.device("cuda", local)
        cld_amd.init_device(local)

    @staticmethod
    def device_count():
        import torch
        return torch.cuda.device_count()          # does not initialise a GPU on this image

    def upload(self, arr):
        return self.torch.from_numpy(arr).to(self.dev)

    def empty(self, nbytes):
        return self.torch.empty(nbytes, dtype=self.torch.uint8, device=self.dev)

    def detect(self, d_buf, d_offs, n, d_out):
        self.cld.detect_batch_device(0, d_buf.data_ptr(), d_offs.data_ptr(), n, d_out.data_ptr(), None)

    def sync(self):
        self.torch.cuda.synchronize()

    def kernel_times(self):
        return self.cld.kernel_times(0)

    def last_stats(self):
        return self.cld.last_stats(0)

    def version(self):
        return self.cld.version()


def backend_class():
    """HipBackend, or the class `Backend` of the file CLD_BENCH_MOCK names (the
    CPU tests of the launcher and rank logic: tests/bench_mock.py)."""
    mock = os.environ.get("CLD_BENCH_MOCK")
    if not mock:
        return HipBackend
    import importlib.util
    spec = importlib.util.spec_from_file_location("cld_bench_mock", mock)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod.Backend


def measure(cfg_name, n, steps, warmup, rank, dist, be):
    import torch
    import cld_amd
    import corpus
    cfg = CONFIGS[cfg_name]
    buf, offs = corpus.GENERATORS[cfg_name](n, seed=corpus.SEEDS[cfg_name] + 7919 * rank)
    d_buf = be.upload(buf)
    d_offs = be.upload(offs.view(np.int64))
    d_out = be.empty(n * 40)

    def step():
        be.detect(d_buf, d_offs, n, d_out)

    for _ in range(warmup):
        step()
    be.sync()
    be.kernel_times()                            # reset the event accumulator
    if dist:
        dist.barrier()
    be.sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    be.sync()
    t1 = time.perf_counter()
    if dist:
        dist.barrier()
    elapsed = t1 - t0
    ms, launches = be.kernel_times()
    per = [m / max(1, launches) for m in ms]
    per_rank = None
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device=be.dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        # every rank's own wall time and kernel times, for balance checks of a multi-GPU record
        mine = torch.tensor([float(rank), t1 - t0] + per + [float(n), float(offs[-1])],
                            dtype=torch.float64, device=be.dev)
        allr = [torch.zeros_like(mine) for _ in range(dist.get_world_size())]
        dist.all_gather(allr, mine)
        per_rank = [{"rank": int(v[0]), "elapsed_s": float(v[1]), "wave_ms": float(v[2]), "long_ms": float(v[3]),
                     "general_ms": float(v[4]), "docs": int(v[5]), "doc_bytes": int(v[6])}
                    for v in (x.cpu().tolist() for x in allr)]
    stats = be.last_stats()
    doc_bytes = int(offs[-1])
    alg_bytes = doc_bytes + ALG_BYTES_PER_DOC * n
    kern_ms = per[cfg["kernel"]]                 # the dominant kernel's average launch
    achieved = alg_bytes / (kern_ms / 1e3) / 1e9 if kern_ms > 0 else 0.0
    pmc = pmc_summary(cfg_name)
    traffic = issue = None
    if pmc and pmc.get("docs") == n and kern_ms > 0:
        traffic = pmc.get("hbm_bytes_per_launch")
        c = pmc.get("counters_per_launch", {})
        if "SQ_INSTS_VALU" in c:
            ks = kern_ms / 1e3
            issue = {"valu": {"achieved": c["SQ_INSTS_VALU"] / ks, "peak": VALU_PEAK,
                              "frac": c["SQ_INSTS_VALU"] / ks / VALU_PEAK},
                     "salu": {"achieved": c["SQ_INSTS_SALU"] / ks, "peak": SALU_PEAK,
                              "frac": c["SQ_INSTS_SALU"] / ks / SALU_PEAK},
                     "unit": "wave-instructions/s",
                     "active_inst_frac": pmc.get("frac_active_inst"), "wait_frac": pmc.get("frac_wait_any"),
                     "source": "profiles/pmc_current.json (%s)" % pmc.get("source", "")}
    res = {
        "n": n, "elapsed": elapsed, "steps": steps, "doc_bytes": doc_bytes,
        "value": n * steps / elapsed,
        "input_GBps": doc_bytes * steps / elapsed / 1e9,
        "passes_hist": [int(x) for x in stats.passes[:3]],
        "kernels": {"wave_ms": per[0], "long_ms": per[1], "general_ms": per[2],
                    "last_batch": {"wave_docs": int(stats.short_docs), "long_docs": int(stats.long_docs),
                                   "general_docs": int(stats.general_docs),
                                   "long_requeue_reasons": [int(x) for x in stats.long_requeue]}},
        "roofline": {"bound": "hbm", "kernel": cfg["name"], "achieved": achieved, "peak": HBM_PEAK_GBPS,
                     "unit": "GB/s", "frac": achieved / HBM_PEAK_GBPS, "traffic": traffic,
                     "alg_bytes_per_launch": alg_bytes, "issue": issue},
        "per_rank": per_rank,
    }
    gpu_out = (d_out.cpu().numpy().view(cld_amd.RESULT_DTYPE) if rank == 0 else None)
    del d_buf, d_offs, d_out
    return res, buf, offs, gpu_out


def host_path(n, steps, rank):
    """cld_detect_batch from host memory (C2): pageable numpy buffers (page-
    locked for the call, or staged through the runtime's pinned chunk buffers)
    and pinned ones (cld_host_alloc: DMA'd directly).  Both legs reuse their
    result array, as a service would.  docs/s including PCIe both ways."""
    import cld_amd
    import corpus
    buf, offs = corpus.c2(n, seed=corpus.SEEDS["c2"] + 7919 * rank)
    out = {}
    pb = cld_amd.host_array(len(buf), np.uint8)
    pb[:] = buf
    po = cld_amd.host_array(len(offs), np.uint64)
    po[:] = offs
    pout = cld_amd.host_array(n, cld_amd.RESULT_DTYPE)
    out_pageable = np.zeros(n, dtype=cld_amd.RESULT_DTYPE)
    for kind, (b, o) in (("pageable", (buf, offs)), ("pinned", (pb, po))):
        cld_amd.detect_batch(buf=b, offsets=o, out=out_pageable)   # warm (staging buffers grow once)
        t0 = time.perf_counter()
        for _ in range(steps):
            if kind == "pinned":
                rc = cld_amd.lib().cld_detect_batch(b.ctypes.data, o.ctypes.data, n, pout.ctypes.data, 0)
                assert rc == 0, rc
            else:
                cld_amd.detect_batch(buf=b, offsets=o, out=out_pageable)
        dt = time.perf_counter() - t0
        out[kind] = {"value": n * steps / dt, "unit": "docs/s", "ms_per_step": dt / steps * 1e3,
                     "input_GBps": float(offs[-1]) * steps / dt / 1e9}
    return out


def launch_ranks(n, Backend):
    """`--gpus n` without a launcher: n ranks under torch.distributed.run, as a
    child process (nothing here has touched a GPU), with this command line.
    Returns the exit code."""
    import socket
    import subprocess
    have = Backend.device_count()
    if have < n:
        print("bench.py: --gpus %d asked, but %d GPU(s) are visible; not measuring" % (n, have), file=sys.stderr)
        return 3
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=%d" % n,
           "--master-addr=127.0.0.1", "--master-port=%d" % port, os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=0, help="timed steps (default: per config)")
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--docs", type=int, default=0, help="documents per GPU (default: config size)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-sub", action="store_true", help="skip the C3 sub-measurement of a C2 run")
    ap.add_argument("--no-host", action="store_true", help="skip the host-memory path measurement")
    args = ap.parse_args()
    if args.gpus < 1:
        sys.exit("bench.py: --gpus must be >= 1")
    Backend = backend_class()

    if "WORLD_SIZE" not in os.environ:
        if args.gpus > 1:
            sys.exit(launch_ranks(args.gpus, Backend))
        world = 1
    else:
        world = int(os.environ["WORLD_SIZE"])
        if world != args.gpus:
            sys.exit("bench.py: --gpus %d but the launcher started %d rank(s) (WORLD_SIZE); refusing a "
                     "line whose n_gpus would not be what was asked" % (args.gpus, world))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))

    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group(backend=Backend.dist_backend)
    be = Backend(local)

    cfg = CONFIGS[args.config]
    n = args.docs or cfg["docs"]
    steps = args.steps or cfg["steps"]
    head, buf, offs, gpu_out = measure(args.config, n, steps, args.warmup, rank, dist, be)
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args.config, buf, offs, gpu_out, args.cpu_seconds,
                           200_000 if args.config in ("c2", "c2n", "c4") else 20_000)
    del buf, offs, gpu_out

    sub = None
    if args.config == "c2" and not args.no_sub:
        c3n = CONFIGS["c3"]["docs"] if not args.docs else max(1000, args.docs // 10)
        r3, b3, o3, g3 = measure("c3", c3n, CONFIGS["c3"]["steps"], 1, rank, dist, be)
        sub = {"metric": "docs/sec", "value": r3["value"] * world, "unit": "docs/s",
               "workload": CONFIGS["c3"]["workload"], "docs_per_gpu": c3n, "steps": r3["steps"],
               "ms_per_step": r3["elapsed"] / r3["steps"] * 1e3, "input_GBps": r3["input_GBps"] * world,
               "passes_hist": r3["passes_hist"], "kernels": r3["kernels"], "roofline": r3["roofline"],
               "per_rank": r3["per_rank"],
               "cpu_baseline": (cpu_baseline("c3", b3, o3, g3, args.cpu_seconds, 4_000)
                                if rank == 0 and world == 1 and not args.no_cpu_baseline else None)}
        del b3, o3, g3
    host = None
    if args.config == "c2" and not args.no_host and world == 1:
        host = host_path(n, 10, rank)
        host["kernel_only_docs_per_s"] = head["value"]
        host["pinned_vs_kernel_only"] = host["pinned"]["value"] / head["value"]

    if rank != 0:
        if dist:
            dist.destroy_process_group()
        return
    line = {
        "metric": "docs/sec",
        "value": head["value"] * world,
        "unit": "docs/s",
        "n_gpus": world,
        "steps": steps,
        "warmup": args.warmup,
        "ms_per_step": head["elapsed"] / steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (seeded corpus.py; vocabularies from the reference's octa tables; quadgram table: "
                "the synthetic Q1 (the real quadchrome table is a missing blob))",
        "config": {"workload": cfg["workload"], "docs_per_gpu": n, "bytes_per_gpu": head["doc_bytes"],
                   "mean_doc_bytes": head["doc_bytes"] / n, "parallelism": "document shards, %d rank(s)" % world},
        "input_GBps": (sum(r["doc_bytes"] for r in head["per_rank"]) * steps / head["elapsed"] / 1e9
                       if head["per_rank"] else head["input_GBps"]),
        "passes_hist": head["passes_hist"],
        "kernels": head["kernels"],
        "roofline": head["roofline"],
        "per_rank": head["per_rank"],
        "cpu_baseline": cpu,
        "c3": sub,
        "host_path": host,
        "tables": be.version(),
    }
    print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
