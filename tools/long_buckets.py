"""k_long cost by document length: C5's long documents (one-language C3
pages on or off) bucketed by length, each bucket timed alone (kernel ms per
MB of text).  Usage: long_buckets.py [mono_frac ...]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "language-detector_amd"))


def main():
    import importlib
    fr = sys.argv[1:] or ["0", "0.25"]
    import cld_amd
    cld_amd.init_device(0, tables=cld_amd.SYNTH_TABLES)
    for m in fr:
        os.environ["CLD_C3_MONO_FRAC"] = m
        import corpus
        corpus = importlib.reload(corpus)
        buf, offs = corpus.c5(400_000)
        offs = offs.astype(np.int64)
        lens = np.diff(offs)
        edges = [257, 1024, 2048, 4096, 8192, 16384, 32768, 65537]
        for lo, hi in zip(edges[:-1], edges[1:]):
            idx = np.nonzero((lens >= lo) & (lens < hi))[0]
            if len(idx) == 0:
                continue
            docs = [bytes(buf[offs[i]:offs[i + 1]]) for i in idx]
            b, o = cld_amd.pack(docs)
            cld_amd.detect_batch(buf=b, offsets=o)
            ms = []
            for _ in range(3):
                cld_amd.detect_batch(buf=b, offsets=o)
                ms.append(cld_amd.last_stats(0).long_ms)
            st = cld_amd.last_stats(0)
            mb = len(b) / 1e6
            print("mono %s len [%5d,%5d): %6d docs %7.2f MB  long %8.3f ms  %6.2f ms/MB  passes %s" %
                  (m, lo, hi, len(idx), mb, min(ms), min(ms) / mb, list(st.passes)),
                  flush=True)


if __name__ == "__main__":
    main()
