"""Full-size corpora (BASELINE configs C2/C3/C4, and a C5 sample) for the GPU
suite's reference sweep (tests/test_gpu_zfullsize.py).

Generating them takes minutes of host time (C3: 100K pages of 16 KB; C5's long
documents are cut from 16-64 KB pages), so `prefetch()` -- called from
conftest.py when a session selects the GPU tests -- starts one generator
process per corpus at session start; they write raw .npy files to a cache
directory while the rest of the GPU suite runs, and `load()` waits for them.
Test infrastructure only: the corpora are corpus.py's, bit for bit.

    python tests/fullsize.py <name> <outdir>      (one generator process)
"""
import os
import subprocess
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)

# name -> (generator, documents): C2, C3 and C4 whole, as BASELINE.json sizes
# them; C5 as a 200K-document sample of its 100M stream
CORPORA = {
    "c2": ("c2", 1_000_000),
    "c3": ("c3", 100_000),
    "c4": ("c4", 1_100_000),
    "c5": ("c5", 200_000),
    "html": ("html", 100_000),      # HTML pages (is_plain_text = false), a quarter with 4-byte characters
}


def cache_dir():
    # keyed by the generator's source, so a changed corpus.py never reads a stale cache
    import hashlib
    with open(os.path.join(ROOT, "language-detector_amd", "corpus.py"), "rb") as f:
        key = hashlib.sha256(f.read()).hexdigest()[:12]
    d = os.environ.get("CLD_CORPUS_CACHE") or os.path.join(os.environ.get("TMPDIR", "/tmp"),
                                                          "cld_corpus_%d_%s" % (os.getuid(), key))
    os.makedirs(d, exist_ok=True)
    return d


def _paths(name):
    d = cache_dir()
    return os.path.join(d, name + ".buf.npy"), os.path.join(d, name + ".offs.npy"), os.path.join(d, name + ".done")


_procs = {}


def prefetch(names=None):
    """Start the generators of every corpus not already cached (non-blocking)."""
    for name in names or CORPORA:
        if os.path.exists(_paths(name)[2]) or name in _procs:
            continue
        log = open(os.path.join(cache_dir(), name + ".log"), "w")
        _procs[name] = subprocess.Popen([sys.executable, os.path.abspath(__file__), name, cache_dir()],
                                        stdout=log, stderr=subprocess.STDOUT)


def load(name, timeout=900):
    """(buf, offsets) of corpus `name`, generating it here if no prefetch did."""
    bp, op, done = _paths(name)
    if not os.path.exists(done):
        if name not in _procs:
            prefetch([name])
        p = _procs[name]
        t0 = time.time()
        while p.poll() is None:
            if time.time() - t0 > timeout:
                p.kill()
                raise TimeoutError("corpus %s not generated in %d s" % (name, timeout))
            time.sleep(1)
        if p.returncode != 0 or not os.path.exists(done):
            raise RuntimeError("corpus generator %s failed (%s)" % (name, os.path.join(cache_dir(), name + ".log")))
    return np.load(bp), np.load(op)


def _generate(name, outdir):
    sys.path.insert(0, os.path.join(ROOT, "language-detector_amd"))
    import corpus
    gen, n = CORPORA[name]
    t0 = time.time()
    buf, offs = corpus.html(n, seed=77, emoji=0.25) if gen == "html" else corpus.GENERATORS[gen](n)
    bp, op, done = (os.path.join(outdir, name + s) for s in (".buf.npy", ".offs.npy", ".done"))
    np.save(bp + ".tmp.npy", buf)
    np.save(op + ".tmp.npy", offs)
    os.replace(bp + ".tmp.npy", bp)
    os.replace(op + ".tmp.npy", op)
    with open(done, "w") as f:
        f.write("%d documents, %d bytes, %.1f s\n" % (len(offs) - 1, len(buf), time.time() - t0))


if __name__ == "__main__":
    _generate(sys.argv[1], sys.argv[2])
