"""ctypes binding of oracle/_ref/librefcld2.so -- the reference CLD2 itself,
built in its dynamic-data mode (oracle/refcld/).  TEST INFRASTRUCTURE ONLY:
tests use it to pin the oracle end to end; bench.py may time it as the
"reference" CPU baseline.  The tables are written as a cld2_data_file00 from
a CLDT blob by tools/cld2_data_file.py and read by the reference's loader."""
import ctypes
import os
import subprocess
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
LIB = os.path.join(HERE, "_ref", "librefcld2.so")

RESULT_DTYPE = np.dtype([("lang3", "<i4", 3), ("percent3", "<i4", 3), ("normalized3", "<f8", 3),
                         ("text_bytes", "<i4"), ("summary_lang", "<i4"), ("is_reliable", "<i4"),
                         ("n_chunks", "<i4")])
CHUNK_DTYPE = np.dtype([("offset", "<i4"), ("bytes", "<i4"), ("lang1", "<u2"), ("pad", "<u2")])


class Hints(ctypes.Structure):
    _fields_ = [("content_language_hint", ctypes.c_char_p), ("tld_hint", ctypes.c_char_p),
                ("encoding_hint", ctypes.c_int32), ("language_hint", ctypes.c_int32)]


MANIFEST = os.path.join(HERE, "_ref", "librefcld2.manifest.json")


def available():
    return os.path.exists(LIB) or os.path.isdir("/root/reference/cld2/internal")


def verify_build():
    """Raise unless oracle/_ref/librefcld2.so is present and was built from
    this tree's recipe: its manifest (oracle/refcld/manifest.py, written at
    link time) must name this library's sha256 and the current sha256 of
    oracle/refcld/refcld.cc and oracle/refcld/Makefile.  Returns the manifest."""
    import hashlib
    import json

    def sha(p):
        with open(p, "rb") as f:
            return hashlib.sha256(f.read()).hexdigest()
    if not os.path.exists(LIB):
        raise RuntimeError("reference checker %s is not built (oracle/refcld/Makefile)" % LIB)
    if not os.path.exists(MANIFEST):
        raise RuntimeError("reference checker has no build manifest %s" % MANIFEST)
    with open(MANIFEST) as f:
        m = json.load(f)
    if m["library"]["sha256"] != sha(LIB):
        raise RuntimeError("librefcld2.so does not match its build manifest")
    for rel, h in m["recipe"].items():
        if sha(os.path.join(ROOT, rel)) != h:
            raise RuntimeError("librefcld2.so was built from another %s than this tree's" % rel)
    if len(m.get("reference_sources", {})) < 18:
        raise RuntimeError("librefcld2.so manifest lists too few reference sources")
    return m


def build():
    subprocess.run(["make", "-s", "-C", os.path.join(HERE, "refcld")], check=True)


_loaded = {}


class RefCLD:
    """One process-wide reference instance (its tables are global state)."""

    def __init__(self, cldt_path):
        import sys
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        import cld2_data_file
        import cldt
        if not os.path.exists(LIB):
            build()
        self.lib = lib = ctypes.CDLL(LIB)
        lib.refcld_load.argtypes = [ctypes.c_char_p]
        lib.refcld_detect.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                      ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
        lib.refcld_detect_batch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
        lib.refcld_detect_batch_flags.argtypes = lib.refcld_detect_batch.argtypes + [ctypes.c_int]
        lib.refcld_detect_flags.argtypes = lib.refcld_detect.argtypes + [ctypes.c_int]
        lib.refcld_detect_batch_vec.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                                ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                                ctypes.c_int]
        fd, path = tempfile.mkstemp(suffix=".cld2_data_file00")
        with os.fdopen(fd, "wb") as f:
            f.write(cld2_data_file.build(cldt.Blob.load(cldt_path)))
        rc = lib.refcld_load(path.encode())
        self.data_file = path
        if rc != 0:
            raise RuntimeError("reference loader rejected %s" % path)

    def detect_batch(self, buf, offsets, plain=None, hints=None, threads=1, flags=0):
        """flags: ExtDetectLanguageSummary's (0x0100 kCLDFlagScoreAsQuads, 0x4000 kCLDFlagBestEffort)."""
        buf = np.ascontiguousarray(buf, dtype=np.uint8)
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        n = len(offsets) - 1
        out = np.zeros(n, dtype=RESULT_DTYPE)
        pl = None if plain is None else np.ascontiguousarray(plain, dtype=np.uint8)
        harr = None
        if hints is not None:
            harr = (Hints * n)(*[Hints(h.content_language_hint, h.tld_hint, h.encoding_hint, h.language_hint)
                                 for h in hints])
        bptr = buf.ctypes.data if buf.size else ctypes.addressof(ctypes.c_uint8(0))
        rc = self.lib.refcld_detect_batch_flags(bptr, offsets.ctypes.data, n, None if pl is None else pl.ctypes.data,
                                                ctypes.cast(harr, ctypes.c_void_p) if harr is not None else None,
                                                out.ctypes.data, threads, int(flags))
        if rc != 0:
            raise RuntimeError("refcld_detect_batch rc=%d" % rc)
        return out

    def detect_batch_vec(self, buf, offsets, plain=None, threads=1, flags=0):
        """Vector mode over a batch, `threads` host threads -> (results, chunks, chunk_offsets),
        document i's vector = chunks[chunk_offsets[i]:chunk_offsets[i + 1]]."""
        buf = np.ascontiguousarray(buf, dtype=np.uint8)
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        n = len(offsets) - 1
        out = np.zeros(n, dtype=RESULT_DTYPE)
        base = np.zeros(n + 1, dtype=np.uint64)
        np.cumsum(np.diff(offsets) + 16, out=base[1:])      # a region of len + 16 chunks per document
        ch = np.zeros(max(int(base[-1]), 1), dtype=CHUNK_DTYPE)
        pl = None if plain is None else np.ascontiguousarray(plain, dtype=np.uint8)
        bptr = buf.ctypes.data if buf.size else ctypes.addressof(ctypes.c_uint8(0))
        rc = self.lib.refcld_detect_batch_vec(bptr, offsets.ctypes.data, n, None if pl is None else pl.ctypes.data,
                                              out.ctypes.data, ch.ctypes.data, base.ctypes.data, threads, int(flags))
        if rc != 0:
            raise RuntimeError("refcld_detect_batch_vec rc=%d" % rc)
        cnt = out["n_chunks"].astype(np.int64)
        assert np.all(cnt <= np.diff(base).astype(np.int64))
        coffs = np.zeros(n + 1, dtype=np.uint64)
        np.cumsum(cnt, out=coffs[1:])
        idx = np.repeat(base[:-1].astype(np.int64) - coffs[:-1].astype(np.int64), cnt) + np.arange(int(coffs[-1]))
        return out, ch[idx], coffs

    def detect_vec(self, doc, plain=True, hints=None, flags=0):
        """ExtDetectLanguageSummary with a ResultChunkVector -> (result, chunks)."""
        b = bytes(doc)
        r = np.zeros(1, dtype=RESULT_DTYPE)
        cap = len(b) + 16
        ch = np.zeros(cap, dtype=CHUNK_DTYPE)
        h = None
        if hints is not None:
            h = Hints(hints.content_language_hint, hints.tld_hint, hints.encoding_hint, hints.language_hint)
        self.lib.refcld_detect_flags(b, len(b), int(plain), ctypes.byref(h) if h is not None else None,
                                     r.ctypes.data, ch.ctypes.data, cap, int(flags))
        return r[0], ch[:int(r[0]["n_chunks"])].copy()


def instance(cldt_path):
    """The reference loaded with `cldt_path`'s tables (reloaded when it changes)."""
    global _loaded
    if _loaded.get("path") != cldt_path:
        r = _loaded.get("ref")
        if r is None:
            r = RefCLD(cldt_path)
        else:
            import sys
            sys.path.insert(0, os.path.join(ROOT, "tools"))
            import cld2_data_file
            import cldt
            fd, path = tempfile.mkstemp(suffix=".cld2_data_file00")
            with os.fdopen(fd, "wb") as f:
                f.write(cld2_data_file.build(cldt.Blob.load(cldt_path)))
            if r.lib.refcld_load(path.encode()) != 0:
                raise RuntimeError("reference loader rejected %s" % path)
            r.data_file = path
        _loaded = {"path": cldt_path, "ref": r}
    return _loaded["ref"]
