"""Python host binding of libcld_mi355x.so (the C ABI in include/cld_mi355x.h).

Mirrors the reference's caller-facing interface for this path:
  detect_language(text) -> ISO code       main.go:77-81 Detect_language / wrapper.cc:7-16
  detect_batch(docs)    -> cld_result[]   one DetectLanguageSummaryV2 per document
  prepare_batch(docs, flags)              handlers.go:150-151: StripExtras (handlers.go:198-210)
                                          + the cgo C-string cut, as a GPU kernel
  load_data_from_file(path)               CLD2::loadDataFromFile (run-time tables)
There is no CPU fallback: if the HIP library or a GPU is missing, calls raise.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("CLD_MI355X_LIB") or os.path.join(HERE, "build", "libcld_mi355x.so")
# Product default: Q0, the empty quadgram table (cld_version() says "quad=empty-Q0").
# Tests and the benchmark opt into the synthetic Q1 table through CLD_MI355X_TABLES.
Q0_TABLES = os.path.join(HERE, "data", "cld2_q0.cldt")
SYNTH_TABLES = os.path.join(HERE, "data", "cld2_synth_q1.cldt")
FLAG_STRIP_EXTRAS = 1      # include/cld_mi355x.h CLD_FLAG_STRIP_EXTRAS
FLAG_CSTRING = 2           # include/cld_mi355x.h CLD_FLAG_CSTRING
FLAG_HTML = 4              # include/cld_mi355x.h CLD_FLAG_HTML (cld_detect_batch_ex)
FLAG_SCORE_AS_QUADS = 0x0100   # CLD_FLAG_SCORE_AS_QUADS = kCLDFlagScoreAsQuads (compact_lang_det.h:343)
FLAG_BEST_EFFORT = 0x4000      # CLD_FLAG_BEST_EFFORT = kCLDFlagBestEffort (compact_lang_det.h:349)
UNKNOWN_ENCODING = 23      # encodings.h UNKNOWN_ENCODING
UNKNOWN_LANGUAGE = 26      # generated_language.h UNKNOWN_LANGUAGE
LANG_FAILED = 0xFFFF       # include/cld_mi355x.h CLD_LANG_FAILED: a document without a result
EIO, ENOMEM, ENOSPC = -5, -12, -28   # include/cld_mi355x.h error codes

RESULT_DTYPE = np.dtype([("lang3", "<u2", 3), ("summary_lang", "<u2"), ("percent3", "i1", 3),
                         ("is_reliable", "u1"), ("text_bytes", "<i4"), ("normalized3", "<f8", 3)])
assert RESULT_DTYPE.itemsize == 40

# Every symbol include/cld_mi355x.h declares (checked by tests/test_capi.py)
EXPORTS = ("detect_language", "cld_init", "cld_init_device", "cld_shutdown", "cld_detect_batch",
           "cld_detect_batch_device", "cld_plan_shards", "cld_kernel_time", "cld_language_code",
           "cld_language_name", "cld_last_batch_stats", "cld_version", "cld_stage_cycles",
           "cld_load_data_from_file", "cld_load_data_from_raw_address", "cld_unload_data",
           "cld_is_data_dynamic", "cld_export_tables", "cld_convert_data_file",
           "cld_detect_batch_device_ex", "cld_prepare_batch", "cld_host_alloc", "cld_host_free",
           "cld_kernel_times", "cld_detect_batch_ex", "cld_hint_priors", "cld_detect_batch_vec")
CHUNK_DTYPE = np.dtype([("offset", "<i4"), ("bytes", "<i4"), ("lang1", "<u2"), ("pad", "<u2")])   # cld_chunk


class Hints(ctypes.Structure):
    """CLDHints (compact_lang_det.h:134-139) = include/cld_mi355x.h cld_hints."""
    _fields_ = [("content_language_hint", ctypes.c_char_p), ("tld_hint", ctypes.c_char_p),
                ("encoding_hint", ctypes.c_int32), ("language_hint", ctypes.c_int32)]

    @classmethod
    def make(cls, content_language=None, tld=None, encoding=UNKNOWN_ENCODING, language=UNKNOWN_LANGUAGE):
        enc = lambda v: v.encode() if isinstance(v, str) else v
        return cls(enc(content_language), enc(tld), encoding, language)


class BatchStats(ctypes.Structure):
    _fields_ = [("docs", ctypes.c_uint64), ("short_docs", ctypes.c_uint64), ("general_docs", ctypes.c_uint64),
                ("passes", ctypes.c_uint64 * 4), ("short_ms", ctypes.c_double), ("general_ms", ctypes.c_double),
                ("long_docs", ctypes.c_uint64), ("long_ms", ctypes.c_double),
                ("long_requeue", ctypes.c_uint64 * 8)]


class CldError(RuntimeError):
    pass


class PartialBatchError(CldError):
    """CLD_EIO from a batch call: every result is complete except the documents
    in `failed` (summary_lang == LANG_FAILED), which the GPU could not score even
    alone.  `value` is what the call would have returned."""

    def __init__(self, what, value, failed):
        super().__init__("%s: %d document(s) without a result" % (what, int(np.count_nonzero(failed))))
        self.value = value
        self.failed = failed


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


_lib = None


def lib():
    """Load the in-tree HIP library (never a fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise CldError("libcld_mi355x.so is not built (run __graft_entry__.build())")
        L = ctypes.CDLL(LIB_PATH)
        L.detect_language.argtypes = [ctypes.c_char_p]
        L.detect_language.restype = ctypes.c_char_p
        L.cld_init.argtypes = [ctypes.c_char_p, ctypes.c_int]
        L.cld_detect_batch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_uint32]
        L.cld_detect_batch_device.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                              ctypes.c_void_p, ctypes.c_void_p]
        L.cld_language_code.restype = ctypes.c_char_p
        L.cld_language_name.restype = ctypes.c_char_p
        L.cld_version.restype = ctypes.c_char_p
        L.cld_last_batch_stats.argtypes = [ctypes.c_int, ctypes.POINTER(BatchStats)]
        L.cld_init_device.argtypes = [ctypes.c_char_p, ctypes.c_int]
        L.cld_plan_shards.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
        L.cld_kernel_time.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_double),
                                      ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int)]
        L.cld_kernel_times.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int)]
        L.cld_prepare_batch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32,
                                        ctypes.c_void_p, ctypes.c_void_p]
        L.cld_detect_batch_device_ex.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                                 ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p]
        L.cld_load_data_from_file.argtypes = [ctypes.c_char_p]
        L.cld_load_data_from_raw_address.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
        L.cld_export_tables.argtypes = [ctypes.c_char_p]
        L.cld_convert_data_file.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p]
        L.cld_host_alloc.argtypes = [ctypes.c_size_t]
        L.cld_host_alloc.restype = ctypes.c_void_p
        L.cld_host_free.argtypes = [ctypes.c_void_p]
        L.cld_detect_batch_ex.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
                                          ctypes.c_uint32, ctypes.c_void_p]
        L.cld_detect_batch_vec.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
                                           ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                           ctypes.c_void_p]
        L.cld_hint_priors.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.POINTER(Hints),
                                      ctypes.c_void_p, ctypes.c_void_p]
        _lib = L
    return _lib


def load_data_from_file(path):
    """CLD2::loadDataFromFile (compact_lang_det.h:393): scoring tables from a cld2_data_file00."""
    rc = lib().cld_load_data_from_file(path.encode())
    if rc != 0:
        raise CldError("cld_load_data_from_file(%s) failed: %d" % (path, rc))


def load_data_from_raw_address(data):
    """CLD2::loadDataFromRawAddress (compact_lang_det.h:406) over a bytes-like image."""
    b = bytes(data)
    rc = lib().cld_load_data_from_raw_address(ctypes.c_char_p(b), len(b))
    if rc != 0:
        raise CldError("cld_load_data_from_raw_address failed: %d" % rc)


def unload_data():
    rc = lib().cld_unload_data()
    if rc != 0:
        raise CldError("cld_unload_data failed: %d" % rc)


def is_data_dynamic():
    return bool(lib().cld_is_data_dynamic())


def export_tables(path):
    rc = lib().cld_export_tables(path.encode())
    if rc != 0:
        raise CldError("cld_export_tables failed: %d" % rc)


def convert_data_file(data_file, out_cldt, base_cldt=None):
    """cld2_data_file00 + base CLDT -> CLDT file (host only, no GPU)."""
    rc = lib().cld_convert_data_file(data_file.encode(), base_cldt.encode() if base_cldt else None,
                                     out_cldt.encode())
    if rc != 0:
        raise CldError("cld_convert_data_file(%s) failed: %d" % (data_file, rc))


def init(tables=None, n_devices=0):
    rc = lib().cld_init(tables.encode() if tables else None, n_devices)
    if rc != 0:
        raise CldError("cld_init failed: %d" % rc)


def init_device(device, tables=None):
    """One process per GPU: bind the runtime to HIP device `device` (context 0)."""
    rc = lib().cld_init_device(tables.encode() if tables else None, device)
    if rc != 0:
        raise CldError("cld_init_device(%d) failed: %d" % (device, rc))


def plan_shards(offsets, nshards):
    """Contiguous document shards of equal estimated kernel cost (cld_plan_shards; host-only, no GPU)."""
    offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    cuts = np.zeros(nshards + 1, dtype=np.uint64)
    rc = lib().cld_plan_shards(offsets.ctypes.data, len(offsets) - 1, nshards, cuts.ctypes.data)
    if rc != 0:
        raise CldError("cld_plan_shards failed: %d" % rc)
    return cuts.astype(np.int64)


def kernel_time(ctx=0):
    """(short_ms, general_ms, launches) summed over batches since the last call."""
    a, b, n = ctypes.c_double(), ctypes.c_double(), ctypes.c_int()
    rc = lib().cld_kernel_time(ctx, ctypes.byref(a), ctypes.byref(b), ctypes.byref(n))
    if rc != 0:
        raise CldError("cld_kernel_time failed: %d" % rc)
    return a.value, b.value, n.value


def kernel_times(ctx=0):
    """([wave_ms, long_ms, general_ms], launches) summed over batches since the last call."""
    ms = (ctypes.c_double * 3)()
    n = ctypes.c_int()
    rc = lib().cld_kernel_times(ctx, ms, ctypes.byref(n))
    if rc != 0:
        raise CldError("cld_kernel_times failed: %d" % rc)
    return [ms[0], ms[1], ms[2]], n.value


def stage_cycles(ctx=0):
    """Per-stage cycle sums of the wavefront kernel (CLD_PROFILE_STAGES=1)."""
    c = np.zeros(16, dtype=np.uint64)
    rc = lib().cld_stage_cycles(ctx, ctypes.c_void_p(c.ctypes.data))
    if rc != 0:
        raise CldError("cld_stage_cycles failed: %d" % rc)
    return c


def pack(docs):
    """list of str/bytes -> (uint8 buffer, uint64 offsets[n+1])."""
    bs = [d.encode("utf-8") if isinstance(d, str) else bytes(d) for d in docs]
    offs = np.zeros(len(bs) + 1, dtype=np.uint64)
    np.cumsum([len(b) for b in bs], out=offs[1:])
    buf = np.frombuffer(b"".join(bs), dtype=np.uint8) if bs else np.zeros(0, np.uint8)
    return buf, offs


def detect_batch(docs=None, buf=None, offsets=None, flags=0, out=None):
    """One DetectLanguageSummaryV2 per document; flags = FLAG_STRIP_EXTRAS | FLAG_CSTRING
    prepares each text as POST / does before detecting (handlers.go:150-151);
    FLAG_SCORE_AS_QUADS / FLAG_BEST_EFFORT are CLD2's own flags.  out: an
    existing contiguous RESULT_DTYPE array of n entries to fill (a caller that
    reuses its result buffer, as a service would), else a new one."""
    if docs is not None:
        buf, offsets = pack(docs)
    buf = np.ascontiguousarray(buf, dtype=np.uint8)
    offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    n = len(offsets) - 1
    if out is None:
        out = np.zeros(n, dtype=RESULT_DTYPE)
    elif out.dtype != RESULT_DTYPE or out.shape != (n,) or not out.flags["C_CONTIGUOUS"] or not out.flags["WRITEABLE"]:
        raise ValueError("out must be a writeable contiguous array of %d RESULT_DTYPE entries" % n)
    if n == 0:
        return out
    bptr = buf.ctypes.data if buf.size else ctypes.addressof(ctypes.c_uint8(0))
    rc = lib().cld_detect_batch(bptr, offsets.ctypes.data, n, out.ctypes.data, flags)
    if rc == EIO:
        raise PartialBatchError("cld_detect_batch", out, out["summary_lang"] == LANG_FAILED)
    if rc != 0:
        raise CldError("cld_detect_batch failed: %d" % rc)
    return out


def detect_batch_ex(docs=None, buf=None, offsets=None, hints=None, html=False, flags=0):
    """ExtDetectLanguageSummary per document (compact_lang_det.h:324-335):
    html=True scores every document as HTML (is_plain_text = false); hints is
    None or one Hints per document; flags: FLAG_SCORE_AS_QUADS / FLAG_BEST_EFFORT."""
    if docs is not None:
        buf, offsets = pack(docs)
    buf = np.ascontiguousarray(buf, dtype=np.uint8)
    offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    n = len(offsets) - 1
    out = np.zeros(n, dtype=RESULT_DTYPE)
    if n == 0:
        return out
    harr = None
    if hints is not None:
        if len(hints) != n:
            raise ValueError("need one Hints per document")
        harr = (Hints * n)(*hints)
    bptr = buf.ctypes.data if buf.size else ctypes.addressof(ctypes.c_uint8(0))
    rc = lib().cld_detect_batch_ex(bptr, offsets.ctypes.data, n, ctypes.cast(harr, ctypes.c_void_p) if harr else None,
                                   (FLAG_HTML if html else 0) | flags, out.ctypes.data)
    if rc == EIO:
        raise PartialBatchError("cld_detect_batch_ex", out, out["summary_lang"] == LANG_FAILED)
    if rc != 0:
        raise CldError("cld_detect_batch_ex failed: %d" % rc)
    return out


def detect_batch_vec(docs=None, buf=None, offsets=None, hints=None, html=False, chunk_cap=None, flags=0):
    """ExtDetectLanguageSummary with a ResultChunkVector per document:
    (results, chunks [CHUNK_DTYPE], chunk_offsets[n+1]); document i's vector is
    chunks[chunk_offsets[i]:chunk_offsets[i+1]]."""
    if docs is not None:
        buf, offsets = pack(docs)
    buf = np.ascontiguousarray(buf, dtype=np.uint8)
    offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    n = len(offsets) - 1
    out = np.zeros(n, dtype=RESULT_DTYPE)
    coffs = np.zeros(n + 1, dtype=np.uint64)
    if n == 0:
        return out, np.zeros(0, dtype=CHUNK_DTYPE), coffs
    harr = None
    if hints is not None:
        if len(hints) != n:
            raise ValueError("need one Hints per document")
        harr = (Hints * n)(*hints)
    cap = chunk_cap if chunk_cap is not None else 4 * n + 1024
    bptr = buf.ctypes.data if buf.size else ctypes.addressof(ctypes.c_uint8(0))
    for _ in range(2):                                     # second try with the exact size
        chunks = np.zeros(max(cap, 1), dtype=CHUNK_DTYPE)
        rc = lib().cld_detect_batch_vec(bptr, offsets.ctypes.data, n,
                                        ctypes.cast(harr, ctypes.c_void_p) if harr else None,
                                        (FLAG_HTML if html else 0) | flags, out.ctypes.data, chunks.ctypes.data, cap,
                                        coffs.ctypes.data)
        if rc == 0:
            return out, chunks[:int(coffs[-1])], coffs
        if rc == EIO:                                      # some document got no vector (an empty one)
            raise PartialBatchError("cld_detect_batch_vec", (out, chunks[:int(coffs[-1])], coffs),
                                    out["summary_lang"] == LANG_FAILED)
        if rc != ENOSPC or chunk_cap is not None:
            break
        cap = int(coffs[-1])
    raise CldError("cld_detect_batch_vec failed: %d" % rc)


def hint_priors(doc=b"", html=False, hints=None):
    """Host-only ApplyHints (compact_lang_det_impl.cc:1587-1684): (priors, boosts16).
    priors: the trimmed CLDLangPriors as int16 (weight << 10) + language;
    boosts16: prior boosts latn[4] othr[4], whacks latn[4] othr[4] as langprobs."""
    b = doc.encode() if isinstance(doc, str) else bytes(doc)
    p = np.zeros(14, dtype=np.int16)
    q = np.zeros(16, dtype=np.uint32)
    cb = ctypes.create_string_buffer(b, len(b) + 1)
    rc = lib().cld_hint_priors(cb, len(b), 0 if html else 1, ctypes.byref(hints) if hints is not None else None,
                               p.ctypes.data, q.ctypes.data)
    if rc < 0:
        raise CldError("cld_hint_priors failed: %d" % rc)
    return p[:rc].copy(), q


def detect_batch_device(device, d_buf_ptr, d_offsets_ptr, n, d_out_ptr, stream_ptr=None):
    rc = lib().cld_detect_batch_device(device, d_buf_ptr, d_offsets_ptr, n, d_out_ptr, stream_ptr)
    if rc != 0:
        raise CldError("cld_detect_batch_device failed: %d" % rc)


def last_stats(device=0):
    st = BatchStats()
    rc = lib().cld_last_batch_stats(device, ctypes.byref(st))
    if rc != 0:
        raise CldError("cld_last_batch_stats failed: %d" % rc)
    return st


def detect_language(text):
    """main.go:77-81 / wrapper.cc:7-16: NUL-terminated text -> ISO code ('en' for unknown)."""
    b = text.encode("utf-8") if isinstance(text, str) else bytes(text)
    return lib().detect_language(b).decode()


def version():
    return lib().cld_version().decode()


def host_array(n, dtype):
    """numpy array of n elements in pinned host memory (cld_host_alloc): a
    cld_detect_batch on such buffers skips the staging copy.  The memory is
    released with the array."""
    dtype = np.dtype(dtype)
    nbytes = max(1, n * dtype.itemsize)
    p = lib().cld_host_alloc(nbytes)
    if not p:
        raise CldError("cld_host_alloc(%d) failed" % nbytes)
    raw = (ctypes.c_uint8 * nbytes).from_address(p)
    arr = np.frombuffer(raw, dtype=np.uint8)[:n * dtype.itemsize].view(dtype)
    import weakref
    weakref.finalize(raw, lib().cld_host_free, p)
    return arr


def language_code(lang):
    return lib().cld_language_code(int(lang)).decode()


ENGLISH, UNKNOWN_LANGUAGE = 0, 26     # generated_language.h Language enum values


def result_code(r):
    """compact_lang_det.cc:91-93 + wrapper.cc:14: the ISO code detect_language() returns
    for a cld_result (UNKNOWN -> ENGLISH)."""
    lang = int(r["summary_lang"])
    return language_code(ENGLISH if lang == UNKNOWN_LANGUAGE else lang)


def language_name(lang):
    return lib().cld_language_name(int(lang)).decode()


def prepare_batch(docs=None, buf=None, offsets=None, flags=FLAG_STRIP_EXTRAS | FLAG_CSTRING):
    """handlers.go:150-151 text preparation on the GPU (cld_prepare_batch):
    StripExtras (handlers.go:198-210) and/or the cgo C-string cut.  -> (buf, offsets)."""
    if docs is not None:
        buf, offsets = pack(docs)
    buf = np.ascontiguousarray(buf, dtype=np.uint8)
    offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    n = len(offsets) - 1
    out = np.zeros(int(offsets[-1] - offsets[0]) + n + 1, dtype=np.uint8)
    oo = np.zeros(n + 1, dtype=np.uint64)
    bptr = buf.ctypes.data if buf.size else ctypes.addressof(ctypes.c_uint8(0))
    rc = lib().cld_prepare_batch(bptr, offsets.ctypes.data, n, flags, out.ctypes.data, oo.ctypes.data)
    if rc != 0:
        raise CldError("cld_prepare_batch failed: %d" % rc)
    return out[:int(oo[-1])], oo


def strip_extras(text):
    """handlers.go:198-210 StripExtras for one text (GPU kernel, no C-string cut)."""
    b = text.encode("utf-8") if isinstance(text, str) else bytes(text)
    out, oo = prepare_batch([b], flags=FLAG_STRIP_EXTRAS)
    r = bytes(out[:int(oo[1])])
    return r.decode("utf-8", "surrogateescape") if isinstance(text, str) else r
