"""The C-ABI library loads and exports every symbol include/*.h declares (no GPU calls)."""
import ctypes
import os
import re

import cld_amd

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared(header):
    src = open(os.path.join(ROOT, "include", header)).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return set(re.findall(r"\b([a-z_][a-z0-9_]*)\s*\(", src)) - {"sizeof"}


def test_library_exports_every_declared_symbol():
    assert os.path.exists(cld_amd.LIB_PATH), "run __graft_entry__.build() first"
    lib = ctypes.CDLL(cld_amd.LIB_PATH)
    names = declared("cld_mi355x.h") | declared("wrapper.h")
    assert {"detect_language", "cld_detect_batch"} <= names
    for n in sorted(names):
        assert hasattr(lib, n), n
    assert set(cld_amd.EXPORTS) <= names


def test_wrapper_header_matches_reference_signature():
    src = open(os.path.join(ROOT, "include", "wrapper.h")).read()
    assert "const char* detect_language(const char *text);" in src


def test_result_record_layout():
    assert cld_amd.RESULT_DTYPE.itemsize == 40
    assert [cld_amd.RESULT_DTYPE.fields[f][1] for f in ("lang3", "summary_lang", "percent3", "is_reliable",
                                                       "text_bytes", "normalized3")] == [0, 6, 8, 11, 12, 16]


def test_chunk_record_layout():
    """cld_chunk = ResultChunk (compact_lang_det.h:147-153): int offset, int32 bytes, uint16 lang1, uint16 pad."""
    assert cld_amd.CHUNK_DTYPE.itemsize == 12
    assert [cld_amd.CHUNK_DTYPE.fields[f][1] for f in ("offset", "bytes", "lang1", "pad")] == [0, 4, 8, 10]
