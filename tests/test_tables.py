"""Properties of the CLDT blob that the GPU design relies on (no GPU)."""
import ctypes
import struct

import numpy as np

import cldt


def test_blob_sections(blob):
    for sid in (cldt.META, cldt.SCRIPT_PROP, cldt.LOWER_REPL, cldt.SCAN_NOT, cldt.CJK_UNI_PROP, cldt.CJK_COMPAT,
                cldt.DELTA_BI, cldt.DISTINCT_BI, cldt.QUAD, cldt.QUAD2, cldt.DELTA_OCTA, cldt.DISTINCT_OCTA,
                cldt.EXPECTED_SCORE, cldt.LGPROB, cldt.LANG_TO_PLANG, cldt.PLANG_TO_LANG_LATN,
                cldt.PLANG_TO_LANG_OTHR, cldt.ULSCRIPT_RTYPE, cldt.ULSCRIPT_DEFAULT_LANG, cldt.CLOSEST_ALT,
                cldt.CLOSE_SET, cldt.LANG_CODES, cldt.LANG_NAMES, cldt.ULSCRIPT_CODES, cldt.PROVENANCE):
        assert sid in blob.sections, sid
    m = blob.meta
    assert (m["num_languages"], m["num_ulscripts"], m["english"], m["unknown_language"]) == (614, 102, 0, 26)
    codes = blob.strings(cldt.LANG_CODES)
    assert codes[0] == "en" and codes[26] == "un" and codes[16] == "zh"
    # sizes of the real tables (cld2_generated_deltaoctachrome.cc:166-167, distinct :92-93)
    d, x = blob.table(cldt.DELTA_OCTA), blob.table(cldt.DISTINCT_OCTA)
    assert (d["size"], d["key_mask"], d["size_one"]) == (4096, 0xFFFFF000, 988)
    assert (x["size"], x["key_mask"], x["size_one"]) == (2048, 0xFFFFF800, 75)
    assert b"SYNTHETIC" in blob.raw(cldt.PROVENANCE)


def test_bucket_tables_power_of_two_and_aligned(blob):
    for sid in (cldt.CJK_COMPAT, cldt.DELTA_BI, cldt.DISTINCT_BI, cldt.QUAD, cldt.QUAD2, cldt.DELTA_OCTA,
                cldt.DISTINCT_OCTA):
        t = blob.table(sid)
        assert t["size"] == 0 or t["size"] & (t["size"] - 1) == 0
        off, _ = blob.sections[sid]
        assert (off + 32) % 16 == 0            # 16-byte bucket gathers


def test_scan_fast_path_equivalence(blob):
    """UTF8GenericScan's 8-byte fast loop (utf8statetable.cc:486-507) may only
    skip bytes whose state-0 entry stays in state 0 with no exit; then the
    byte-at-a-time loop both restatements run is equivalent."""
    raw = blob.raw(cldt.SCAN_NOT)
    state0, s0size, total, shift, bpe, losub, hiadd, n_remap, n_rstr, has_fast = struct.unpack_from("<10I", raw, 0)
    tbl = np.frombuffer(raw, dtype=np.uint8, count=total, offset=48)
    off = (48 + total + 15) & ~15
    fast = np.frombuffer(raw, dtype=np.uint8, count=256, offset=off)
    lo, hi = losub & 0xFF, hiadd & 0xFF
    for c in range(256):
        if (lo <= c and c + hi < 0x80) or fast[c] == 0:
            assert tbl[state0 + c] == 0, hex(c)


def test_lowercase_is_per_character_with_bounded_growth(oracle, blob):
    """No replace-and-resume remaps (so lowering never carries state across a
    character) and no character grows by more than 1.5x -- the bound the
    kernels size their lowercase buffers by and the reason the reference's
    kExitDstSpaceFull branch is unreachable for spans <= 40,935 bytes."""
    raw = blob.raw(cldt.LOWER_REPL)
    h = struct.unpack_from("<12I", raw, 0)
    off = (48 + h[2] + 15) & ~15
    rem = [struct.unpack_from("4B", raw, off + 4 * i) for i in range(h[7])]
    assert not any(e[0] & 0x80 for e in rem)
    L = oracle.lib
    L.cldo_lower.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_int]
    out = ctypes.create_string_buffer(64)
    worst = 0.0
    for cp in list(range(0, 0x3000)) + list(range(0x3000, 0x110000, 37)):
        if 0xD800 <= cp < 0xE000:
            continue
        b = chr(cp).encode("utf-8")
        n = L.cldo_lower(b, len(b), out, 64)
        worst = max(worst, n / len(b))
    assert worst <= 1.5
    src = "ABC Straße ÀÉÎ".encode()
    n = L.cldo_lower(src, len(src), out, 64)
    assert out.raw[:n].decode() == "abc straße àéî"
