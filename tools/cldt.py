"""Reader/writer for the CLDT table blob (layout: language-detector_amd/csrc/cldt_format.h).

Build-time and test-time helper only.  Also carries the two small byte-level
helpers the table tools need (script lookup, quadgram chain + hash), written
from the reference's published algorithm:
  * GetUTF8LetterScriptNum   getonescriptspan.cc:1083 -> utf8statetable.cc:362-411
  * GetQuadHits chain walk   cldutil.cc:315-405
  * QuadHashV2 / Mix         cldutil_shared.cc:167-202
"""
import struct

import numpy as np

MAGIC = 0x54444C43
VERSION = 1

META, SCRIPT_PROP, LOWER_REPL, SCAN_NOT, CJK_UNI_PROP = 1, 2, 3, 4, 5
CJK_COMPAT, DELTA_BI, DISTINCT_BI, QUAD, QUAD2, DELTA_OCTA, DISTINCT_OCTA = 10, 11, 12, 13, 14, 15, 16
EXPECTED_SCORE, LGPROB, LANG_TO_PLANG, PLANG_TO_LANG_LATN, PLANG_TO_LANG_OTHR = 20, 21, 22, 23, 24
ULSCRIPT_RTYPE, ULSCRIPT_DEFAULT_LANG, CLOSEST_ALT, CLOSE_SET = 25, 26, 27, 28
LANG_CODES, LANG_NAMES, ULSCRIPT_CODES, PROVENANCE = 29, 30, 31, 40

META_FIELDS = ("num_languages num_ulscripts lang_to_plang_size english unknown_language "
               "tg_unknown_language chinese chinese_t french italian german spanish hawaiian "
               "ulscript_common ulscript_latin ulscript_cyrillic ulscript_arabic ulscript_hani "
               "ulscript_inherited").split()


class Blob:
    def __init__(self, data: bytes):
        self.data = bytes(data)
        magic, ver, n, _, tbl, _ = struct.unpack_from("<IIIIQQ", self.data, 0)
        if magic != MAGIC or ver != VERSION:
            raise ValueError("not a CLDT v1 blob")
        self.sections = {}
        for i in range(n):
            sid, _, off, size, _ = struct.unpack_from("<IIQQQ", self.data, tbl + 32 * i)
            self.sections[sid] = (off, size)
        self.meta = dict(zip(META_FIELDS, struct.unpack_from("<19I", self.raw(META))))

    @classmethod
    def load(cls, path):
        with open(path, "rb") as f:
            return cls(f.read())

    def raw(self, sid):
        off, size = self.sections[sid]
        return self.data[off:off + size]

    def u8(self, sid):
        return np.frombuffer(self.raw(sid), dtype=np.uint8)

    def u16(self, sid):
        return np.frombuffer(self.raw(sid), dtype="<u2")

    def strings(self, sid):
        b = self.raw(sid)
        n = struct.unpack_from("<I", b, 0)[0]
        offs = struct.unpack_from("<%dI" % (n + 1), b, 4)
        base = 4 + 4 * (n + 1)
        out = []
        for i in range(n):
            s = b[base + offs[i]: base + offs[i + 1] - 1]
            out.append(s.decode("utf-8"))
        return out

    def table(self, sid):
        """CLD2TableSummary section -> dict(size_one,size,key_mask,build_date,buckets,ind)."""
        b = self.raw(sid)
        size_one, size, key_mask, build_date, n_ind, n_b = struct.unpack_from("<6I", b, 0)
        hdr = 32
        buckets = np.frombuffer(b, dtype="<u4", count=4 * n_b, offset=hdr).reshape(n_b, 4)
        ind = np.frombuffer(b, dtype="<u4", count=n_ind, offset=hdr + 16 * n_b)
        return dict(size_one=size_one, size=size, key_mask=key_mask,
                    build_date=build_date, buckets=buckets, ind=ind)

    def script_prop(self):
        b = self.raw(SCRIPT_PROP)
        state0, s0size, total, shift, bpe = struct.unpack_from("<5I", b, 0)
        tbl = np.frombuffer(b, dtype="<u2", count=total, offset=48)
        return state0, shift, tbl


def table_section_bytes(size_one, size, key_mask, build_date, buckets, ind):
    buckets = np.asarray(buckets, dtype="<u4").reshape(-1, 4)
    ind = np.asarray(ind, dtype="<u4")
    hdr = struct.pack("<8I", size_one, size, key_mask, build_date, len(ind), len(buckets), 0, 0)
    return hdr + buckets.tobytes() + ind.tobytes()


def write_blob(path, sections):
    """sections: list of (id, bytes) in order."""
    out = bytearray(32)
    table = []
    for sid, payload in sections:
        while len(out) % 16:
            out.append(0)
        table.append((sid, len(out), len(payload)))
        out += payload
    while len(out) % 16:
        out.append(0)
    tbl_off = len(out)
    for sid, off, size in table:
        out += struct.pack("<IIQQQ", sid, 0, off, size, 0)
    struct.pack_into("<IIIIQQ", out, 0, MAGIC, VERSION, len(table), 0, tbl_off, 0)
    with open(path, "wb") as f:
        f.write(out)


# ---------------------------------------------------------------- byte helpers

def script_num(blob_prop, s: bytes, i: int) -> int:
    """GetUTF8LetterScriptNum(s+i): 1..4-level uint16 state machine, 0 = non-letter."""
    state0, shift, tbl = blob_prop
    c = s[i]
    n = len(s) - i
    base = state0
    if c < 0x80:
        return int(tbl[base + c])
    if (c & 0xE0) == 0xC0 and n >= 2:
        nbytes = 2
    elif (c & 0xF0) == 0xE0 and n >= 3:
        nbytes = 3
    elif (c & 0xF8) == 0xF0 and n >= 4:
        nbytes = 4
    else:
        return 0
    e = int(tbl[base + c])
    for k in range(1, nbytes):
        e = int(tbl[base + (e << shift) + s[i + k]])
    return e


def adv_but_space(c):       # kAdvanceOneCharButSpace, cldutil_shared.h:462
    return 0 if c <= 0x20 else 1 if c < 0xC0 else 2 if c < 0xE0 else 3 if c < 0xF0 else 4


def adv_space_vowel(c):     # kAdvanceOneCharSpaceVowel, cldutil_shared.h:476
    return 1 if (c <= 0x20 or c in b"AEIOUaeiou" or 0x80 <= c < 0xC0) else 0


_MASK0 = (0xFFFFFFFF, 0x000000FF, 0x0000FFFF, 0x00FFFFFF)


def _ld32(t, p):
    return int.from_bytes(t[p:p + 4].ljust(4, b"\0"), "little")


def quad_hash_v2(t: bytes, p: int, n: int) -> int:
    """QuadHashV2(t+p, n), cldutil_shared.cc:196-202 / :167-194."""
    if n == 0:
        return 0
    pre = 0
    if t[p - 1] == 0x20:
        pre |= 0x00004444
    if t[p + n] == 0x20:
        pre |= 0x44440000
    M = 0xFFFFFFFF
    if n <= 4:
        w0 = _ld32(t, p) & _MASK0[n & 3]
        w0 ^= w0 >> 3
        return (w0 ^ pre) & M
    if n <= 8:
        w0 = _ld32(t, p); w0 ^= w0 >> 3
        w1 = _ld32(t, p + 4) & _MASK0[n & 3]; w1 = (w1 ^ (w1 << 4)) & M
        return ((w0 ^ pre) + w1) & M
    w0 = _ld32(t, p); w0 ^= w0 >> 3
    w1 = _ld32(t, p + 4); w1 = (w1 ^ (w1 << 4)) & M
    w2 = _ld32(t, p + 8) & _MASK0[n & 3]; w2 = (w2 ^ (w2 << 2)) & M
    return ((w0 ^ pre) + w1 + w2) & M


def word_quads(word: bytes):
    """Quadgram (offset, len) chain of GetQuadHits over the span ' word ' (cldutil.cc:338-392)."""
    t = b" " + word + b" " + b"  \0" + b"\0" * 16
    limit = len(word) + 2
    src = 1
    out = []
    while src < limit:
        e = src
        e += adv_but_space(t[e]); e += adv_but_space(t[e])
        mid = e
        e += adv_but_space(t[e]); e += adv_but_space(t[e])
        out.append((src, e - src, quad_hash_v2(t, src, e - src)))
        src = e if t[e] == 0x20 else mid
        if src < limit:
            src += adv_space_vowel(t[src])
        else:
            src = limit
    return out
