"""Write / read CLD2 dynamic data files ("cld2_data_file00") -- test and tooling helper.

Restates the reference's writer and reader for the format in
cld2/internal/cld2_dynamic_data.h:22-147:
  * header size          cld2_dynamic_data.cc:45-49 (16-byte marker + 20 u32 + 10 u32 per table)
  * field order          cld2_dynamic_data_extractor.cc:71-108
  * block layout         cld2_dynamic_data_extractor.cc:110-158 (data block order) and
                         alignAll :199-290 (every block 16-byte aligned; NUL-terminated
                         remap string / fast state / recognized-scripts string)
  * table order          cld2_dynamic_data_extractor.cc:53-60 == loader :253-260
The tables come from a CLDT blob (tools/cldt.py).  CLDT does not keep the
tables' kRecognizedLangScripts strings (debug text, never read on the
detection path), so the writer stores `recognized` (default "") for each.

Used by tests/test_dynamic_data.py to produce data files the product library
must import (cld_load_data_from_file / cld_convert_data_file).

    python tools/cld2_data_file.py CLDT_IN DATA_FILE_OUT
"""
import struct
import sys

import cldt

MARKER = b"cld2_data_file00"
TABLE_SECTIONS = (cldt.CJK_COMPAT, cldt.DELTA_BI, cldt.DISTINCT_BI, cldt.QUAD, cldt.QUAD2,
                  cldt.DELTA_OCTA, cldt.DISTINCT_OCTA)
UTF8_FIELDS = ("state0", "state0_size", "total_size", "max_expand", "entry_shift", "bytes_per_entry",
               "losub", "hiadd")
TABLE_FIELDS = ("size_one", "size", "key_mask", "build_date", "t_off", "t_len", "i_off", "i_len",
                "s_off", "s_len")


def header_size(n_tables):
    return 16 + 20 * 4 + n_tables * 10 * 4


def _align(off, a=16):
    return (off + a - 1) // a * a


def unigram_from_blob(blob):
    """The CJK unigram property machine (cld_generated_CjkUni_obj) of a CLDT blob."""
    b = blob.raw(cldt.CJK_UNI_PROP)
    state0, s0size, total, shift, bpe, losub, hiadd = struct.unpack_from("<7I", b, 0)
    assert bpe == 1
    return dict(state0=state0, state0_size=s0size, total_size=total, max_expand=0, entry_shift=shift,
                bytes_per_entry=1, losub=losub, hiadd=hiadd, state_table=b[48:48 + total])


def build(blob, recognized=b"", n_tables=7):
    """CLDT blob -> bytes of a cld2_data_file00 (writeDataFile, extractor :45-158)."""
    u = unigram_from_blob(blob)
    remap_base = bytes(4)                 # one {0,0,0} RemapEntry (cld_generated_cjk_uni_prop_80.cc:7092)
    remap_string = b"\0"                  # strlen("")+1
    expected = blob.raw(cldt.EXPECTED_SCORE)
    tables = [blob.table(s) for s in TABLE_SECTIONS[:n_tables]]
    # alignAll: offsets of every block
    off = header_size(len(tables))
    blocks = []

    def place(data):
        nonlocal off
        off = _align(off)
        blocks.append((off, data))
        start = off
        off += len(data)
        return start, len(data)

    st = place(u["state_table"])
    rb = place(remap_base)
    rs = place(remap_string)
    off = _align(off)                     # fast_state absent: offset 0, length 0
    es = place(expected)
    th = []
    for t in tables:
        nb = t["size"]
        tb = place(t["buckets"][:nb].tobytes())
        ib = place(t["ind"].tobytes())
        sb = place(recognized + b"\0")
        th.append((t["size_one"], t["size"], t["key_mask"], t["build_date"]) + tb + ib + sb)
    total = off
    out = bytearray(total)
    out[0:16] = MARKER
    hdr = [total] + [u[f] for f in UTF8_FIELDS] + [st[0], st[1], rb[0], rb[1], rs[0], rs[1], 0, 0,
                                                  es[0], es[1], len(tables)]
    struct.pack_into("<%dI" % len(hdr), out, 16, *hdr)
    pos = 16 + 4 * len(hdr)
    for row in th:
        struct.pack_into("<10I", out, pos, *row)
        pos += 40
    assert pos == header_size(len(tables))
    for o, data in blocks:
        out[o:o + len(data)] = data
    return bytes(out)


def parse(data):
    """cld2_data_file00 bytes -> dict (loadInternal, loader :41-146)."""
    if data[:16] != MARKER:
        raise ValueError("Malformed header: bad file marker!")
    v = struct.unpack_from("<20I", data, 16)
    hdr = dict(zip(("total",) + UTF8_FIELDS + ("st_off", "st_len", "rb_off", "rb_len", "rs_off", "rs_len",
                                              "fs_off", "fs_len", "es_off", "es_len", "n_tables"), v))
    hdr["tables"] = [dict(zip(TABLE_FIELDS, struct.unpack_from("<10I", data, 96 + 40 * i)))
                     for i in range(hdr["n_tables"])]
    if hdr["total"] != len(data):
        raise ValueError("File size mismatch")
    return hdr


def main():
    blob = cldt.Blob.load(sys.argv[1])
    data = build(blob)
    with open(sys.argv[2], "wb") as f:
        f.write(data)
    print("wrote %s: %d bytes, 7 tables" % (sys.argv[2], len(data)))


if __name__ == "__main__":
    main()
