"""Service text preparation and request handling.

* StripExtras + the cgo C-string cut (handlers.go:150-151, :198-210,
  main.go:77-81) as a GPU kernel (cld_prepare_batch / CLD_FLAG_*), checked
  byte-for-byte against the oracle's sequential rune-by-rune restatement
  (oracle/cld_oracle.c prepare_one) on fuzzed text.
* LanguageDetectorService.handle (handlers.go:31-183, main.go:165-191) against
  the HTTP cases of main_test.go (tests/golden/main_test.json http_cases).
  The es/ms answers of TestStripNames / TestStripLinks need the real quadgram
  table (a missing blob): those two are "parity unpinned" and are compared with
  the oracle on the tables in use instead of the literal.
"""
import json
import os
import random

import numpy as np
import pytest

import cld_amd
import corpus
from service import LanguageDetectorService

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
Q0 = os.path.join(ROOT, "language-detector_amd", "data", "cld2_q0.cldt")


@pytest.fixture(scope="module")
def main_test():
    with open(os.path.join(ROOT, "tests", "golden", "main_test.json"), encoding="utf-8") as f:
        return json.load(f)


def prep(oracle, docs, flags):
    buf, offs = cld_amd.pack(docs)
    b, o = oracle.prepare_batch(buf, offs, flags)
    return [bytes(b[o[i]:o[i + 1]]) for i in range(len(docs))]


# ------------------------------------------------------------ CPU: oracle
def test_oracle_strip_extras_semantics(oracle):
    docs = [b"RT @VictoriaMo02: @SoofyAcosta al fin me contesto \xc3\xa9l wpp jajaja te amo sofy",
            b"Mengalami Turbulensi Dahsyat, 23 Penumpang Avianca Airbus Terluka https://t.co/6SvpzBOKHT "
            b"https://t.co/qYzmaPv7Od",
            b"", b" \t\n\v\f\r ", b"x@y httpx xhttp http @", b"a\xe3\x80\x80b\xc2\xa0c\xc2\x85d\xe2\x80\x8ae",
            b"a\x1cb\x1fc", b"\xe2\x80\x8b zero-width-not-space", b"\xff\xfe @\xff x", b"a\xc2", b"\xe2\x80"]
    want = [b"RT al fin me contesto \xc3\xa9l wpp jajaja te amo sofy ",
            b"Mengalami Turbulensi Dahsyat, 23 Penumpang Avianca Airbus Terluka ",
            b"", b"", b"x@y xhttp ", b"a b c d e ", b"a\x1cb\x1fc ", b"\xe2\x80\x8b zero-width-not-space ",
            b"\xff\xfe x ", b"a\xc2 ", b"\xe2\x80 "]
    assert prep(oracle, docs, 1) == want
    # C-string cut after stripping: a NUL inside a dropped word does not cut
    assert prep(oracle, [b"a\x00b c", b"@x\x00 y", b"\x00"], 3) == [b"a", b"y ", b""]
    assert prep(oracle, [b"a\x00b c"], 2) == [b"a"]


# ------------------------------------------------------------ CPU: handler plumbing
def stub_codes(texts):
    return ["xx" if t.startswith(b"zz") else "en" for t in texts]


def test_handler_cases_without_detection(main_test):
    svc = LanguageDetectorService(dict(main_test["known_languages"]), detect_codes=stub_codes)
    for c in main_test["http_cases"]:
        if c["test"] in ("TestStripNames", "TestStripLinks"):
            continue
        st, body = svc.handle(c["method"], c["path"], "application/json", c["body"].encode())
        assert (st, body.decode()) == (c["status"], c["expected"]), c["test"]


def test_handler_rejects_non_standard_constants(main_test):
    """rapidjson's default parse rejects NaN / Infinity (handlers.go:51-58 -> 400)."""
    svc = LanguageDetectorService(dict(main_test["known_languages"]), detect_codes=stub_codes)
    bad = b'{"error":"Unable to parse request - invalid JSON detected"}'
    for lit in (b"NaN", b"Infinity", b"-Infinity"):
        assert svc.handle("POST", "/", "application/json", b'{"request": [{"text": "a", "n": ' + lit + b'}]}') == (400, bad)


def test_serve_reads_at_most_the_body_limit(main_test):
    """io.LimitReader semantics: a large Content-Length never makes the server
    read (or buffer) past the limit."""
    import http.client
    import threading
    from http.server import ThreadingHTTPServer
    import service as svc_mod
    svc = LanguageDetectorService(dict(main_test["known_languages"]), detect_codes=stub_codes, body_limit=64)
    got = []
    orig = svc.handle
    svc.handle = lambda m, p, ct, body: (got.append(len(body)), orig(m, p, ct, body))[1]
    srv = []
    real = ThreadingHTTPServer.__init__

    def capture(self, *a, **kw):
        real(self, *a, **kw)
        srv.append(self)
    ThreadingHTTPServer.__init__ = capture
    try:
        t = threading.Thread(target=svc_mod.serve, args=(svc, 0), daemon=True)
        t.start()
        while not srv:
            pass
    finally:
        ThreadingHTTPServer.__init__ = real
    port = srv[0].server_address[1]
    body = b'{"request": [{"text": "hello"}]}' + b" " * 4096
    c = http.client.HTTPConnection("127.0.0.1", port, timeout=10)
    c.request("POST", "/", body=body, headers={"Content-Type": "application/json"})
    r = c.getresponse()
    r.read()
    srv[0].shutdown()
    assert got == [64]


def test_serve_oversized_body_is_drained(main_test, monkeypatch):
    """A body past the limit is read to its end and discarded (the reply is
    not lost to a TCP reset, and the keep-alive connection stays usable, as
    with Go's net/http); past DRAIN_LIMIT the server replies and closes."""
    import http.client
    import threading
    import service as svc_mod
    svc = LanguageDetectorService(dict(main_test["known_languages"]), detect_codes=stub_codes, body_limit=64)
    srv = svc_mod.make_server(svc, 0, "127.0.0.1")
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    port = srv.server_address[1]
    try:
        c = http.client.HTTPConnection("127.0.0.1", port, timeout=10)
        body = b'{"request": [{"text": "hello"}]}' + b" " * 200000
        for _ in range(2):                                   # same connection twice
            c.request("POST", "/", body=body, headers={"Content-Type": "application/json"})
            r = c.getresponse()
            assert r.status in (200, 203) and b"iso6391code" in r.read()
        monkeypatch.setattr(svc_mod, "DRAIN_LIMIT", 1000)
        c = http.client.HTTPConnection("127.0.0.1", port, timeout=10)
        c.request("POST", "/", body=body, headers={"Content-Type": "application/json"})
        r = c.getresponse()
        assert r.status in (200, 203) and r.getheader("Connection") == "close" and b"iso6391code" in r.read()
    finally:
        srv.shutdown()


def test_handler_edge_semantics(main_test):
    svc = LanguageDetectorService(dict(main_test["known_languages"]), detect_codes=stub_codes)
    ok = b'{"request": [{"text": "hi"}]}'
    assert svc.handle("POST", "/", "text/plain", ok) == (400, b'{"error":"Content-Type must be set to application/json"}')
    assert svc.handle("PUT", "/", "application/json", ok)[0] == 404
    assert svc.handle("POST", "/", "application/json", b"null") == (200, b"")
    assert svc.handle("POST", "/", "application/json", b'{"req": []}')[0] == 400
    assert svc.handle("POST", "/", "application/json", b"[1]")[0] == 400
    assert svc.handle("POST", "/", "application/json", b'{"request": 5}') == (200, b'{"response":[]}')
    # non-string text -> "" -> en; unknown code -> "Unknown" + 203; the last status assignment wins
    st, body = svc.handle("POST", "/", "application/json",
                          b'{"request": [{"text": 7}, {"x": 1}, {"text": "zz"}]}')
    assert st == 203 and body == (b'{"response":[{"iso6391code":"en","name":"English"},'
                                  b'{"error":"Missing text key"},{"iso6391code":"xx","name":"Unknown"}]}')
    st, _ = svc.handle("POST", "/", "application/json", b'{"request": [{"text": "zz"}, {"x": 1}]}')
    assert st == 400
    # first member of a duplicated name wins (rapidjson FindMember)
    seen = []
    svc2 = LanguageDetectorService({}, detect_codes=lambda t: seen.extend(t) or ["en"] * len(t))
    svc2.handle("POST", "/", "application/json", b'{"request": [{"text": "a", "text": "b"}]}')
    assert seen == [b"a"]
    # body limit: a truncated body is invalid JSON
    big = b'{"request": [{"text": "' + b"a" * (1 << 20) + b'"}]}'
    assert svc.handle("POST", "/", "application/json", big)[0] == 400
    # raw non-UTF-8 bytes in a string survive to the detector unchanged
    seen.clear()
    svc2.handle("POST", "/", "application/json", b'{"request": [{"text": "\xff\xfe\\u0000x"}]}')
    assert seen == [b"\xff\xfe\x00x"]


# ------------------------------------------------------------ GPU
def fuzz_docs(n, seed):
    rng = random.Random(seed)
    atoms = [b" ", b"  ", b"\t", b"\n", b"\r\n", b"\x0b", b"\x0c", b"\xc2\x85", b"\xc2\xa0", b"\xe1\x9a\x80",
             b"\xe2\x80\x80", b"\xe2\x80\x8a", b"\xe2\x80\x8b", b"\xe2\x80\xa8", b"\xe2\x80\xa9", b"\xe2\x80\xaf",
             b"\xe2\x81\x9f", b"\xe3\x80\x80", b"\xe3\x80\x81", b"@", b"@user", b"http", b"https://t.co/x",
             b"htt", b"ht", b"word", b"caf\xc3\xa9", b"\xd0\xbc\xd0\xb8\xd1\x80", b"\x00", b"\xff", b"\xc2",
             b"\xe2\x80", b"\xe2", b"\x80", b"\xed\xa0\x80", b"\xf0\x9f\x98\x80", b"\x1c", b"x", b"RT", b":"]
    docs = []
    for _ in range(n):
        k = rng.choice([0, 1, 3, 8, 20, 40, 90])
        docs.append(b"".join(rng.choice(atoms) for _ in range(k)))
    return docs


@pytest.mark.gpu
@pytest.mark.parametrize("flags", [1, 2, 3])
def test_gpu_prepare_matches_oracle(gpu, oracle, flags):
    docs = fuzz_docs(20000, 7 + flags)
    b2, o2 = corpus.c2(3000)
    docs += [bytes(b2[o2[i]:o2[i + 1]]) for i in range(3000)]
    b5, o5 = corpus.c5(300)
    docs += [bytes(b5[o5[i]:o5[i + 1]]) for i in range(300)]
    buf, offs = cld_amd.pack(docs)
    gb, go = cld_amd.prepare_batch(buf=buf, offsets=offs, flags=flags)
    rb, ro = oracle.prepare_batch(buf, offs, flags)
    assert np.array_equal(go, ro)
    bad = [i for i in range(len(docs)) if bytes(gb[go[i]:go[i + 1]]) != bytes(rb[ro[i]:ro[i + 1]])]
    assert not bad, (bad[:5], docs[bad[0]])


@pytest.mark.gpu
def test_gpu_detect_with_preparation_flags(gpu, oracle):
    docs = fuzz_docs(3000, 99)
    b2, o2 = corpus.c2(3000)
    docs += [b"@user " + bytes(b2[o2[i]:o2[i + 1]]) + b" http://x.y/z" for i in range(3000)]
    b3, o3 = corpus.c3(20)
    docs += [bytes(b3[o3[i]:o3[i + 1]]) for i in range(20)]
    buf, offs = cld_amd.pack(docs)
    got = cld_amd.detect_batch(buf=buf, offsets=offs, flags=3)
    pb, po = oracle.prepare_batch(buf, offs, 3)
    ref = oracle.detect_batch(pb, po, threads=8)
    for f in ("lang3", "summary_lang", "percent3", "is_reliable", "text_bytes", "normalized3"):
        assert np.array_equal(got[f], ref[f]), f


@pytest.mark.gpu
def test_gpu_service_http_cases(gpu, oracle, main_test, tmp_path):
    import cld2_data_file
    import cldt
    svc = LanguageDetectorService(dict(main_test["known_languages"]))
    names = dict(main_test["known_languages"])
    for c in main_test["http_cases"]:
        st, body = svc.handle(c["method"], c["path"], "application/json", c["body"].encode())
        if c["test"] in ("TestStripNames", "TestStripLinks", "TestValidInput"):
            # synthetic quadgram table in use: the answer is the oracle's on the prepared text
            text = json.loads(c["body"])["request"][0]["text"].encode()
            pb, po = oracle.prepare_batch(np.frombuffer(text, np.uint8), np.array([0, len(text)], np.uint64), 3)
            lang = int(oracle.detect_batch(pb, po)[0]["summary_lang"])
            code = oracle.code(oracle.english if lang == oracle.unknown else lang)
            want = {"response": [{"iso6391code": code, "name": names.get(code, "Unknown")}]}
            assert json.loads(body) == want and st == (200 if code in names else 203), c["test"]
        else:
            assert (st, body.decode()) == (c["status"], c["expected"]), c["test"]
    # with the empty quadgram table (loaded as CLD2 dynamic data) TestValidInput's literal holds
    dyn = tmp_path / "q0.cld2_data_file00"
    dyn.write_bytes(cld2_data_file.build(cldt.Blob.load(Q0)))
    cld_amd.load_data_from_file(str(dyn))
    try:
        c = next(c for c in main_test["http_cases"] if c["test"] == "TestValidInput")
        st, body = svc.handle("POST", "/", "application/json", c["body"].encode())
        assert (st, body.decode()) == (c["status"], c["expected"])
    finally:
        cld_amd.unload_data()
