"""Generate tests/golden/*.json fixtures from the reference's own test data.

Run in the build container only (reads /root/reference as text; the GPU box
never sees the reference).  Produces DATA fixtures, not copies of source:

  cld2_unittest.json   For every document of cld2_unittest.cc:51-190 (input
                       strings from unittest_data.h) and every document
                       dumped in cld2/docs/CLD2UnitTestOutput.html: the input
                       text, the DocTote dump(s), "N chunks scored" and the
                       summary line printed by DetectLanguageSummaryV2
                       (compact_lang_det_impl.cc:1949-2043, tote.cc:253-264).
  cld2_verbose.json    Per-document hit-buffer / linear-buffer / chunk-summary
                       dumps of CLD2UnitTestOutputVerbose.html
                       (scoreonescriptspan.cc:561-661).
  main_test.json       main_test.go known-answer strings (:144-305) and the
                       README example with their expected codes.
"""
import html
import json
import os
import re
import unicodedata

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))


def _unescape(lit):
    data = bytearray()
    for piece in re.findall(rb'"((?:[^"\\]|\\.)*)"', lit):
        i = 0
        while i < len(piece):
            c = piece[i]
            if c == 0x5C:                # backslash escape
                n = piece[i + 1]
                if n == ord("x"):
                    j = i + 2
                    while j < len(piece) and chr(piece[j]) in "0123456789abcdefABCDEF":
                        j += 1
                    data.append(int(piece[i + 2:j], 16) & 0xFF)
                    i = j
                    continue
                data.append({ord("n"): 10, ord("t"): 9, ord('"'): 34, ord("\\"): 92}.get(n, n))
                i += 2
                continue
            data.append(c)
            i += 1
    return bytes(data)


def c_string_literals():
    """name -> bytes for every kTeststr_* in unittest_data.h (UTF-8 literal
    branch; first definition wins).  Commented-out older versions (which the
    checked-in HTML goldens were produced from) are kept as name@old<k>."""
    out = {}
    src = open(os.path.join(REF, "cld2/internal/unittest_data.h"), "rb").read()
    src = src[:src.index(b"#else")]      # UTF-8 literal branch only
    nold = {}
    for m in re.finditer(rb'(//)?const char\* (kTeststr_\w+)\s*=((?:\s*(?://)?\s*"(?:[^"\\]|\\.)*")+)\s*;', src):
        name = m.group(2).decode()
        lit = re.sub(rb"\n\s*//", b"\n", m.group(3))
        if m.group(1):
            k = nold.get(name, 0)
            nold[name] = k + 1
            out["%s@old%d" % (name, k)] = _unescape(lit)
        elif name not in out:
            out[name] = _unescape(lit)
    # kTeststr_en lives in cld2_unittest.cc itself (:30-42), split over lines
    src = open(os.path.join(REF, "cld2/internal/cld2_unittest.cc"), "rb").read()
    m = re.search(rb'const char\* kTeststr_en =((?:\s*"(?:[^"\\]|\\.)*")+);', src)
    out["kTeststr_en"] = _unescape(m.group(1))
    return out


def test_pairs():
    src = open(os.path.join(REF, "cld2/internal/cld2_unittest.cc"), encoding="utf-8").read()
    body = src[src.index("static const TestPair kTestPair[] = {"):]
    body = body[:body.index("{UNKNOWN_LANGUAGE, NULL}")]
    pairs = []
    for line in body.splitlines():
        if line.strip().startswith("//"):
            continue
        m = re.match(r"\s*\{(\w+),\s*(kTeststr_\w+)\}", line)
        if m:
            pairs.append((m.group(1), m.group(2)))
    return pairs


def letters_key(b):
    """Letters and marks only (the span scanner keeps exactly those), lowercased."""
    t = b.decode("utf-8", "replace") if isinstance(b, bytes) else b
    return "".join(ch for ch in t.lower() if unicodedata.category(ch)[0] in "LM")


def parse_unittest_html(path):
    s = open(path, encoding="utf-8").read()
    docs = []
    pos = 0
    summ_re = re.compile(r"\n([^\n<]*?)(\d+) bytes = ([A-Za-z_\-]+)([ *]) <br><br>\n")
    while True:
        m = summ_re.search(s, pos)
        if not m:
            break
        block = s[pos:m.start()]
        texts = re.findall(r'<span style="background[^"]*">\n(.*?)</span>', block, re.S)
        dumps = []
        for d in re.finditer(r"DocTote::Dump\n((?:\[[^\n]*\n)*)  (\d+) chunks scored", block):
            rows = []
            for row in d.group(1).strip().splitlines():
                r = re.match(r"\[\s*(\d+)\]\s+(\S+)\s+(-?\d+)B\s+(-?\d+)p\s+(-?\d+)R,", row)
                rows.append([int(r.group(1)), r.group(2), int(r.group(3)), int(r.group(4)), int(r.group(5))])
            dumps.append({"slots": rows, "chunks": int(d.group(2))})
        langs = re.findall(r"(\S+)\.(\d+)R\((\d+)%\)", m.group(1))
        docs.append({
            "shown_text": html.unescape("".join(texts)),
            "dumps": dumps,
            "top3": [[l, int(r), int(p)] for l, r, p in langs],
            "text_bytes": int(m.group(2)),
            "summary_name": m.group(3),
            "summary_reliable": m.group(4) == " ",
        })
        pos = m.end()
    return docs


def parse_verbose_html(path):
    s = open(path, encoding="utf-8").read()
    out = []
    for doc_i, doc in enumerate(s.split("DocTote::Dump")):
      for seg in doc.split("<br>ScoreOneScriptSpan(")[1:]:
          m = re.match(r"(\w+),(-?\d+)\) '(.*?)'<br>", seg, re.S)
          rec = {"doc": doc_i, "script": m.group(1), "text_bytes": int(m.group(2)),
                 "span_text": html.unescape(m.group(3)), "rounds": []}
          for hb in re.finditer(r"DumpHitBuffer\[(\w+), next_base/delta/distinct (\d+), (\d+), (\d+)\)<br>\n(.*?)<br>\nLinear\[\) <br>DumpLinearBuffer\[(\d+)\)<br>\n(.*?)<br>\nDumpChunkStart\[(\d+)\]<br>\n(.*?)<br>\n(.*?)<br>DumpSummaryBuffer\[(\d+)\]<br>\n[^\n]*\n(.*?)<br>\n<br>", seg, re.S):
              # Q[next_base] is the dummy end-of-scan entry the dump appends (:590-596)
              base = [[int(a), int(b)] for i, a, b in re.findall(r"Q\[(\d+)\](-?\d+),(-?\d+),", hb.group(5))
                      if int(i) < int(hb.group(2))]
              delta = [[int(a), int(b)] for a, b in re.findall(r"L\[\d+\](-?\d+),(-?\d+),", hb.group(5))]
              distinct = [[int(a), int(b)] for a, b in re.findall(r"(?<![A-Z])D\[\d+\](-?\d+),(-?\d+),", hb.group(5))]
              linear = [[int(i), int(o), t, int(lp, 16)] for i, o, t, lp in
                        re.findall(r"\[(\d+)\](-?\d+),([UQLD])=([0-9a-f]{8}),", hb.group(7))]
              cstart = [int(x) for x in re.findall(r"\[\d+\](\d+)", hb.group(9))]
              summ = []
              for row in re.findall(r"\[\d+\] ([^\n]*?)<br>", hb.group(12)):
                  r = re.match(r"(\d+) lin\[(\d+)\] (\S+)\.(\d+) (\S+)\.(\d+) (\d+)B (\d+)# (\w+) (\d+)Rd (\d+)Rs", row)
                  summ.append([int(r.group(1)), int(r.group(2)), r.group(3), int(r.group(4)), r.group(5),
                               int(r.group(6)), int(r.group(7)), int(r.group(8)), r.group(9),
                               int(r.group(10)), int(r.group(11))])
              rec["rounds"].append({
                  "next_base": int(hb.group(2)), "next_delta": int(hb.group(3)), "next_distinct": int(hb.group(4)),
                  "base": base, "delta": delta, "distinct": distinct, "next_linear": int(hb.group(6)),
                  "linear": linear, "chunk_start": cstart, "summary": summ})
          out.append(rec)
    return out


def main():
    lits = c_string_literals()
    pairs = test_pairs()
    docs = parse_unittest_html(os.path.join(REF, "cld2/docs/CLD2UnitTestOutput.html"))
    keys = {name: letters_key(b) for name, b in lits.items()}
    used = set()
    for d in docs:
        shown = letters_key(d["shown_text"])
        cands = [n for n, k in keys.items() if k[:30] and shown[:30] == k[:30]]
        if not cands:
            cands = [n for n, k in keys.items() if shown[:24] and shown[:24] in k]
        if len(cands) > 1:
            cands = [n for n in cands if n not in used] or cands
        d["var"] = cands[0] if cands else None
        if d["var"]:
            used.add(d["var"])
            d["text_hex"] = lits[d["var"]].hex()
            # The HTML shows every scored letter; equality of the letter streams
            # says the dump was produced from exactly this input version.
            d["exact_input"] = letters_key(d["shown_text"]) == keys[d["var"]]
    doc_vars = {d["var"] for d in docs}
    test_list = [{"expected": e, "var": v, "text_hex": lits[v].hex(), "in_html": v in doc_vars}
                 for e, v in pairs if v in lits]
    json.dump({"source": "cld2/docs/CLD2UnitTestOutput.html + unittest_data.h + cld2_unittest.cc:51-190",
               "html_docs": docs, "test_pairs": test_list},
              open(os.path.join(HERE, "cld2_unittest.json"), "w"), ensure_ascii=False, indent=1)
    verbose = parse_verbose_html(os.path.join(REF, "cld2/docs/CLD2UnitTestOutputVerbose.html"))
    json.dump({"source": "cld2/docs/CLD2UnitTestOutputVerbose.html", "spans": verbose},
              open(os.path.join(HERE, "cld2_verbose.json"), "w"), ensure_ascii=False, indent=0)

    # main_test.go KATs
    mt = open(os.path.join(REF, "main_test.go"), encoding="utf-8").read()
    kats = []
    for m in re.finditer(r'testText :?= "((?:[^"\\]|\\.)*)"\s*\n\s*code :?= Detect_language\(testText\)\s*\n\s*assert\.Equal\(t, "(\w+)", code\)', mt):
        kats.append({"text": m.group(1).encode().decode("unicode_escape").encode("latin-1").decode("utf-8"),
                     "expected": m.group(2)})
    readme = "This is an example input message."
    kats.append({"text": readme, "expected": "en", "source": "README.md:19"})
    kats.append({"text": "This is a valid input test.", "expected": "en", "source": "main_test.go:124-142"})
    # main_test.go HTTP cases: method, path, request body, expected status and body
    http_cases = []
    for m in re.finditer(r'func (Test\w+)\(t \*testing\.T\) \{(.*?)\n\}', mt, re.S):
        name, fn = m.group(1), m.group(2)
        st = re.search(r'assert\.Equal\(t, (\d+), resp\.StatusCode', fn)
        exp = re.search(r'expected := `([^`]*)`', fn)
        if not st or not exp:
            continue
        req = re.search(r'strings\.NewReader\(`([^`]*)`\)', fn)
        get = re.search(r'http\.Get\(serverUrl( \+ "(\w+)")?\)', fn)
        http_cases.append({"test": name, "method": "POST" if req else "GET",
                           "path": "/" + (get.group(2) or "" if get else ""),
                           "body": req.group(1) if req else "", "status": int(st.group(1)),
                           "expected": exp.group(1)})
    # the known-language map the service answers names from (main.go:114-124, LANG_FILE)
    known = json.load(open(os.path.join(REF, "data", "cld_codes.json"), encoding="utf-8"))
    json.dump({"source": "main_test.go:144-305 (kats), main_test.go:52-345 (http_cases), "
                         "data/cld_codes.json (known_languages)",
               "kats": kats, "http_cases": http_cases, "known_languages": sorted(known.items())},
              open(os.path.join(HERE, "main_test.json"), "w"), ensure_ascii=False, indent=1)
    print("html docs", len(docs), "matched", sum(1 for d in docs if d["var"]),
          "test pairs", len(test_list), "verbose spans", len(verbose), "kats", len(kats))


if __name__ == "__main__":
    main()
