"""data/cjk_charsets.json: the letter characters of the reference's CJK unit-test
documents (unittest_data.h kTeststr_{zh_Hans,zh_Hant,ja_Hani,ko_Hani}, taken from
the committed fixture tests/golden/cld2_unittest.json), used by corpus.c4."""
import json, os, unicodedata
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
g = json.load(open(os.path.join(ROOT, "tests/golden/cld2_unittest.json"), encoding="utf-8"))
texts = {t["var"]: bytes.fromhex(t["text_hex"]).decode("utf-8", "replace") for t in g["test_pairs"]}
out = {}
for lang, var in (("zh", "kTeststr_zh_Hans"), ("zh-Hant", "kTeststr_zh_Hant"), ("ja", "kTeststr_ja_Hani"), ("ko", "kTeststr_ko_Hani")):
    out[lang] = sorted({c for c in texts[var] if unicodedata.category(c).startswith("L") and ord(c) > 0x2E80})
json.dump(out, open(os.path.join(ROOT, "language-detector_amd/data/cjk_charsets.json"), "w", encoding="utf-8"), ensure_ascii=False)
print({k: len(v) for k, v in out.items()})
