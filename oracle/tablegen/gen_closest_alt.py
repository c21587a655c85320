"""Turn kClosestAltLanguage (compact_lang_det_impl.cc:259-427, a static array
the extractor cannot link) into an include file of enum expressions that the
extractor compiles against the reference's own Language enum.  Reads the
reference source as text; writes only the .inc named on the command line."""
import re, sys

src = open(sys.argv[1], encoding="utf-8").read()
start = src.index("static const Language kClosestAltLanguage[] = {")
body = src[start:src.index("};", start)]
out = []
for line in body.splitlines()[1:]:
    m = re.match(r"\s*\(\s*(\d+)\s*>=\s*kMinCorrPercent\)\s*\?\s*(\w+)\s*:\s*UNKNOWN_LANGUAGE,", line)
    if not m:
        continue
    thr, lang = int(m.group(1)), m.group(2)
    if lang == "Unknown":          # static Language Unknown = UNKNOWN_LANGUAGE (:255)
        lang = "UNKNOWN_LANGUAGE"
    out.append("  (%d >= 24) ? %s : UNKNOWN_LANGUAGE," % (thr, lang))   # kMinCorrPercent (:252)
open(sys.argv[2], "w").write("\n".join(out) + "\n")
print("closest-alt entries:", len(out))
