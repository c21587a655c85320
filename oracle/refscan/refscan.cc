// refscan.cc -- TEST INFRASTRUCTURE ONLY.  Runs pieces of the reference that
// need no scoring table, compiled from /root/reference where they lie
// (oracle/refscan/Makefile), so the restatements can be pinned to them:
//   spans <plain>  ScriptScanner::GetOneScriptSpanLower over each document
//                  (getonescriptspan.cc:799-1065), HTML mode when plain = 0
//   tags           ScanToPossibleLetter (getonescriptspan.cc:503-541)
//   entities       ReadEntity (getonescriptspan.cc:393-451)
//   hints          the CLDLangPriors the hint code builds
//                  (compact_lang_det_hint_code.cc: SetCLDLangTagsHint from
//                  GetLangTagsFromHtml, content-language, TLD, encoding and
//                  language hints, then TrimCLDLangPriors(4), as ApplyHints
//                  does at compact_lang_det_impl.cc:1587-1643)
// Input on stdin: records of u32 length + bytes.  Output on stdout, binary:
//   spans:    u32 n_spans, then per span u32 ulscript, u32 text_bytes, bytes
//   tags:     i32 per record
//   entities: i32 value, i32 consumed per record
//   hints:    record = 5 fields (u32 len + bytes each): html body (empty =
//             plain text), content-language, tld, encoding (decimal), language
//             (decimal); output u32 n, then n int16 priors
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#include "compact_lang_det_hint_code.h"
#include "getonescriptspan.h"

namespace CLD2 {
int ScanToPossibleLetter(const char* isrc, int len, int max_exit_state);
int ReadEntity(const char* src, int srcn, int* src_consumed);
std::string GetLangTagsFromHtml(const char* utf8_body, int32 utf8_body_len, int32 max_scan_bytes);
}  // namespace CLD2
using namespace CLD2;

static bool read_rec(std::string* out) {
  uint32_t n;
  if (fread(&n, 4, 1, stdin) != 1) return false;
  out->resize(n);
  return n == 0 || fread(&(*out)[0], 1, n, stdin) == n;
}
static void put32(uint32_t v) { fwrite(&v, 4, 1, stdout); }

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  const std::string mode = argv[1];
  std::string rec;
  if (mode == "spans") {
    const bool plain = argc > 2 && atoi(argv[2]) != 0;
    while (read_rec(&rec)) {
      std::string doc = rec + std::string(16, '\0');        // NUL-terminated, as the wrapper hands it over
      ScriptScanner ss(doc.data(), (int)rec.size(), plain);
      LangSpan span;
      std::vector<std::string> out;
      std::vector<int> scripts;
      while (ss.GetOneScriptSpanLower(&span)) {
        // invalid UTF-8 can leave the lowercaser short of its 3 pad bytes:
        // text_bytes < 0 is reported as an empty span with the raw value
        out.emplace_back(span.text, span.text_bytes > 0 ? span.text_bytes : 0);
        scripts.push_back(span.ulscript | (span.text_bytes < 0 ? (uint32_t)(-span.text_bytes) << 16 : 0u));
      }
      put32((uint32_t)out.size());
      for (size_t i = 0; i < out.size(); ++i) {
        put32((uint32_t)scripts[i]);
        put32((uint32_t)out[i].size());
        fwrite(out[i].data(), 1, out[i].size(), stdout);
      }
    }
  } else if (mode == "tags") {
    while (read_rec(&rec)) {
      std::string doc = rec + std::string(16, '\0');
      put32((uint32_t)ScanToPossibleLetter(doc.data(), (int)rec.size(), 1));
    }
  } else if (mode == "entities") {
    while (read_rec(&rec)) {
      std::string doc = rec + std::string(16, '\0');
      int consumed = 0;
      const int v = ReadEntity(doc.data(), (int)rec.size(), &consumed);
      put32((uint32_t)v);
      put32((uint32_t)consumed);
    }
  } else if (mode == "hints") {
    for (;;) {
      std::string html, cl, tld, enc, lang;
      if (!read_rec(&html) || !read_rec(&cl) || !read_rec(&tld) || !read_rec(&enc) || !read_rec(&lang)) break;
      CLDLangPriors lp;
      InitCLDLangPriors(&lp);
      if (!html.empty()) {
        std::string body = html + std::string(16, '\0');
        SetCLDLangTagsHint(GetLangTagsFromHtml(body.data(), (int)html.size(), 8 << 10), &lp);
      }
      if (!cl.empty()) SetCLDContentLangHint(cl.c_str(), &lp);
      if (!tld.empty()) SetCLDTLDHint(tld.c_str(), &lp);
      const int e = atoi(enc.c_str());
      if (e != UNKNOWN_ENCODING) SetCLDEncodingHint((Encoding)e, &lp);
      const int l = atoi(lang.c_str());
      if (l != UNKNOWN_LANGUAGE) SetCLDLanguageHint((Language)l, &lp);
      TrimCLDLangPriors(4, &lp);
      put32((uint32_t)lp.n);
      fwrite(lp.prior, 2, lp.n, stdout);
    }
  }
  return 0;
}
