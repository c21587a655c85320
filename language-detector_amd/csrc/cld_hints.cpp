// cld_hints.cpp -- CLDHints -> prior boosts and whacks, on the host.
//
// Restates the reference's hint code (compact_lang_det_hint_code.cc) and the
// prior half of ApplyHints (compact_lang_det_impl.cc:1524-1684) over tables
// extracted into the CLDT blob.  A document's hints become 16 langprobs that
// the kernels add to (boosts) or zero in (whacks) every chunk tote, exactly
// where ScoreBoosts does (scoreonescriptspan.cc:125-152).  Pinned against the
// reference's own hint code by tests/test_html_hints.py (oracle/refscan).
#include "cld_hints.h"

#include <stdlib.h>
#include <string.h>

#include <string>

#include "cldt_format.h"

namespace cld {
namespace {

struct Lookup {
  const char* key;
  const char* code;
  int16_t p1, p2;
};

// Binary search of a CLDT hint table (DoLangTagLookup / DoTLDLookup, :1007-1046).
bool lookup(const uint8_t* sec, const char* key, Lookup* out) {
  const uint32_t n = *(const uint32_t*)sec;
  const cldt_hint_entry* e = (const cldt_hint_entry*)(sec + 4);
  const char* pool = (const char*)(e + n);
  uint32_t lo = 0, hi = n;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    const int c = strcmp(pool + e[mid].key_off, key);
    if (c < 0) lo = mid + 1;
    else if (c > 0) hi = mid;
    else {
      out->key = pool + e[mid].key_off;
      out->code = e[mid].code_off == 0xFFFFFFFFu ? nullptr : pool + e[mid].code_off;
      out->p1 = e[mid].prior1;
      out->p2 = e[mid].prior2;
      return true;
    }
  }
  return false;
}

struct Priors {
  int n = 0;
  int16_t p[kMaxPriors];
};
int weight(int16_t olp) { return olp >> 10; }                 // GetCLDPriorWeight (.h:41-43)
int lang_of(int16_t olp) { return olp & 0x3FF; }              // GetCLDPriorLang (.h:44-46)
void set_weight(int w, int16_t* olp) { *olp = (int16_t)((*olp & 0x3FF) + (w << 10)); }

void merge_max(int16_t olp, Priors* lps) {                    // MergeCLDLangPriorsMax :941-956
  if (olp == 0) return;
  for (int i = 0; i < lps->n; ++i)
    if (lang_of(lps->p[i]) == lang_of(olp)) {
      const int a = weight(lps->p[i]), b = weight(olp);
      set_weight(a >= b ? a : b, &lps->p[i]);
      return;
    }
  if (lps->n < kMaxPriors) lps->p[lps->n++] = olp;
}
void merge_boost(int16_t olp, Priors* lps) {                  // MergeCLDLangPriorsBoost :958-972
  if (olp == 0) return;
  for (int i = 0; i < lps->n; ++i)
    if (lang_of(lps->p[i]) == lang_of(olp)) {
      set_weight(weight(lps->p[i]) + 2, &lps->p[i]);
      return;
    }
  if (lps->n < kMaxPriors) lps->p[lps->n++] = olp;
}
void trim(int max_entries, Priors* lps) {                     // TrimCLDLangPriors :975-996
  if (lps->n <= max_entries) return;
  for (int i = 0; i < lps->n; ++i) {                          // insertion sort by |weight|, stable
    const int16_t t = lps->p[i];
    const int w = abs(weight(t));
    int k = i;
    for (; k > 0 && abs(weight(lps->p[k - 1])) < w; --k) lps->p[k] = lps->p[k - 1];
    lps->p[k] = t;
  }
  lps->n = max_entries;
}

// Each tag of a lowercased comma list, via table 1, else its part before the
// first hyphen via table 2 (SetCLDLangTagsHint :1394-1437).
void lang_tags_hint(const HintView& v, const std::string& tags, Priors* lps) {
  if (tags.empty()) return;
  int commas = 0;
  for (char c : tags) commas += c == ',';
  if (commas > 4) return;
  size_t pos = 0;
  while (pos < tags.size()) {
    size_t comma = tags.find(',', pos);
    if (comma == std::string::npos) comma = tags.size();
    const size_t len = comma - pos;
    if (len <= 16) {
      char tmp[20];
      memcpy(tmp, tags.data() + pos, len);
      tmp[len] = 0;
      Lookup e;
      if (lookup(v.langtag1, tmp, &e)) {
        merge_max(e.p1, lps);
        merge_max(e.p2, lps);
      } else {
        if (char* hy = strchr(tmp, '-')) *hy = 0;
        if (strlen(tmp) <= 3 && lookup(v.langtag2, tmp, &e)) {
          merge_max(e.p1, lps);
          merge_max(e.p2, lps);
        }
      }
    }
    pos = comma + 1;
  }
}

// The three-state language-attribute copier (CopyOneQuotedString :1355-1380).
std::string copy_one_quoted(const HintView& v, const char* s, int pos, int max_pos) {
  std::string out;
  int state = 1;
  for (int i = pos; i < max_pos; ++i) {
    const unsigned char c = (unsigned char)s[i];
    const int e = v.action[c] >> (3 * state);
    state = e & 3;
    if (e & 4) out.push_back(state == 0 ? (char)v.remap[c] : ',');
  }
  if (state == 0) out.push_back(',');
  return out;
}

// GetLangTagsFromHtml (:1557-1646) and its scanners (:1209-1353).
int find_tag_start(const char* b, int pos, int max_pos) {
  for (int i = pos; i < max_pos; ++i)
    if (b[i] == '<') return i;
  return -1;
}
int find_tag_end(const char* b, int pos, int max_pos) {
  for (int i = pos; i < max_pos; ++i) {
    const char c = b[i];
    if (c == '>') return i;
    if (c == '<' || c == '&') return i - 1;
  }
  return -1;
}
int find_quote_start(const char* b, int pos, int max_pos) {
  for (int i = pos; i < max_pos; ++i) {
    const char c = b[i];
    if (c == '"' || c == '\'') return i;
    if (c != ' ') return -1;
  }
  return -1;
}
int find_quote_end(const char* b, int pos, int max_pos) {
  for (int i = pos; i < max_pos; ++i) {
    const char c = b[i];
    if (c == '"' || c == '\'') return i;
    if (c == '>' || c == '=' || c == '<' || c == '&') return i - 1;
  }
  return -1;
}
int find_equal_sign(const char* b, int pos, int max_pos) {
  for (int i = pos; i < max_pos; ++i) {
    const char c = b[i];
    if (c == '=') return i;
    if (c == '"' || c == '\'') {                 // skip the quoted run (backslash escapes)
      int j = i + 1;
      for (; j < max_pos; ++j) {
        if (b[j] == c) break;
        if (b[j] == '\\') ++j;
      }
      i = j;
    }
  }
  return -1;
}
bool find_before(const char* b, int min_pos, int pos, const char* s) {
  const int len = (int)strlen(s);
  if (pos - min_pos < len) return false;
  int i = pos;
  while (i > min_pos + len && b[i - 1] == ' ') --i;
  i -= len;
  if (i < min_pos) return false;
  for (int j = 0; j < len; ++j)
    if ((b[i + j] | 0x20) != s[j]) return false;
  return true;
}
bool find_after(const char* b, int pos, int max_pos, const char* s) {
  const int len = (int)strlen(s);
  if (max_pos - pos < len) return false;
  int i = pos;
  while (i < max_pos - len) {
    const unsigned char c = (unsigned char)b[i];
    if (c == ' ' || c == '"' || c == '\'') ++i;
    else break;
  }
  for (int j = 0; j < len; ++j)
    if ((b[i + j] | 0x20) != s[j]) return false;
  return true;
}
std::string copy_quoted(const HintView& v, const char* b, int pos, int max_pos) {
  const int q0 = find_quote_start(b, pos, max_pos);
  if (q0 < 0) return std::string();
  const int q1 = find_quote_end(b, q0 + 1, max_pos);
  if (q1 < 0) return std::string();
  return copy_one_quoted(v, b, q0 + 1, q1);
}
std::string lang_tags_from_html(const HintView& v, const char* b, int len, int max_scan) {
  std::string out;
  if (max_scan > len) max_scan = len;
  int k = 0;
  while (k < max_scan) {
    const int st = find_tag_start(b, k, max_scan);
    if (st < 0) break;
    const int en = find_tag_end(b, st + 1, max_scan);
    if (en < 0) break;
    if (find_after(b, st + 1, en, "!--") || find_after(b, st + 1, en, "font ") ||
        find_after(b, st + 1, en, "script ") || find_after(b, st + 1, en, "link ") ||
        find_after(b, st + 1, en, "img ") || find_after(b, st + 1, en, "a ")) {
      k = en + 1;
      continue;
    }
    const bool in_meta = find_after(b, st + 1, en, "meta ");
    bool content_is_lang = false;
    int kk = st + 1, eq;
    while ((eq = find_equal_sign(b, kk, en)) >= 0) {
      if (in_meta) {
        if (find_before(b, kk, eq, " http-equiv") && find_after(b, eq + 1, en, "content-language ")) {
          content_is_lang = true;
        } else if (find_before(b, kk, eq, " name") &&
                   (find_after(b, eq + 1, en, "dc.language ") || find_after(b, eq + 1, en, "language "))) {
          content_is_lang = true;
        }
      }
      if ((content_is_lang && find_before(b, kk, eq, " content")) || find_before(b, kk, eq, " lang") ||
          find_before(b, kk, eq, ":lang")) {
        const std::string t = copy_quoted(v, b, eq + 1, en);
        if (!t.empty() && out.find(t) == std::string::npos) out += t;
      }
      kk = eq + 1;
    }
    k = en + 1;
  }
  if (out.size() > 1) out.erase(out.size() - 1);
  return out;
}

// IsLatnLanguage / IsOthrLanguage (lang_script.cc:344-353)
bool is_latn(const HintView& v, int lang) {
  return lang >= 0 && (uint32_t)lang < v.l2p_size && lang == v.p2l_latn[v.l2p[lang]];
}
bool is_othr(const HintView& v, int lang) {
  return lang >= 0 && (uint32_t)lang < v.l2p_size && lang == v.p2l_othr[v.l2p[lang]];
}
int close_set(const HintView& v, int lang) {
  return (lang >= 0 && (uint32_t)lang < v.n_langs) ? v.close_set[lang] : 0;
}
// MakeLangProb (cldutil.cc:610-614) with kLgProbV2TblBackmap (cldutil_shared.h:311-314).
// Weights above 12 read past the reference's 13-entry table (undefined there);
// they are clamped to 12 here.
uint32_t make_lang_prob(const HintView& v, int lang, int qprob) {
  static const uint8_t kBackmap[13] = {0, 0, 1, 3, 6, 10, 15, 21, 28, 36, 45, 55, 66};
  const uint32_t ps = (lang >= 0 && (uint32_t)lang < v.l2p_size) ? v.l2p[lang] : 0;
  return (ps << 8) | kBackmap[qprob > 12 ? 12 : qprob];
}

struct Rings {
  uint32_t lp[4][4] = {};   // boost latn, boost othr, whack latn, whack othr
  int n[4] = {0, 0, 0, 0};
  void push(int r, uint32_t v) { lp[r][n[r]] = v; n[r] = (n[r] + 1) & 3; }
};

void add_one_whack(const HintView& v, int whacker, int whackee, Rings* r) {   // AddOneWhack :1545-1561
  const uint32_t lp = make_lang_prob(v, whackee, 1);
  if (is_latn(v, whacker) && is_latn(v, whackee)) r->push(2, lp);
  if (is_othr(v, whacker) && is_othr(v, whackee)) r->push(3, lp);
}
void add_close_lang_whack(const HintView& v, int lang, Rings* r) {           // AddCloseLangWhack :1563-1585
  if ((uint32_t)lang == v.chinese) { add_one_whack(v, lang, (int)v.chinese_t, r); return; }
  if ((uint32_t)lang == v.chinese_t) { add_one_whack(v, lang, (int)v.chinese, r); return; }
  const int base = close_set(v, lang);
  if (base == 0) return;
  for (uint32_t i = 0; i < v.l2p_size; ++i)
    if (close_set(v, (int)i) == base && (int)i != lang) add_one_whack(v, lang, (int)i, r);
}

}  // namespace

int hint_priors(const HintView& v, const uint8_t* doc, size_t len, bool plain, const cld_hints* h,
                int16_t out[kMaxPriors]) {
  Priors lps;
  if (!plain && doc && len) {
    // GetLangTagsFromHtml reads a few bytes past a tag end; give it a padded copy
    const size_t scan = len < (8u << 10) ? len : (8u << 10);
    std::string body((const char*)doc, scan);
    body.append(16, '\0');
    lang_tags_hint(v, lang_tags_from_html(v, body.data(), (int)scan, 8 << 10), &lps);
  }
  if (h) {
    if (h->content_language_hint && h->content_language_hint[0]) {
      const char* cl = h->content_language_hint;
      lang_tags_hint(v, copy_one_quoted(v, cl, 0, (int)strlen(cl)), &lps);
    }
    if (h->tld_hint && h->tld_hint[0] && strlen(h->tld_hint) <= 3) {     // SetCLDTLDHint :1446-1464
      char t[4] = {0, 0, 0, 0};
      strncpy(t, h->tld_hint, 3);
      for (int i = 0; t[i]; ++i) t[i] |= 0x20;
      Lookup e;
      if (lookup(v.tld, t, &e)) {
        merge_boost(e.p1, &lps);
        merge_boost(e.p2, &lps);
      }
    }
    if (h->encoding_hint != CLD_UNKNOWN_ENCODING && h->encoding_hint >= 0 &&
        (uint32_t)h->encoding_hint < v.n_enc)                              // SetCLDEncodingHint :1466-1501
      merge_boost(v.enc[h->encoding_hint], &lps);
    if (h->language_hint != (int32_t)v.unknown_language)                  // SetCLDLanguageHint :1503-1507
      merge_boost((int16_t)((8 << 10) + h->language_hint), &lps);
  }
  trim(4, &lps);
  for (int i = 0; i < lps.n; ++i) out[i] = lps.p[i];
  return lps.n;
}

void hint_boosts(const HintView& v, const int16_t* p, int n, uint32_t out16[16]) {
  Rings r;
  for (int i = 0; i < n; ++i) {                                           // prior boosts :1645-1652
    const int lang = lang_of(p[i]), q = weight(p[i]);
    if (q > 0) {
      const uint32_t lp = make_lang_prob(v, lang, q);
      if (is_latn(v, lang)) r.push(0, lp);
      if (is_othr(v, lang)) r.push(1, lp);
    }
  }
  constexpr int kCloseSetSize = 10;                                       // lang_script.cc:258
  int count[kCloseSetSize + 1] = {};
  for (int i = 0; i < n; ++i) {
    const int lang = lang_of(p[i]);
    const int cs = close_set(v, lang);
    if (cs >= 0 && cs <= kCloseSetSize) ++count[cs];
    if ((uint32_t)lang == v.chinese || (uint32_t)lang == v.chinese_t) ++count[kCloseSetSize];
  }
  for (int i = 0; i < n; ++i) {                                           // close-set whacks :1666-1683
    const int lang = lang_of(p[i]), q = weight(p[i]);
    if (q <= 0) continue;
    const int cs = close_set(v, lang);
    if (cs > 0 && cs <= kCloseSetSize && count[cs] == 1) add_close_lang_whack(v, lang, &r);
    if (((uint32_t)lang == v.chinese || (uint32_t)lang == v.chinese_t) && count[kCloseSetSize] == 1)
      add_close_lang_whack(v, lang, &r);
  }
  for (int k = 0; k < 4; ++k)
    for (int j = 0; j < 4; ++j) out16[4 * k + j] = r.lp[k][j];
}

}  // namespace cld
