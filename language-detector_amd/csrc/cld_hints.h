// cld_hints.h -- host-side hint processing (CLDHints -> per-document prior
// boosts / whacks), the runtime's restatement of the reference's hint code.
#ifndef CLD_HINTS_H_
#define CLD_HINTS_H_
#include <stddef.h>
#include <stdint.h>

#include "../../include/cld_mi355x.h"

namespace cld {

// Views into the CLDT blob (cldt_format.h: CLDT_HINT_* and the language maps).
struct HintView {
  const uint8_t* langtag1 = nullptr;
  const uint8_t* langtag2 = nullptr;
  const uint8_t* tld = nullptr;
  const uint8_t* action = nullptr;     // kLangCodeAction[256]
  const uint8_t* remap = nullptr;      // kLangCodeRemap[256]
  const int16_t* enc = nullptr;        // prior per Encoding value
  uint32_t n_enc = 0;
  const uint8_t* l2p = nullptr;        // kLanguageToPLang
  uint32_t l2p_size = 0;
  const uint16_t* p2l_latn = nullptr;
  const uint16_t* p2l_othr = nullptr;
  const uint8_t* close_set = nullptr;
  uint32_t n_langs = 0;
  uint32_t chinese = 0, chinese_t = 0, unknown_language = 26;
  bool ok() const { return langtag1 && langtag2 && tld && action && remap && enc && l2p && p2l_latn && p2l_othr && close_set; }
};

constexpr int kMaxPriors = 14;         // kMaxOneCLDLangPrior (compact_lang_det_hint_code.h:34)

// The CLDLangPriors ApplyHints builds (compact_lang_det_impl.cc:1587-1643):
// lang= tags of the first 8 KB of an HTML document, then the content-language,
// TLD, encoding and language hints, trimmed to 4.  Returns the count.
int hint_priors(const HintView& v, const uint8_t* doc, size_t len, bool plain, const cld_hints* h,
                int16_t out[kMaxPriors]);

// The scoring context those priors become (:1645-1684): 16 langprobs, prior
// boosts latn[4] and othr[4], then close-language whacks latn[4] and othr[4].
void hint_boosts(const HintView& v, const int16_t* priors, int n, uint32_t out16[16]);

}  // namespace cld
#endif
