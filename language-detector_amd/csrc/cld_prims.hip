// cld_prims.hip -- the device primitives every kernel shares (k_wave,
// k_long and its staged stages, k_html_rewrite): byte helpers, the table
// state machines (script numbers, the lowercaser), gram hashes and bucket
// probes, the document tote, reliability, the HTML tag / entity scanner
// pieces and the summary.  Each is a small function with the reference lines
// whose semantics it implements; the per-document pipelines that compose them
// are the wave-parallel kernels (cld_wave.hip, cld_long.hip, cld_seq.hip).
//
//  * Scoring tables stay in HBM and are gathered through L2/MALL.
//  * The only floating point is ReliabilityExpected; this file is compiled
//    with -ffp-contract=off so its double ops round exactly like the oracle.

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "cld_device.h"

namespace cld {

// ----------------------------------------------------------------- constants
enum : int {
  kExitIllegalStructure = 240, kExitOK = 241, kExitReplace1 = 243, kExitReplace2 = 244,
  kExitReplace3 = 245, kExitReplace21 = 246, kExitReplace31 = 247, kExitReplace32 = 248,
  kExitReplaceOffset1 = 249, kExitReplaceOffset2 = 250, kExitReplace1S0 = 251,
  kExitSpecial = 252, kExitDoAgain = 253, kExitRejectAlt = 254
};
constexpr int kMaxScriptBuffer = 40960;
constexpr int kMaxScriptLowerBuffer = kMaxScriptBuffer * 3 / 2;
constexpr int kMaxScriptBytes = kMaxScriptBuffer - 32;
constexpr int kWithinScriptTail = 32;
constexpr int kMaxBoosts = 4;
constexpr int kChunksizeQuads = 20;
constexpr int kChunksizeUnis = 50;
constexpr int kMaxScoringHits = 1000;
constexpr int kMaxSummaries = kMaxScoringHits / kChunksizeQuads;
constexpr int kPredictionTableSize = 4096;
constexpr int kCLDFlagFinish = 1, kCLDFlagSqueeze = 2, kCLDFlagRepeats = 4, kCLDFlagTop40 = 8,
              kCLDFlagShort = 16, kCLDFlagUseWords = 64;
// The public result-affecting flags (compact_lang_det.h:343, :349), as the
// caller passes them (CLD_FLAG_SCORE_AS_QUADS / CLD_FLAG_BEST_EFFORT)
constexpr int kCLDFlagScoreAsQuads = 0x0100, kCLDFlagBestEffort = 0x4000;
constexpr uint16_t kUnusedKey = 0xFFFF;
enum { UNIHIT = 0, QUADHIT = 1, DELTAHIT = 2, DISTINCTHIT = 3 };
enum { RTypeNone = 0, RTypeOne = 1, RTypeMany = 2, RTypeCJK = 3 };

// -------------------------------------------------------- small byte helpers
__device__ __forceinline__ int utf8_len(uint8_t c) {          // utf8statetable.h:266-281
  return c < 0xC0 ? 1 : c < 0xE0 ? 2 : c < 0xF0 ? 3 : 4;
}
__device__ __forceinline__ int adv_but_space(uint8_t c) {     // cldutil_shared.h:462-473
  return c <= 0x20 ? 0 : c < 0xC0 ? 1 : c < 0xE0 ? 2 : c < 0xF0 ? 3 : 4;
}
__device__ __forceinline__ int adv_space_vowel(uint8_t c) {   // cldutil_shared.h:476-487
  return (c <= 0x20) | (c == 'A') | (c == 'E') | (c == 'I') | (c == 'O') | (c == 'U') |
         (c == 'a') | (c == 'e') | (c == 'i') | (c == 'o') | (c == 'u') | ((c & 0xC0) == 0x80);
}

// Document bytes: reads past the end return NUL, as for the NUL-terminated
// string wrapper.cc hands to CLD2.
struct DocView {
  const uint8_t* p;
  int len;
  // (rewritten HTML documents only, cld_html.hip) one byte per position, 1
  // where the original had an entity's '&': a script lookahead landing there
  // sees that '&' (script 0), not the decoded character
  const uint8_t* hf = nullptr;
  // (rewritten pages of kMaxScriptBytes and more) each byte's page offset and,
  // after dropped '&'s, where they began (cld_html.hip hpos / hgap): the span
  // soft limit reads the page's raw bytes left (getonescriptspan.cc:814-819)
  const uint32_t* hp = nullptr;
  const uint32_t* hg = nullptr;
  __device__ __forceinline__ uint8_t at(int i) const { return (unsigned)i < (unsigned)len ? p[i] : 0; }
};

// Loads from the table set (and the k_long slot) through pointers the compiler
// cannot prove global -- the pointers held in DevTables, a reference captured
// by a lambda.  A plain dereference becomes a FLAT load, which also counts
// against LGKM, so every later LDS or scalar wait would wait for the gather
// too.  Only for memory that is always global (never a private or LDS copy).
template <class V>
__device__ __forceinline__ V gld(const V* p) {
  return *(const __attribute__((address_space(1))) V*)p;
}
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 gld4(const uint32_t* p) {      // one 16-byte load (p 16-byte aligned)
  const u32x4_t v = gld(reinterpret_cast<const u32x4_t*>(p));
  return make_uint4(v.x, v.y, v.z, v.w);
}

// ---------------------------------------------------------- state machines
__device__ __forceinline__ uint32_t sm16(const DevSM& sm, int64_t i) {
  return (i < 0 || i >= (int64_t)sm.total) ? 0u : (uint32_t)gld(sm.t16 + i);
}
__device__ __forceinline__ int32_t sm8(const DevSM& sm, int64_t i) {
  return (i < 0 || i >= (int64_t)sm.total) ? 0 : (int32_t)gld(sm.t8 + i);
}

// GetUTF8LetterScriptNum -> UTF8GenericPropertyTwoByte
// getonescriptspan.cc:1083-1088, utf8statetable.cc:362-411
template <class Src>
__device__ int script_num_sm(const DevSM& sm, const Src& s, int i) {
  uint8_t c = s.at(i);
  int64_t b = sm.state0;
  if (c < 0x80) return (int)(uint8_t)sm16(sm, b + c);
  int n = utf8_len(c);
  uint32_t e;
  if ((c & 0xE0) == 0xC0 && n >= 2) {
    e = sm16(sm, b + c);
    e = sm16(sm, b + ((int64_t)e << sm.shift) + s.at(i + 1));
  } else if ((c & 0xF0) == 0xE0 && n >= 3) {
    e = sm16(sm, b + c);
    e = sm16(sm, b + ((int64_t)e << sm.shift) + s.at(i + 1));
    e = sm16(sm, b + ((int64_t)e << sm.shift) + s.at(i + 2));
  } else if ((c & 0xF8) == 0xF0 && n >= 4) {
    e = sm16(sm, b + c);
    e = sm16(sm, b + ((int64_t)e << sm.shift) + s.at(i + 1));
    e = sm16(sm, b + ((int64_t)e << sm.shift) + s.at(i + 2));
    e = sm16(sm, b + ((int64_t)e << sm.shift) + s.at(i + 3));
  } else {
    e = 0;
  }
  return (int)(uint8_t)e;
}
template <class Src>
__device__ __forceinline__ int script_num(const DevTables& T, const Src& s, int i) { return script_num_sm(T.script, s, i); }

// UTF8GenericPropertyBigOneByte on the CJK unigram machine, srclen =
// kAdvanceOneChar[lead] (cldutil.cc:221-226, utf8statetable.cc:271-320)
__device__ int uni_prop(const DevTables& T, const uint8_t* s, int srclen) {
  const DevSM& sm = T.uni;
  int64_t b0 = sm.state0;
  int sh = (int)sm.shift;
  uint8_t c = s[0];
  int32_t e;
  if (c < 0x80) return sm8(sm, b0 + c);
  if ((c & 0xE0) == 0xC0 && srclen >= 2) {
    e = sm8(sm, b0 + c);
    e = sm8(sm, b0 + ((int64_t)e << sh) + s[1]);
  } else if ((c & 0xF0) == 0xE0 && srclen >= 3) {
    e = sm8(sm, b0 + c);
    int64_t tb = b0 + ((int64_t)e << (sh + 4));
    e = (int8_t)sm8(sm, tb + s[1]);
    tb += (int64_t)e << sh;
    e = sm8(sm, tb + s[2]);
  } else if ((c & 0xF8) == 0xF0 && srclen >= 4) {
    e = sm8(sm, b0 + c);
    e = sm8(sm, b0 + ((int64_t)e << sh) + s[1]);
    int64_t tb = b0 + ((int64_t)e << (sh + 4));
    e = (int8_t)sm8(sm, tb + s[2]);
    tb += (int64_t)e << sh;
    e = sm8(sm, tb + s[3]);
  } else {
    e = 0;
  }
  return (uint8_t)e;
}

__device__ __forceinline__ bool in_state_zero(const DevSM& sm, int64_t tb) {
  return (uint64_t)(tb - sm.state0) < sm.state0_size;
}

// ScanToLetterOrSpecial -> UTF8GenericScan(utf8scannot_lettermarkspecial),
// getonescriptspan.cc:480-485, utf8statetable.cc:460-554.  Byte loop only;
// the extractor proved the 8-byte fast loop skips exactly bytes whose
// state-0 entry is 0, so results are identical.
__device__ int scan_to_letter_or_special(const DevTables& T, const DocView& d, int start, int len) {
  if (len <= 0) return 0;
  const DevSM& sm = T.scan;
  int src = start;
  const int lim = start + len;
  const int64_t tb0 = sm.state0;
  int e;
  for (;;) {
    int64_t tb = tb0;
    e = 0;
    while (src < lim) {
      uint8_t c = d.at(src);
      e = sm8(sm, tb + c);
      ++src;
      if (e >= kExitIllegalStructure) break;
      tb = tb0 + ((int64_t)e << sm.shift);
    }
    if (e >= kExitIllegalStructure) {
      --src;
      if (!in_state_zero(sm, tb)) {
        do { --src; } while (src > start && (d.at(src) & 0xC0) == 0x80);
      }
    } else if (!in_state_zero(sm, tb)) {
      e = kExitIllegalStructure;
      do { --src; } while (src > start && (d.at(src) & 0xC0) == 0x80);
    } else {
      e = kExitOK;
    }
    if (e != kExitDoAgain) break;
  }
  return src - start;
}

// UTF8GenericReplace(utf8repl_lettermarklower, plain text) without the offset
// map: utf8statetable.cc:608-867 plus the kExitDoAgain driver :1138-1169.
// `olen` is the reference's logical output capacity (kMaxScriptLowerBuffer);
// the physical buffer only needs 1.5x the input (max per-char expansion of
// this table, verified by tests/test_tables.py) plus padding.
// om (nullable): the map2uplow_ offset map being built (ResultChunkVector
// mode), any type with copy / insert / del (cld_seq.hip RangeStream).
struct NoMap {
  __device__ void copy(int) {}
  __device__ void insert(int) {}
  __device__ void del(int) {}
};
template <class M = NoMap>
__device__ int lower_replace_sm(const DevSM& sm, const uint8_t* in0, int ilen, uint8_t* out0, int olen,
                                bool plain = true, M* om = nullptr) {
  const int sh = (int)sm.shift;
  const int nEntries = 1 << sh;
  int total_filled = 0;
  const uint8_t* in = in0;
  int inlen = ilen;
  uint8_t* out = out0;
  int outlen = olen;
  for (;;) {
    const uint8_t* src = in;
    const uint8_t* copystart = in;            // the map2uplow_ bookkeeping (ResultChunkVector mode)
    const uint8_t* srclimit = in + inlen;
    uint8_t* dst = out;
    uint8_t* dstlimit = out + outlen;
    int e = 0;
    const int64_t tb0 = sm.state0;
    int64_t tb = tb0;
    uint8_t c = 0;
    if ((dstlimit - dst) < (srclimit - src)) {
      e = 239;  // kExitDstSpaceFull, no backup
    } else {
      for (;;) {                 // Do_state_table (:645)
        tb = tb0; e = 0; c = 0;
      newe:                      // Do_state_table_newe (:651)
        while (src < srclimit) {
          c = *src;
          e = sm8(sm, tb + c);
          *dst = c;
          ++src; ++dst;
          if (e >= kExitIllegalStructure) break;
          tb = tb0 + ((int64_t)e << sh);
        }
        if (e < kExitIllegalStructure) break;   // source consumed
        int offset = 0;
        bool again = true;
        switch (e) {
          case kExitReplace31:
            dst -= 2;
            if (om) { om->copy((int)(src - copystart) - 2); om->del(2); copystart = src; }
            dst[-1] = (uint8_t)sm8(sm, tb + c + nEntries * 1); break;
          case kExitReplace32:
            dst -= 1;
            if (om) { om->copy((int)(src - copystart) - 1); om->del(1); copystart = src; }
            dst[-2] = (uint8_t)sm8(sm, tb + c + nEntries * 2);
            dst[-1] = (uint8_t)sm8(sm, tb + c + nEntries * 1); break;
          case kExitReplace21:
            dst -= 1;
            if (om) { om->copy((int)(src - copystart) - 1); om->del(1); copystart = src; }
            dst[-1] = (uint8_t)sm8(sm, tb + c + nEntries * 1); break;
          case kExitReplace3:
            dst[-3] = (uint8_t)sm8(sm, tb + c + nEntries * 3);
            dst[-2] = (uint8_t)sm8(sm, tb + c + nEntries * 2);
            dst[-1] = (uint8_t)sm8(sm, tb + c + nEntries * 1); break;
          case kExitReplace2:
            dst[-2] = (uint8_t)sm8(sm, tb + c + nEntries * 2);
            dst[-1] = (uint8_t)sm8(sm, tb + c + nEntries * 1); break;
          case kExitReplace1:
            dst[-1] = (uint8_t)sm8(sm, tb + c + nEntries * 1); break;
          case kExitReplace1S0:
            dst[-1] = (uint8_t)sm8(sm, tb + c + 256 * 1); break;
          case kExitReplaceOffset2:
          case kExitSpecial:
          case kExitReplaceOffset1: {
            bool z = (nEntries != 256) && in_state_zero(sm, tb);
            if (e == kExitReplaceOffset2)
              offset += (uint8_t)sm8(sm, tb + c + (z ? 256 : nEntries) * 2) << 8;
            offset += (uint8_t)sm8(sm, tb + c + (z ? 256 : nEntries) * 1);
            if ((uint32_t)offset >= sm.n_remap) { e = kExitIllegalStructure; again = false; break; }
            const uint8_t* re = sm.remap + 4 * offset;
            int del_len = re[0] & 0x7F;
            int add_len = re[1] & 0x7F;
            if ((re[1] & 0x80) && !plain && (uint32_t)offset + 1 < sm.n_remap) {   // HTML half of the pair (:755-762)
              re += 4;
              add_len = re[1] & 0x7F;
            }
            int soff = re[2] | (re[3] << 8);
            uint8_t* newdst = dst - del_len + add_len;
            if ((dstlimit - newdst) < (srclimit - src)) { e = 239; again = false; break; }
            dst -= del_len;
            for (int k = 0; k < add_len; ++k)
              dst[k] = ((uint32_t)(soff + k) < sm.n_rstr) ? sm.rstr[soff + k] : 0;
            dst += add_len;
            if (om) {
              if (add_len > del_len) {
                om->copy((int)(src - copystart)); om->insert(add_len - del_len); copystart = src;
              } else if (add_len < del_len) {
                om->copy((int)(src - copystart) + add_len - del_len); om->del(del_len - add_len);
                copystart = src;
              }
            }
            if (re[0] & 0x80) {
              int ne = ((uint32_t)(soff + add_len) < sm.n_rstr) ? sm.rstr[soff + add_len] : 0;
              tb = tb0 + ((int64_t)ne << sh);
              goto newe;
            }
            break;
          }
          default:
            again = false;
            break;
        }
        if (!again) break;
      }
      if (e >= 239) {           // exit code: back up over the rejected character
        --src; --dst;
        if (!in_state_zero(sm, tb)) {
          do { --src; --dst; } while (src > in && (src[0] & 0xC0) == 0x80);
        }
      } else if (!in_state_zero(sm, tb)) {
        e = kExitIllegalStructure;
        do { --src; --dst; } while (src > in && (src[0] & 0xC0) == 0x80);
      } else {
        e = kExitOK;
      }
      if (om && src > copystart) { om->copy((int)(src - copystart)); copystart = src; }
    }
    int consumed = (int)(src - in), filled = (int)(dst - out);
    total_filled += filled;
    if (e != kExitDoAgain) break;
    in += consumed; inlen -= consumed; out += filled; outlen -= filled;
  }
  return total_filled;
}


// ------------------------------------------------------------ lang/script
__device__ __forceinline__ int rtype_of(const DevTables& T, int s) {        // lang_script.cc:154-160
  if (s < 0 || (uint32_t)s >= T.n_scripts) s = 0;
  return gld(T.rtype + (s));
}
__device__ __forceinline__ int default_language(const DevTables& T, int s) { // :314-318
  if (s < 0 || (uint32_t)s >= T.n_scripts) return (int)T.unknown_lang;
  return gld(T.deflang + (s));
}
__device__ __forceinline__ uint32_t per_script_number_latin(const DevTables& T, int lang) { // :320-326
  if (gld(T.rtype + (T.latin)) == RTypeNone) return 1;
  if (lang < 0 || (uint32_t)lang >= T.l2p_size) return 0;
  return gld(T.l2p + (lang));
}
__device__ __forceinline__ int from_per_script_number(const DevTables& T, int s, uint8_t ps) { // :328-341
  if (s < 0 || (uint32_t)s >= T.n_scripts) return (int)T.unknown_lang;
  int rt = gld(T.rtype + (s));
  if (rt == RTypeNone || rt == RTypeOne) return gld(T.deflang + (s));
  if ((uint32_t)s == T.latin) return gld(T.p2l_latn + (ps));
  return gld(T.p2l_othr + (ps));
}
__device__ __forceinline__ int close_set(const DevTables& T, int lang) {      // :261-310
  if (lang < 0 || (uint32_t)lang >= T.n_langs) return 0;
  return gld(T.close_set + (lang));
}
__device__ __forceinline__ int lscript4(const DevTables& T, int s) {          // :552-557
  return (uint32_t)s == T.latin ? 0 : (uint32_t)s == T.cyrillic ? 1 : (uint32_t)s == T.arabic ? 2 : 3;
}

// -------------------------------------------------------------- hashing
__device__ __forceinline__ uint32_t ld32(const uint8_t* p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
__constant__ uint32_t kWordMask0[4] = {0xFFFFFFFFu, 0x000000FFu, 0x0000FFFFu, 0x00FFFFFFu};

// QuadHashV2 / QuadHashV2Mix  cldutil_shared.cc:167-202
__device__ uint32_t quad_hash_v2(const uint8_t* w, int n) {
  if (n == 0) return 0;
  uint32_t pre = 0;
  if (w[-1] == ' ') pre |= 0x00004444u;
  if (w[n] == ' ') pre |= 0x44440000u;
  uint32_t w0, w1, w2;
  if (n <= 4) {
    w0 = ld32(w) & kWordMask0[n & 3]; w0 ^= w0 >> 3;
    return w0 ^ pre;
  } else if (n <= 8) {
    w0 = ld32(w); w0 ^= w0 >> 3;
    w1 = ld32(w + 4) & kWordMask0[n & 3]; w1 ^= w1 << 4;
    return (w0 ^ pre) + w1;
  }
  w0 = ld32(w); w0 ^= w0 >> 3;
  w1 = ld32(w + 4); w1 ^= w1 << 4;
  w2 = ld32(w + 8) & kWordMask0[n & 3]; w2 ^= w2 << 2;
  return (w0 ^ pre) + w1 + w2;
}
// BiHashV2 cldutil_shared.cc:107-122
__device__ uint32_t bi_hash_v2(const uint8_t* w, int n) {
  if (n == 0) return 0;
  uint32_t w0, w1;
  if (n <= 4) { w0 = ld32(w) & kWordMask0[n & 3]; return w0 ^ (w0 >> 3); }
  w0 = ld32(w); w0 ^= w0 >> 3;
  w1 = ld32(w + 4) & kWordMask0[n & 3]; w1 ^= w1 << 18;
  return w0 + w1;
}
// OctaHash40 / OctaHash40Mix cldutil_shared.cc:234-354 (64-bit carries kept)
__device__ uint64_t octa_hash40(const uint8_t* w, int n) {
  if (n == 0) return 0;
  uint64_t pre = 0;
  if (w[-1] == ' ') pre |= 0x00004444u;
  if (w[n] == ' ') pre |= 0x44440000u;
  int q = (n - 1) >> 2;
  if (q > 5) q = 5;
  uint64_t w0 = ld32(w);
  if (q == 0) w0 &= kWordMask0[n & 3];
  uint64_t sum = w0;
  w0 ^= w0 >> 3;
  for (int i = 1; i <= q; ++i) {
    uint64_t w1 = ld32(w + 4 * i);
    if (i == q) w1 &= kWordMask0[n & 3];
    sum += w1;
    switch (i) {
      case 1: w1 ^= w1 << 4; break;
      case 2: w1 ^= w1 << 2; break;
      case 3: w1 ^= w1 >> 8; break;
      case 4: w1 ^= w1 >> 4; break;
      default: w1 ^= w1 >> 6; break;
    }
    w0 += w1;
  }
  sum += sum >> 17;
  sum += sum >> 9;
  sum = (sum & 0xFF) << 32;
  return (w0 ^ pre) + sum;
}
__device__ __forceinline__ uint64_t pair_hash(uint64_t a, uint64_t b) {   // cldutil_shared.cc:384-386
  return ((a >> 13) | (a << 51)) + b;
}

// QuadHashV3Lookup4 / OctaHashV3Lookup4 cldutil_shared.h:380-454: one 16-byte
// bucket gather, first of four slots whose masked key matches.
__device__ __forceinline__ uint32_t lookup4(const DevTbl& t, uint32_t sub, uint32_t key) {
  if (t.n_buckets == 0) return 0;
  const uint4 b = gld4(t.b + 4 * (size_t)sub);
  if (((key ^ b.x) & t.key_mask) == 0) return b.x;
  if (((key ^ b.y) & t.key_mask) == 0) return b.y;
  if (((key ^ b.z) & t.key_mask) == 0) return b.z;
  if (((key ^ b.w) & t.key_mask) == 0) return b.w;
  return 0;
}
__device__ __forceinline__ uint32_t quad_lookup(const DevTbl& t, uint32_t h) {
  return lookup4(t, (h + (h >> 12)) & (t.size - 1), h & t.key_mask);
}
// GetQuadHits' probe (cldutil.cc:356-363): QuadHashV3Lookup4 on the first
// quadgram table, then on the second one only on a miss.  Both buckets are
// gathered at once -- the second load need not wait for the first answer --
// so a miss costs one L2 round trip, not two.  ind: the indirect subscript,
// bit 31 set for the second table.  Returns the matching keyvalue or 0.
__device__ __forceinline__ uint32_t quad_probe(const DevTbl& q1, const DevTbl& q2, uint32_t h, uint32_t& ind) {
  const bool two = q2.size != 0 && q2.n_buckets != 0;
  const uint4 b1 = q1.n_buckets ? gld4(q1.b + 4 * (size_t)((h + (h >> 12)) & (q1.size - 1))) : make_uint4(0, 0, 0, 0);
  const uint4 b2 = two ? gld4(q2.b + 4 * (size_t)((h + (h >> 12)) & (q2.size - 1))) : make_uint4(0, 0, 0, 0);
  auto match = [](uint4 b, uint32_t key, uint32_t mask) -> uint32_t {
    if (((key ^ b.x) & mask) == 0) return b.x;
    if (((key ^ b.y) & mask) == 0) return b.y;
    if (((key ^ b.z) & mask) == 0) return b.z;
    if (((key ^ b.w) & mask) == 0) return b.w;
    return 0u;
  };
  uint32_t probs = q1.n_buckets ? match(b1, h & q1.key_mask, q1.key_mask) : 0u;
  ind = 0;
  if (probs == 0 && q2.size != 0) {
    probs = two ? match(b2, h & q2.key_mask, q2.key_mask) : 0u;
    if (probs) ind = (probs & ~q2.key_mask) | 0x80000000u;
  } else if (probs) {
    ind = probs & ~q1.key_mask;
  }
  return probs;
}
__device__ __forceinline__ uint32_t octa_lookup(const DevTbl& t, uint64_t h) {
  uint32_t sub = (uint32_t)((h + (h >> 12)) & (uint64_t)(t.size - 1));
  return lookup4(t, sub, (uint32_t)(h >> 4) & t.key_mask);
}
__device__ __forceinline__ uint32_t ind_at(const DevTbl& t, uint32_t i) { return i < t.n_ind ? gld(t.ind + i) : 0u; }

// ------------------------------------------------------------------ totes
struct DocTote {                                              // tote.h:65-107
  int incr_count;
  int sorted;
  uint16_t key[24];
  int value[24], score[24], rel[24];
  __device__ void init() {
    incr_count = 0; sorted = 0;
    for (int i = 0; i < 24; ++i) key[i] = kUnusedKey;
  }
  __device__ void add(uint16_t k, int bytes, int sc, int r) { // tote.cc:127-175
    ++incr_count;
    int s0 = k & 15, s1 = s0 ^ 8, s2 = (k & 7) + 16;
    int s = key[s0] == k ? s0 : key[s1] == k ? s1 : key[s2] == k ? s2 : -1;
    if (s >= 0) { value[s] += bytes; score[s] += sc; rel[s] += r * bytes; return; }
    int a;
    if (key[s0] == kUnusedKey) a = s0;
    else if (key[s1] == kUnusedKey) a = s1;
    else if (key[s2] == kUnusedKey) a = s2;
    else {
      a = s0;
      if (value[s1] < value[a]) a = s1;
      if (value[s2] < value[a]) a = s2;
    }
    key[a] = k; value[a] = bytes; score[a] = sc; rel[a] = r * bytes;
  }
  __device__ int find(uint16_t k) const {                     // tote.cc:178-202
    if (sorted) {
      for (int s = 0; s < 24; ++s) if (key[s] == k) return s;
      return -1;
    }
    int s0 = k & 15;
    if (key[s0] == k) return s0;
    if (key[s0 ^ 8] == k) return s0 ^ 8;
    if (key[(k & 7) + 16] == k) return (k & 7) + 16;
    return -1;
  }
  __device__ void sort3() {                                   // tote.cc:221-250 (n = 3)
    for (int s = 0; s < 3; ++s) {
      if (key[s] == kUnusedKey) value[s] = -1;
      for (int s2 = s + 1; s2 < 24; ++s2) {
        if (key[s2] == kUnusedKey) value[s2] = -1;
        if (value[s] < value[s2]) {
          uint16_t tk = key[s]; key[s] = key[s2]; key[s2] = tk;
          int t = value[s]; value[s] = value[s2]; value[s2] = t;
          t = score[s]; score[s] = score[s2]; score[s2] = t;
          t = rel[s]; rel[s] = rel[s2]; rel[s2] = t;
        }
      }
    }
    sorted = 1;
  }
};

// ReliabilityDelta cldutil.cc:553-571
__device__ int reliability_delta(int v1, int v2, int grams) {
  int maxr = grams < 8 ? 12 * grams : 100;
  int thr = (grams * 5) >> 3;
  thr = thr < 3 ? 3 : thr > 16 ? 16 : thr;
  int d = v1 - v2;
  if (d >= thr) return maxr;
  if (d <= 0) return 0;
  int r = (100 * d) / thr;
  return r < maxr ? r : maxr;
}
// ReliabilityExpected cldutil.cc:585-605 -- double, no contraction
__device__ int reliability_expected(int actual, int expected) {
  if (expected == 0) return 100;
  if (actual == 0) return 0;
  double ratio = expected > actual ? (1.0 * expected) / actual : (1.0 * actual) / expected;
  if (ratio <= 1.5) return 100;
  if (ratio > 4.0) return 0;
  double num = __dmul_rn(100.0, 4.0 - ratio);
  return (int)__ddiv_rn(num, 2.5);
}

// ------------------------------------------------------------ HTML mode
// IsSpecial (getonescriptspan.cc:470-477)
__device__ __forceinline__ bool is_special(uint8_t c) { return c == '<' || c == '>' || c == '&'; }

// ScanToPossibleLetter (getonescriptspan.cc:150-203, 503-541): the cheap tag
// parser as a transition function over the reference's byte classes (the
// same restatement the oracle pins against the reference, tests/test_html_hints.py).
enum { TC_LT, TC_GT, TC_EX, TC_HY, TC_QU, TC_AP, TC_SL, TC_S, TC_C, TC_R, TC_I, TC_P, TC_T, TC_Y, TC_L, TC_E,
       TC_CR, TC_NL, TC_PL };
__device__ int tag_class(uint8_t c) {
  switch (c) {
    case '<': return TC_LT; case '>': return TC_GT; case '!': return TC_EX; case '-': return TC_HY;
    case '"': return TC_QU; case '\'': return TC_AP; case '/': return TC_SL; case '\n': case '\r': return TC_CR;
    case '&': case '@': case '`': return TC_PL;
    default: break;
  }
  if ((c >= 'A' && c <= 'Z') || (c >= 'a' && c <= 'z')) {
    switch (c | 0x20) {
      case 's': return TC_S; case 'c': return TC_C; case 'r': return TC_R; case 'i': return TC_I;
      case 'p': return TC_P; case 't': return TC_T; case 'y': return TC_Y; case 'l': return TC_L;
      case 'e': return TC_E; default: return TC_PL;
    }
  }
  return c >= 0xC0 ? TC_PL : TC_NL;
}
__device__ __forceinline__ int tag_common(int k, int other) {
  return k == TC_LT ? 1 : k == TC_GT ? 2 : k == TC_QU ? 10 : k == TC_AP ? 11 : other;
}
__device__ int tag_next(int s, int k) {
  switch (s) {
    case 0: case 2: return k == TC_LT ? 3 : ((k >= TC_S && k <= TC_E) || k == TC_PL) ? 0 : 2;
    case 3: return k == TC_EX ? 4 : k == TC_S ? 13 : (k == TC_HY || k == TC_SL) ? 9 : tag_common(k, 9);
    case 4: return k == TC_HY ? 5 : tag_common(k, 9);
    case 5: return k == TC_HY ? 6 : tag_common(k, 9);
    case 6: return k == TC_HY ? 7 : 6;
    case 7: return k == TC_HY ? 8 : 6;
    case 8: return k == TC_GT ? 2 : k == TC_HY ? 8 : 6;
    case 9: return tag_common(k, 9);
    case 10: return k == TC_QU ? 9 : k == TC_CR ? 12 : 10;
    case 11: return k == TC_AP ? 9 : k == TC_CR ? 12 : 11;
    case 12: return k == TC_LT ? 1 : k == TC_GT ? 2 : 12;
    case 13: return k == TC_C ? 14 : k == TC_T ? 28 : tag_common(k, 9);
    case 14: return k == TC_R ? 15 : tag_common(k, 9);
    case 15: return k == TC_I ? 16 : tag_common(k, 9);
    case 16: return k == TC_P ? 17 : tag_common(k, 9);
    case 17: return k == TC_T ? 18 : tag_common(k, 9);
    case 18: return (k == TC_GT || k == TC_CR || k == TC_NL) ? 19 : tag_common(k, 9);
    case 19: return k == TC_LT ? 20 : 19;
    case 20: return k == TC_SL ? 21 : 19;
    case 21: return k == TC_S ? 22 : (k == TC_CR || k == TC_NL) ? 21 : 19;
    case 22: return k == TC_C ? 23 : 19;
    case 23: return k == TC_R ? 24 : 19;
    case 24: return k == TC_I ? 25 : 19;
    case 25: return k == TC_P ? 26 : 19;
    case 26: return k == TC_T ? 27 : 19;
    case 27: return k == TC_GT ? 2 : 19;
    case 28: return k == TC_Y ? 29 : tag_common(k, 9);
    case 29: return k == TC_L ? 30 : tag_common(k, 9);
    case 30: return k == TC_E ? 31 : tag_common(k, 9);
    case 31: return (k == TC_GT || k == TC_CR || k == TC_NL) ? 32 : tag_common(k, 9);
    case 32: return k == TC_LT ? 33 : 32;
    case 33: return k == TC_SL ? 34 : 32;
    case 34: return k == TC_S ? 35 : (k == TC_CR || k == TC_NL) ? 34 : 32;
    case 35: return k == TC_T ? 36 : 32;
    case 36: return k == TC_Y ? 37 : 32;
    case 37: return k == TC_L ? 38 : 32;
    case 38: return k == TC_E ? 39 : 32;
    case 39: return k == TC_GT ? 2 : 32;
    default: return 1;
  }
}
__device__ int scan_to_possible_letter(const DocView& d, int start, int len) {
  int src = start, e = 0, st = 0;
  const int lim = start + len;
  while (src < lim) {
    e = tag_next(st, tag_class(d.at(src++)));
    if (e <= 1) { --src; break; }
    st = e;
  }
  if (src >= lim) return len;
  if (e != 0 && e != 2) {
    int off = src - start - 1;
    while (0 < off && d.at(start + off) != '<') --off;
    return off + 1;
  }
  return src - start;
}
// FixUnicodeValue (fixunicodevalue.cc)
__device__ int32_t fix_unicode_value(const DevTables& T, int32_t uv) {
  const uint32_t u = (uint32_t)uv;
  if (u < 0x100) return T.cp1252 ? (int32_t)T.cp1252[u] : uv;
  if (u < 0xD800) return uv;
  if ((u & ~0x0Fu) == 0xFDD0 || (u & ~0x0Fu) == 0xFDE0 || (u & 0xFFFEu) == 0xFFFE) return 0xFFFD;
  if (0xE000 <= u && u <= 0x10FFFF) return uv;
  return 0xFFFD;
}
__device__ __forceinline__ bool is_digit_c(uint8_t c) { return c >= '0' && c <= '9'; }
__device__ __forceinline__ bool is_xdigit_c(uint8_t c) {
  return is_digit_c(c) || (c >= 'a' && c <= 'f') || (c >= 'A' && c <= 'F');
}
__device__ __forceinline__ bool is_alnum_c(uint8_t c) { return is_digit_c(c) || ((c | 0x20) >= 'a' && (c | 0x20) <= 'z'); }
// strto32_base10 / _base16 (getonescriptspan.cc:325-391), quirks kept
__device__ int32_t entity_number(const DevTables& T, const DocView& d, int p, int lim, bool hex, int* endp) {
  *endp = p;
  while (p < lim && d.at(p) == '0') ++p;
  if (p == lim || !(hex ? is_xdigit_c(d.at(p)) : is_digit_c(d.at(p)))) return -1;
  int e = p;
  while (e < lim && (hex ? is_xdigit_c(d.at(e)) : is_digit_c(d.at(e)))) ++e;
  *endp = e;
  const int n = e - p;
  bool fits;
  if (hex) {
    fits = n < 8 || (n == 8 && d.at(p) < '8');
  } else {
    fits = n < 9;
    if (n == 10) {                                 // memcmp(p, "2147483647", 10) <= 0
      const char* mx = "2147483647";
      int c = 0;
      for (int i = 0; i < 10 && c == 0; ++i) c = (int)d.at(p + i) - (int)(uint8_t)mx[i];
      fits = c <= 0;
    }
  }
  if (!fits) return 0xFFFD;
  int32_t v = 0;
  for (; p < e; ++p) {
    const uint8_t c = d.at(p);
    v = hex ? (int32_t)(((uint32_t)v << 4) + (uint32_t)(is_digit_c(c) ? c - '0' : (c | 0x20) - 'a' + 10))
            : v * 10 + (c - '0');
  }
  return fix_unicode_value(T, v);
}
// LookupEntity (:292-300): binary search of the sorted entity names
__device__ int32_t lookup_entity(const DevTables& T, const DocView& d, int p, int n) {
  if (n >= 16 || !T.ent_names) return -1;
  const uint32_t cnt = *reinterpret_cast<const uint32_t*>(T.ent_names);
  const uint32_t* off = reinterpret_cast<const uint32_t*>(T.ent_names + 4);
  const char* base = reinterpret_cast<const char*>(T.ent_names + 4 + 4 * (cnt + 1));
  uint32_t lo = 0, hi = cnt;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    const char* s = base + off[mid];
    int c = 0, i = 0;
    for (;; ++i) {                                 // strcmp(name, key)
      const int a = (uint8_t)s[i], b = i < n ? d.at(p + i) : 0;
      if (a != b || a == 0) { c = a - b; break; }
    }
    if (c < 0) lo = mid + 1;
    else if (c > 0) hi = mid;
    else return T.ent_values[mid];
  }
  return -1;
}
// ReadEntity (:393-451) at document position p, srcn bytes available
__device__ int32_t read_entity(const DevTables& T, const DocView& d, int p, int srcn, int* consumed) {
  const int end = p + srcn;
  if (srcn == 0 || d.at(p) != '&') { *consumed = 0; return -1; }
  *consumed = 1;
  const int st = p + 1;
  int en;
  int32_t v;
  if (st < end && d.at(st) == '#') {
    if (st + 2 >= end) return -1;
    const uint8_t x = d.at(st + 1);
    v = (x == 'x' || x == 'X') ? entity_number(T, d, st + 2, end, true, &en) : entity_number(T, d, st + 1, end, false, &en);
    if (v == -1 || en > end) return -1;
  } else {
    for (en = st; en < end && is_alnum_c(d.at(en)); ++en) {}
    v = lookup_entity(T, d, st, en - st);
    if (v < 0) return -1;
    if (v >= 256 && !(en < end && d.at(en) == ';')) return -1;
  }
  if (en < end && d.at(en) == ';') ++en;
  *consumed = en - p;
  return v;
}
// runetochar (:249-286)
__device__ int rune_to_utf8(uint8_t* s, uint32_t c) {
  if (c <= 0x7F) { s[0] = (uint8_t)c; return 1; }
  if (c <= 0x7FF) { s[0] = (uint8_t)(0xC0 | (c >> 6)); s[1] = (uint8_t)(0x80 | (c & 0x3F)); return 2; }
  if (c > 0x10FFFF) c = 0xFFFD;
  if (c <= 0xFFFF) {
    s[0] = (uint8_t)(0xE0 | (c >> 12)); s[1] = (uint8_t)(0x80 | ((c >> 6) & 0x3F)); s[2] = (uint8_t)(0x80 | (c & 0x3F));
    return 3;
  }
  s[0] = (uint8_t)(0xF0 | (c >> 18)); s[1] = (uint8_t)(0x80 | ((c >> 12) & 0x3F));
  s[2] = (uint8_t)(0x80 | ((c >> 6) & 0x3F)); s[3] = (uint8_t)(0x80 | (c & 0x3F));
  return 4;
}
// EntityToBuffer (:454-468)
__device__ void entity_to_buffer(const DevTables& T, const DocView& d, int p, int len, uint8_t* dst, int* tlen,
                                 int* plen) {
  const int32_t v = read_entity(T, d, p, len, tlen);
  if (v > 0) {
    *plen = rune_to_utf8(dst, (uint32_t)v);
  } else {
    *tlen = 1;
    *plen = 0;
  }
}
// GetUTF8LetterScriptNum over a small local buffer (a decoded entity)
struct BufView {
  const uint8_t* p;
  __device__ __forceinline__ uint8_t at(int i) const { return p[i]; }
};

// ------------------------------------------------------- close sets
__device__ __forceinline__ bool same_close_set(const DevTables& T, int l1, int l2) {   // :44-56
  int c1 = close_set(T, l1);
  return c1 != 0 && c1 == close_set(T, l2);
}
__device__ uint8_t per_script_number(const DevTables& T, int ulscript, int lang) {  // lang_script.cc:320-326
  if (ulscript < 0 || (uint32_t)ulscript >= T.n_scripts) return 0;
  if (gld(T.rtype + (ulscript)) == RTypeNone) return 1;
  if (lang < 0 || (uint32_t)lang >= T.l2p_size) return 0;
  return gld(T.l2p + (lang));
}
// BetterBoundary scoreonescriptspan.cc:671-720
// ------------------------------------------------------ document level
// RefineScoredClosePairs + MoveLang1ToLang2 compact_lang_det_impl.cc:1105-1203
struct Extract { int lang3[3], pct3[3], rp3[3], text_bytes; bool reliable; double ns3[3]; };

// ExtractLangEtc :1276-1384 with GetNormalizedScore :1269-1273
__device__ __forceinline__ bool is_figs(const DevTables& T, int l) {
  return l == (int)T.french || l == (int)T.italian || l == (int)T.german || l == (int)T.spanish;
}
__device__ __forceinline__ bool is_efigs(const DevTables& T, int l) { return l == (int)T.english || is_figs(T, l); }

// a[i] for a runtime i in 0..2 as selects, so Extract stays in registers
// (a dynamically indexed member array would put the whole struct in scratch)
template <class V>
__device__ __forceinline__ V sel3(const V (&a)[3], int i) { return i == 0 ? a[0] : i == 1 ? a[1] : a[2]; }

// CalcSummaryLang :1414-1522 (best_effort: kCLDFlagBestEffort, :1493)
__device__ __forceinline__ int calc_summary_lang(const DevTables& T, int total, const Extract& x, bool& rel,
                                                 bool best_effort = false) {
  const int unk = (int)T.unknown_lang, en = (int)T.english;
  int slot_count = 3;
  int active[3] = {0, 1, 2};
  int ignore = 0;
  int ret_pct = x.pct3[0];
  int summary = x.lang3[0];
  rel = true;
  if (x.pct3[0] < 2) rel = false;
  for (int i = 0; i < 3; ++i) {
    if (x.lang3[i] == (int)T.tg_unknown) {
      ignore += x.pct3[i];
      for (int j = i + 1; j < 3; ++j) active[j - 1] = active[j];
      --slot_count;
      ret_pct = (x.pct3[0] * 100) / (101 - ignore);
      summary = sel3(x.lang3, active[0]);
      if (sel3(x.pct3, active[0]) < 2) rel = false;
    }
  }
  int second_bytes = (total * sel3(x.pct3, active[1])) / 100;
  int l0 = sel3(x.lang3, active[0]), l1 = sel3(x.lang3, active[1]);
  int p0 = sel3(x.pct3, active[0]), p1 = sel3(x.pct3, active[1]);
  if (l0 == en && l1 != en && l1 != unk && p1 >= 17 && second_bytes >= 15) {
    ignore += p0; ret_pct = (p1 * 100) / (101 - ignore); summary = l1;
    if (p1 < 2) rel = false;
  } else if (is_figs(T, l0) && !is_efigs(T, l1) && l1 != unk && p1 >= 20 && second_bytes >= 15) {
    ignore += p0; ret_pct = (p1 * 100) / (101 - ignore); summary = l1;
    if (p1 < 2) rel = false;
  } else if (l1 == en && l0 != en) {
    ignore += p1; ret_pct = (p0 * 100) / (101 - ignore);
  } else if (is_figs(T, l1) && !is_efigs(T, l0)) {
    ignore += p1; ret_pct = (p0 * 100) / (101 - ignore);
  }
  if (ret_pct < 26 && !best_effort) { summary = unk; rel = false; }
  if (ret_pct < 51) rel = false;
  if (100 - (x.pct3[0] + x.pct3[1] + x.pct3[2]) > 20) rel = false;
  if (slot_count == 0) { summary = unk; rel = false; }
  return summary;
}

__device__ void write_result(cld_result* r, const Extract& x, int summary, bool rel) {
  cld_result o;
  for (int i = 0; i < 3; ++i) {
    o.lang3[i] = (uint16_t)x.lang3[i];
    o.percent3[i] = (int8_t)x.pct3[i];
    o.normalized3[i] = x.ns3[i];
  }
  o.summary_lang = (uint16_t)summary;
  o.is_reliable = rel ? 1 : 0;
  o.text_bytes = x.text_bytes;
  *r = o;
}

// A document the kernels could not score: no language, summary CLD_LANG_FAILED.
__device__ void mark_failed(const DevTables& T, cld_result* r) {
  for (int k = 0; k < 3; ++k) {
    r->lang3[k] = (uint16_t)T.unknown_lang;
    r->percent3[k] = 0;
    r->normalized3[k] = 0.0;
  }
  r->summary_lang = (uint16_t)CLD_LANG_FAILED;
  r->is_reliable = 0;
  r->text_bytes = 0;
}

}  // namespace cld
