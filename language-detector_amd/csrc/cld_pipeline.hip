// cld_pipeline.hip -- the CLD2 DetectLanguage hot path as gfx950 device code.
//
// One document per lane.  A wavefront carries 64 independent documents
// through span segmentation, lowercasing, gram hashing + bucket probes, chunk
// totes and the document tote/summary.  Design notes:
//
//  * No per-round hit buffers of the reference size: quad/octa/uni/bi hits are
//    kept as packed (u16 offset, u32 indirect) streams sized to the kernel's
//    document-length bucket; LinearizeAll's linear[] array is never built --
//    the three sorted hit streams are merge-walked directly into the chunk
//    totes (ChunkAll + ScoreAllHits fused), so a round touches each hit once.
//  * Scoring tables stay in HBM and are gathered through L2/MALL (they are
//    ~0.8 MB, far below one XCD's 4 MB L2); per-lane state lives in private
//    (scratch) memory in the short-document kernel and in a per-lane global
//    arena in the general kernel.
//  * The only floating point is ReliabilityExpected; this file is compiled
//    with -ffp-contract=off so its double ops round exactly like the oracle.
//
// Every function cites the reference lines whose semantics it implements.

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
struct DevMap;
__device__ void dm_copy(DevMap& m, int b);
__device__ void dm_insert(DevMap& m, int b);
__device__ void dm_delete(DevMap& m, int b);
__device__ int lower_replace_sm(const DevSM& sm, const uint8_t* in0, int ilen, uint8_t* out0, int olen,
                                bool plain = true, DevMap* om = nullptr) {
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
            if (om) { dm_copy(*om, (int)(src - copystart) - 2); dm_delete(*om, 2); copystart = src; }
            dst[-1] = (uint8_t)sm8(sm, tb + c + nEntries * 1); break;
          case kExitReplace32:
            dst -= 1;
            if (om) { dm_copy(*om, (int)(src - copystart) - 1); dm_delete(*om, 1); copystart = src; }
            dst[-2] = (uint8_t)sm8(sm, tb + c + nEntries * 2);
            dst[-1] = (uint8_t)sm8(sm, tb + c + nEntries * 1); break;
          case kExitReplace21:
            dst -= 1;
            if (om) { dm_copy(*om, (int)(src - copystart) - 1); dm_delete(*om, 1); copystart = src; }
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
                dm_copy(*om, (int)(src - copystart)); dm_insert(*om, add_len - del_len); copystart = src;
              } else if (add_len < del_len) {
                dm_copy(*om, (int)(src - copystart) + add_len - del_len); dm_delete(*om, del_len - add_len);
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
      if (om && src > copystart) { dm_copy(*om, (int)(src - copystart)); copystart = src; }
    }
    int consumed = (int)(src - in), filled = (int)(dst - out);
    total_filled += filled;
    if (e != kExitDoAgain) break;
    in += consumed; inlen -= consumed; out += filled; outlen -= filled;
  }
  return total_filled;
}

__device__ __forceinline__ int lower_replace(const DevTables& T, const uint8_t* in0, int ilen, uint8_t* out0, int olen,
                                             bool plain = true, DevMap* om = nullptr) {
  return lower_replace_sm(T.lower, in0, ilen, out0, olen, plain, om);
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
struct Tote {                                                 // tote.h:33-61
  uint16_t score[256];      // first: 8-byte aligned groups of four keys
  uint64_t in_use;
  int score_count;
  __device__ void reinit() { in_use = 0; score_count = 0; }
  __device__ void add(uint8_t key, int delta) {              // tote.cc:52-61
    int g = key >> 2;
    uint64_t m = 1ull << g;
    if (!(in_use & m)) {
      *reinterpret_cast<uint64_t*>(&score[g * 4]) = 0;
      in_use |= m;
    }
    score[key] = (uint16_t)(score[key] + delta);
  }
  __device__ void top3(int* key3) const {                    // tote.cc:65-101
    key3[0] = key3[1] = key3[2] = -1;
    int s0 = -1, s1 = -1, s2 = -1;
    uint64_t m = in_use;
    while (m) {
      int g = __ffsll((unsigned long long)m) - 1;
      m &= m - 1;
      for (int i = 0; i < 4; ++i) {
        int k = g * 4 + i;
        int v = score[k];
        if (v > s2) {
          if (v > s1) {
            s2 = s1; key3[2] = key3[1];
            if (v > s0) { s1 = s0; key3[1] = key3[0]; s0 = v; key3[0] = k; }
            else { s1 = v; key3[1] = k; }
          } else {
            s2 = v; key3[2] = k;
          }
        }
      }
    }
  }
};

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

struct Boosts { int n; uint32_t lp[kMaxBoosts]; };            // scoreonescriptspan.h:116-120

// ProcessProbV2Tote cldutil.cc:128-138
__device__ __forceinline__ void add_lang_prob(const DevTables& T, uint32_t lp, Tote& t) {
  const uint8_t* e = T.lgprob + 8 * (lp & 0xFF);
  uint8_t k1 = (lp >> 8) & 0xFF, k2 = (lp >> 16) & 0xFF, k3 = (lp >> 24) & 0xFF;
  if (k1) t.add(k1, e[5]);
  if (k2) t.add(k2, e[6]);
  if (k3) t.add(k3, e[7]);
}

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

// ------------------------------------------------------------- workspaces
// Per-lane state.  Capacities are template constants so the short kernel can
// keep everything in private memory; the general kernel instantiates the
// reference maxima in a global per-lane arena.
template <int SB_, int LB_, int HB_, bool MULTIPASS_>
struct Work {
  static constexpr int SB = SB_, LB = LB_, HB = HB_;
  static constexpr bool MULTIPASS = MULTIPASS_;
  uint8_t sbuf[SB + 16];
  uint8_t lbuf[LB + 16];
  uint16_t b_off[HB + 1]; uint32_t b_ind[HB + 1];
  uint16_t d_off[HB + 1]; uint32_t d_ind[HB + 1];
  uint16_t x_off[HB + 1]; uint32_t x_ind[HB + 1];
  Tote tote;
  int predict[MULTIPASS_ ? kPredictionTableSize : 1];
  int sqz[MULTIPASS_ ? kPredictionTableSize : 1];
};

struct Span { uint8_t* text; int text_bytes; int ulscript; };

// Thrown (as a flag) when a short-kernel capacity would be exceeded or more
// passes are needed: the document is re-queued for the general kernel.
struct Status { bool requeue; };

// ------------------------------------------------- ResultChunkVector mode
// OffsetMap (offsetmap.cc:43-453): copy / insert / delete ranges from the
// document (A) to the text built from it (A'), one byte per range in the
// reference's coding (2-bit op, 6-bit length, prefix bytes for long ranges,
// adjacent copies merged).  Built by the scanner (map2original_) and the
// lowercaser (map2uplow_) only when a document asks for its chunk vector.
enum { DM_PREFIX = 0, DM_COPY = 1, DM_INSERT = 2, DM_DELETE = 3 };
struct DevMap {
  uint8_t* d; int n, cap;
  int pend_op, pend_len, max_a, max_ap;
  bool over;                                  // capacity exceeded: the document reports an error
  // MapBack's resume point: the start (byte index, A and A' offsets) of the
  // range the last lookup settled on.  Entries before it never change (the
  // map only grows at its end), and every range before it ends at or below
  // its A' offset, so a lookup at or past that offset may start there: the
  // summary buffer maps its chunks in increasing order, which made MapBack
  // quadratic in the span length when every lookup walked from the start.
  int cur_i, cur_a, cur_ap;
};
__device__ void dm_push(DevMap& m, int op, int len) {           // Emit :203-206
  if (m.n >= m.cap) { m.over = true; return; }
  m.d[m.n++] = (uint8_t)((op << 6) | (len & 0x3F));
}
__device__ void dm_clear(DevMap& m) {
  m.n = 0; m.pend_op = DM_COPY; m.pend_len = 0; m.max_a = 0; m.max_ap = 0;
  m.cur_i = 0; m.cur_a = 0; m.cur_ap = 0;
}
__device__ void dm_flush(DevMap& m) {                           // Flush :158-187
  if (m.pend_len == 0) return;
  if (m.pend_op == DM_COPY && m.n > 0) {
    const uint8_t c = m.d[m.n - 1];
    if ((c >> 6) == DM_COPY && (c & 0x3F) + m.pend_len <= 0x3F) {
      m.d[m.n - 1] = (uint8_t)(c + m.pend_len);
      m.pend_len = 0;
      return;
    }
  }
  if (m.pend_len > 0x3F) {
    bool nz = false;
    for (int shift = 30; shift > 0; shift -= 6) {
      const int prefix = (m.pend_len >> shift) & 0x3F;
      if (prefix > 0 || nz) { dm_push(m, DM_PREFIX, prefix); nz = true; }
    }
  }
  dm_push(m, m.pend_op, m.pend_len & 0x3F);
  m.pend_len = 0;
}
__device__ void dm_copy(DevMap& m, int b) {                     // Copy :107-118
  if (b == 0) return;
  m.max_a += b; m.max_ap += b;
  if (m.pend_op == DM_COPY) m.pend_len += b;
  else { dm_flush(m); m.pend_op = DM_COPY; m.pend_len = b; }
}
__device__ void dm_insert(DevMap& m, int b) {                   // Insert :122-138
  if (b == 0) return;
  m.max_ap += b;
  if (m.pend_op == DM_INSERT) m.pend_len += b;
  else if (b == 1 && m.pend_op == DM_DELETE && m.pend_len == 1) m.pend_op = DM_COPY;
  else { dm_flush(m); m.pend_op = DM_INSERT; m.pend_len = b; }
}
__device__ void dm_delete(DevMap& m, int b) {                   // Delete :141-156
  if (b == 0) return;
  m.max_a += b;
  if (m.pend_op == DM_DELETE) m.pend_len += b;
  else if (b == 1 && m.pend_op == DM_INSERT && m.pend_len == 1) m.pend_op = DM_COPY;
  else { dm_flush(m); m.pend_op = DM_DELETE; m.pend_len = b; }
}
__device__ void dm_reset(DevMap& m) {                           // Reset -> MaybeFlushAll :190-200
  if (0 < m.pend_len || m.n == 0) { dm_copy(m, 1); dm_flush(m); }
}
// MapBack :428-452: the range of non-zero A' width that holds ap (the
// reference's window walk settles on the same one).
__device__ int dm_map_back(DevMap& m, int ap) {
  dm_reset(m);
  if (ap < 0) return 0;
  if (m.max_ap <= ap) return (ap - m.max_ap) + m.max_a;
  int lo_a = 0, lo_ap = 0, i = 0;
  if (m.cur_ap <= ap) { i = m.cur_i; lo_a = m.cur_a; lo_ap = m.cur_ap; }
  while (i < m.n) {
    const int i0 = i;
    int op = DM_PREFIX, len = 0;
    while (i < m.n && op == DM_PREFIX) {
      const uint8_t c = m.d[i++];
      op = c >> 6;
      len = (len << 6) + (c & 0x3F);
    }
    if (op == DM_PREFIX) break;
    const int hi_a = lo_a + (op == DM_INSERT ? 0 : len), hi_ap = lo_ap + (op == DM_DELETE ? 0 : len);
    if (ap < hi_ap) {
      m.cur_i = i0; m.cur_a = lo_a; m.cur_ap = lo_ap;
      const int a = ap - (lo_ap - lo_a);
      return a >= hi_a ? hi_a : a;
    }
    lo_a = hi_a; lo_ap = hi_ap;
  }
  return (ap - m.max_ap) + m.max_a;
}

// SetChunkSummary's fields (scoreonescriptspan.h:240-252) as the vector path keeps them
struct ChunkSum { uint16_t offset, chunk_start, lang1, lang2, score1, bytes; uint8_t rd, rs; };
constexpr int kVecLinear = 4 * (kMaxScoringHits + 8) + 8;

// Per-document vector state (in the lane's arena) for k_general_vec.
struct VecOut {
  DevMap orig, low;                           // map2original_, map2uplow_
  cld_chunk* v; int n, cap; bool over;        // the document's ResultChunkVector (its pool region)
  const uint8_t* doc; int doc_len;            // the original document (SummaryBufferToVector backs up in it)
  uint32_t lin_lp[kVecLinear];                // this round's linear[] langprobs and offsets
  uint16_t lin_off[kVecLinear];
  ChunkSum sb[kMaxSummaries + 1];             // the round's summary buffer + the dummy off the end
};

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

// ------------------------------------------------------------- scanner
// ScriptScanner::SkipToFrontOfSpan: getonescriptspan.cc:592-642
__device__ int skip_to_front_of_span(const DevTables& T, const DocView& d, int start, int len, int* script,
                                     bool plain) {
  int sc = 0, skip = 0, tlen = 0, plen = 0;
  while (skip < len) {
    skip += scan_to_letter_or_special(T, d, start + skip, len - skip);
    if (skip >= len) { *script = sc; return len; }
    const uint8_t c = d.at(start + skip);
    if (!plain && is_special(c)) {
      if (c == '<') {
        tlen = scan_to_possible_letter(d, start + skip, len - skip);
        sc = 0;
      } else if (c == '>') {
        tlen = 1;
        sc = 0;
      } else {                                   // '&': expand, no advance
        uint8_t tmp[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        entity_to_buffer(T, d, start + skip, len - skip, tmp, &tlen, &plen);
        if (plen > 0) sc = script_num(T, BufView{tmp}, 0);
      }
    } else {
      tlen = utf8_len(c);
      sc = script_num(T, d, start + skip);
    }
    if (sc != 0) break;
    skip += tlen;
  }
  *script = sc;
  return skip;
}

// ScriptScanner::GetOneScriptSpan: getonescriptspan.cc:799-1027 (HTML mode
// when !plain: tags skipped, entities decoded into the span).
// `next`/`remaining` are next_byte_ - start_byte_ and byte_length_.
template <class W>
__device__ bool get_one_script_span(const DevTables& T, const DocView& d, int& next, int& remaining,
                                    W& w, Span& span, Status& st, bool plain = true, DevMap* mo = nullptr) {
  const int common = (int)T.common, inherited = (int)T.inherited;
  span.text = w.sbuf; span.text_bytes = 0; span.ulscript = 0;
  if (mo) { dm_clear(*mo); dm_delete(*mo, next); }    // map2original_: MapBack(0) = span offset (:835-836)
  int put_soft_limit = kMaxScriptBytes - kWithinScriptTail;
  if (kMaxScriptBytes <= remaining && remaining < 2 * kMaxScriptBytes) put_soft_limit = remaining / 2;
  int spanscript, sc = 0, tlen = 0, plen = 0;
  uint8_t* sb = w.sbuf;
  sb[0] = ' '; sb[1] = 0;
  int take = 0, put = 1;
  int skip = skip_to_front_of_span(T, d, next, remaining, &spanscript, plain);
  next += skip; remaining -= skip;
  if (mo) {
    if (skip != 1) { dm_delete(*mo, skip); dm_insert(*mo, 1); }
    else dm_copy(*mo, 1);
  }
  if (remaining <= 0) { if (mo) dm_reset(*mo); return false; }
  span.ulscript = spanscript;
  const int base = next, bl = remaining;
  while (take < bl) {
    bool need_break = false;
    while (take < bl) {
      uint8_t c0 = d.at(base + take);
      if (put + 4 > W::SB) { st.requeue = true; return false; }
      if (!plain && is_special(c0)) {
        if (c0 == '<' || c0 == '>') { sc = 0; break; }
        entity_to_buffer(T, d, base + take, bl - take, sb + put, &tlen, &plen);   // '&': copy entity, no advance
        if (plen > 0) sc = script_num(T, BufView{sb + put}, 0);
      } else {
        tlen = plen = utf8_len(c0);
        if (take < bl - 3) {
          sb[put] = c0; sb[put + 1] = d.at(base + take + 1);
          sb[put + 2] = d.at(base + take + 2); sb[put + 3] = d.at(base + take + 3);
        } else {
          for (int k = 0; k < plen; ++k) sb[put + k] = d.at(base + take + k);
        }
        sc = script_num(T, d, base + take);
      }
      if (sc != spanscript && sc != inherited) {
        if (sc == common) {
          need_break = true;
        } else {
          int sc2 = script_num(T, d, base + take + tlen);
          if (sc2 != common && sc2 != spanscript) need_break = true;
        }
      }
      if (need_break) break;
      take += tlen; put += plen;
      if (mo) {
        if (tlen == plen) dm_copy(*mo, tlen);
        else if (tlen < plen) { dm_copy(*mo, tlen); dm_insert(*mo, plen - tlen); }
        else { dm_copy(*mo, plen); dm_delete(*mo, tlen - plen); }
      }
      if (put >= kMaxScriptBytes) break;
    }
    while (take < bl) {
      tlen = scan_to_letter_or_special(T, d, base + take, bl - take);
      take += tlen;
      if (mo) dm_delete(*mo, tlen);
      if (take >= bl) break;
      const uint8_t c1 = d.at(base + take);
      if (!plain && is_special(c1)) {
        if (c1 == '<') {
          tlen = scan_to_possible_letter(d, base + take, bl - take);
          sc = 0;
        } else if (c1 == '>') {
          tlen = 1;
          sc = 0;
        } else {                                 // '&': expand, no advance
          if (put + 4 > W::SB) { st.requeue = true; return false; }
          entity_to_buffer(T, d, base + take, bl - take, sb + put, &tlen, &plen);
          if (plen > 0) sc = script_num(T, BufView{sb + put}, 0);
        }
      } else {
        tlen = utf8_len(c1);
        sc = script_num(T, d, base + take);
      }
      if (sc != 0) break;
      take += tlen;
      if (mo) dm_delete(*mo, tlen);
    }
    if (put + 1 > W::SB) { st.requeue = true; return false; }
    sb[put++] = ' ';
    if (mo) dm_insert(*mo, 1);
    if (sc != spanscript && sc != inherited) break;
    if (put >= put_soft_limit) break;
  }
  while (0 < take && take < bl && (d.at(base + take) & 0xC0) == 0x80) { --take; --put; }
  next += take; remaining -= take;
  if (put + 4 > W::SB) { st.requeue = true; return false; }
  sb[put] = ' '; sb[put + 1] = ' '; sb[put + 2] = ' '; sb[put + 3] = 0;
  if (mo) { dm_insert(*mo, 4); dm_reset(*mo); }
  span.text_bytes = put;
  return true;
}

// ScriptScanner::LowerScriptSpan getonescriptspan.cc:1033-1054
template <class W>
__device__ void lower_script_span(const DevTables& T, W& w, Span& span, Status& st, bool plain = true,
                                  DevMap* ml = nullptr) {
  int ilen = span.text_bytes + 3;
  // HTML mode may map a character to more bytes (the &amp;-style half of a
  // remap pair): then only the reference's own capacity bounds it
  if ((plain ? (ilen * 3) / 2 + 4 : kMaxScriptLowerBuffer) > W::LB) { st.requeue = true; return; }
  if (ml) dm_clear(*ml);
  int filled = lower_replace(T, span.text, ilen, w.lbuf, kMaxScriptLowerBuffer, plain, ml);
  w.lbuf[filled] = 0; w.lbuf[filled + 1] = 0; w.lbuf[filled + 2] = 0; w.lbuf[filled + 3] = 0;
  span.text = w.lbuf;
  span.text_bytes = filled - 3;
  if (ml) dm_reset(*ml);
}

// ---------------------------------------------------------- squeezing
__device__ int backscan_to_space(const uint8_t* src, int limit) {        // :491-504
  int n = 0;
  if (limit > 32) limit = 32;
  while (n < limit) { if (src[-n - 1] == ' ') return n; ++n; }
  n = 0;
  while (n < limit) { if ((src[-n] & 0xC0) != 0x80) return n; ++n; }
  return 0;
}
__device__ int forwardscan_to_space(const uint8_t* src, int limit) {     // :509-522
  int n = 0;
  if (limit > 32) limit = 32;
  while (n < limit) { if (src[n] == ' ') return n + 1; ++n; }
  n = 0;
  while (n < limit) { if ((src[n] & 0xC0) != 0x80) return n; ++n; }
  return 0;
}
__device__ __forceinline__ int next_char_code(const uint8_t* src, int* incr) {
  int c = src[0];
  *incr = 1;
  if (c < 0xC0) {
  } else if ((c & 0xE0) == 0xC0) { c = (c << 8) | src[1]; *incr = 2; }
  else if ((c & 0xF0) == 0xE0) { c = (c << 16) | (src[1] << 8) | src[2]; *incr = 3; }
  else { c = (int)(((uint32_t)c << 24) | ((uint32_t)src[1] << 16) | ((uint32_t)src[2] << 8) | src[3]); *incr = 4; }
  return c;
}
__device__ int count_predicted_bytes(const uint8_t* src, int len, int* hash, int* tbl) {  // :541-580
  int p_count = 0, h = *hash;
  const uint8_t* lim = src + len;
  while (src < lim) {
    int incr;
    int c = next_char_code(src, &incr);
    src += incr;
    int p = tbl[h];
    tbl[h] = c;
    if (c == p) p_count += incr;
    h = ((h << 4) ^ c) & 0xFFF;
  }
  *hash = h;
  return p_count;
}
__device__ int count_spaces4(const uint8_t* src, int len) {              // :586-595
  int s = 0;
  for (int i = 0; i < (len & ~3); i += 4)
    s += (src[i] == ' ') + (src[i + 1] == ' ') + (src[i + 2] == ' ') + (src[i + 3] == ' ');
  return s;
}
__device__ int cheap_rep_words_inplace(uint8_t* isrc, int src_len, int* hash, int* tbl) {  // :610-692
  const uint8_t* src = isrc;
  const uint8_t* lim = isrc + src_len;
  uint8_t* dst = isrc;
  int h = *hash;
  uint8_t* word_dst = dst;
  int good = 0, wlen = 0;
  while (src < lim) {
    int c = src[0];
    *dst++ = (uint8_t)c;
    if (c == ' ') {
      if (good * 2 > wlen) dst = word_dst;
      word_dst = dst; good = 0; wlen = 0;
    }
    int incr = 1;
    if (c < 0xC0) {
    } else if ((c & 0xE0) == 0xC0) { *dst++ = src[1]; c = (c << 8) | src[1]; incr = 2; }
    else if ((c & 0xF0) == 0xE0) { *dst++ = src[1]; *dst++ = src[2]; c = (c << 16) | (src[1] << 8) | src[2]; incr = 3; }
    else {
      *dst++ = src[1]; *dst++ = src[2]; *dst++ = src[3];
      c = (int)(((uint32_t)c << 24) | ((uint32_t)src[1] << 16) | ((uint32_t)src[2] << 8) | src[3]); incr = 4;
    }
    src += incr;
    wlen += incr;
    int p = tbl[h];
    tbl[h] = c;
    if (c == p) good += incr;
    h = ((h << 4) ^ c) & 0xFFF;
  }
  *hash = h;
  if ((dst - isrc) < (src_len - 3)) { dst[0] = ' '; dst[1] = ' '; dst[2] = ' '; dst[3] = 0; }
  else if ((dst - isrc) < src_len) { dst[0] = ' '; }
  return (int)(dst - isrc);
}
__device__ int cheap_squeeze_inplace(uint8_t* isrc, int src_len, int* tbl) {  // :785-865
  uint8_t* src = isrc;
  uint8_t* dst = src;
  uint8_t* lim = src + src_len;
  bool skipping = false;
  int hash = 0;
  for (int i = 0; i < kPredictionTableSize; ++i) tbl[i] = 0;
  const int chunksize = 48, space_thresh = (48 * 25) / 100, predict_thresh = (48 * 40) / 100;
  while (src < lim) {
    int remaining = (int)(lim - src);
    int len = remaining < chunksize ? remaining : chunksize;
    while ((src[len] & 0xC0) == 0x80) ++len;
    int space_n = count_spaces4(src, len);
    int predb_n = count_predicted_bytes(src, len, &hash, tbl);
    if (space_n >= space_thresh || predb_n >= predict_thresh) {
      if (!skipping) {
        int n = backscan_to_space(dst, (int)(dst - isrc));
        dst -= n;
        if (dst == isrc) *dst++ = ' ';
        skipping = true;
      }
    } else {
      if (skipping) {
        int n = forwardscan_to_space(src, len);
        src += n; remaining -= n; len -= n;
        skipping = false;
      }
      if (len > 0) {
        for (int k = 0; k < len; ++k) dst[k] = src[k];   // memmove, dst <= src
        dst += len;
      }
    }
    src += len;
  }
  if ((dst - isrc) < (src_len - 3)) { dst[0] = ' '; dst[1] = ' '; dst[2] = ' '; dst[3] = 0; }
  else if ((dst - isrc) < src_len) { dst[0] = ' '; }
  return (int)(dst - isrc);
}
// ResultChunkVector mode keeps offsets: the Overwrite variants turn the
// dropped text into '.' runs in place (:697-765, :869-939).
__device__ int cheap_rep_words_inplace_overwrite(uint8_t* isrc, int src_len, int* hash, int* tbl) {
  const uint8_t* src = isrc;
  const uint8_t* lim = isrc + src_len;
  uint8_t* dst = isrc;
  int h = *hash;
  uint8_t* word_dst = dst;
  int good = 0, wlen = 0;
  while (src < lim) {
    int c = src[0];
    *dst++ = (uint8_t)c;
    if (c == ' ') {
      if (good * 2 > wlen)
        for (uint8_t* q = word_dst; q < dst - 1; ++q) *q = '.';
      word_dst = dst; good = 0; wlen = 0;
    }
    int incr = 1;
    if (c < 0xC0) {
    } else if ((c & 0xE0) == 0xC0) { *dst++ = src[1]; c = (c << 8) | src[1]; incr = 2; }
    else if ((c & 0xF0) == 0xE0) { *dst++ = src[1]; *dst++ = src[2]; c = (c << 16) | (src[1] << 8) | src[2]; incr = 3; }
    else {
      *dst++ = src[1]; *dst++ = src[2]; *dst++ = src[3];
      c = (int)(((uint32_t)c << 24) | ((uint32_t)src[1] << 16) | ((uint32_t)src[2] << 8) | src[3]); incr = 4;
    }
    src += incr;
    wlen += incr;
    int p = tbl[h];
    tbl[h] = c;
    if (c == p) good += incr;
    h = ((h << 4) ^ c) & 0xFFF;
  }
  *hash = h;
  if ((dst - isrc) < (src_len - 3)) { dst[0] = ' '; dst[1] = ' '; dst[2] = ' '; dst[3] = 0; }
  else if ((dst - isrc) < src_len) { dst[0] = ' '; }
  return (int)(dst - isrc);
}
__device__ int cheap_squeeze_inplace_overwrite(uint8_t* isrc, int src_len, int* tbl) {
  uint8_t* src = isrc;
  uint8_t* dst = src;
  uint8_t* lim = src + src_len;
  bool skipping = false;
  int hash = 0;
  for (int i = 0; i < kPredictionTableSize; ++i) tbl[i] = 0;
  const int chunksize = 48, space_thresh = (48 * 25) / 100, predict_thresh = (48 * 40) / 100;
  ++src; ++dst;                                      // always keep the leading space
  while (src < lim) {
    int remaining = (int)(lim - src);
    int len = remaining < chunksize ? remaining : chunksize;
    while ((src[len] & 0xC0) == 0x80) ++len;
    int space_n = count_spaces4(src, len);
    int predb_n = count_predicted_bytes(src, len, &hash, tbl);
    if (space_n >= space_thresh || predb_n >= predict_thresh) {
      if (!skipping) {
        int n = backscan_to_space(dst, (int)(dst - isrc));
        for (uint8_t* q = dst - n; q < dst; ++q) *q = '.';
        skipping = true;
      }
      for (uint8_t* q = dst; q < dst + len; ++q) *q = '.';
      dst[len - 1] = ' ';
    } else if (skipping) {
      int n = forwardscan_to_space(src, len);
      for (uint8_t* q = dst; q < dst + n - 1; ++q) *q = '.';
      skipping = false;
    }
    dst += len;
    src += len;
  }
  if ((dst - isrc) < (src_len - 3)) { dst[0] = ' '; dst[1] = ' '; dst[2] = ' '; dst[3] = 0; }
  else if ((dst - isrc) < src_len) { dst[0] = ' '; }
  return (int)(dst - isrc);
}
__device__ bool cheap_squeeze_trigger_test(const uint8_t* src, int src_len, int* tbl) {  // :952-971
  const int testsize = 256;
  if (src_len < testsize) return false;
  if (count_spaces4(src, testsize) >= (testsize * 25) / 100) return true;
  for (int i = 0; i < kPredictionTableSize; ++i) tbl[i] = 0;
  int hash = 0;
  return count_predicted_bytes(src, testsize, &hash, tbl) >= (testsize * 67) / 100;
}

// ------------------------------------------------------------ hit streams
// GetQuadHits cldutil.cc:315-405
template <class W>
__device__ int get_quad_hits(const DevTables& T, const uint8_t* text, int off, int limit, W& w, int& nb, Status& st) {
  const uint8_t* src = text + off;
  const uint8_t* lim = text + limit;
  int npq = 0;
  uint32_t pq0 = 0, pq1 = 0;
  if (src[0] == ' ') ++src;
  while (src < lim) {
    const uint8_t* e = src;
    e += adv_but_space(e[0]); e += adv_but_space(e[0]);
    const uint8_t* mid = e;
    e += adv_but_space(e[0]); e += adv_but_space(e[0]);
    uint32_t h = quad_hash_v2(src, (int)(e - src));
    if (h != pq0 && h != pq1) {
      uint32_t flag = 0;
      const DevTbl* hit = &T.quad;
      uint32_t probs = quad_lookup(T.quad, h);
      if (probs == 0 && T.quad2.size != 0) {
        flag = 0x80000000u; hit = &T.quad2;
        probs = quad_lookup(T.quad2, h);
      }
      if (probs != 0) {
        if (npq == 0) pq0 = h; else pq1 = h;
        npq ^= 1;
        if (nb >= W::HB) { st.requeue = true; return 0; }
        w.b_off[nb] = (uint16_t)(src - text);
        w.b_ind[nb] = (probs & ~hit->key_mask) | flag;
        ++nb;
      }
    }
    src = (e[0] == ' ') ? e : mid;
    if (src < lim) src += adv_space_vowel(src[0]);
    else src = lim;
    if (nb >= kMaxScoringHits) break;
  }
  w.b_off[nb] = (uint16_t)(src - text);
  w.b_ind[nb] = 0;
  return (int)(src - text);
}

// GetOctaHits cldutil.cc:416-533
template <class W>
__device__ void get_octa_hits(const DevTables& T, const uint8_t* text, int off, int limit, W& w,
                              int& nd, int& nx, Status& st) {
  const uint8_t* src = text + off;
  const uint8_t* lim = text + limit + 1;
  int npo = 0;
  uint64_t po[2] = {0, 0};
  int charcount = 0;
  if (src[0] == ' ') ++src;
  const uint8_t* prior_word_start = src;
  const uint8_t* word_start = src;
  const uint8_t* word_end = src;
  while (src < lim) {
    if (src[0] == ' ') {
      uint64_t wh = octa_hash40(word_start, (int)(word_end - word_start));
      if (wh != po[0] && wh != po[1]) {
        po[npo] = wh; npo = 1 - npo;
        uint64_t tph = po[npo];
        if (nx + 2 > W::HB || nd + 1 > W::HB) { st.requeue = true; return; }
        if (tph != 0 && tph != wh) {
          uint32_t probs = octa_lookup(T.distinctocta, pair_hash(tph, wh));
          if (probs) {
            w.x_off[nx] = (uint16_t)(prior_word_start - text);
            w.x_ind[nx] = probs & ~T.distinctocta.key_mask;
            ++nx;
          }
        }
        uint32_t probs = octa_lookup(T.distinctocta, wh);
        if (probs) {
          w.x_off[nx] = (uint16_t)(word_start - text);
          w.x_ind[nx] = probs & ~T.distinctocta.key_mask;
          ++nx;
        }
        probs = octa_lookup(T.deltaocta, wh);
        if (probs) {
          w.d_off[nd] = (uint16_t)(word_start - text);
          w.d_ind[nd] = probs & ~T.deltaocta.key_mask;
          ++nd;
        }
      }
      charcount = 0;
      prior_word_start = word_start;
      word_start = src + 1;
      word_end = word_start;
    } else {
      ++charcount;
    }
    src += utf8_len(src[0]);
    if (charcount <= 8) word_end = src;
    if (nd >= kMaxScoringHits) break;
    if (nx >= kMaxScoringHits - 1) break;
  }
  uint16_t dummy = (uint16_t)(src - text);
  w.d_off[nd] = dummy; w.d_ind[nd] = 0;
  w.x_off[nx] = dummy; w.x_ind[nx] = 0;
}

// GetUniHits cldutil.cc:201-244
template <class W>
__device__ int get_uni_hits(const DevTables& T, const uint8_t* text, int off, int limit, W& w, int& nb, Status& st) {
  const uint8_t* src = text + off;
  const uint8_t* lim = text + limit;
  if (src[0] == ' ') ++src;
  while (src < lim) {
    const uint8_t* us = src;
    int len = utf8_len(us[0]);
    src += len;
    int propval = uni_prop(T, us, len);
    if (propval > 0) {
      if (nb >= W::HB) { st.requeue = true; return 0; }
      w.b_off[nb] = (uint16_t)(src - text);
      w.b_ind[nb] = (uint32_t)propval;
      ++nb;
    }
    if (nb >= kMaxScoringHits) break;
  }
  w.b_off[nb] = (uint16_t)(src - text);
  w.b_ind[nb] = 0;
  return (int)(src - text);
}

// GetBiHits cldutil.cc:248-310
template <class W>
__device__ void get_bi_hits(const DevTables& T, const uint8_t* text, int off, int limit, W& w,
                            int& nd, int& nx, Status& st) {
  const uint8_t* src = text + off;
  const uint8_t* lim = text + limit;
  while (src < lim) {
    int len = utf8_len(src[0]);
    int len2 = utf8_len(src[len]) + len;
    if (6 <= len2) {
      uint32_t bh = bi_hash_v2(src, len2);
      if (nd + 1 > W::HB || nx + 1 > W::HB) { st.requeue = true; return; }
      uint32_t probs = quad_lookup(T.deltabi, bh);
      if (probs) {
        w.d_off[nd] = (uint16_t)(src - text); w.d_ind[nd] = probs & ~T.deltabi.key_mask; ++nd;
      }
      probs = quad_lookup(T.distinctbi, bh);
      if (probs) {
        w.x_off[nx] = (uint16_t)(src - text); w.x_ind[nx] = probs & ~T.distinctbi.key_mask; ++nx;
      }
    }
    src += len;
    if (nd >= kMaxScoringHits) break;
    if (nx >= kMaxScoringHits - 1) break;
  }
  uint16_t dummy = (uint16_t)(src - text);
  w.d_off[nd] = dummy; w.d_ind[nd] = 0;
  w.x_off[nx] = dummy; w.x_ind[nx] = 0;
}

// ------------------------------------------------- linearize + chunk (fused)
// LinearizeAll (scoreonescriptspan.cc:856-975) as a generator: yields the
// linear[] entries in order without materialising the array.
struct LinearEntry { int offset; int type; uint32_t langprob; };

template <class W>
struct Linearizer {
  const DevTables* T;
  const W* w;
  const DevTbl *base_obj, *base_obj2, *delta_obj, *distinct_obj;
  int base_hit;
  int bi, di, xi, bl, dl, xl;
  bool seed_pending;
  uint32_t seed_lp;
  int seed_off;
  bool pend2;                 // second langprob of a two-langprob base hit
  LinearEntry pend;

  __device__ void init(const DevTables& TT, const W& ww, bool cjk, int nb, int nd, int nx, int lowest,
                       uint32_t seed) {
    T = &TT; w = &ww;
    if (cjk) { base_obj = &TT.compat; base_obj2 = &TT.compat; delta_obj = &TT.deltabi; distinct_obj = &TT.distinctbi; base_hit = UNIHIT; }
    else { base_obj = &TT.quad; base_obj2 = &TT.quad2; delta_obj = &TT.deltaocta; distinct_obj = &TT.distinctocta; base_hit = QUADHIT; }
    bi = di = xi = 0; bl = nb; dl = nd; xl = nx;
    seed_pending = true; seed_lp = seed; seed_off = lowest; pend2 = false;
  }

  __device__ bool next(LinearEntry& e) {
    if (seed_pending) {
      seed_pending = false;
      e.offset = seed_off; e.type = base_hit; e.langprob = seed_lp;
      return true;
    }
    if (pend2) { pend2 = false; e = pend; return true; }
    while (bi < bl || di < dl || xi < xl) {
      int boff = w->b_off[bi], doff = w->d_off[di], xoff = w->x_off[xi];
      if (di < dl && doff <= boff && doff <= xoff) {
        uint32_t lp = ind_at(*delta_obj, w->d_ind[di]);
        ++di;
        if (lp > 0) { e.offset = doff; e.type = DELTAHIT; e.langprob = lp; return true; }
      } else if (xi < xl && xoff <= boff && xoff <= doff) {
        uint32_t lp = ind_at(*distinct_obj, w->x_ind[xi]);
        ++xi;
        if (lp > 0) { e.offset = xoff; e.type = DISTINCTHIT; e.langprob = lp; return true; }
      } else {
        uint32_t ind = w->b_ind[bi];
        const DevTbl* lb = base_obj;
        if (ind & 0x80000000u) { lb = base_obj2; ind &= ~0x80000000u; }
        ++bi;
        if (ind < lb->size_one) {
          uint32_t lp = ind_at(*lb, ind);
          if (lp > 0) { e.offset = boff; e.type = base_hit; e.langprob = lp; return true; }
        } else {
          ind += ind - lb->size_one;
          uint32_t lp = ind_at(*lb, ind), lp2 = ind_at(*lb, ind + 1);
          if (lp > 0 && lp2 > 0) {
            e.offset = boff; e.type = base_hit; e.langprob = lp;
            pend.offset = boff; pend.type = base_hit; pend.langprob = lp2; pend2 = true;
            return true;
          }
          if (lp > 0) { e.offset = boff; e.type = base_hit; e.langprob = lp; return true; }
          if (lp2 > 0) { e.offset = boff; e.type = base_hit; e.langprob = lp2; return true; }
        }
      }
    }
    return false;
  }
};

struct Ctx {
  int ulscript;
  Boosts latn, othr;        // ScoringContext::distinct_boost (scoreonescriptspan.h:139)
  // ApplyHints result (compact_lang_det_impl.cc:1645-1684): langprior_boost
  // latn[4] othr[4], then langprior_whack latn[4] othr[4]; null for none
  const uint32_t* priors;
  VecOut* vo;               // ResultChunkVector being built (k_general_vec), else null
  int flags;                // the caller's public flags (kCLDFlagScoreAsQuads / kCLDFlagBestEffort)
};

// SetChunkSummary scoreonescriptspan.cc:60-96
__device__ ChunkSum chunk_summary(const DevTables& T, int ulscript, int lo, int hi, int first_linear, const Tote& t) {
  int key3[3];
  t.top3(key3);
  int lang1 = from_per_script_number(T, ulscript, (uint8_t)key3[0]);
  int lang2 = from_per_script_number(T, ulscript, (uint8_t)key3[1]);
  int len = hi - lo;
  int sc1 = key3[0] >= 0 ? t.score[key3[0]] : 0;
  int sc2 = key3[1] >= 0 ? t.score[key3[1]] : 0;
  int actual = 0;
  if (len > 0) actual = (int)((uint32_t)sc1 << 10) / len;
  int esub = lang1 * 4 + lscript4(T, ulscript);
  int expected = (esub >= 0 && (uint32_t)esub < T.n_expected) ? gld(T.expected + (esub)) : 0;
  ChunkSum cs;
  cs.offset = (uint16_t)lo;
  cs.chunk_start = (uint16_t)first_linear;
  cs.lang1 = (uint16_t)lang1;
  cs.lang2 = (uint16_t)lang2;
  cs.score1 = (uint16_t)sc1;
  cs.bytes = (uint16_t)len;
  uint16_t grams = (uint16_t)t.score_count;
  int rd = (uint8_t)reliability_delta((uint16_t)sc1, (uint16_t)sc2, grams);
  int c1 = close_set(T, lang1);
  if (c1 != 0 && c1 == close_set(T, lang2)) rd = 100;
  cs.rd = (uint8_t)rd;
  cs.rs = (uint8_t)reliability_expected(actual, expected);
  return cs;
}
// SummaryBufferToDocTote :305-315, one entry
__device__ __forceinline__ void chunk_to_doc(const ChunkSum& cs, DocTote& dt) {
  int rel = cs.rd < cs.rs ? cs.rd : cs.rs;
  dt.add(cs.lang1, cs.bytes, cs.score1, rel);
}

// ---------------------------------------------- chunk vector (vec mode)
__device__ __forceinline__ bool same_close_set(const DevTables& T, int l1, int l2) {   // :44-56
  int c1 = close_set(T, l1);
  return c1 != 0 && c1 == close_set(T, l2);
}
__device__ int get_lang_score(const DevTables& T, uint32_t lp, uint8_t pslang) {     // cldutil.cc:141-152
  const uint8_t* e = T.lgprob + 8 * (lp & 0xFF);
  int r = 0;
  if (((lp >> 8) & 0xFF) == pslang) r += e[5];
  if (((lp >> 16) & 0xFF) == pslang) r += e[6];
  if (((lp >> 24) & 0xFF) == pslang) r += e[7];
  return r;
}
__device__ uint8_t per_script_number(const DevTables& T, int ulscript, int lang) {  // lang_script.cc:320-326
  if (ulscript < 0 || (uint32_t)ulscript >= T.n_scripts) return 0;
  if (gld(T.rtype + (ulscript)) == RTypeNone) return 1;
  if (lang < 0 || (uint32_t)lang >= T.l2p_size) return 0;
  return gld(T.l2p + (lang));
}
// BetterBoundary scoreonescriptspan.cc:671-720
__device__ int better_boundary(const DevTables& T, const VecOut& vo, uint8_t ps0, uint8_t ps1, int lin0, int lin1,
                               int lin2) {
  if (lin2 - lin0 <= 8) return lin1;
  int running = 0, diff[8];
  for (int i = lin0; i < lin0 + 8; ++i) {
    uint32_t lp = vo.lin_lp[i];
    diff[i & 7] = get_lang_score(T, lp, ps0) - get_lang_score(T, lp, ps1);
    if (i < lin0 + 4) running += diff[i & 7]; else running -= diff[i & 7];
  }
  int best_value = 0, best = lin1;
  for (int i = lin0; i < lin2 - 8; ++i) {
    if (best_value < running) {
      bool plus = false, minus = false;
      for (int kk = 0; kk < 8; ++kk) { plus |= diff[kk] > 0; minus |= diff[kk] < 0; }
      if (plus && minus) { best_value = running; best = i + 4; }
    }
    uint32_t lp = vo.lin_lp[i + 8];
    int nd = get_lang_score(T, lp, ps0) - get_lang_score(T, lp, ps1);
    int md = diff[(i + 4) & 7], od = diff[i & 7];
    diff[i & 7] = nd;
    running += 2 * md - od - nd;
  }
  return best;
}
// SharpenBoundaries :764-829 over vo.sb[0..n] (sb[n] = the dummy off the end)
__device__ void sharpen_boundaries(const DevTables& T, VecOut& vo, int ulscript, int n) {
  int prior_linear = vo.sb[0].chunk_start;
  uint16_t prior_lang = vo.sb[0].lang1;
  for (int i = 1; i < n; ++i) {
    ChunkSum& cs = vo.sb[i];
    const uint16_t this_lang = cs.lang1;
    if (this_lang == prior_lang) { prior_linear = cs.chunk_start; continue; }
    const int this_linear = cs.chunk_start, next_linear = vo.sb[i + 1].chunk_start;
    if (same_close_set(T, prior_lang, this_lang)) { prior_linear = this_linear; prior_lang = this_lang; continue; }
    const uint8_t ps0 = per_script_number(T, ulscript, prior_lang), ps1 = per_script_number(T, ulscript, this_lang);
    const int better = better_boundary(T, vo, ps0, ps1, prior_linear, this_linear, next_linear);
    const int old_off = vo.lin_off[this_linear], new_off = vo.lin_off[better];
    cs.chunk_start = (uint16_t)better;
    cs.offset = (uint16_t)new_off;
    cs.bytes = (uint16_t)(cs.bytes - (new_off - old_off));
    vo.sb[i - 1].bytes = (uint16_t)(vo.sb[i - 1].bytes + (new_off - old_off));
    prior_linear = better;
    prior_lang = this_lang;
  }
}
__device__ __forceinline__ int scanner_map_back(VecOut& vo, int t) {      // ScriptScanner::MapBack :1076-1078
  return dm_map_back(vo.orig, dm_map_back(vo.low, t));
}
__device__ void item_to_vector(VecOut& vo, int new_lang, int mapped_offset, int mapped_len) {  // ItemToVector :322-355
  if (vo.n > 0) {
    cld_chunk& prior = vo.v[vo.n - 1];
    if (new_lang == prior.lang1) { prior.bytes = (mapped_offset + mapped_len) - prior.offset; return; }
  }
  if (vo.n >= vo.cap) { vo.over = true; return; }
  cld_chunk rc;
  rc.offset = mapped_offset; rc.bytes = mapped_len; rc.lang1 = (uint16_t)new_lang; rc.pad = 0;
  vo.v[vo.n++] = rc;
}
// SummaryBufferToVector :386-495
__device__ void summary_buffer_to_vector(const DevTables& T, VecOut& vo, int n) {
  const int unk = (int)T.unknown_lang;
  for (int i = 0; i < n; ++i) {
    const ChunkSum cs = vo.sb[i];
    const int unmapped_offset = cs.offset, unmapped_len = cs.bytes;
    int mapped_offset = scanner_map_back(vo, unmapped_offset);
    if (mapped_offset > 0) {
      const int prior_size = vo.n > 0 ? vo.v[vo.n - 1].bytes : 0;
      int n_limit = prior_size - 3 < mapped_offset ? prior_size - 3 : mapped_offset;
      if (n_limit > 12) n_limit = 12;
      auto at = [&](int k) -> uint8_t {           // us[-k - 1] in the original document
        const int q = mapped_offset - k - 1;
        return (unsigned)q < (unsigned)vo.doc_len ? vo.doc[q] : 0;
      };
      int k = 0;
      while (k < n_limit && at(k) >= 0x41) ++k;
      if (k >= n_limit) k = 0;
      if (k < n_limit) {
        const uint8_t ch = at(k);
        if (ch == '\'' || ch == '"' || ch == '#' || ch == '@') ++k;
      }
      if (k > 0) { vo.v[vo.n - 1].bytes -= k; mapped_offset -= k; }
    }
    const int mapped_len = scanner_map_back(vo, unmapped_offset + unmapped_len) - mapped_offset;
    int new_lang = cs.lang1;
    bool delta_bad = cs.rd < 75, score_bad = cs.rs < 75;       // kUnreliablePercentThreshold (:33)
    const uint16_t prior_lang = vo.n > 0 ? vo.v[vo.n - 1].lang1 : (uint16_t)unk;
    if (prior_lang == cs.lang1) delta_bad = false;
    if (same_close_set(T, cs.lang1, prior_lang)) { new_lang = prior_lang; delta_bad = false; }
    if (same_close_set(T, cs.lang1, cs.lang2) && prior_lang == cs.lang2) { new_lang = prior_lang; delta_bad = false; }
    const uint16_t next_lang = (i + 1 >= n) ? (uint16_t)unk : vo.sb[i + 1].lang1;
    if (delta_bad && prior_lang == cs.lang2 && next_lang == cs.lang2) { new_lang = prior_lang; delta_bad = false; }
    if (delta_bad || score_bad) new_lang = unk;
    item_to_vector(vo, new_lang, mapped_offset, mapped_len);
  }
}
__device__ void just_one_item_to_vector(VecOut& vo, int lang1, int unmapped_offset, int unmapped_len) {  // :499-530
  const int mapped_offset = scanner_map_back(vo, unmapped_offset);
  const int mapped_len = scanner_map_back(vo, unmapped_offset + unmapped_len) - mapped_offset;
  item_to_vector(vo, lang1, mapped_offset, mapped_len);
}
// MoveLang1ToLang2's vector half (compact_lang_det_impl.cc:1122-1147)
__device__ void move_lang1_to_lang2_vec(const DevTables& T, VecOut& vo, int lang1, int lang2) {
  int k = 0;
  uint16_t prior_lang = (uint16_t)T.unknown_lang;
  for (int i = 0; i < vo.n; ++i) {
    cld_chunk rc = vo.v[i];
    if (rc.lang1 == lang1) rc.lang1 = (uint16_t)lang2;
    if (rc.lang1 == prior_lang && k > 0) {
      vo.v[k - 1].bytes += rc.bytes;
    } else {
      vo.v[k] = rc;
      ++k;
    }
    prior_lang = rc.lang1;
  }
  vo.n = k;
}

// ProcessHitBuffer (:1067-1116) for one round: LinearizeAll + ChunkAll +
// ScoreAllHits (+ScoreOneChunk/ScoreBoosts/AddDistinctBoost2) + doc tote.
template <class W>
__device__ void score_round(const DevTables& T, Ctx& cx, W& w, bool cjk, int nb, int nd, int nx,
                            int lowest, int ulscript, DocTote& dt) {
  Linearizer<W> lin;
  uint32_t seed = ((uint32_t)per_script_number_latin(T, default_language(T, cx.ulscript)) << 8) | 0u;
  // MakeLangProb(lang, 1): kLgProbV2TblBackmap[1] == 0 (cldutil_shared.h:310-313)
  lin.init(T, w, cjk, nb, nd, nx, lowest, seed);
  const int chunksize = cjk ? kChunksizeUnis : kChunksizeQuads;
  const int base_hit = cjk ? UNIHIT : QUADHIT;
  const int dummy_off = w.b_off[nb];      // linear[next_linear].offset
  Boosts& db = ((uint32_t)cx.ulscript == T.latin) ? cx.latn : cx.othr;
  Tote& t = w.tote;

  LinearEntry cur;
  bool have = lin.next(cur);               // the seed always exists
  int left = nb;
  int nchunks = 0;
  VecOut* vo = cx.vo;
  int li = 0;                              // linear[] subscript (chunk_start values)
  int nsb = 0;
  // ChunkAll: with no base hits, one dummy chunk holding every entry
  bool single = (left <= 0);
  while (single || left > 0) {
    int blen = chunksize;
    if (left < chunksize + (chunksize >> 1)) blen = left;
    else if (left < 2 * chunksize) blen = (left + 1) >> 1;
    bool last = single || (left - blen <= 0);
    t.reinit();
    int lo = have ? cur.offset : dummy_off;
    const int first_li = li;
    int cnt = 0;
    while (have && (last || cnt < blen)) {
      if (vo) { vo->lin_lp[li] = cur.langprob; vo->lin_off[li] = (uint16_t)cur.offset; }
      ++li;
      add_lang_prob(T, cur.langprob, t);
      if (cur.type <= QUADHIT) t.score_count++;
      if (cur.type == DISTINCTHIT) { db.lp[db.n] = cur.langprob; db.n = (db.n + 1) & (kMaxBoosts - 1); }
      if (cur.type == base_hit) ++cnt;
      have = lin.next(cur);
    }
    // ScoreBoosts (scoreonescriptspan.cc:125-152): prior boosts, distinct
    // boosts, then the prior whacks zero their languages (ZeroPSLang :39-42)
    const int so = ((uint32_t)cx.ulscript == T.latin) ? 0 : 4;
    if (cx.priors)
      for (int k = 0; k < kMaxBoosts; ++k) if (cx.priors[so + k] > 0) add_lang_prob(T, cx.priors[so + k], t);
    for (int k = 0; k < kMaxBoosts; ++k) if (db.lp[k] > 0) add_lang_prob(T, db.lp[k], t);
    if (cx.priors)
      for (int k = 0; k < kMaxBoosts; ++k)
        if (cx.priors[8 + so + k] > 0) t.score[(cx.priors[8 + so + k] >> 8) & 0xFF] = 0;
    int hi = have ? cur.offset : dummy_off;
    if (nchunks < kMaxSummaries) {
      const ChunkSum cs = chunk_summary(T, ulscript, lo, hi, first_li, t);
      if (vo) vo->sb[nsb++] = cs;
      else chunk_to_doc(cs, dt);
    }
    ++nchunks;
    if (single) break;
    left -= blen;
  }
  if (vo) {
    // ProcessHitBuffer with a vector (:1097-1115): dummy entry off the end
    // (ScoreAllHits :289-297), SharpenBoundaries, then the doc tote and the vector
    ChunkSum& dm = vo->sb[nsb];
    dm = ChunkSum{};
    dm.offset = (uint16_t)dummy_off;
    dm.chunk_start = (uint16_t)li;
    vo->lin_off[li] = (uint16_t)dummy_off;
    sharpen_boundaries(T, *vo, cx.ulscript, nsb);
    for (int i = 0; i < nsb; ++i) chunk_to_doc(vo->sb[i], dt);
    summary_buffer_to_vector(T, *vo, nsb);
  }
}

// ScoreOneScriptSpan :1302-1333 with ScoreEntireScriptSpan :1132-1160,
// ScoreCJKScriptSpan :1163-1214, ScoreQuadScriptSpan :1231-1277
template <class W>
__device__ void score_one_script_span(const DevTables& T, Ctx& cx, W& w, const Span& span, DocTote& dt, Status& st) {
  int rt = rtype_of(T, span.ulscript);
  if ((cx.flags & kCLDFlagScoreAsQuads) && rt != RTypeCJK) rt = RTypeMany;   // :1318-1320
  if (rt == RTypeNone || rt == RTypeOne) {
    int bytes = span.text_bytes;
    dt.add((uint16_t)default_language(T, span.ulscript), bytes, bytes, 100);
    if (cx.vo) just_one_item_to_vector(*cx.vo, default_language(T, span.ulscript), 1, bytes - 1);
    return;
  }
  const bool cjk = (rt == RTypeCJK);
  int off = 1;
  int lowest = off;
  const int limit = span.text_bytes;
  while (off < limit) {
    int nb = 0, nd = 0, nx = 0, next;
    if (cjk) {
      next = get_uni_hits(T, span.text, off, limit, w, nb, st);
      if (st.requeue) return;
      get_bi_hits(T, span.text, off, next, w, nd, nx, st);
    } else {
      next = get_quad_hits(T, span.text, off, limit, w, nb, st);
      if (st.requeue) return;
      get_octa_hits(T, span.text, off, next, w, nd, nx, st);
    }
    if (st.requeue) return;
    score_round(T, cx, w, cjk, nb, nd, nx, lowest, span.ulscript, dt);
    lowest = next;        // SpliceHitBuffer :1118-1127
    off = next;
  }
}

// ------------------------------------------------------ document level
// RefineScoredClosePairs + MoveLang1ToLang2 compact_lang_det_impl.cc:1105-1203
__device__ __forceinline__ void refine_scored_close_pairs(const DevTables& T, DocTote& d, VecOut* vo = nullptr) {
  for (int s = 0; s < 24; ++s) {
    int cs = close_set(T, d.key[s]);
    if (cs == 0) continue;
    for (int s2 = s + 1; s2 < 24; ++s2) {
      if (close_set(T, d.key[s2]) == cs) {
        int from, to;
        if (d.value[s] < d.value[s2]) { from = s; to = s2; } else { from = s2; to = s; }
        const int from_lang = d.key[from], to_lang = d.key[to];
        d.value[to] += d.value[from]; d.score[to] += d.score[from]; d.rel[to] += d.rel[from];
        d.key[from] = kUnusedKey; d.score[from] = 0; d.rel[from] = 0;
        if (vo) move_lang1_to_lang2_vec(T, *vo, from_lang, to_lang);
        break;
      }
    }
  }
}
// RemoveUnreliableLanguages :997-1101 (score field receives newbytes, as there)
__device__ __forceinline__ void remove_unreliable_languages(const DevTables& T, DocTote& d) {
  for (int s = 0; s < 24; ++s) {
    int lang = d.key[s];
    if (lang == kUnusedKey) continue;
    int bytes = d.value[s], reli = d.rel[s];
    if (bytes == 0) continue;
    int rp = reli / bytes;
    if (rp >= 41) continue;
    int alt = (int)T.unknown_lang;
    if ((uint32_t)lang <= T.hawaiian && (uint32_t)lang < T.n_closest) alt = gld(T.closest + (lang));
    if (alt == (int)T.unknown_lang) continue;
    int as = d.find((uint16_t)alt);
    if (as < 0) continue;
    int bytes2 = d.value[as], reli2 = d.rel[as];
    if (bytes2 == 0) continue;
    int rp2 = reli2 / bytes2;
    int to = as, from = s;
    if (rp2 < rp || (rp2 == rp && lang < alt)) { to = s; from = as; }
    int np = rp > rp2 ? rp : rp2;
    if (np < 41) np = 41;
    int nbytes = bytes + bytes2;
    d.key[from] = kUnusedKey; d.score[from] = 0; d.rel[from] = 0;
    d.score[to] = nbytes; d.rel[to] = np * nbytes;
  }
  for (int s = 0; s < 24; ++s) {
    if (d.key[s] == kUnusedKey) continue;
    int bytes = d.value[s], reli = d.rel[s];
    if (bytes == 0) continue;
    if (reli / bytes >= 41) continue;
    d.key[s] = kUnusedKey; d.score[s] = 0; d.rel[s] = 0;
  }
}

struct Extract { int lang3[3], pct3[3], rp3[3], text_bytes; bool reliable; double ns3[3]; };

// ExtractLangEtc :1276-1384 with GetNormalizedScore :1269-1273
__device__ __forceinline__ void extract_lang_etc(const DevTables& T, const DocTote& d, int total, Extract& x) {
  const int unk = (int)T.unknown_lang;
  int bc[3] = {0, 0, 0};
  for (int i = 0; i < 3; ++i) { x.rp3[i] = 0; x.lang3[i] = unk; x.pct3[i] = 0; x.ns3[i] = 0.0; }
  x.reliable = false;
  for (int i = 0; i < 3; ++i) {
    int k = d.key[i];
    if (k != kUnusedKey && k != unk) {
      x.lang3[i] = k;
      bc[i] = d.value[i];
      x.rp3[i] = d.rel[i] / (bc[i] ? bc[i] : 1);
      x.ns3[i] = bc[i] <= 0 ? 0.0 : (double)((int32_t)((uint32_t)d.score[i] << 10) / bc[i]);
    }
  }
  int t12 = bc[0] + bc[1], t123 = t12 + bc[2];
  if (total < t123) total = t123;
  int div = total > 1 ? total : 1;
  x.pct3[0] = (bc[0] * 100) / div;
  x.pct3[1] = (t12 * 100) / div;
  x.pct3[2] = (t123 * 100) / div;
  x.pct3[2] -= x.pct3[1];
  x.pct3[1] -= x.pct3[0];
  if (x.pct3[1] < x.pct3[2]) { ++x.pct3[1]; --x.pct3[2]; }
  if (x.pct3[0] < x.pct3[1]) { ++x.pct3[0]; --x.pct3[1]; }
  x.text_bytes = total;
  int k0 = d.key[0];
  if (k0 != kUnusedKey && k0 != unk) {
    int b0 = d.value[0];
    x.reliable = (d.rel[0] / (b0 ? b0 : 1)) >= 41;
  }
  if (100 - (x.pct3[0] + x.pct3[1] + x.pct3[2]) > 20) x.reliable = false;
}

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

// DetectLanguageSummaryV2 compact_lang_det_impl.cc:1707-2106 (HTML mode when
// !plain, the ApplyHints priors when given, a ResultChunkVector when vo;
// cflags: the caller's public flags, kCLDFlagScoreAsQuads / kCLDFlagBestEffort);
// recursion unrolled into passes.  Returns the number of passes, or 0 with
// st.requeue set.
template <class W>
__device__ int detect_doc(const DevTables& T, const DocView& d, W& w, cld_result* out, Status& st,
                          bool plain = true, const uint32_t* priors = nullptr, VecOut* vo = nullptr,
                          uint32_t cflags = 0) {
  const int unk = (int)T.unknown_lang;
  int flags = (int)(cflags & (kCLDFlagScoreAsQuads | kCLDFlagBestEffort));
  int passes = 0;
  Extract x;
  if (vo) vo->n = 0;
  if (d.len == 0) {
    for (int i = 0; i < 3; ++i) { x.lang3[i] = unk; x.pct3[i] = 0; x.ns3[i] = 0.0; x.rp3[i] = 0; }
    x.text_bytes = 0;
    write_result(out, x, unk, false);
    return 1;
  }
  for (;;) {
    ++passes;
    DocTote dt;
    dt.init();
    Ctx cx;
    cx.ulscript = 0;
    cx.latn.n = 0; cx.othr.n = 0;
    cx.priors = priors;
    cx.vo = vo;
    cx.flags = flags;
    if (vo) vo->n = 0;                       // resultchunkvector->clear() (:1730-1732)
    for (int k = 0; k < kMaxBoosts; ++k) { cx.latn.lp[k] = 0; cx.othr.lp[k] = 0; }
    int next = 0, remaining = d.len;
    int hash = 0;
    if constexpr (W::MULTIPASS) {
      if (flags & kCLDFlagRepeats) for (int i = 0; i < kPredictionTableSize; ++i) w.predict[i] = 0;
    }
    int total = 0;
    bool restart = false;
    Span span;
    while (get_one_script_span(T, d, next, remaining, w, span, st, plain, vo ? &vo->orig : nullptr)) {
      lower_script_span(T, w, span, st, plain, vo ? &vo->low : nullptr);
      if (st.requeue) return 0;
      if (flags & kCLDFlagSqueeze) {
        if constexpr (W::MULTIPASS)
          span.text_bytes = vo ? cheap_squeeze_inplace_overwrite(span.text, span.text_bytes, w.sqz)
                               : cheap_squeeze_inplace(span.text, span.text_bytes, w.sqz);
      } else if (2048 < span.text_bytes && !(flags & kCLDFlagFinish)) {
        if constexpr (W::MULTIPASS) {
          if (cheap_squeeze_trigger_test(span.text, span.text_bytes, w.sqz)) {
            flags |= kCLDFlagSqueeze; restart = true; break;
          }
        } else {
          st.requeue = true; return 0;
        }
      }
      if (flags & kCLDFlagRepeats) {
        if constexpr (W::MULTIPASS)
          span.text_bytes = vo ? cheap_rep_words_inplace_overwrite(span.text, span.text_bytes, &hash, w.predict)
                               : cheap_rep_words_inplace(span.text, span.text_bytes, &hash, w.predict);
      }
      cx.ulscript = span.ulscript;
      score_one_script_span(T, cx, w, span, dt, st);
      if (st.requeue) return 0;
      total += span.text_bytes;
    }
    if (st.requeue) return 0;
    if (restart) continue;
    refine_scored_close_pairs(T, dt, vo);
    dt.sort3();
    extract_lang_etc(T, dt, total, x);
    bool good = (flags & kCLDFlagFinish) || total <= 256 ||
                (x.reliable && x.pct3[0] >= 70) || (x.reliable && x.pct3[0] + x.pct3[1] >= 93);
    if (good) {
      if (!(flags & kCLDFlagBestEffort)) remove_unreliable_languages(T, dt);   // :1998-2000
      dt.sort3();
      extract_lang_etc(T, dt, total, x);
      bool rel;
      int summary = calc_summary_lang(T, total, x, rel, (flags & kCLDFlagBestEffort) != 0);
      write_result(out, x, summary, rel);
      if (vo && vo->n > 0) {                 // FinishResultVector(0, buffer_length) (:1688-1702)
        cld_chunk& a = vo->v[0];
        if (a.offset > 0) { a.bytes += a.offset; a.offset = 0; }
        cld_chunk& z = vo->v[vo->n - 1];
        if (z.offset + z.bytes < d.len) z.bytes += d.len - (z.offset + z.bytes);
      }
      return passes;
    }
    if constexpr (!W::MULTIPASS) { st.requeue = true; return 0; }
    flags |= kCLDFlagTop40 | kCLDFlagRepeats | kCLDFlagFinish;
    if (total < 256) flags |= kCLDFlagShort | kCLDFlagUseWords;
  }
}

}  // namespace cld
