// cld_long.hip -- one wavefront per document of any length up to kDocCap (k_long).
//
// The wavefront kernel (cld_wave.hip) keeps a <=256-byte document in LDS.
// Longer documents -- multi-span pages, 1000-hit rounds, the Repeats pass --
// run here: the 64 lanes still share one document, but the per-span buffers
// (lowered text up to the reference's 61,440 bytes, word lists, quad chain,
// hit and emission streams, the 4096-entry predictor) sit in a per-wave slot
// in HBM that stays L2/MALL resident while the wave works on it; LDS holds the
// chunk tote, chunk plan and DocTote.
//
//   stage                              reference                         across lanes
//   per-byte script/scanner classes    getonescriptspan.cc:480-485,      bytes; checked to be a per-
//                                      utf8statetable.cc:362-554         character (local) formulation
//   GetOneScriptSpan + LowerScriptSpan getonescriptspan.cc:799-1054      bytes: run/gap state from the
//     (fused)                                                            last break / letter-stop event
//                                                                        (ballot masks), per-char lowering,
//                                                                        prefix-sum compaction; soft/hard
//                                                                        span limits from prefix sums
//   CheapSqueezeTriggerTest            compact_lang_det_impl.cc:952-971  chars (predictor below)
//   CheapRepWordsInplace (pass 2)      compact_lang_det_impl.cc:610-692  chars: 12-bit hash from the last
//                                                                        three chars, equal hashes inside a
//                                                                        window matched by 12 ballots;
//                                                                        segment sums; compaction
//   GetQuadHits                        cldutil.cc:315-405                the chain enters every word at its
//                                                                        first byte: one lane walks one
//                                                                        word; hashes/probes per entry; the
//                                                                        last-two-hits filter by ballot with a
//                                                                        scalar resolve on conflict; 1000 cut
//   GetOctaHits                        cldutil.cc:416-533                words; same filter scheme; caps
//   GetUniHits / GetBiHits             cldutil.cc:201-310                chars
//   LinearizeAll/ChunkAll/ScoreAllHits scoreonescriptspan.cc:856-1031,   chunk k = contiguous range of each
//                                      208-302                           stream (rank arithmetic); LDS tote
//   DocTote / summary                  tote.cc, compact_lang_det_impl    lane 0
//
// Anything this formulation cannot reproduce exactly (a document longer than
// kDocCap, a non-local scanner/lowercaser state, the Squeeze restart, a
// capacity overflow) is appended to seq_list and redone from scratch by
// k_long's SEQ instantiation, whose spans come from the sequential span
// source (cld_seq.hip).

namespace cld {
namespace lng {

using wave::excl_scan;
using wave::lower_char;
using wave::lower_char_sm;
using wave::lanemask_lt;
using wave::rdl;
using wave::rdl64;
using wave::rdlu;
using wave::ufl;
using wave::ufl64;
using wave::uflu;
using wave::wmax;
using wave::wor64;
using wave::wsum;
using wave::wsync;

constexpr int kDocCap = 1 << 20;                     // longest document taken (C5 caps at 64 KB; the slot holds 1 bit per byte)
constexpr int kLB = kMaxScriptLowerBuffer + 256;     // lowered span + pads + hash read slack
constexpr int kDocWords = kDocCap / 64 + 2;
// No per-byte state is stored: classify() and the span builder both derive
// the classes from the document bytes (round 2 measured storing them, 8 B per
// byte written once and streamed back, as slower: C3 828K vs 867K docs/s).
constexpr int kSpanWords = kLB / 64 + 1;
constexpr int kListCap = kLB / 2;                    // words / spaces / chain entries per span
constexpr int kHB = 1024;                            // hits per round (reference: <= 1000)
constexpr int kEB = 2048;                            // base emissions per round (<= 2 per hit)
constexpr int kMaxCh = 64;                           // chunks per round (<= 50 + 1)
// Span cache: pass 1 builds every lowered span into lbd (16-byte aligned, each
// followed by its pads), so pass 2 (Repeats) reads them back instead of
// re-running the span builder over the per-byte classes.
constexpr int kLbdCap = 512 * 1024;
constexpr int kMaxSpans = 4096;
constexpr uint32_t kInf = 0xFFFFFFFFu;
// A lowered span of up to kLdsText - 48 bytes (pads included) is scored from
// LDS: the chain walk, the gram hashes and the word scans then read the text
// at LDS latency instead of through the per-wave HBM slot.  Longer spans run
// the same code on the slot copy.
#ifndef LNG_TEXT
#define LNG_TEXT 6128                    // fills the 8 KB the scoring state shares with the Repeats predictor
#endif
constexpr int kLdsText = LNG_TEXT;
// Read-ahead of the slot's streams (bit 1 word starts, 2 quad chain, 4 octa
// word ends): overlap vs the registers it costs (measured: only 4 pays).
#ifndef LNG_PF
#define LNG_PF 4
#endif
// Inlining of the two largest stages (A/B: a call keeps the caller's
// registers free, inlining lets the slot / LDS accesses stay global / ds).
#ifndef LNG_SR_INL
#define LNG_SR_INL __device__ __forceinline__
#endif
#ifndef LNG_NS_INL
#define LNG_NS_INL __device__ __forceinline__
#endif

// Per-wave working set in HBM (one per resident wavefront of the persistent grid).
struct Slot {
  uint32_t epoch, epoch2;
  uint32_t pad_[30];
  uint64_t pred[kPredictionTableSize];   // Repeats predictor (doc-wide): (epoch << 32) | last char after hash h
  uint64_t pred2[kPredictionTableSize];  // Squeeze / trigger-test predictor (per span), epoch2
  uint64_t lsm[kDocWords];               // letter stops: char start, scanner stops, script != 0
  uint64_t spm[kSpanWords];              // spaces of the lowered span (Repeats, Squeeze)
  uint64_t delm[kSpanWords];             // Repeats: delete flags at segment-ending spaces; Squeeze: predicted starts
  uint64_t aux[2][kSpanWords];           // Squeeze: predicted starts of 2/4-byte, 3/4-byte characters
  uint64_t chm[kSpanWords];              // Squeeze: chunk starts
  alignas(16) uint8_t lb[2][kLB];        // lowered span text; [1] = after CheapRepWords
  alignas(16) uint8_t lbd[kLbdCap];      // pass 1's lowered spans, back to back (span cache)
  int32_t sp_off[kMaxSpans];             //   their offsets in lbd, text_bytes and scripts
  int32_t sp_tb[kMaxSpans];
  int32_t sp_ul[kMaxSpans];
  uint16_t wst[kListCap];                // quad chain entry points (word starts)
  uint16_t wsp[kListCap];                // word-ending spaces (octa words)
  uint16_t chain[kListCap];              // quad chain of the span
  uint16_t b_off[kHB];                   // base hits (debug dump only)
  uint32_t b_ind[kHB];
  uint16_t d_off[kHB];                   // delta / distinct emissions (offsets; adds below)
  uint32_t d_ind[kHB];                   // delta / distinct hits (debug dump only)
  uint16_t x_off[kHB];
  uint32_t x_ind[kHB];
  uint16_t d_hoff[kHB];                  // delta / distinct hit offsets (debug dump only)
  uint16_t x_hoff[kHB];
  uint16_t be_off[kEB];
  uint32_t be_ai[kEB];                   // per emission: its tote adds' index in the per-GPU adds
  uint32_t d_ai[kHB];                    //   table (adds_index), base / delta / distinct
  uint32_t x_ai[kHB];
};

// Per-wave LDS (16-byte aligned: the tote is zeroed and read as uint4).  The
// scoring state and the Repeats predictor are never live together (pass 2
// runs CheapRepWordsInplace over every cached span before scoring any, see
// rep_all), so they share the first 8 KB.  The staged kernels (k_lspan /
// k_lscore / k_lrep) score without the predictor and with a smaller text
// window: SmemT<TEXT, false> (the stage functions take either layout).
template <int TEXT, bool PRED, bool REC = false>
struct alignas(16) SmemT {
  // REC (the span-parallel scoring of k_lgroup): DocTote adds are recorded
  // in order at rec[rec_n++] instead of added, and replayed by k_lfinish
  static constexpr bool kRec = REC;
  union {
    struct {
      uint8_t text[TEXT];                // a window of the current span's lowered text (Win)
      uint32_t tote[256];                // chunk tote, one key per word (uint16 wrap applied at read)
      uint32_t lo[kMaxCh];               // first offset of chunk k
      union {
        struct {                         // round-at-a-time scoring (score_round: CJK spans)
          int32_t theta[kMaxCh];         // chunk k takes delta/distinct emissions with offset <= theta_k
          uint16_t E[kMaxCh];            // base emission number closing chunk k
          uint16_t bst[kMaxCh + 1];
          uint16_t st[2][kMaxCh + 1];    // first delta [0] / distinct [1] emission of chunk k
        };
      };
    };
    uint16_t pred[PRED ? kPredictionTableSize : 1];   // Repeats predictor, 16-bit codes (pred_code)
  };
  uint64_t ring[2][4];                   // distinct boosts (as tote adds), latn / othr, oldest first
  uint64_t pri_add[2][4];                // ApplyHints prior boosts (as tote adds), latn / othr (has_pri)
  uint8_t pri_wk[2][4];                  // ApplyHints prior whacks: the key each zeroes, 0 = none
  int has_pri;                           // the document carries priors (cld_detect_batch_ex hints)
  DocTote dt;
  uint32_t* dbg;                         // debug dump of one document (CLD_DEBUG_DOC), else null
  uint32_t dbg_pos;
  unsigned long long* prof;              // per-stage cycle sums (CLD_PROFILE_STAGES=1), else null
  uint64_t* rec;                         // (REC) where this span's DocTote adds go
  uint32_t rec_n, rec_cap;
  int rec_over;                          // (REC) more adds than rec_cap
};
using Smem = SmemT<kLdsText, true>;
// A DocTote add as recorded (REC): key | bytes << 16 | score << 32 | reliability << 48.
__device__ __forceinline__ uint64_t dt_rec(int key, int bytes, int score, int rel) {
  return (uint64_t)(uint16_t)key | ((uint64_t)(uint16_t)bytes << 16) | ((uint64_t)(uint16_t)score << 32) |
         ((uint64_t)(uint8_t)rel << 48);
}
template <class SM>
__device__ __forceinline__ void dt_add(SM& s, int key, int bytes, int score, int rel) {   // lane 0
  if constexpr (SM::kRec) {
    if (s.rec_n < s.rec_cap) s.rec[s.rec_n] = dt_rec(key, bytes, score, rel);
    else s.rec_over = 1;
    ++s.rec_n;
  } else {
    s.dt.add((uint16_t)key, bytes, score, rel);
  }
}
static_assert(sizeof(Smem) <= 10240, "k_long LDS per wave: 4 blocks of 4 waves per CU must fit 160 KB");

// ------------------------------------------------ ResultChunkVector (vec mode)
// cld_detect_batch_vec runs k_long<.., VEC = true> over every plain document:
// the same span, hit and scoring stages, plus what the reference's vector
// needs (scoreonescriptspan.cc:389-548, 671-845; offsetmap.cc):
//   * the span builder records, per byte of the span text, the document offset
//     ScriptScanner::MapBack returns for it (omap): map2original_'s ops are
//     Copy for letters, Delete + Insert(1) for a gap turned into one space
//     (Copy(1) when the gap is one byte), Insert(4) for the pads; map2uplow_ is
//     the identity because vec mode keeps documents whose lowering changes a
//     character's length on the sequential span source;
//   * Repeats overwrite instead of cutting (CheapRepWordsInplaceOverwrite), so
//     those offsets stay valid; Squeeze documents go to the sequential span source;
//   * per round, linear[] is materialised from the emission streams (rank =
//     merge position, LinearizeAll's tie order) for SharpenBoundaries, whose
//     BetterBoundary window scan runs across lanes; the sharpened chunk bytes
//     feed the DocTote, as there;
//   * SummaryBufferToVector / ItemToVector, the close-pair relabelling and
//     FinishResultVector append to the document's region of the vector pool.
constexpr int kLinCap = 1 + kEB + 2 * kHB + 1;        // seed + base + delta + distinct emissions + dummy
struct VecSlot {                                       // per resident wave, HBM
  uint32_t omap[kLB];                                  // span text position -> document offset
  uint32_t lin_off[kLinCap];                           // the round's linear[]: offsets
  uint64_t lin_add[kLinCap];                           //   langprobs as tote adds
  int32_t vd[kLinCap];                                 // BetterBoundary: pslang0 - pslang1 score per entry
};
struct VecState {                                      // wave-uniform
  VecSlot* vs;
  cld_chunk* v;                                        // the document's region of the pool
  int cap, n;
  bool over;                                           // the vector outgrew its region
  const uint8_t* doc;
  int L;
  int last_off, last_bytes, last_lang;                 // v[n - 1], mirrored
  const uint32_t* hpos;                                // a rewritten HTML page: byte -> page offset, else null
  const uint32_t* hgap;                                //   and where dropped '&'s before a byte began
  bool seq;                                            // spans from seq_span (cld_seq.hip): omap covers any span
};

// Stage cycle accounting: 0 classify, 1 span+lowercase, 2 squeeze test,
// 3 repeats, 4 word lists + quad chain, 5 quad hits, 6 octa/uni/bi hits,
// 7 linearize/chunk/score.  Built with -DLNG_PROF_SUB, slots 0-5 instead split
// score_round (mark_sub) and every other stage lands in slot 6.
#ifdef LNG_PROF_SUB
constexpr bool kProfSub = true;
#else
constexpr bool kProfSub = false;
#endif
template <class SM>
__device__ __forceinline__ void mark(SM& s, int lane, int stage, long long& t) {
  if (kProfSub && stage != 7) stage = 6;
  if (s.prof) {
    const long long now = (long long)clock64();
    if (lane == 0) atomicAdd(&s.prof[stage], (unsigned long long)(now - t));
    t = now;
  }
}
template <class SM>
__device__ __forceinline__ void mark_sub(SM& s, int lane, int stage, long long& t) {
  if (kProfSub && s.prof) {
    const long long now = (long long)clock64();
    if (lane == 0) atomicAdd(&s.prof[stage], (unsigned long long)(now - t));
    t = now;
  }
}

// Debug dump records (u32 words): 'S' span {ul, tb, pass} and 'T' its text
// {tb, bytes packed}; 'R' round {off, next,
// nb, nd, nx, then nb+nd+nx (offset, indirect) pairs}; 'C' chunk {lo, hi, lang1,
// lang2, score1, score2, grams, rel_delta, rel_score}.
template <class SM>
__device__ void dbg_words(SM& s, int lane, const uint32_t* v, int n) {
  if (!s.dbg) return;
  if (lane == 0) {
    for (int i = 0; i < n; ++i) s.dbg[1 + s.dbg_pos + i] = v[i];
    s.dbg_pos += n;
    s.dbg[0] = s.dbg_pos;
  }
  wave::wsync();
}

// 'T' record: a span's text as scored (after Squeeze / Repeats), tb bytes
// packed four to a word.
template <class SM>
__device__ void dbg_text(SM& s, int lane, const uint8_t* text, int tb) {
  if (!s.dbg) return;
  const int n = tb > 0 ? (tb + 3) >> 2 : 0;
  uint32_t* o = s.dbg + 1 + s.dbg_pos;
  if (lane == 0) { o[0] = 'T'; o[1] = (uint32_t)tb; }
  for (int i = lane; i < n; i += 64) {
    uint32_t w = 0;
    for (int k = 0; k < 4; ++k)
      if (4 * i + k < tb) w |= (uint32_t)text[4 * i + k] << (8 * k);
    o[2 + i] = w;
  }
  wave::wsync();
  if (lane == 0) {
    s.dbg_pos += 2 + n;
    s.dbg[0] = s.dbg_pos;
  }
  wave::wsync();
}

// Debug trace (CLD_TRACE=1): lane 0 of each wave stores (document, stage,
// value) into pinned host memory so a stuck batch names its document.
__device__ __forceinline__ void trace(uint32_t* tr, int lane, uint32_t doc, uint32_t stage, uint32_t v) {
  const uint64_t act = __ballot(1);
  if (tr && lane == __builtin_ctzll(act)) {
    __hip_atomic_store(&tr[0], doc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&tr[1], stage | ((uint32_t)__popcll(act) << 16) | ((uint32_t)lane << 24), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&tr[2], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_fetch_add(&tr[3], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// Per-byte class word built by classify():
//   bits 0-7 script number (GetUTF8LetterScriptNum), 8-15 script of the next
//   character, 16-18 character length, 19 lead byte, 20 letter stop,
//   21 cut by the document end, 22 not lowerable here, 24-27 lowered length.
__device__ __forceinline__ int cls_sn(uint32_t c) { return c & 0xFF; }
__device__ __forceinline__ int cls_sn2(uint32_t c) { return (c >> 8) & 0xFF; }
__device__ __forceinline__ int cls_n(uint32_t c) { return (c >> 16) & 7; }
__device__ __forceinline__ bool cls_lead(uint32_t c) { return (c >> 19) & 1; }
__device__ __forceinline__ bool cls_cut(uint32_t c) { return (c >> 21) & 1; }
__device__ __forceinline__ bool cls_nolow(uint32_t c) { return (c >> 22) & 1; }
__device__ __forceinline__ int cls_olen(uint32_t c) { return (c >> 24) & 15; }

__device__ __forceinline__ int topbit(uint64_t m) { return 63 - __builtin_clzll(m); }
__device__ __forceinline__ uint64_t mask_le(int lane) { return lane >= 63 ? ~0ull : ((2ull << lane) - 1); }
__device__ __forceinline__ int nth_bit(uint64_t m, int n) {
  for (int i = 0; i < n; ++i) m &= m - 1;
  return __builtin_ctzll(m);
}
__device__ __forceinline__ uint32_t shfl32(uint32_t v, int l) { return (uint32_t)__shfl((int)v, l, 64); }
__device__ __forceinline__ uint64_t shfl64(uint64_t v, int l) {
  return ((uint64_t)shfl32((uint32_t)(v >> 32), l) << 32) | shfl32((uint32_t)v, l);
}
// Orders global-memory traffic between the lanes of one wavefront (the slot
// is private to the wave; workgroup scope = same CU, same L1).
__device__ __forceinline__ void gsync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

#include "cld_seq.hip"   // spans of the documents the parallel span builder cannot formulate

// LDS window over a lowered span for the hit stages (score_span): s.text
// holds span bytes [w0, w1).  A span longer than the LDS text buffer stays in
// the slot (g); every block of those stages first makes its byte range
// resident (win_text) and reads the text through the biased LDS pointer it
// returns, so the chain walk, the gram hashes and the word scans read LDS at
// any span length (a window reload is a few 16-byte loads per lane, once per
// ~6 KB of text per stage).  g null: the whole span is in s.text already.
// The pointer returned is LDS only: a biased LDS pointer (s.text - w0) must
// never meet a global one in the same value -- the compiler then widens it to
// a flat address before the caller adds its position back, and a window past
// s.text's LDS offset wraps into an address outside every aperture.  So a
// block wider than the window fails here (ok = false); the parallel kernels
// hand that document on, and the sequential span source's instantiation
// reads such spans in place instead (WinG below).
struct Win {
  static constexpr bool kSeq = false;
  const uint8_t* g;
  int w0, w1;
  int len;                                     // bytes of the span buffer that may be copied
};
// (Smem is defined above; the window copy writes s.text.)
template <class SM>
__device__ __forceinline__ const uint8_t* win_text(Win& w, SM& s, int lo, int hi, bool& ok, int lane) {
  hi = hi < w.len ? hi : w.len;
  lo = lo > 0 ? lo : 0;
  if (lo < w.w0 || hi > w.w1) {
    const int a = (lo - 32 > 0 ? lo - 32 : 0) & ~15;
    if (!w.g || hi > a + (int)sizeof(s.text) - 15) {   // (a block wider than the buffer: handed on)
      ok = false;
      return s.text - w.w0;
    }
    const int b = min(w.len, a + (int)sizeof(s.text) - 15);
    const int n16 = (b - a + 15) >> 4;
    wsync();                                     // every lane is done with the previous window
    for (int i = lane; i < n16; i += 64)
      reinterpret_cast<uint4*>(s.text)[i] = gld4(reinterpret_cast<const uint32_t*>(w.g + a) + 4 * i);
    wsync();
    w.w0 = a;
    w.w1 = a + 16 * n16;
  }
  return s.text - w.w0;
}

// The window of detect<.., SEQ> (the sequential span source's documents, the
// ones handed on): a span held whole in LDS (g null) is read there, unbiased;
// a longer one is read in place from the slot (g), at any block width.  The
// two pointers may meet as one flat value: neither is biased.
// kSeq: its span text may hold malformed characters (a lead byte claiming
// bytes that are not continuations, ' ' included), so the hit stages take
// their character starts from the sequential decode (char_starts) instead of
// "not a continuation byte", and a word ends only at a space that starts a
// character -- the positions the reference's walks visit (cldutil.cc:201-533).
struct WinG {
  static constexpr bool kSeq = true;
  const uint8_t* g;
  int w0, w1;
  int len;
};
template <class SM>
__device__ __forceinline__ const uint8_t* win_text(WinG& w, SM& s, int lo, int hi, bool& ok, int lane) {
  (void)lo; (void)hi; (void)ok; (void)lane;
  return w.g ? w.g : s.text;
}
template <bool G> struct WinSel { using type = Win; };
template <> struct WinSel<true> { using type = WinG; };
template <bool G> using WinOf = typename WinSel<G>::type;

// First set bit at or after `from` in a bitmask over positions [0, L); L if none.
__device__ int find_first_g(const uint64_t* m, int from, int L) {
  from = ufl(from);
  if (from >= L) return L;
  int w = from >> 6;
  uint64_t x = ufl64(m[w]) & (~0ull << (from & 63));
  for (;;) {
    if (x) {
      const int r = (w << 6) + __builtin_ctzll(x);
      return r < L ? r : L;
    }
    ++w;
    if ((w << 6) >= L) return L;
    x = ufl64(m[w]);
  }
}

// ----------------------------------------------------- stage 0: classify
// ScanToLetterOrSpecial (getonescriptspan.cc:480-485, utf8statetable.cc:460-554)
// as a per-character property: from state 0 the character either exits on its
// first byte (the scan stops here: 1), or on a later byte from a non-zero state
// (the reference backs up to the lead byte: 1), or returns to state 0 after its
// last byte (the scan continues with the next character: 0).  Anything else
// (-1) makes the sequential scan depend on earlier characters.
// A character cut by the end of the document (`cut`) runs out of input
// instead: the scan ends there, and unless it is back in state 0 it backs up
// to the lead byte (a stop), exactly as at :538-546.
__device__ int scan_char_sm(const DevSM& sm, const DocView& d, int p, int n, bool cut) {
  const int64_t tb0 = sm.state0;
  int64_t tb = tb0;
  for (int k = 0; k < n; ++k) {
    const int e = sm8(sm, tb + d.at(p + k));
    if (e >= kExitIllegalStructure) {
      if (e == kExitDoAgain) return -1;
      if (k == 0) return 1;
      return in_state_zero(sm, tb) ? -1 : 1;
    }
    tb = tb0 + ((int64_t)e << sm.shift);
  }
  if (cut) return in_state_zero(sm, tb) ? (tb == tb0 ? 0 : -1) : 1;
  return tb == tb0 ? 0 : -1;
}
__device__ __forceinline__ int scan_char(const DevTables& T, const DocView& d, int p, int n, bool cut) {
  return scan_char_sm(T.scan, d, p, n, cut);
}

// Character property table: for every well-formed 1-, 2- and 3-byte UTF-8
// sequence (indexed by its bytes, so overlong forms keep their own entry) the
// outcome of the three per-character machines -- GetUTF8LetterScriptNum,
// the ScanToLetterOrSpecial class and the LowerScriptSpan bytes.  Built once
// per GPU by k_build_cpt from the very device functions below; 4-byte and
// malformed sequences still run the machines.
//   bits 0-7 script, 8-9 scan class (0 continue, 1 stop, 3 non-local),
//   10 lowerable here, 11-14 lowered length, 16 lowered differently in HTML
//   mode (the HTML half of a remap pair, utf8statetable.cc:755-762), 32-63
//   lowered bytes
constexpr int kCptSize = 128 + 2048 + 65536;
constexpr uint64_t kCptHtmlLower = 1ull << 16;
using wave::cpt_index;
__device__ uint64_t cpt_eval(const DevTables& T, const uint8_t* b, int n) {
  const DocView dv{b, n};
  const int sn = script_num(T, dv, 0);
  const int st = scan_char(T, dv, 0, n, false);
  uint64_t o = 0;
  int olen = 0;
  const bool lowok = lower_char(T, b, n, o, olen) && olen <= 4;
  uint8_t lp[16], lh[16];
  const int fp = lower_replace_sm(T.lower, b, n, lp, 16, true), fh = lower_replace_sm(T.lower, b, n, lh, 16, false);
  bool hdiff = fp != fh;
  for (int k = 0; k < fp && k < 16; ++k) hdiff |= lp[k] != lh[k];
  return (uint64_t)(sn & 0xFF) | ((uint64_t)(st < 0 ? 3 : st) << 8) | ((uint64_t)lowok << 10) |
         ((uint64_t)(lowok ? olen : 0) << 11) | (hdiff ? kCptHtmlLower : 0ull) |
         ((lowok ? (o & 0xFFFFFFFFull) : 0ull) << 32);
}

// The rare characters the property table does not cover (4-byte or cut by
// the document end): the three machines, out of line so their state does not
// count against the span builder's registers.  The machines go by value (see
// lower_tail).  -> sn | (int8)st << 8 | lowok << 16 | olen << 20 | lowered << 32
__device__ __noinline__ uint64_t char_slow(DevSM script, DevSM scan, DevSM lower, DocView dv, int p, int n,
                                           int avail) {
  const int sn = script_num_sm(script, dv, p);
  const int st = scan_char_sm(scan, dv, p, avail, avail < n);
  uint64_t o = 0;
  int olen = 0;
  const bool lowok = avail == n && lower_char_sm(lower, dv.p + p, n, o, olen) && olen <= 4;
  if (!lowok) { olen = 0; o = 0; }
  return (uint64_t)(sn & 0xFF) | ((uint64_t)(uint8_t)(int8_t)st << 8) | ((uint64_t)lowok << 16) |
         ((uint64_t)olen << 20) | ((o & 0xFFFFFFFFull) << 32);
}

// The document bytes p..p+7 (NULs past its end) as three aligned dwords: a
// dword is loaded only if it holds a byte of the document, so nothing past
// the buffer is touched.  Lanes load them a window ahead (raw_load), and
// raw_bytes realigns them when the window is processed.
__device__ __forceinline__ void raw_load(const DocView& dv, int p, uint32_t& d0, uint32_t& d1, uint32_t& d2) {
  const uintptr_t a = (uintptr_t)(dv.p + p) & ~(uintptr_t)3, end = (uintptr_t)(dv.p + dv.len);
  const uint32_t* q = reinterpret_cast<const uint32_t*>(a);
  d0 = a < end ? gld(q) : 0u;              // (the document is always in global memory)
  d1 = a + 4 < end ? gld(q + 1) : 0u;
  d2 = a + 8 < end ? gld(q + 2) : 0u;
}
__device__ __forceinline__ void raw_bytes(const DocView& dv, int p, uint32_t d0, uint32_t d1, uint32_t d2, uint32_t& lo,
                                          uint32_t& hi) {
  const uint32_t sh = (uint32_t)((uintptr_t)(dv.p + p) & 3);
  lo = __builtin_amdgcn_alignbyte(d1, d0, sh);
  hi = __builtin_amdgcn_alignbyte(d2, d1, sh);
  const int v = dv.len - p;                      // bytes of the document from p on
  if (v < 8) {
    if (v <= 0) lo = hi = 0;
    else if (v < 4) { lo &= (1u << (8 * v)) - 1u; hi = 0; }
    else hi &= v == 4 ? 0u : (1u << (8 * (v - 4))) - 1u;
  }
}

// Per byte p of the document: the class word (cls_* above) and, for a lead
// byte, the lowered bytes of its character (LowerScriptSpan is per character
// once each one starts and ends in state 0, checked by lower_char).  The 8
// bytes a lane needs come in as lo/hi (raw_bytes); the property-table gathers
// for this character and the next one are issued first, then pf() (the
// caller's prefetch of its next window, so that those loads overlap this
// window's gathers and work), then the gathers are used.  4-byte and cut
// characters run the machines.  bad: the character breaks the local
// formulation; need/conts count the continuation bytes the lead bytes claim /
// that are present.  Nothing is stored: classify() and the span builder both
// call this, so the per-wave slot holds no per-byte state.
// Property-table indices of the character at p (i1; 0 when it needs the
// machines or is not a lead byte) and of the next character (i2; -1 when its
// bytes are not a well-formed 1-3 byte sequence).
__device__ __forceinline__ void cp_index(const DocView& dv, int p, uint32_t lo, uint32_t hi, int& i1, int& i2) {
  const int L = dv.len;
  const uint32_t b0 = lo & 0xFF, b1 = (lo >> 8) & 0xFF, b2 = (lo >> 16) & 0xFF;
  const int n = utf8_len((uint8_t)b0);
  const int avail = p + n > L ? L - p : n;
  const bool fast = p < L && (b0 & 0xC0) != 0x80 && avail == n && n <= 3;
  i1 = fast ? cpt_index(b0, b1, b2, n) : 0;
  // the next character's bytes are bytes n..n+3 of lo:hi
  const uint64_t w = ((uint64_t)hi << 32) | lo;
  const uint32_t nx = (uint32_t)(w >> (8 * (n < 4 ? n : 4)));
  const uint32_t c2 = nx & 0xFF, d1 = (nx >> 8) & 0xFF, d2 = (nx >> 16) & 0xFF;
  const int n2 = utf8_len((uint8_t)c2);
  i2 = -1;
  if (c2 < 0x80) i2 = (int)c2;
  else if (n2 == 2 && (c2 & 0xE0) == 0xC0 && (d1 & 0xC0) == 0x80) i2 = cpt_index(c2, d1, 0, 2);
  else if (n2 == 3 && (d1 & 0xC0) == 0x80 && (d2 & 0xC0) == 0x80) i2 = cpt_index(c2, d1, d2, 3);
}
// The gathers themselves: e = entry i1, e2 = the low word (script) of entry i2.
template <bool SN2>
__device__ __forceinline__ void cp_gather(const DevTables& T, int i1, int i2, uint64_t& e, uint32_t& e2) {
  e = gld(T.cpt + (i1));
  e2 = SN2 ? gld(reinterpret_cast<const uint32_t*>(T.cpt) + 2 * (i2 >= 0 ? i2 : 0)) : 0u;
}
// The class word of byte p from its bytes and gathered entries (cls_* above).
template <bool SN2>
__device__ __forceinline__ uint32_t cp_decode(const DevTables& T, const DocView& dv, int p, uint32_t lo, uint32_t hi,
                                              uint64_t e, uint32_t e2, int i2, uint32_t& lw, int& bad, int& need,
                                              int& conts) {
  const int L = dv.len;
  lw = 0;
  if (p >= L) return 0u;
  const uint32_t c = lo & 0xFF;
  if ((c & 0xC0) == 0x80) {
    ++conts;
    return 0u;
  }
  const int n = utf8_len((uint8_t)c);
  const int avail = p + n > L ? L - p : n;   // a final character cut by the document end
  const bool fast = avail == n && n <= 3;
  bool wf = true;
#pragma unroll
  for (int k = 1; k < 4; ++k)
    if (k < avail) wf &= ((lo >> (8 * k)) & 0xC0) == 0x80;
  bad |= !wf;
  need += avail - 1;
  int sn, st, olen = 0;
  bool lowok;
  if (fast) {
    sn = (int)(e & 0xFF);
    st = (int)((e >> 8) & 3);
    if (st == 3) st = -1;
    lowok = (e >> 10) & 1;
    olen = (int)((e >> 11) & 15);
    lw = (uint32_t)(e >> 32);
  } else {                                   // 4-byte or cut: run the machines (out of line)
    const uint64_t es = char_slow(T.script, T.scan, T.lower, dv, p, n, avail);
    sn = (int)(es & 0xFF);
    st = (int)(int8_t)((es >> 8) & 0xFF);
    lowok = (es >> 16) & 1;
    olen = (int)((es >> 20) & 15);
    lw = (uint32_t)(es >> 32);
  }
  int sn2 = 0;
  if constexpr (SN2) sn2 = i2 >= 0 ? (int)(e2 & 0xFF) : script_num(T, dv, p + n);
  if (st < 0) bad = 1;
  const bool ls = st > 0 && sn != 0;
  (void)hi;
  return (uint32_t)sn | ((uint32_t)sn2 << 8) | ((uint32_t)n << 16) | (1u << 19) | ((uint32_t)ls << 20) |
         ((uint32_t)(avail < n) << 21) | ((uint32_t)!lowok << 22) | ((uint32_t)olen << 24);
}
// All three in one: gathers, then pf() (the caller's read-ahead), then decode.
template <bool SN2, class Pf>
__device__ __forceinline__ uint32_t char_props_b(const DevTables& T, const DocView& dv, int p, uint32_t lo, uint32_t hi,
                                                 uint32_t& lw, int& bad, int& need, int& conts, Pf&& pf) {
  int i1, i2;
  cp_index(dv, p, lo, hi, i1, i2);
  uint64_t e;
  uint32_t e2;
  cp_gather<SN2>(T, i1, i2, e, e2);
  pf();
  return cp_decode<SN2>(T, dv, p, lo, hi, e, e2, i2, lw, bad, need, conts);
}
struct NoPf {
  __device__ __forceinline__ void operator()() const {}
};
template <bool SN2 = true>
__device__ __forceinline__ uint32_t char_props(const DevTables& T, const DocView& dv, int p, uint32_t& lw, int& bad,
                                               int& need, int& conts) {
  uint32_t d0, d1, d2, lo, hi;
  raw_load(dv, p, d0, d1, d2);
  raw_bytes(dv, p, d0, d1, d2, lo, hi);
  return char_props_b<SN2>(T, dv, p, lo, hi, lw, bad, need, conts, NoPf{});
}

// Validity of the per-character formulation over the whole document, and the
// letter-stop bitmap (one bit per byte) the span builder searches for span
// starts.  False if the document does not tile into characters with local
// scanner behaviour (then the sequential span source redoes it).
__device__ __forceinline__ bool classify(const DevTables& T, const DocView& dv, Slot& S, bool& cut, int lane,
                                         uint64_t* lsm_ext = nullptr) {
  uint64_t* const lsm = lsm_ext ? lsm_ext : S.lsm;   // (documents over kDocCap: a bitmap in the staged store)
  lane = wave::lane_here();
  const int L = dv.len;
  int bad = 0, conts = 0, need = 0;
  cut = false;
  const int nw = (L + 63) >> 6;
  // software pipeline as in next_span: window w+1's gathers and window w+2's
  // raw bytes are in flight while window w is decoded
  uint32_t r0, r1, r2, lo, hi, e2;
  uint64_t e;
  int i1, i2;
  raw_load(dv, lane, r0, r1, r2);
  raw_bytes(dv, lane, r0, r1, r2, lo, hi);
  cp_index(dv, lane, lo, hi, i1, i2);
  cp_gather<false>(T, i1, i2, e, e2);
  raw_load(dv, lane + 64, r0, r1, r2);
  for (int w = 0; w < nw; ++w) {
    const int p = (w << 6) + lane;
    uint32_t lw, lo1, hi1, e2n;
    uint64_t en;
    int j1, j2;
    raw_bytes(dv, p + 64, r0, r1, r2, lo1, hi1);
    cp_index(dv, p + 64, lo1, hi1, j1, j2);
    cp_gather<false>(T, j1, j2, en, e2n);
    if (w + 2 < nw) raw_load(dv, p + 128, r0, r1, r2);
    const uint32_t cw = cp_decode<false>(T, dv, p, lo, hi, e, e2, i2, lw, bad, need, conts);
    lo = lo1;
    hi = hi1;
    e = en;
    i2 = j2;
    const uint64_t m = __ballot((cw >> 20) & 1);
    if (lane == 0) lsm[w] = m;
    cut |= __ballot(cls_cut(cw)) != 0;
  }
  bad |= (wsum(conts) != wsum(need)) ? 1 : 0;
  gsync();
  return __ballot(bad != 0) == 0;
}

// The sequential lowercaser for the rare cut-character tail, kept out of
// line so its state does not count against the kernel's registers.
// The machine goes by value: a reference into the kernel's DevTables
// argument would make every wave copy the whole struct to scratch at entry.
__device__ __noinline__ int lower_tail(DevSM sm, const uint8_t* in, int ilen, uint8_t* out, int olen) {
  return lower_replace_sm(sm, in, ilen, out, olen);
}

// --------------------------------------- stage 1: span text, lowered
// GetOneScriptSpan (getonescriptspan.cc:799-1027, plain text) followed by
// LowerScriptSpan (:1033-1054), straight into lb.  Span text = ' ' + run +
// ' ' + run + ' ' ... + "   \0".  A run starts at a letter stop of the span
// script (or Inherited) and ends at the first break character; the gap after
// it runs to the next letter stop, which continues the span (span script /
// Inherited) or ends it.  Within a 64-byte window every byte's state is the
// type of the last event at or before it (break -> gap, continuing letter
// stop -> run), so all lanes decide at once.  The soft limit (put >=
// put_soft_limit after a run's space) and the hard limit (put >=
// kMaxScriptBytes after a character) come from a prefix sum of the raw byte
// count; the lowered bytes were precomputed per character by classify().
// A final character cut by the document end that lands in a run is copied
// with NUL bytes (DocView), and the lowercaser stops at its lead byte: that
// tail is lowered sequentially by lane 0, so text_bytes can even be < 1 there.
// status: 1 span (returns its lowered text_bytes), 0 no span left, -1 re-queue.
// First letter stop at or after y (the end of a gap the reference's
// non-letter loop deletes), L if none; per lane.
__device__ __forceinline__ int next_stop(const uint64_t* lsm, int y, int L) {
  if (y >= L) return L;
  int w = y >> 6;
  uint64_t m = lsm[w] & (~0ull << (y & 63));
  while (!m) {
    if ((++w << 6) >= L) return L;
    m = lsm[w];
  }
  const int r = (w << 6) + __builtin_ctzll(m);
  return r < L ? r : L;
}

// The span builder's software pipeline, carried from one span of a document
// to the next (the staged span kernel's loop, st_spans): the window the span
// ended in (raw bytes and property gathers), the next window's (gathers
// issued) and the raw words of the one after.  Short spans (C3's pages hold
// 200-760 in 16 KB) start in the window the previous one stopped in, so the
// next call decodes it at once instead of paying a raw load and a dependent
// property gather -- two L2 round trips -- per span.  w < 0: nothing carried.
struct SpanCursor {
  int w = -1;
  uint32_t lo, hi;                               // window w
  uint64_t e;
  int i2;
  uint32_t nlo, nhi;                             // window w + 1
  uint64_t ne;
  int ni2;
  uint32_t r0, r1, r2;                           // raw words of window w + 2
  int mw = -1;                                   // letter-stop bitmap word mw (positions >= the last stop)
  uint64_t mv;
};

// find_first_g with the cursor's bitmap word: the next span's start is
// usually in the word the previous span stopped in (no slot read then).
__device__ __forceinline__ int find_first_c(const uint64_t* m, int from, int L, const SpanCursor* cur) {
  if (!cur) return find_first_g(m, from, L);
  from = ufl(from);
  if (from >= L) return L;
  int w = from >> 6;
  uint64_t x = (cur->mw == w ? cur->mv : ufl64(m[w])) & (~0ull << (from & 63));
  for (;;) {
    if (x) {
      const int r = (w << 6) + __builtin_ctzll(x);
      return r < L ? r : L;
    }
    ++w;
    if ((w << 6) >= L) return L;
    x = ufl64(m[w]);
  }
}

// vec mode: omap receives map2original_'s MapBack per span text byte; hpos
// (a rewritten HTML page, cld_html.hip) maps each byte of dv to its offset in
// the page as given -- offsets in omap are always page offsets.
constexpr int kResumeRange = 1 << 30;           // next_span's *rlo: a range's low end, not an exact offset
// HB: a rewritten HTML page of kMaxScriptBytes and more (dv.hp set): the
// soft limit from page offsets and the resume bookkeeping below.  Its own
// instantiation, so plain documents' span loop carries none of its state.
template <bool VEC = false, bool HB = false>
LNG_NS_INL int next_span(const DevTables& T, const DocView& dv, Slot& S, uint8_t* lb, int& next, int& ulscript,
                         int& status, int lane, uint32_t* omap = nullptr, const uint32_t* hpos = nullptr,
                         const uint32_t* hgap = nullptr, const uint64_t* lsm_ext = nullptr, int* rlo = nullptr,
                         SpanCursor* cur = nullptr) {
  const uint64_t* const lsm = lsm_ext ? lsm_ext : S.lsm;
  lane = wave::lane_here();
  const int L = dv.len;
  const int common = (int)T.common, inherited = (int)T.inherited;
  // the soft limit (getonescriptspan.cc:814-819) from the raw bytes left: on
  // a rewritten page the page offset of the resume point.  Where the
  // reference's scan stops at a dropped '&' (a stale script: the scan's
  // script is not reset by an undecodable entity, :874-883, 974-987) it
  // resumes up to a run of dropped '&'s earlier than the letter the span
  // builder resumes at; the previous span left in *rlo either that offset
  // (a letter stop of another script) or, with kResumeRange, the earliest one
  // (after the hard limit); -1: none; no rlo: any resume point right after
  // dropped '&'s counts as a range.
  // A document whose soft limit differs across that range, or whose range
  // straddles a regime, is handed on (the sequential span source scans the page itself).
  auto soft_of = [](int r) {
    return (kMaxScriptBytes <= r && r < 2 * kMaxScriptBytes) ? r / 2 : kMaxScriptBytes - kWithinScriptTail;
  };
  auto regime = [](int r) { return r < kMaxScriptBytes ? 0 : r < 2 * kMaxScriptBytes ? 1 : 2; };
  int remaining = L - next;
  const int rl = (HB && rlo) ? *rlo : -2;
  if (HB && rlo) *rlo = -1;
  if (HB && dv.hp && next > 0 && next < L) {
    remaining = L - (int)gld(dv.hp + next);
    if (rl >= 0 && !(rl & kResumeRange)) remaining = L - rl;   // the exact resume offset
    const int lo = rl >= 0 ? ((rl & kResumeRange) ? rl & ~kResumeRange : -1)
                           : (rl == -2 && (gld(dv.hf + next) & 2)) ? (int)gld(dv.hg + next) : -1;
    if (lo >= 0) {
      const int r0 = L - lo;
      if (soft_of(r0) != soft_of(remaining) || regime(r0) != regime(remaining)) {
        status = -1;
        return 0;
      }
    }
  }
  const int soft = soft_of(remaining);
  const int q = find_first_c(lsm, next, L, cur);
  status = 1;
  if (q >= L) {
    next = L;
    status = 0;
    return 0;
  }
  int ss = 0;                                    // the span script: read off q's lane in the first window
  if (lane == 0) lb[0] = ' ';
  // vec mode: where a scan that reaches the document end stops.  A final
  // character cut by the end is consumed whole (UTF8OneCharLen) by the
  // reference's loops, so its claimed bytes run past L.
  int dend = L;
  if constexpr (VEC) {
    int xc = L - 1;
    while (xc > 0 && xc > L - 4 && (dv.p[xc] & 0xC0) == 0x80) --xc;
    if (xc >= 0 && L > 0) {
      const int nc = utf8_len(dv.p[xc]);
      if (xc + nc > L) dend = xc + nc;
    }
  }
  // position r of dv -> page offset (past the end: where the scan stops)
  auto orig = [&](int r) -> int { return r >= L ? dend : (hpos ? (int)gld(hpos + r) : r); };
  if constexpr (VEC) {
    // map2original_ at the leading space (getonescriptspan.cc:835-848):
    // Delete(offset) Delete(skip) Insert(1) maps it past the skipped bytes, to
    // the first letter q; skip == 1 is a Copy(1) of the skipped byte; and
    // Delete(1) Insert(1) (offset 1, skip 0) merges into Copy(1) of byte 0
    const int n0 = next == 0 ? 0 : orig(next), q0 = orig(q);
    if (lane == 0) omap[0] = (uint32_t)((q0 - n0 == 1) ? n0 : (q0 == 1 && n0 == 1 ? 0 : q0));
  }
  int put = 1, lpos = 1, grow = 0, bad = 0, nxt = L, cutx = -1;
  bool run = false;
  // software pipeline: while window w is processed, window w+1's property
  // gathers and window w+2's raw bytes are in flight
  uint32_t r0 = 0, r1 = 0, r2 = 0, lo = 0, hi = 0, e2 = 0;
  uint64_t e = 0;
  int i2 = -1;
  // the carried pipeline (cur): window q >> 6 decoded from it at once, or its
  // next window as the usual pipeline state; else a fresh start
  const int w0 = q >> 6;
  bool next_ready = false;
  uint32_t nlo = 0, nhi = 0;
  uint64_t ne = 0;
  int ni2 = -1;
  if (cur && cur->w == w0) {
    lo = cur->lo; hi = cur->hi; e = cur->e; i2 = cur->i2;
    nlo = cur->nlo; nhi = cur->nhi; ne = cur->ne; ni2 = cur->ni2;
    r0 = cur->r0; r1 = cur->r1; r2 = cur->r2;
    next_ready = true;
  } else if (cur && cur->w >= 0 && cur->w + 1 == w0) {
    lo = cur->nlo; hi = cur->nhi; e = cur->ne; i2 = cur->ni2;
    r0 = cur->r0; r1 = cur->r1; r2 = cur->r2;
  } else {
    const int x0 = (w0 << 6) + lane;
    raw_load(dv, x0, r0, r1, r2);
    raw_bytes(dv, x0, r0, r1, r2, lo, hi);
    int i1;
    cp_index(dv, x0, lo, hi, i1, i2);
    cp_gather<false>(T, i1, i2, e, e2);
    raw_load(dv, x0 + 64, r0, r1, r2);          // (guarded: nothing past the document is read)
  }
  uint32_t slo = 0, shi = 0;                     // (cur) the decoded window's own state
  uint64_t se = 0;
  int si2 = -1;
  for (int w = w0;; ++w) {
    const int x = (w << 6) + lane;
    uint32_t lw = 0, cw = 0;
    int cur_i2 = -1;                             // property index of the next character (cp_index)
    {
      uint32_t lo1, hi1, e2n = 0;
      uint64_t en;
      int j2;
      if (next_ready) {                          // (carried: window w + 1 gathered, w + 2 loaded)
        lo1 = nlo; hi1 = nhi; en = ne; j2 = ni2;
        next_ready = false;
      } else {
        int j1;
        raw_bytes(dv, x + 64, r0, r1, r2, lo1, hi1);
        cp_index(dv, x + 64, lo1, hi1, j1, j2);
        cp_gather<false>(T, j1, j2, en, e2n);
        raw_load(dv, x + 128, r0, r1, r2);
      }
      int ignore2 = 0;
      cw = cp_decode<false>(T, dv, x, lo, hi, e, e2, i2, lw, ignore2, ignore2, ignore2);
      cur_i2 = i2;
      if (cur) { slo = lo; shi = hi; se = e; si2 = i2; }
      lo = lo1;
      hi = hi1;
      e = en;
      e2 = e2n;
      i2 = j2;
      if (x < q) {
        cw = 0;
        lw = 0;
      }
      if (w == (q >> 6)) ss = rdl(cls_sn(cw), q & 63);
    }
    const bool lead = cls_lead(cw);
    const int n = cls_n(cw);
    bool brk = false, ok = false, foreign = false;
    if (lead) {
      const int sc = cls_sn(cw);
      if (sc != ss && sc != inherited) {
        if (sc == common) {
          brk = true;
        } else {
          // the next character's script, only for a letter of another script
          // (rare inside a span): gathered here rather than for every byte
          int sc2 = cur_i2 >= 0 ? (int)(gld(reinterpret_cast<const uint32_t*>(T.cpt) + 2 * cur_i2) & 0xFF)
                                : script_num(T, dv, x + n);
          if (dv.hf && x + n < L && gld(dv.hf + x + n)) sc2 = 0;   // onto a rewritten HTML entity: the raw '&'
          brk = sc2 != common && sc2 != ss;
        }
      }
      if ((cw >> 20) & 1) {
        if (sc == ss || sc == inherited) ok = true;
        else foreign = true;
      }
    }
    const uint64_t Bm = __ballot(brk), Om = __ballot(ok);
    const uint64_t evm = Bm | Om;
    const uint64_t ev_le = evm & mask_le(lane), ev_lt = evm & lanemask_lt(lane);
    const bool inrun = ev_le ? ((Om >> topbit(ev_le)) & 1) : run;
    const bool prev_run = ev_lt ? ((Om >> topbit(ev_lt)) & 1) : run;
    const bool endc = foreign && (brk || !prev_run);     // a letter stop of another script after a gap
    const bool sep = brk && prev_run;                    // a run ends here: its ' '
    const bool cutc = cls_cut(cw);                       // only the last character
    const bool chr = lead && inrun;
    const int raw = chr ? n : (sep ? 1 : 0);
    const int pre = excl_scan(raw, lane);
    const uint64_t Em = __ballot(endc);
    const uint64_t Hm = __ballot(chr && !cutc && put + pre + n >= kMaxScriptBytes);
    const uint64_t Sm = __ballot(sep && put + pre + 1 >= soft);
    const uint64_t stopm = Em | Hm | Sm;
    const int stop = stopm ? __builtin_ctzll(stopm) : 64;
    const bool act = lane <= stop;
    const bool hard_here = lane == stop && ((Hm >> lane) & 1);
    const bool out_chr = act && chr && !cutc;
    if (out_chr && cls_nolow(cw)) bad = 1;
    const int olen = out_chr ? cls_olen(cw) : 0;
    grow += olen > n ? olen - n : 0;
    const int tl = olen + ((act && (sep || hard_here)) ? 1 : 0);
    const int opre = excl_scan(tl, lane);
    if constexpr (VEC) {
      if (out_chr && olen != n) bad = 1;         // map2uplow_ not the identity: the sequential span source maps it
      if (out_chr)
        for (int k = 0; k < olen; ++k) omap[lpos + opre + k] = (uint32_t)orig(x + k);   // Copy
      if (act && (sep || hard_here)) {
        // the run's ' ': Delete(gap) then Insert(1) maps it to the letter after
        // the gap; a gap of one byte makes that a Copy(1) of the gap byte, no
        // gap an Insert at the run end (:955-993)
        const int fr = sep ? x : x + n;
        const int nl = orig(next_stop(lsm, fr, L));
        int from = orig(fr);
        // dropped '&'s just before the break (hflag bit 1 on the byte after
        // them) are deleted in the letter loop, and that Delete merges with
        // the gap's: the gap starts where they began (hgap)
        if (dv.hf && fr < L && (gld(dv.hf + fr) & 2)) {
          if (sep) from = (int)gld(hgap + fr);
          else bad = 1;                          // (after the hard limit: the sequential span source)
        }
        omap[lpos + opre + olen] = (uint32_t)(nl - from >= 2 ? nl : from);
      }
    }
    if (out_chr)
      for (int k = 0; k < olen; ++k) lb[lpos + opre + k] = (uint8_t)(lw >> (8 * k));
    if (act && (sep || hard_here)) lb[lpos + opre + olen] = ' ';
    if (act && chr && cutc) cutx = x;
    lpos += rdl(opre + tl, 63);
    // raw bytes of the lanes up to the stop (a prefix-sum read, not another
    // reduction), plus the hard limit's ' '
    put += rdl(pre + raw, stop < 64 ? stop : 63) + ((stop < 64 && ((Hm >> stop) & 1)) ? 1 : 0);
    // (lb / omap room for the next window; put itself never passes
    // kMaxScriptBytes + 1: the hard limit stops the span)
    if (lpos + 64 > kLB) {
      bad = 1;
      if (cur) cur->w = -1;
      break;
    }
    if (stop < 64) {
      if (cur) {                                 // the next span starts at or after this window
        cur->mw = w;                             // (its letter stops at and after the stop: bit 20 of cw)
        cur->mv = __ballot((cw >> 20) & 1);
        cur->w = w;
        cur->lo = slo; cur->hi = shi; cur->e = se; cur->i2 = si2;
        cur->nlo = lo; cur->nhi = hi; cur->ne = e; cur->ni2 = i2;
        cur->r0 = r0; cur->r1 = r1; cur->r2 = r2;
      }
      const int xs = (w << 6) + stop;
      if ((Hm >> stop) & 1) {
        const int xe = xs + rdl(n, stop);
        nxt = find_first_c(lsm, xe, L, cur);
        // after the hard limit the reference's gap scan keeps the last
        // letter's script: the first dropped '&' in the gap stops it
        if (HB && rlo && dv.hp) {
          const int e = nxt < L ? nxt : L - 1;
          for (int y = xe; y <= e; y += 64) {
            const uint64_t dm = __ballot(y + lane <= e && (gld(dv.hf + y + lane) & 2));
            if (dm) {
              *rlo = (int)gld(dv.hg + y + __builtin_ctzll(dm)) | kResumeRange;
              break;
            }
          }
        }
      } else if ((Sm >> stop) & 1) {
        nxt = find_first_c(lsm, xs, L, cur);                          // the gap scan starts at the break char
      } else {
        nxt = xs;                                                     // another script's letter stop
        // dropped '&'s right before it: after a letter of a third script (the
        // single-letter continuation) the reference's script is stale there,
        // and its scan stops at the last of them (:916-931: the next byte's
        // script decides); after a letter of the span's own script it
        // consumes them
        if (HB && rlo && dv.hp && (gld(dv.hf + xs) & 2)) {
          int pc = xs - 1;
          while (pc > 0 && (dv.p[pc] & 0xC0) == 0x80) --pc;
          const int scp = pc >= 0 ? script_num(T, dv, pc) : 0;
          if (scp != 0 && scp != common && scp != ss && scp != inherited) *rlo = (int)gld(dv.hp + xs) - 1;
        }
        // vec mode: dropped '&'s right before it may stop the reference's scan
        // at the first of them (a stale script after a foreign letter,
        // getonescriptspan.cc:876-931), one offset earlier: the sequential span source
        if (VEC && dv.hf && (gld(dv.hf + xs) & 2)) {
          // (only when the run's last character is a letter of another script
          // -- the single-letter continuation -- is the reference's script
          // stale there; after a letter of the span's own script it consumes them)
          int pc = xs - 1;
          while (pc > 0 && (dv.p[pc] & 0xC0) == 0x80) --pc;
          const int scp = pc >= 0 ? script_num(T, dv, pc) : 0;
          if (scp != 0 && scp != common && scp != ss && scp != inherited) bad = 1;
        }
      }
      break;
    }
    if (evm) run = (Om >> topbit(evm)) & 1;
    if ((w << 6) + 64 >= L) {                                         // end of document
      if (cur) cur->w = -1;
      if (run && wmax((uint32_t)(cutx + 1)) == 0) {                 // (a cut character brings its own)
        if (lane == 0) lb[lpos] = ' ';
        if (VEC && lane == 0) omap[lpos] = (uint32_t)dend;           // Insert(1) at the document end
        ++lpos;
        ++put;
      }
      nxt = L;
      break;
    }
  }
  next = nxt;
  ulscript = ss;
  cutx = (int)wmax((uint32_t)(cutx + 1)) - 1;
  if (cutx >= 0) {                               // the cut last character: lowercaser tail
    int filled = 0;
    if (lane == 0) {
      uint8_t tail[12];
      const int nc = utf8_len(dv.p[cutx]);
      for (int k = 0; k < nc; ++k) tail[k] = (uint8_t)dv.at(cutx + k);
      for (int k = 0; k < 4; ++k) tail[nc + k] = ' ';                 // separator + "   " (ilen stops before \0)
      filled = lower_tail(T.lower, tail, nc + 4, lb + lpos, kMaxScriptLowerBuffer - lpos);
      if constexpr (VEC) {
        // the cut character is copied whole (Copy(n): its missing bytes map
        // past the document end), then the ' ' and the pads map to where its
        // claimed bytes end; the lowercaser must leave these bytes as they are
        for (int k = 0; k < filled; ++k) {
          omap[lpos + k] = (uint32_t)(cutx + (k < nc ? k : nc));
          if (k < nc + 4 && lb[lpos + k] != tail[k]) bad = 1;
        }
      }
    }
    lpos += rdl(filled, 0);
    for (int k = lane; k < 40; k += 64) lb[lpos + k] = 0;
    lpos -= 3;                                                        // text_bytes = filled - 3
  } else {
    for (int k = lane; k < 40; k += 64) lb[lpos + k] = k < 3 ? ' ' : 0;   // "   " (lowered pads), NULs
    if (VEC && lane < 4) omap[lpos + lane] = (uint32_t)orig(nxt);     // Insert(4): where the scan stopped
  }
  // the reference's lowercaser would stop early (kExitDstSpaceFull) only for
  // spans near the 40 KB limit that also grow; re-queue those.
  if (put + 3 + wsum(grow) > kMaxScriptLowerBuffer - 8) bad = 1;
  gsync();
  if (__ballot(bad != 0)) status = -1;
  return lpos;
}

// The sequential walk of char_starts for a window holding a malformed
// character (or the tail of one), out of line: it is rare, and its loop would
// otherwise add to the span builders' registers.
__device__ __noinline__ uint64_t char_starts_walk(const uint8_t* text, int base, int len, const uint64_t* resets,
                                                  int& carry) {
  auto reset_after = [&](int p) -> int {          // first reset position > p, or a large value
    if (!resets) return 0x7FFFFFFF;
    for (int q = p + 1; q < base + 64 + 4; ++q)
      if ((ufl64(resets[q >> 6]) >> (q & 63)) & 1) return q;
    return 0x7FFFFFFF;
  };
  const int end = min(base + 64, len);
  int p = base + carry;
  if (carry > 0) {
    const int r = reset_after(base - 1);
    if (r < p) p = r;
  }
  uint64_t m = 0;
  while (p < end) {
    m |= 1ull << (p - base);
    const int q = p + utf8_len(ufl(text[p]));
    const int r = reset_after(p);
    p = r < q ? r : q;
  }
  carry = p > end ? p - end : 0;      // in the last window: the last character runs past len
  return m;
}

// Character starts of the sequential UTF-8 decode that CountPredictedBytes
// and CheapRepWordsInplace run (compact_lang_det_impl.cc:541-580, 610-692):
// a lead byte consumes the count its value claims, continuation bytes or not.
// For well-formed text that is "every byte that is not 10xxxxxx"; a malformed
// character (a document cut inside a character leaves one at a span end)
// swallows the bytes it claims.  Window [base, base + 64) of text[0, len);
// decoding restarts at every set bit of `resets` (null: only at 0); carry =
// bytes of this window the previous window's last character still claims.
__device__ __forceinline__ uint64_t char_starts(const uint8_t* text, int base, int len, const uint64_t* resets,
                                                int& carry, bool careful, int lane) {
  const int x = base + lane;
  if (!careful)                                  // no cut character in the document: well-formed span text
    return __ballot(x < len && (text[x] & 0xC0) != 0x80);
  const bool valid = x < len;
  const uint8_t b = valid ? text[x] : (uint8_t)0;
  const bool nc = valid && (b & 0xC0) != 0x80;
  const int n = utf8_len(b);
  bool mal = false;
  if (nc) {
    for (int k = 1; k < n; ++k) mal |= (text[x + k] & 0xC0) != 0x80;
  } else if (valid && x >= base + carry) {
    // a continuation byte that no lead byte before it claims is a character
    // of its own in the sequential decode (0x80-0xBF advance one byte): the
    // walk takes the window (the carried bytes are checked below)
    const uint32_t p1 = x >= 1 ? text[x - 1] : 0u, p2 = x >= 2 ? text[x - 2] : 0u, p3 = x >= 3 ? text[x - 3] : 0u;
    const bool k1 = (p1 & 0xC0) == 0x80, k2 = (p2 & 0xC0) == 0x80;
    mal = !(p1 >= 0xC0 || (k1 && p2 >= 0xE0) || (k1 && k2 && p3 >= 0xF0));
  }
  const uint64_t ncm = __ballot(nc);
  const int end = min(base + 64, len);
  // well-formed window whose carried bytes (the tail of a character begun in
  // the previous window) are continuation bytes: starts = non-continuation bytes
  const bool carry_ok = carry == 0 || (carry < 64 && (ncm & ((1ull << carry) - 1)) == 0);
  if (!__ballot(mal) && carry_ok) {
    if (ncm) {                                    // the last character may claim bytes of the next window
      const int last = base + topbit(ncm);
      const int q = last + utf8_len(ufl(text[last]));
      carry = q > end ? q - end : 0;
    } else {                                      // no start here: the carried character ends in this window
      carry = base + carry > end ? base + carry - end : 0;   // (or runs past the text's end)
    }
    return ncm;
  }
  // rare: walk the window (uniform scalar loop, out of line)
  return char_starts_walk(text, base, len, resets, carry);
}

// ------------------------------------------------------ predictor (squeeze/repeats)
// The predictor's character code: a lead byte and the bytes its value claims,
// continuation bytes or not, big-endian; *incr = their count
// (compact_lang_det_impl.cc:641-667, the same decode in CountPredictedBytes).
__device__ __forceinline__ int next_char_code(const uint8_t* src, int* incr) {
  const uint32_t c = src[0];
  const int n = c < 0xC0 ? 1 : (c & 0xE0) == 0xC0 ? 2 : (c & 0xF0) == 0xE0 ? 3 : 4;
  *incr = n;
  uint32_t v = c;
  for (int k = 1; k < n; ++k) v = (v << 8) | src[k];
  return (int)v;
}
// A fresh predictor table: a new epoch makes every older entry read as 0.
__device__ uint32_t new_epoch(uint32_t& epoch, uint64_t* tbl, int lane) {
  uint32_t e = uflu(epoch) + 1u;
  if (e == 0) {                                     // wrapped: clear for real
    for (int i = lane; i < kPredictionTableSize; i += 64) tbl[i] = 0;
    e = 1;
  }
  gsync();
  if (lane == 0) epoch = e;
  return e;
}

// One window of CountPredictedBytes / CheapRepWordsInplace's predictor
// (compact_lang_det_impl.cc:541-580, 610-692) over the characters whose lead
// bytes are the lanes of lm, in lane order: p = tbl[h]; tbl[h] = c;
// predicted = (c == p); h = ((h << 4) ^ c) & 0xFFF.  h after a character
// depends only on it and the two before it, so every lane computes its own;
// lanes with equal table keys are matched with 12 ballots and the latest
// earlier one supplies p.  hcarry is the hash after the last character.
__device__ bool predict_window(uint64_t* tbl, uint32_t epoch, uint64_t lm, uint32_t c, uint32_t& hcarry, int lane) {
  if (!lm) return false;
  const bool me = (lm >> lane) & 1;
  const uint64_t below = lm & lanemask_lt(lane);
  const int p1 = below ? topbit(below) : -1;
  const uint64_t below2 = p1 > 0 ? (below & lanemask_lt(p1)) : 0ull;
  const int p2 = below2 ? topbit(below2) : -1;
  const uint32_t c1 = shfl32(c, p1 < 0 ? lane : p1);
  const uint32_t c2 = shfl32(c, p2 < 0 ? lane : p2);
  uint32_t h;
  if (p1 < 0) h = (c ^ (hcarry << 4)) & 0xFFFu;
  else if (p2 < 0) h = (c ^ (c1 << 4) ^ (hcarry << 8)) & 0xFFFu;
  else h = (c ^ (c1 << 4) ^ (c2 << 8)) & 0xFFFu;
  const uint32_t hp = shfl32(h, p1 < 0 ? lane : p1);
  const uint32_t key = p1 < 0 ? hcarry : hp;
  uint64_t eq = lm;
#pragma unroll
  for (int b = 0; b < 12; ++b) {
    const bool bit = (key >> b) & 1;
    const uint64_t m = __ballot(bit);
    eq &= bit ? m : ~m;
  }
  const uint64_t earlier = eq & lanemask_lt(lane);
  uint32_t pc = shfl32(c, earlier ? topbit(earlier) : lane);
  if (me && !earlier) {
    const uint64_t e = tbl[key];
    pc = (uint32_t)(e >> 32) == epoch ? (uint32_t)e : 0u;
  }
  const bool last = (eq & ~mask_le(lane)) == 0;
  if (me && last) tbl[key] = ((uint64_t)epoch << 32) | c;
  hcarry = rdlu(h, topbit(lm));
  gsync();
  return me && c == pc;
}

// The Repeats predictor in LDS.  The reference's table holds the packed UTF-8
// bytes of a character (next_char_code; up to 32 bits); the LDS table holds a
// 16-bit code that is one-to-one on every value a table entry is compared
// against, except a sentinel class whose full value goes to the slot's
// overflow table (S.pred, low 32 bits):
//   1 byte (c < 0xC0)                        c                  0x0000-0x00BF
//   2 bytes, continuation second byte        0xD800 | 11 bits   0xD800-0xDFFF
//   3 bytes, well formed, not overlong,      the 16-bit scalar  0x0800-0xFFFF
//     not a surrogate                                           minus 0xD800-0xDFFF
//   anything else (4 bytes, malformed)       kPredSent          0x07FF
// The ranges are disjoint, so equal codes <=> equal values outside the
// sentinel class.  The empty table (all 0) reads as the reference's 0.
constexpr uint32_t kPredSent = 0x07FF;
__device__ __forceinline__ uint32_t pred_code(uint32_t b0, uint32_t b1, uint32_t b2, int incr) {
  if (incr == 1) return b0;
  const bool c1 = (b1 & 0xC0) == 0x80, c2 = (b2 & 0xC0) == 0x80;
  if (incr == 2) return c1 ? 0xD800u | ((b0 & 0x1F) << 6) | (b1 & 0x3F) : kPredSent;
  if (incr == 3 && c1 && c2) {
    const uint32_t v = ((b0 & 0xF) << 12) | ((b1 & 0x3F) << 6) | (b2 & 0x3F);
    if (v >= 0x800 && (v < 0xD800 || v > 0xDFFF)) return v;
  }
  return kPredSent;
}

// predict_window on the LDS table: the first lane of a key in the window
// reads the code (and, for the sentinel, the overflow value); the last lane of
// a key writes it.
__device__ __forceinline__ bool predict_window_lds(uint16_t* tbl, uint64_t* ovf, uint64_t lm, uint32_t c,
                                                   uint32_t code, uint32_t& hcarry, int lane) {
  const bool me = (lm >> lane) & 1;
  const uint64_t below = lm & lanemask_lt(lane);
  const int p1 = below ? topbit(below) : -1;
  const uint64_t below2 = p1 > 0 ? (below & lanemask_lt(p1)) : 0ull;
  const int p2 = below2 ? topbit(below2) : -1;
  const uint32_t c1 = shfl32(c, p1 < 0 ? lane : p1);
  const uint32_t c2 = shfl32(c, p2 < 0 ? lane : p2);
  uint32_t h;
  if (p1 < 0) h = (c ^ (hcarry << 4)) & 0xFFFu;
  else if (p2 < 0) h = (c ^ (c1 << 4) ^ (hcarry << 8)) & 0xFFFu;
  else h = (c ^ (c1 << 4) ^ (c2 << 8)) & 0xFFFu;
  const uint32_t hp = shfl32(h, p1 < 0 ? lane : p1);
  const uint32_t key = p1 < 0 ? hcarry : hp;
  uint64_t eq = lm;
#pragma unroll
  for (int b = 0; b < 12; ++b) {
    const bool bit = (key >> b) & 1;
    const uint64_t m = __ballot(bit);
    eq &= bit ? m : ~m;
  }
  const uint64_t earlier = eq & lanemask_lt(lane);
  const uint32_t pc = shfl32(c, earlier ? topbit(earlier) : lane);
  bool pr = me && earlier && c == pc;
  if (me && !earlier) {
    const uint32_t pcode = tbl[key];
    pr = pcode == kPredSent ? (uint32_t)ovf[key] == c : pcode == code;
  }
  const bool last = (eq & ~mask_le(lane)) == 0;
  const bool wr = me && last;
  if (wr) tbl[key] = (uint16_t)code;
  hcarry = rdlu(h, topbit(lm));
  if (__ballot(wr && code == kPredSent)) {
    if (wr && code == kPredSent) ovf[key] = c;
    gsync();
  }
  return pr;
}

// CheapRepWordsInplace (compact_lang_det_impl.cc:610-692) on one span of the
// span cache, in place, in one pass: like the reference, every byte goes to
// dst as it is read, and a space whose segment was mostly predicted rewinds
// dst to the start of its word.  Per 64-byte window the pieces that end at a
// space of the window are decided; a deleted piece is not written (the
// reference writes it and then rewinds over it: only bytes past the final
// length differ, and nothing reads those), a kept piece and the open piece at
// the window end are written at their dst positions (<= their source
// positions, so in place is safe).  The next window's bytes are loaded while
// the current one is processed.  hcarry carries from span to span.
__device__ __forceinline__ int rep_span_lds(uint16_t* tbl, uint64_t* ovf, uint8_t* text, int len, uint32_t& hcarry, bool careful,
                            bool& ok, int lane) {
  lane = wave::lane_here();
  const int nw = (len + 63) >> 6;
  int D = 0, WD = 0;                     // dst, word_dst (as offsets)
  int cwl = 0, cgd = 0;                  // open segment: bytes / predicted bytes so far
  int carry = 0;
  uint32_t n0 = text[lane], n1 = text[lane + 1], n2 = text[lane + 2];
  for (int w = 0; w < nw; ++w) {
    const int base = w << 6, x = base + lane;
    const uint32_t b0 = n0, b1 = n1, b2 = n2;
    if (w + 1 < nw) {
      n0 = text[x + 64];
      n1 = text[x + 65];
      n2 = text[x + 66];
    }
    const bool valid = x < len;
    // (well-formed text: the starts come from the bytes already in registers)
    const uint64_t st = careful ? char_starts(text, base, len, nullptr, carry, careful, lane)
                                : __ballot(valid && (b0 & 0xC0) != 0x80);
    const bool lead = valid && ((st >> lane) & 1);
    int incr = 1;
    uint32_t c = 0, code = 0;
    if (lead) {
      incr = b0 < 0xC0 ? 1 : (b0 & 0xE0) == 0xC0 ? 2 : (b0 & 0xF0) == 0xE0 ? 3 : 4;
      if (incr == 1) c = b0;
      else if (incr == 2) c = (b0 << 8) | b1;
      else if (incr == 3) c = (b0 << 16) | (b1 << 8) | b2;
      else c = (b0 << 24) | (b1 << 16) | (b2 << 8) | (uint32_t)text[x + 3];
      code = pred_code(b0, b1, b2, incr);
    }
    const uint64_t lm = __ballot(lead);
    const bool pr = lm ? predict_window_lds(tbl, ovf, lm, c, code, hcarry, lane) : false;
    const int wl = lead ? incr : 0, gd = (lead && pr) ? incr : 0;
    const bool sp = lead && b0 == ' ';
    const uint64_t spm = __ballot(sp);
    const int ewl = excl_scan(wl, lane), egd = excl_scan(gd, lane);
    const uint64_t psp = spm & lanemask_lt(lane);
    const int ps = psp ? topbit(psp) : lane;
    const int ewl_ps = __shfl(ewl, ps, 64), egd_ps = __shfl(egd, ps, 64);
    const int swl = psp ? ewl - ewl_ps : cwl + ewl;
    const int sgd = psp ? egd - egd_ps : cgd + egd;
    const uint64_t dm = __ballot(sp && sgd * 2 > swl);
    const int twl = rdl(ewl + wl, 63), tgd = rdl(egd + gd, 63);
    // pieces: a byte belongs to the first space at or after it in the window
    const uint64_t ge = spm & ~lanemask_lt(lane);
    const bool write = valid && (!ge || !((dm >> __builtin_ctzll(ge)) & 1));
    const uint64_t km = __ballot(write);
    const int bD = (spm && ((dm >> __builtin_ctzll(spm)) & 1)) ? WD : D;   // first piece deleted: rewind
    if (write) text[bD + __popcll(km & lanemask_lt(lane))] = (uint8_t)b0;
    if (spm) {
      const int ls = topbit(spm);
      WD = bD + __popcll(km & mask_le(ls));
      cwl = twl - rdl(ewl, ls);
      cgd = tgd - rdl(egd, ls);
    } else {
      cwl += twl;
      cgd += tgd;
    }
    D = bD + __popcll(km);
  }
  // a last character claiming bytes past the span (a span cut inside a
  // character, malformed text): the reference copies the bytes it claims,
  // the pad bytes after the span included (:640-662)
  if (carry > 0) {
    if (lane == 0)
      for (int k = 0; k < carry; ++k) text[D + k] = text[len + k];
    D += carry;
  }
  ok = true;
  // "   \0" if at least 4 bytes went, else a single ' ' if any went (:684-689)
  if (D < len - 3) {
    if (lane < 4) text[D + lane] = lane < 3 ? ' ' : 0;
  } else if (D < len) {
    if (lane == 0) text[D] = ' ';
  }
  gsync();
  return D;
}

// CheapSqueezeTriggerTest (compact_lang_det_impl.cc:952-971) on a lowered span
// of more than 2048 bytes: >= 25% spaces or >= 67% predicted bytes in the first
// 256 bytes (fresh table, hash 0).
__device__ __forceinline__ bool squeeze_trigger(Slot& S, const uint8_t* text, bool careful, int lane) {
  lane = wave::lane_here();
  int sp = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) sp += text[lane * 4 + k] == ' ';
  if (wsum(sp) >= (256 * 25) / 100) return true;
  const uint32_t ep = new_epoch(S.epoch2, S.pred2, lane);
  uint32_t h = 0;
  int pc = 0, carry = 0;
  for (int w = 0; w < 4; ++w) {
    const int x = (w << 6) + lane;
    const uint64_t st = char_starts(text, w << 6, 256, nullptr, carry, careful, lane);
    const bool lead = (st >> lane) & 1;
    int incr = 1;
    const uint32_t c = lead ? (uint32_t)next_char_code(text + x, &incr) : 0u;
    const uint64_t lm = __ballot(lead);
    const bool pr = predict_window(S.pred2, ep, lm, c, h, lane);
    pc += (lead && pr) ? incr : 0;
  }
  return wsum(pc) >= (256 * 67) / 100;
}

// CheapRepWordsInplace (compact_lang_det_impl.cc:610-692), src -> dst.  The
// predictor table and hash carry over from span to span within the pass.  A
// segment runs from a space (inclusive: its byte counts for the next word) to
// the next space; at that space the bytes after the previous space, this space
// included, are dropped if more than half of the segment was predicted.
// OW (vec mode): CheapRepWordsInplaceOverwrite (:697-770) -- the same
// segments and predictions, but a mostly-predicted segment's bytes before its
// closing space become '.' and the text keeps its length.
template <bool OW = false>
__device__ __forceinline__ int rep_words(Slot& S, const uint8_t* src, uint8_t* dst, int len, uint32_t& hcarry, uint32_t ep,
                         bool careful, bool& ok, int lane) {
  lane = wave::lane_here();
  const int nw = (len + 63) >> 6;
  int cwl = 0, cgd = 0;                  // open segment: bytes / predicted bytes so far
  int carry = 0;
  for (int w = 0; w < nw; ++w) {
    const int x = (w << 6) + lane;
    const bool valid = x < len;
    const uint8_t b = valid ? src[x] : (uint8_t)0;
    const uint64_t st = char_starts(src, w << 6, len, nullptr, carry, careful, lane);
    const bool lead = valid && ((st >> lane) & 1);
    int incr = 1;
    const uint32_t c = lead ? (uint32_t)next_char_code(src + x, &incr) : 0u;
    const uint64_t lm = __ballot(lead);
    const bool pr = predict_window(S.pred, ep, lm, c, hcarry, lane);
    const int wl = lead ? incr : 0, gd = (lead && pr) ? incr : 0;
    const bool sp = lead && b == ' ';
    const uint64_t spm = __ballot(sp);
    const int ewl = excl_scan(wl, lane), egd = excl_scan(gd, lane);
    const uint64_t psp = spm & lanemask_lt(lane);
    const int ps = psp ? topbit(psp) : lane;
    const int ewl_ps = __shfl(ewl, ps, 64), egd_ps = __shfl(egd, ps, 64);
    const int swl = psp ? ewl - ewl_ps : cwl + ewl;
    const int sgd = psp ? egd - egd_ps : cgd + egd;
    const uint64_t dm = __ballot(sp && sgd * 2 > swl);
    if (lane == 0) {
      S.spm[w] = spm;
      S.delm[w] = dm;
    }
    const int twl = rdl(ewl + wl, 63), tgd = rdl(egd + gd, 63);
    if (spm) {
      const int ls = topbit(spm);
      cwl = twl - rdl(ewl, ls);
      cgd = tgd - rdl(egd, ls);
    } else {
      cwl += twl;
      cgd += tgd;
    }
  }
  gsync();
  // a last character claiming bytes past the span (a span cut inside a
  // character, malformed text) copies the bytes it claims, pads included, and
  // the text grows by them (:640-662; the open piece is never deleted)
  ok = true;
  if constexpr (OW) {
    for (int w = 0; w < nw; ++w) {
      const int x = (w << 6) + lane;
      if (x < len) {
        int ww = w;
        uint64_t m = S.spm[w] & (~0ull << lane);
        while (!m && ((ww + 1) << 6) < len) m = S.spm[++ww];
        bool dot = false;
        if (m) {
          const int sp = __builtin_ctzll(m);
          dot = ((S.delm[ww] >> sp) & 1) && !(ww == w && sp == lane);   // the closing space stays
        }
        dst[x] = dot ? (uint8_t)'.' : src[x];
      }
    }
    if (dst != src)
      for (int k = lane; k < 48; k += 64) dst[len + k] = src[len + k];   // pads as they are (:758-767)
    gsync();
    // (a span whose lowercaser stopped early can have len < 1: the
    // reference's loop then copies nothing and the span has 0 bytes)
    return len > 0 ? len + carry : 0;
  }
  int dpos = 0;
  for (int w = 0; w < nw; ++w) {
    const int x = (w << 6) + lane;
    bool keep = false;
    if (x < len) {
      int ww = w;
      uint64_t m = S.spm[w] & (~0ull << lane);
      while (!m && ((ww + 1) << 6) < len) m = S.spm[++ww];
      keep = true;
      if (m) {
        const int s = __builtin_ctzll(m);
        keep = !((S.delm[ww] >> s) & 1);
      }
    }
    const uint64_t km = __ballot(keep);
    if (keep) dst[dpos + __popcll(km & lanemask_lt(lane))] = src[x];
    dpos += __popcll(km);
  }
  if (carry > 0) {                               // (positions >= dpos are not written yet: in place is safe)
    gsync();
    if (lane == 0)
      for (int k = 0; k < carry; ++k) dst[dpos + k] = src[len + k];
    dpos += carry;
    gsync();
  }
  // in place, the bytes from dpos on keep their old values; then "   \0" if
  // at least 4 bytes went, else a single ' ' if any went (:684-689)
  for (int k = lane; k < 48; k += 64) {
    uint8_t v = src[dpos + k];
    if (dpos < len - 3 && k < 4) v = k < 3 ? ' ' : 0;
    else if (dpos < len && k == 0) v = ' ';
    dst[dpos + k] = v;
  }
  gsync();
  return dpos;
}

// CheapSqueezeInplace (compact_lang_det_impl.cc:785-865) on a lowered span,
// in place.  Chunk boundaries (48 bytes, extended past continuation bytes)
// depend on the text alone and are found first.  The chunks' CountPredictedBytes
// calls share one fresh table and hash, so the predictor runs over the span's
// characters in order -- block-parallel, as for Repeats -- with the decode
// restarting at every chunk start; each chunk's predicted-byte and
// CountSpaces4 counts are popcounts over per-byte bitmasks.  The keep / skip
// assembly then walks the chunks: BackscanToSpace and ForwardscanToSpace
// (:491-522) are ballots over <= 32 bytes, and a kept chunk (<= 51 bytes)
// moves in one lane-parallel step, reads before writes, exactly as memmove.
__device__ __forceinline__ int range_pop(const uint64_t* m, int a, int b) {   // set bits in [a, b)
  int c = 0;
  while (a < b) {
    const int w = a >> 6, o = a & 63, e = min(b - (w << 6), 64);
    const uint64_t bits = ufl64(m[w]) >> o;
    const int n = e - o;
    c += __popcll(n >= 64 ? bits : bits & ((1ull << n) - 1));
    a += n;
  }
  return c;
}

// Out of line: Squeeze is rare, and inlined its state would count against the
// registers of every pass.
// OW (vec mode): CheapSqueezeInplaceOverwrite (:869-940) -- the chunks start
// after the leading space, and a squeezed stretch becomes '.'s (each skipped
// chunk closing with a ' ') instead of being cut, so the text keeps its
// length and the offset map stays valid.
template <bool OW = false>
__device__ __noinline__ int squeeze_span(Slot& S, uint8_t* text, int len, bool careful, int lane) {
  constexpr int kChunk = 48;
  constexpr int s0 = OW ? 1 : 0;                 // (OW: the first byte, a space, is always kept)
  const int nw = (len + 63) >> 6;
  // chunk starts
  for (int i = lane; i < nw + 1; i += 64) S.chm[i] = 0;
  gsync();
  {
    int src = s0, cw = 0;
    uint64_t cur = 0;
    while (src < len) {
      if ((src >> 6) != cw) {
        if (lane == 0) S.chm[cw] = cur;
        cur = 0;
        cw = src >> 6;
      }
      cur |= 1ull << (src & 63);
      int clen = min(kChunk, len - src);
      while ((ufl(text[src + clen]) & 0xC0) == 0x80) ++clen;
      src += clen;
    }
    if (lane == 0) S.chm[cw] = cur;
  }
  gsync();
  // predictions, decode restarting at each chunk start
  const uint32_t ep = new_epoch(S.epoch2, S.pred2, lane);
  uint32_t h = 0;
  int carry = 0;
  for (int w = 0; w < nw; ++w) {
    const int x = (w << 6) + lane;
    const bool valid = x >= s0 && x < len;
    const uint8_t b = valid ? text[x] : (uint8_t)0;
    const uint64_t st = char_starts(text, w << 6, len, S.chm, carry, careful, lane);
    const bool lead = valid && ((st >> lane) & 1);
    int incr = 1;
    const uint32_t c = lead ? (uint32_t)next_char_code(text + x, &incr) : 0u;
    const uint64_t lm = __ballot(lead);
    const bool pr = predict_window(S.pred2, ep, lm, c, h, lane);
    const bool ps = lead && pr;                  // CountPredictedBytes adds incr for it
    const uint64_t m0 = __ballot(ps), m1 = __ballot(ps && ((incr - 1) & 1)), m2 = __ballot(ps && ((incr - 1) & 2));
    const uint64_t sm = __ballot(valid && b == ' ');
    if (lane == 0) {
      S.delm[w] = m0;
      S.aux[0][w] = m1;
      S.aux[1][w] = m2;
      S.spm[w] = sm;
    }
  }
  gsync();
  constexpr int kSpaceThresh = (kChunk * 25) / 100, kPredictThresh = (kChunk * 40) / 100;
  if constexpr (OW) {
    bool skipping = false;
    for (int src = 1; src < len;) {
      int clen = min(kChunk, len - src);
      while ((ufl(text[src + clen]) & 0xC0) == 0x80) ++clen;   // move past continuation bytes
      const int space_n = range_pop(S.spm, src, src + (clen & ~3));
      const int predb_n = range_pop(S.delm, src, src + clen) + range_pop(S.aux[0], src, src + clen) +
                          2 * range_pop(S.aux[1], src, src + clen);
      if (space_n >= kSpaceThresh || predb_n >= kPredictThresh) {
        if (!skipping) {                         // keeping -> skipping: the word before becomes '.'s
          const int lim = min(src, 32);
          const uint64_t spc = __ballot(lane < lim && text[src - lane - 1] == ' ');
          int n = 0;
          if (spc) {
            n = __builtin_ctzll(spc);
          } else {
            const uint64_t cb = __ballot(lane < lim && (text[src - lane] & 0xC0) != 0x80);
            n = cb ? __builtin_ctzll(cb) : 0;
          }
          gsync();
          if (lane < n) text[src - n + lane] = '.';
          skipping = true;
        }
        gsync();
        if (lane < clen) text[src + lane] = lane == clen - 1 ? ' ' : '.';   // (clen <= 51)
      } else if (skipping) {                     // skipping -> keeping: up to the next word start
        const int lim = min(clen, 32);
        const uint64_t spc = __ballot(lane < lim && text[src + lane] == ' ');
        int n = 0;
        if (spc) {
          n = __builtin_ctzll(spc) + 1;
        } else {
          const uint64_t cb = __ballot(lane < lim && (text[src + lane] & 0xC0) != 0x80);
          n = cb ? __builtin_ctzll(cb) : 0;
        }
        gsync();
        if (lane < n - 1) text[src + lane] = '.';
        skipping = false;
      }
      gsync();
      src += clen;
    }
    return len;                                  // (no pads: the text keeps its length)
  }
  int src = 0, dst = 0;
  bool skipping = false;
  while (src < len) {
    int clen = min(kChunk, len - src);
    while ((ufl(text[src + clen]) & 0xC0) == 0x80) ++clen;    // move past continuation bytes
    const int space_n = range_pop(S.spm, src, src + (clen & ~3));
    const int predb_n = range_pop(S.delm, src, src + clen) + range_pop(S.aux[0], src, src + clen) +
                        2 * range_pop(S.aux[1], src, src + clen);
    if (space_n >= kSpaceThresh || predb_n >= kPredictThresh) {
      if (!skipping) {                           // keeping -> skipping: back to a word start
        const int lim = min(dst, 32);
        const uint64_t spc = __ballot(lane < lim && text[dst - lane - 1] == ' ');
        int n = 0;
        if (spc) {
          n = __builtin_ctzll(spc);
        } else {
          const uint64_t cb = __ballot(lane < lim && (text[dst - lane] & 0xC0) != 0x80);
          n = cb ? __builtin_ctzll(cb) : 0;
        }
        dst -= n;
        if (dst == 0) {                          // force a leading space if the first chunk goes
          if (lane == 0) text[0] = ' ';
          dst = 1;
        }
        skipping = true;
      }
    } else {
      int s2 = src, l2 = clen;
      if (skipping) {                            // skipping -> keeping: forward to a word start
        const int lim = min(clen, 32);
        const uint64_t spc = __ballot(lane < lim && text[src + lane] == ' ');
        int n = 0;
        if (spc) {
          n = __builtin_ctzll(spc) + 1;
        } else {
          const uint64_t cb = __ballot(lane < lim && (text[src + lane] & 0xC0) != 0x80);
          n = cb ? __builtin_ctzll(cb) : 0;
        }
        s2 += n;
        l2 -= n;
        skipping = false;
      }
      if (l2 > 0) {                              // memmove(dst, src, l2), l2 <= 51
        const uint8_t v = lane < l2 ? text[s2 + lane] : (uint8_t)0;
        gsync();
        if (lane < l2) text[dst + lane] = v;
        dst += l2;
      }
    }
    gsync();
    src += clen;
  }
  // pad: "   \0", or one ' ' when fewer than 4 bytes went (:852-862)
  if (lane < 4 && dst < len - 3) text[dst + lane] = lane < 3 ? ' ' : 0;
  else if (lane == 0 && dst < len) text[dst] = ' ';
  gsync();
  return dst;
}

// Emissions keep 32-bit indices, not the 8-byte adds: the seven tables' adds
// sit back to back in one per-GPU array that starts at compat's
// (cld_build_adds), so entry i of table t is adds_index(T, t, i) there, and an
// emission stream costs 4 bytes of slot per entry instead of 8 (the streams
// were ~45% of k_long's HBM writes at C3, profiles/round4f_emission_index.txt).
__device__ __forceinline__ uint32_t adds_index(const DevTables& T, const DevTbl& t, uint32_t i) {
  return (uint32_t)(t.adds - T.compat.adds) + i;
}
__device__ __forceinline__ uint64_t adds_by_index(const DevTables& T, uint32_t g) { return gld(T.compat.adds + g); }
// A chunk's add before its gather (chunk_ref / resolve_ref): bit 62 marks an
// index into the adds array; anything else is the add itself (the seed, a
// prior or a ring boost: tote adds use bits 0-47 and 63, never 62).
constexpr uint64_t kRefIndex = 1ull << 62;
__device__ __forceinline__ uint64_t resolve_ref(const DevTables& T, uint64_t r) {
  return (r & kRefIndex) ? adds_by_index(T, (uint32_t)r) : r;
}

// Base emissions of one base hit (LinearizeAll, scoreonescriptspan.cc:856-960):
// one or two langprobs as tote adds, zero langprobs dropped.  ind bit 31
// selects the second quad table.
// The emission test is the langprob itself (ind_at, 4 bytes): a zero
// langprob is exactly a zero add (k_build_adds); the adds are gathered only
// when the chunk is scored (chunk_ref / resolve_ref).
__device__ __forceinline__ void base_adds(const DevTables& T, const DevTbl& t1, const DevTbl& t2, uint32_t ind,
                                          uint32_t& l1, uint32_t& l2, uint32_t& g1, uint32_t& g2) {
  const DevTbl* lb = &t1;
  if (ind & 0x80000000u) {
    lb = &t2;
    ind &= ~0x80000000u;
  }
  l2 = 0;
  g2 = 0;
  if (ind < lb->size_one) {
    l1 = ind_at(*lb, ind);
    g1 = adds_index(T, *lb, ind);
  } else {
    ind += ind - lb->size_one;
    l1 = ind_at(*lb, ind);
    l2 = ind_at(*lb, ind + 1);
    g1 = adds_index(T, *lb, ind);
    g2 = g1 + 1;
    if (!l1) {
      l1 = l2;
      l2 = 0;
      g1 = g2;
    }
  }
}

// ---------------------------------------------------- quad chain of a span
// GetQuadHits' chain (cldutil.cc:349-401): from src, e = 4 chars on (stopping
// at a space), mid = 2 chars on; next = e + 1 if text[e] is the word's space,
// else mid (+1 on a vowel).  It never jumps over a space, so it enters every
// word at its first byte and a word's entries depend on that word alone.
template <class SM, class WN>
__device__ __forceinline__ bool word_lists(WN& win, SM& s, int tb, int start, Slot& S, int& nws, int& nsp, int lane) {
  lane = wave::lane_here();
  nws = 0;
  nsp = 0;
  bool ok = true;
  int carry = 0;
  bool prev_sp = false;                          // (WN::kSeq) a word-ending space at w0 - 1
  for (int w0 = start; w0 <= tb; w0 += 64) {
    const uint8_t* text = win_text(win, s, w0 - 1, w0 + 65, ok, lane);
    if (!ok) return false;
    const int x = w0 + lane;
    bool isws, issp;
    if constexpr (WN::kSeq) {
      const uint64_t cs = char_starts(text, w0, tb + 1, nullptr, carry, true, lane);
      issp = x <= tb && ((cs >> lane) & 1) && text[x] == ' ';
      const uint64_t spm = __ballot(issp);
      isws = x < tb && (x == start || (lane == 0 ? prev_sp : ((spm >> (lane - 1)) & 1) != 0));
      prev_sp = (spm >> 63) != 0;
    } else {
      isws = x < tb && (x == start || text[x - 1] == ' ');
      issp = x <= tb && text[x] == ' ';
    }
    const uint64_t m1 = __ballot(isws), m2 = __ballot(issp);
    if (isws) {
      const int k = nws + __popcll(m1 & lanemask_lt(lane));
      if (k < kListCap) S.wst[k] = (uint16_t)x;
    }
    if (issp) {
      const int k = nsp + __popcll(m2 & lanemask_lt(lane));
      if (k < kListCap) S.wsp[k] = (uint16_t)x;
    }
    nws += __popcll(m1);
    nsp += __popcll(m2);
  }
  gsync();
  return nws <= kListCap && nsp <= kListCap;
}

// The first four entries are also returned packed (r01: entries 0-1, r23:
// entries 2-3, 16 bits each), so build_chain writes most words without a
// second walk.
__device__ __forceinline__ int walk_word(const uint8_t* text, int s, int tb, uint16_t* out, uint32_t& r01, uint32_t& r23) {
  int cnt = 0, src = s;
  r01 = 0;
  r23 = 0;
  for (;;) {
    if (out) out[cnt] = (uint16_t)src;
    if (cnt < 4) {
      const uint32_t v = (uint32_t)src << (16 * (cnt & 1));
      if (cnt < 2) r01 |= v;
      else r23 |= v;
    }
    ++cnt;
    int e = src;
    e += adv_but_space(text[e]);
    e += adv_but_space(text[e]);
    const int mid = e;
    e += adv_but_space(text[e]);
    e += adv_but_space(text[e]);
    if (text[e] == ' ') break;                    // next = e + 1: the next word start, or the end
    if (mid >= tb) break;                         // next = limit
    src = mid + adv_space_vowel(text[mid]);
    if (src >= tb) break;
  }
  return cnt;
}

template <class SM, class WN>
__device__ __forceinline__ int build_chain(WN& win, SM& sm, int tb, Slot& S, int nws, int lane) {
  lane = wave::lane_here();
  int nch = 0;
  int sn = (LNG_PF & 1) && lane < nws ? S.wst[lane] : 0;       // word starts one block ahead
  for (int i0 = 0; i0 < nws; i0 += 64) {
    // the block's words: from its first start to the next block's first (a walk stops at its word's space)
    bool ok = true;
    const uint8_t* text = win_text(win, sm, ufl(S.wst[i0]), (i0 + 64 < nws ? ufl(S.wst[i0 + 64]) : tb) + 24, ok, lane);
    if (!ok) return -1;
    const int i = i0 + lane;
    int cnt = 0;
    const int s = (LNG_PF & 1) ? sn : (i < nws ? S.wst[i] : 0);
    if (LNG_PF & 1) sn = i + 64 < nws ? S.wst[i + 64] : 0;
    uint32_t r01 = 0, r23 = 0;
    if (i < nws) cnt = walk_word(text, s, tb, nullptr, r01, r23);
    const int pre = excl_scan(cnt, lane);
    const int tot = rdl(pre + cnt, 63);
    if (nch + tot > kListCap) return -1;
    uint16_t* o = S.chain + nch + pre;
    if (cnt > 4) {
      walk_word(text, s, tb, o, r01, r23);         // long word: walk again
    } else {
      if (cnt > 0) o[0] = (uint16_t)r01;
      if (cnt > 1) o[1] = (uint16_t)(r01 >> 16);
      if (cnt > 2) o[2] = (uint16_t)r23;
      if (cnt > 3) o[3] = (uint16_t)(r23 >> 16);
    }
    nch += tot;
  }
  gsync();
  return nch;
}

// GetQuadHits for one round from chain entry c0 (cldutil.cc:315-405): probes
// per entry, the "not one of the last two hits" filter, the 1000-hit cut.
// Each kept hit's base emissions go straight to be_off / be_ai (eb of
// them), so score_round does not read the hits back; the hit list itself is
// kept only for the debug dump (D).  Returns the round end (the reference's
// `next`); c0 advances.
template <bool D, class SM, class WN>
__device__ __forceinline__ int quad_round(const DevTables& T, WN& win, SM& sm, int tb, Slot& S, int nch, int& c0, int& nb,
                          int& eb, bool& ok, int lane) {
  lane = wave::lane_here();
  nb = 0;
  eb = 0;
  uint32_t A = 0, B = 0;                 // last two kept hashes (pq0 / pq1 as a set)
  int pn = (LNG_PF & 2) && c0 + lane < nch ? S.chain[c0 + lane] : 0;   // chain entries one block ahead
  for (int i0 = c0; i0 < nch; i0 += 64) {
    // the block's chain entries: each reads its quad (<= 4 chars) and one byte either side
    const uint8_t* text = win_text(win, sm, ufl(S.chain[i0]) - 1, ufl(S.chain[min(i0 + 63, nch - 1)]) + 24, ok, lane);
    if (!ok) return tb;
    const int i = i0 + lane;
    bool hit = false;
    uint32_t hv = 0, ind = 0;
    int p = 0;
    const int pc = (LNG_PF & 2) ? pn : (i < nch ? S.chain[i] : 0);
    if (LNG_PF & 2) pn = i + 64 < nch ? S.chain[i + 64] : 0;
    if (i < nch) {
      p = pc;
      int e = p;
      e += adv_but_space(text[e]);
      e += adv_but_space(text[e]);
      e += adv_but_space(text[e]);
      e += adv_but_space(text[e]);
      hv = quad_hash_v2(text + p, e - p);
      const uint32_t probs = quad_probe(T.quad, T.quad2, hv, ind);
      hit = probs != 0;
    }
    const uint64_t hm = __ballot(hit);
    // every hit kept so far => its two predecessors are the previous hit lanes
    const uint64_t hb = hm & lanemask_lt(lane);
    const int q1 = hb ? topbit(hb) : -1;
    const uint64_t hb2 = q1 > 0 ? (hb & lanemask_lt(q1)) : 0ull;
    const int q2 = hb2 ? topbit(hb2) : -1;
    const uint32_t h1 = shfl32(hv, q1 < 0 ? lane : q1), h2 = shfl32(hv, q2 < 0 ? lane : q2);
    const uint32_t a = q1 < 0 ? A : h1;
    const uint32_t bb = q1 < 0 ? B : (q2 < 0 ? A : h2);
    const uint64_t cm = __ballot(hit && (hv == a || hv == bb));
    uint64_t keep = hm;
    uint32_t nA, nB;
    if (cm) {
      const int f = __builtin_ctzll(cm);
      keep = hm & lanemask_lt(f);
      uint32_t xA = rdlu(a, f), xB = rdlu(bb, f);
      for (uint64_t r = hm & ~lanemask_lt(f); r; r &= r - 1) {
        const int l = __builtin_ctzll(r);
        const uint32_t v = rdlu(hv, l);
        if (v == xA || v == xB) continue;
        xB = xA;
        xA = v;
        keep |= 1ull << l;
      }
      nA = xA;
      nB = xB;
    } else if (hm) {
      const int t1 = topbit(hm);
      nA = rdlu(hv, t1);
      const uint64_t r2 = hm & ~(1ull << t1);
      nB = r2 ? rdlu(hv, topbit(r2)) : A;
    } else {
      nA = A;
      nB = B;
    }
    const int kc = __popcll(keep);
    int lastl = 64;
    if (nb + kc >= kMaxScoringHits) {
      lastl = nth_bit(keep, kMaxScoringHits - nb - 1);
      keep &= mask_le(lastl);
    }
    const bool kept = (keep >> lane) & 1;
    if (D && kept) {
      const int k = nb + __popcll(keep & lanemask_lt(lane));
      S.b_off[k] = (uint16_t)p;
      S.b_ind[k] = ind;
    }
    nb += __popcll(keep);
    {
      uint32_t l1 = 0, l2 = 0, g1 = 0, g2 = 0;
      if (kept) base_adds(T, T.quad, T.quad2, ind, l1, l2, g1, g2);
      const int c = (l1 != 0) + (l2 != 0);
      const int o = eb + excl_scan(c, lane);
      eb = rdl(o + c, 63);
      if (l1) {
        S.be_off[o] = (uint16_t)p;
        S.be_ai[o] = g1;
      }
      if (l2) {
        S.be_off[o + 1] = (uint16_t)p;
        S.be_ai[o + 1] = g2;
      }
    }
    if (lastl < 64) {
      c0 = i0 + lastl + 1;
      gsync();
      return c0 < nch ? ufl(S.chain[c0]) : tb;
    }
    A = nA;
    B = nB;
  }
  c0 = nch;
  gsync();
  return tb;
}

// GetOctaHits (cldutil.cc:416-533) over [off, next]: one lane per word (words
// end at the spaces in [start, next]); the two-word repeat filter updates the
// pair partner even when the probes miss; caps: 1000 delta / 999 distinct
// hits.  As in quad_round, the hits become emissions here (ed delta / ex
// distinct with non-zero langprobs, in hit order); the hit lists are kept
// only for the debug dump (D).
template <bool D, class SM, class WN>
__device__ __forceinline__ void octa_round(const DevTables& T, WN& win, SM& sm, Slot& S, int nsp, int& j0, int off, int next,
                           int& nd, int& nx, int& edm, int& exm, bool& ok, int lane) {
  lane = wave::lane_here();
  edm = 0;
  exm = 0;
  const int start = off + (ufl(win_text(win, sm, off, off + 1, ok, lane)[off]) == ' ' ? 1 : 0);
  if (!ok) return;
  const int lim = next + 1;
  nd = 0;
  nx = 0;
  uint64_t A = 0, B = 0;                 // last two kept word hashes
  // word-ending spaces one block ahead; a word's start and the one before
  // come from the previous lanes (lanes 0/1: the previous block's last two)
  int en = (LNG_PF & 4) && j0 + lane < nsp ? S.wsp[j0 + lane] : 0x7FFFFFFF;
  int c1 = start - 1, c2 = start - 1;    // wsp[jb - 1], wsp[jb - 2] as "start - 1" before jfirst
  for (int jb = j0;; jb += 64) {
    // the block's words end at spaces below lim: text from the space before the first on
    const uint8_t* text =
        jb < nsp ? win_text(win, sm, c1, min((int)ufl(S.wsp[min(jb + 63, nsp - 1)]), lim) + 8, ok, lane) : sm.text;
    if (!ok) return;
    const int j = jb + lane;
    const int ej = (LNG_PF & 4) ? en : (j < nsp ? S.wsp[j] : 0x7FFFFFFF);
    if (LNG_PF & 4) en = j + 64 < nsp ? S.wsp[j + 64] : 0x7FFFFFFF;
    const bool v = j < nsp && ej < lim;
    const uint64_t vm = __ballot(v);
    if (!vm) break;
    const int nv = __popcll(vm);
    const int e1 = (int)wave::wshr1((uint32_t)ej, (uint32_t)c1);          // wsp[j - 1]
    const int e2 = (int)wave::wshr1((uint32_t)e1, (uint32_t)c2);          // wsp[j - 2]
    c1 = rdl(ej, 63);
    c2 = rdl(ej, 62);
    int a = start, pws = start, e = 0;
    uint64_t wh = 0;
    if (v) {
      e = ej;
      a = e1 + 1;
      pws = e2 + 1;
      int we = a, q = a, cc = 0;
      while (q < e) {
        ++cc;
        q += utf8_len(text[q]);
        if (cc <= 8) we = q;
        else break;
      }
      wh = octa_hash40(text + a, we - a);
    }
    // filter (every word takes part): fast path assumes no drop in this block
    const uint64_t h1 = wave::wshr1_64(wh), h2 = wave::wshr1_64(h1);   // lanes - 1, - 2 (used from lanes 1, 2 on)
    const uint64_t pa = lane >= 1 ? h1 : A;
    const uint64_t pb = lane >= 2 ? h2 : (lane == 1 ? A : B);
    const uint64_t cm = __ballot(v && (wh == pa || wh == pb));
    uint64_t keep = vm;
    uint32_t tlo = (uint32_t)pa, thi = (uint32_t)(pa >> 32);    // pair partner = previous kept word
    uint64_t nA, nB;
    if (cm) {
      const int f = __builtin_ctzll(cm);
      keep = vm & lanemask_lt(f);
      uint64_t xA = rdl64(pa, f), xB = rdl64(pb, f);
      for (int l = f; l < nv; ++l) {
        const uint64_t hv = rdl64(wh, l);
        if (hv == xA || hv == xB) continue;
        if (lane == l) {
          tlo = (uint32_t)xA;
          thi = (uint32_t)(xA >> 32);
        }
        xB = xA;
        xA = hv;
        keep |= 1ull << l;
      }
      nA = xA;
      nB = xB;
    } else {
      nA = rdl64(wh, nv - 1);
      nB = nv >= 2 ? rdl64(wh, nv - 2) : A;
    }
    uint32_t pp = 0, xp = 0, dp = 0;
    if ((keep >> lane) & 1) {
      const uint64_t tph = ((uint64_t)thi << 32) | tlo;
      if (tph != 0 && tph != wh) pp = octa_lookup(T.distinctocta, pair_hash(tph, wh));
      xp = octa_lookup(T.distinctocta, wh);
      dp = octa_lookup(T.deltaocta, wh);
    }
    // tote adds of the hits (issued before the cap arithmetic they do not depend on)
    const uint32_t xm = ~T.distinctocta.key_mask, dmk = ~T.deltaocta.key_mask;
    const uint32_t apx = pp ? ind_at(T.distinctocta, pp & xm) : 0u;
    const uint32_t axp = xp ? ind_at(T.distinctocta, xp & xm) : 0u;
    const uint32_t adp = dp ? ind_at(T.deltaocta, dp & dmk) : 0u;
    const int cx = (pp != 0) + (xp != 0), cd = (dp != 0);
    const int ex = excl_scan(cx, lane), ed = excl_scan(cd, lane);
    const uint64_t capm = __ballot(v && (nx + ex + cx >= kMaxScoringHits - 1 || nd + ed + cd >= kMaxScoringHits));
    const int cut = capm ? __builtin_ctzll(capm) : 64;
    {
      const bool in = lane <= cut;
      const int mx = in ? (apx != 0) + (axp != 0) : 0, md = in ? (adp != 0) : 0;
      int ox = exm + excl_scan(mx, lane);
      const int od = edm + excl_scan(md, lane);
      exm = rdl(ox + mx, 63);
      edm = rdl(od + md, 63);
      if (in && apx) {
        S.x_off[ox] = (uint16_t)pws;
        S.x_ai[ox] = adds_index(T, T.distinctocta, pp & xm);
        ++ox;
      }
      if (in && axp) {
        S.x_off[ox] = (uint16_t)a;
        S.x_ai[ox] = adds_index(T, T.distinctocta, xp & xm);
      }
      if (in && adp) {
        S.d_off[od] = (uint16_t)a;
        S.d_ai[od] = adds_index(T, T.deltaocta, dp & dmk);
      }
    }
    if (D && lane <= cut) {
      int o = nx + ex;
      if (pp) {
        S.x_hoff[o] = (uint16_t)pws;
        S.x_ind[o] = pp & xm;
        ++o;
      }
      if (xp) {
        S.x_hoff[o] = (uint16_t)a;
        S.x_ind[o] = xp & xm;
      }
      if (dp) {
        S.d_hoff[nd + ed] = (uint16_t)a;
        S.d_ind[nd + ed] = dp & dmk;
      }
    }
    const int lastl = cut < 64 ? cut : 63;
    nx += rdl(ex + cx, lastl);
    nd += rdl(ed + cd, lastl);
    if (cut < 64 || nv < 64) break;
    A = nA;
    B = nB;
  }
  // next round's words start after `next` (a chain position, never a space)
  int lo = j0, hi = nsp;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if ((int)ufl(S.wsp[mid]) < lim) lo = mid + 1;
    else hi = mid;
  }
  j0 = lo;
  gsync();
}

// GetUniHits + GetBiHits (cldutil.cc:201-310) for one round from off.
// As in quad_round / octa_round, the hits become emissions here (eb base,
// edm delta, exm distinct); the hit lists are kept only for the debug dump.
template <bool D, class SM, class WN>
__device__ __forceinline__ int cjk_round(const DevTables& T, WN& win, SM& sm, int tb, Slot& S, int off, int& nb, int& nd,
                         int& nx, int& eb, int& edm, int& exm, bool& ok, int lane) {
  lane = wave::lane_here();
  const int start = off + (ufl(win_text(win, sm, off, off + 1, ok, lane)[off]) == ' ' ? 1 : 0);
  if (!ok) return tb;
  nb = 0;
  eb = 0;
  edm = 0;
  exm = 0;
  int next = -1;
  uint32_t endmax = (uint32_t)start;
  int carry = 0;
  for (int w0 = start; w0 < tb; w0 += 64) {
    const uint8_t* text = win_text(win, sm, w0, w0 + 64 + 8, ok, lane);
    if (!ok) return tb;
    const int x = w0 + lane;
    int prop = 0, len = 0;
    bool cst;
    if constexpr (WN::kSeq) cst = (char_starts(text, w0, tb, nullptr, carry, true, lane) >> lane) & 1;
    else cst = (text[x] & 0xC0) != 0x80;
    if (x < tb && cst) {
      len = utf8_len(text[x]);
      prop = uni_prop(T, text + x, len);
      endmax = (uint32_t)(x + len) > endmax ? (uint32_t)(x + len) : endmax;
    }
    uint64_t hm = __ballot(prop > 0);
    int lastl = 64;
    if (nb + __popcll(hm) >= kMaxScoringHits) {
      lastl = nth_bit(hm, kMaxScoringHits - nb - 1);
      hm &= mask_le(lastl);
    }
    const bool kept = (hm >> lane) & 1;
    if (D && kept) {
      const int k = nb + __popcll(hm & lanemask_lt(lane));
      S.b_off[k] = (uint16_t)(x + len);
      S.b_ind[k] = (uint32_t)prop;
    }
    nb += __popcll(hm);
    {
      uint32_t l1 = 0, l2 = 0, g1 = 0, g2 = 0;
      if (kept) base_adds(T, T.compat, T.compat, (uint32_t)prop, l1, l2, g1, g2);
      const int c = (l1 != 0) + (l2 != 0);
      const int o = eb + excl_scan(c, lane);
      eb = rdl(o + c, 63);
      if (l1) {
        S.be_off[o] = (uint16_t)(x + len);
        S.be_ai[o] = g1;
      }
      if (l2) {
        S.be_off[o + 1] = (uint16_t)(x + len);
        S.be_ai[o + 1] = g2;
      }
    }
    if (lastl < 64) {
      next = rdl(x + len, lastl);
      break;
    }
  }
  if (next < 0) next = (int)wave::wmax(endmax);
  nd = 0;
  nx = 0;
  carry = 0;
  for (int w0 = off; w0 < next; w0 += 64) {
    const uint8_t* text = win_text(win, sm, w0, w0 + 64 + 12, ok, lane);
    if (!ok) return tb;
    const int x = w0 + lane;
    uint32_t dp = 0, xp = 0;
    bool cst;
    if constexpr (WN::kSeq) cst = (char_starts(text, w0, next, nullptr, carry, true, lane) >> lane) & 1;
    else cst = (text[x] & 0xC0) != 0x80;
    const bool v = x < next && cst;
    if (v) {
      const int len = utf8_len(text[x]);
      const int len2 = utf8_len(text[x + len]) + len;
      if (6 <= len2) {
        const uint32_t bh = bi_hash_v2(text + x, len2);
        dp = quad_lookup(T.deltabi, bh);
        xp = quad_lookup(T.distinctbi, bh);
      }
    }
    const uint32_t adp = dp ? ind_at(T.deltabi, dp & ~T.deltabi.key_mask) : 0u;
    const uint32_t axp = xp ? ind_at(T.distinctbi, xp & ~T.distinctbi.key_mask) : 0u;
    const int cd = dp != 0, cx = xp != 0;
    const int ed = excl_scan(cd, lane), ex = excl_scan(cx, lane);
    const uint64_t capm = __ballot(v && (nd + ed + cd >= kMaxScoringHits || nx + ex + cx >= kMaxScoringHits - 1));
    const int cut = capm ? __builtin_ctzll(capm) : 64;
    {
      const bool in = lane <= cut;
      const int md = in ? (adp != 0) : 0, mx = in ? (axp != 0) : 0;
      const int od = edm + excl_scan(md, lane), ox = exm + excl_scan(mx, lane);
      edm = rdl(od + md, 63);
      exm = rdl(ox + mx, 63);
      if (md) {
        S.d_off[od] = (uint16_t)x;
        S.d_ai[od] = adds_index(T, T.deltabi, dp & ~T.deltabi.key_mask);
      }
      if (mx) {
        S.x_off[ox] = (uint16_t)x;
        S.x_ai[ox] = adds_index(T, T.distinctbi, xp & ~T.distinctbi.key_mask);
      }
    }
    if (D && lane <= cut) {
      if (dp) {
        S.d_hoff[nd + ed] = (uint16_t)x;
        S.d_ind[nd + ed] = dp & ~T.deltabi.key_mask;
      }
      if (xp) {
        S.x_hoff[nx + ex] = (uint16_t)x;
        S.x_ind[nx + ex] = xp & ~T.distinctbi.key_mask;
      }
    }
    const int lastl = cut < 64 ? cut : 63;
    nd += rdl(ed + cd, lastl);
    nx += rdl(ex + cx, lastl);
    if (cut < 64) break;
  }
  gsync();
  return next;
}

// ProcessProbV2Tote (cldutil.cc:128-138) precomputed per emission: the three
// (key, score) tote adds of a langprob, packed k1 | s1 << 8 | k2 << 16 |
// s2 << 24 | k3 << 32 | s3 << 40 (bytes 5..7 of its kLgProbV2Tbl row).
__device__ __forceinline__ uint64_t tote_adds(const DevTables& T, uint32_t lp) {
  const uint32_t e = gld(reinterpret_cast<const uint32_t*>(T.lgprob + 8 * (lp & 0xFF) + 4));
  return (uint64_t)((lp >> 8) & 0xFF) | ((uint64_t)((e >> 8) & 0xFF) << 8) | ((uint64_t)((lp >> 16) & 0xFF) << 16) |
         ((uint64_t)((e >> 16) & 0xFF) << 24) | ((uint64_t)(lp >> 24) << 32) | ((uint64_t)(e >> 24) << 40);
}


// Per (script, key): language | close set << 16 | expected score << 32
// (FromPerScriptNumber, close sets, kAvgDeltaOctaScore: lang_script.cc:328-341,
// 261-310; scoreonescriptspan.cc:75-80), one table per GPU built by
// k_build_keytab, L2-resident and shared by every wave (it used to be a
// per-wave LDS copy; the LDS now goes to occupancy).
__device__ uint64_t keytab_eval(const DevTables& T, int ulscript, int k) {
  const int lang = from_per_script_number(T, ulscript, (uint8_t)k);
  const int esub = lang * 4 + lscript4(T, ulscript);
  const int16_t ex = (esub >= 0 && (uint32_t)esub < T.n_expected) ? gld(T.expected + (esub)) : (int16_t)0;
  return (uint64_t)(uint16_t)lang | ((uint64_t)close_set(T, lang) << 16) | ((uint64_t)(uint16_t)ex << 32);
}

// Chunk k's adds (score_round): t < seedn the seed, then its base, delta and
// distinct emissions, then the four boosts (the last four distinct langprobs
// so far) -- as refs (kRefIndex): the emissions' gathers are issued later
// (resolve_ref), once their indices are in.  Plain functions rather than
// lambdas: a captured reference loses its address space, and the slot / LDS
// reads would become FLAT.
template <class SM>
__device__ __forceinline__ uint64_t chunk_ref(const Slot& S, const SM& s, uint64_t seed, int rs, int t, int k, int tot,
                                              int bs, int nB, int ds, int nD, int xs, int nX, int xe) {
  if (t >= tot) return 0ull;
  int u = t;
  const int seedn = k == 0 ? 1 : 0;
  if (u < seedn) return seed;
  if ((u -= seedn) < nB) return kRefIndex | S.be_ai[bs + u];
  if ((u -= nB) < nD) return kRefIndex | S.d_ai[ds + u];
  if ((u -= nD) < nX) return kRefIndex | S.x_ai[xs + u];
  if (u - nX >= kMaxBoosts) return s.pri_add[rs][u - nX - kMaxBoosts];   // prior boosts (has_pri)
  const int v = xe - kMaxBoosts + (u - nX);
  return v < 0 ? s.ring[rs][v + kMaxBoosts] : (kRefIndex | gld(&S.x_ai[v]));   // (gld: no LDS/global pointer select)
}
// Chunk plan of k: emission ranges and the number of adds.
template <class SM>
__device__ __forceinline__ int chunk_plan(const SM& s, int K, int eb, int k, int& bs, int& nB, int& ds, int& nD,
                                          int& xs, int& nX, int& xe) {
  bs = s.bst[k];
  const int be = k == K - 1 ? eb : s.bst[k + 1];
  ds = s.st[0][k];
  xs = s.st[1][k];
  xe = s.st[1][k + 1];
  nB = be - bs;
  nD = s.st[0][k + 1] - ds;
  nX = xe - xs;
  return (k == 0 ? 1 : 0) + nB + nD + nX + kMaxBoosts + (s.has_pri ? kMaxBoosts : 0);
}

// ---------------------------------------------------- vec mode helpers
// GetLangScore (cldutil.cc:141-152) on a langprob's tote adds: the scores of
// the keys equal to pslang.
__device__ __forceinline__ int add_score(uint64_t a, uint32_t ps) {
  int r = 0;
  if ((uint32_t)(a & 0xFF) == ps) r += (int)((a >> 8) & 0xFF);
  if ((uint32_t)((a >> 16) & 0xFF) == ps) r += (int)((a >> 24) & 0xFF);
  if ((uint32_t)((a >> 32) & 0xFF) == ps) r += (int)((a >> 40) & 0xFF);
  return r;
}
// ScriptScanner::MapBack (getonescriptspan.cc:1076-1078) for y <= text_bytes:
// map2original_.MapBack(map2uplow_.MapBack(y)).  The inner MapBack of a
// negative y is 0 (offsetmap.cc:430; a span whose lowercaser stopped early on
// a malformed character has text_bytes < 1), and the outer one maps that to
// the span's page offset, omap[0] -- not to 0.
__device__ __forceinline__ int vec_map_back(const VecState& V, int y) { return (int)gld(V.vs->omap + (y < 0 ? 0 : y)); }
__device__ __forceinline__ void vec_store(VecState& V, int lane) {
  if (lane == 0 && !V.over && V.n > 0) {
    cld_chunk c;
    c.offset = V.last_off;
    c.bytes = V.last_bytes;
    c.lang1 = (uint16_t)V.last_lang;
    c.pad = 0;
    V.v[V.n - 1] = c;
  }
}
// ItemToVector (scoreonescriptspan.cc:323-360): extend the last item when the
// language repeats (over any gap), else append
__device__ __forceinline__ void vec_item(VecState& V, int lang, int off, int len, int lane) {
  if (V.n > 0 && lang == V.last_lang) {
    V.last_bytes = off + len - V.last_off;
  } else {
    if (V.n >= V.cap) {
      V.over = true;
      return;
    }
    ++V.n;
    V.last_off = off;
    V.last_bytes = len;
    V.last_lang = lang;
  }
  vec_store(V, lane);
}
__device__ __forceinline__ uint64_t wmax64(uint64_t v) {
#pragma unroll
  for (int o = 32; o; o >>= 1) {
    const uint64_t t = shfl64(v, wave::lane_here() ^ o);
    v = t > v ? t : v;
  }
  return v;
}
// Entries of a sorted u16 stream <= o (le) or < o.
__device__ __forceinline__ int count_upto(const uint16_t* a, int n, int o, bool le) {
  int lo = 0, hi = n;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    const int v = a[mid];
    if (le ? v <= o : v < o) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}
// BetterBoundary (scoreonescriptspan.cc:671-720) across lanes: the window
// sum at left end i is R(i) = d[i..i+3] - d[i+4..i+7]; the scan keeps the first
// i with the largest R(i) > 0 among windows holding both a positive and a
// negative d, and moves the boundary to i + 4.
__device__ int better_boundary_w(VecSlot* vs, uint32_t ps0, uint32_t ps1, int lin0, int lin1, int lin2, int lane) {
  if (lin2 - lin0 <= 8) return lin1;
  for (int j = lin0 + lane; j < lin2; j += 64) {
    const uint64_t a = vs->lin_add[j];
    vs->vd[j] = add_score(a, ps0) - add_score(a, ps1);
  }
  gsync();
  uint64_t best = 0;
  for (int i = lin0 + lane; i < lin2 - 8; i += 64) {
    int r = 0;
    bool plus = false, minus = false;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int dv = vs->vd[i + k];
      r += k < 4 ? dv : -dv;
      plus |= dv > 0;
      minus |= dv < 0;
    }
    if (plus && minus && r > 0) {
      const uint64_t key = ((uint64_t)(uint32_t)r << 32) | (uint32_t)(0xFFFFFFFFu - (uint32_t)i);
      best = key > best ? key : best;
    }
  }
  best = wmax64(best);
  gsync();
  return best ? (int)(0xFFFFFFFFu - (uint32_t)best) + 4 : lin1;
}

// ------------------------------------- linearize + chunk + score (one round)
// LinearizeAll / ChunkAll / ScoreAllHits (scoreonescriptspan.cc:856-1031,
// 208-302) without materialising linear[].  Linear order = the seed (offset
// `lowest`), then (offset, delta < distinct < base, index).  Base emission t
// is base entry t+2 (the seed is #1) and chunk k closes after base entry E_k,
// so chunk k holds base emissions [E_{k-1}-1, E_k-1).  A delta/distinct
// emission at offset o follows 1 + #(base emissions with offset < o) base
// entries and lands in the first chunk k with that count < E_k, i.e. with
// o <= theta_k = be_off[E_k - 2].  Every chunk is therefore one contiguous
// range of each stream.
template <bool D, bool VEC = false, class SM = Smem>
LNG_SR_INL void score_round(const DevTables& T, Slot& S, SM& s, int ulscript, bool cjk, int nb, int nd, int nx,
                            int lowest, int dummy_off, int lane, int eb, int ed, int ex, VecState* V = nullptr) {
  lane = wave::lane_here();
  // The hit rounds (quad_round / octa_round / cjk_round) already turned their
  // nb / nd / nx hits into eb base, ed delta and ex distinct emissions (tote
  // adds, zero langprobs dropped) in be_* / d_* / x_*.
  (void)nd;
  (void)nx;
  const int chunksize = cjk ? kChunksizeUnis : kChunksizeQuads;
  long long t2 = (D && kProfSub && s.prof) ? (long long)clock64() : 0;
  // chunk plan from the base-hit count (ChunkAll :978-1031)
  int K = 0;
  if (nb <= 0) {
    K = 1;
    if (lane == 0) s.E[0] = 0xFFFF;
  } else {
    int left = nb, e = 0;
    while (left > 0) {
      int blen = chunksize;
      if (left < chunksize + (chunksize >> 1)) blen = left;
      else if (left < 2 * chunksize) blen = (left + 1) >> 1;
      e += blen;
      if (lane == 0) s.E[K] = (uint16_t)e;
      ++K;
      left -= blen;
    }
    if (lane == 0) s.E[K - 1] = 0xFFFF;   // the last chunk takes everything that is left
  }
  gsync();                                  // emissions visible; E in LDS
  for (int k = lane; k <= K; k += 64) {
    if (k < K) {
      int th = 0x7FFFFFFF;
      if (k < K - 1) {
        const int idx = (int)s.E[k] - 2;
        th = idx < 0 ? -1 : (idx < eb ? (int)S.be_off[idx] : 0x7FFFFFFF);
      }
      s.theta[k] = th;
      const int bs = k == 0 ? 0 : min(max((int)s.E[k - 1] - 1, 0), eb);
      s.bst[k] = (uint16_t)bs;
    } else {
      s.bst[K] = (uint16_t)eb;
    }
    s.st[0][k] = (uint16_t)ed;
    s.st[1][k] = (uint16_t)ex;
  }
  wsync();
  // chunk of every delta / distinct emission; chunk k's range starts at the
  // first emission whose chunk is >= k (LDS indexed directly: a selected
  // generic pointer would turn these into flat stores, unordered against
  // the ds_write initialisation above)
  for (int pass = 0; pass < 2; ++pass) {
    const int n = pass == 0 ? ed : ex;
    const uint16_t* offs = pass == 0 ? S.d_off : S.x_off;
    int pch = -1;
    for (int i0 = 0; i0 < n; i0 += 64) {
      const int i = i0 + lane;
      int ch = K - 1;
      if (i < n) {
        const int o = offs[i];
        int lo = 0, hi = K - 1;
        while (lo < hi) {
          const int mid = (lo + hi) >> 1;
          if (o <= s.theta[mid]) hi = mid;
          else lo = mid + 1;
        }
        ch = lo;
      }
      const int prev = (int)wave::wshr1((uint32_t)ch, (uint32_t)pch);   // lane - 1's chunk; lane 0: the last block's
      if (i < n)
        for (int k = prev + 1; k <= ch; ++k) s.st[pass][k] = (uint16_t)i;
      pch = rdl(ch, 63);
    }
  }
  wsync();
  // lo[k] = first offset of chunk k (chunk 0 opens with the seed at `lowest`)
  for (int k = lane; k < K; k += 64) {
    uint32_t m = k == 0 ? (uint32_t)lowest : kInf;
    const int bs = s.bst[k], be = k == K - 1 ? eb : s.bst[k + 1];
    const int ds = s.st[0][k], de = s.st[0][k + 1], xs = s.st[1][k], xe = s.st[1][k + 1];
    if (bs < be) m = min(m, (uint32_t)S.be_off[bs]);
    if (ds < de) m = min(m, (uint32_t)S.d_off[ds]);
    if (xs < xe) m = min(m, (uint32_t)S.x_off[xs]);
    s.lo[k] = m;
  }
  wsync();
  if constexpr (D) mark_sub(s, lane, 2, t2);
  if (D && kProfSub && s.prof && lane == 0) atomicAdd(&s.prof[5], ((unsigned long long)K << 20) | 1ull);   // chunks, rounds
  const uint64_t seed = tote_adds(T, (uint32_t)per_script_number_latin(T, default_language(T, ulscript)) << 8);
  const int rs = ((uint32_t)ulscript == T.latin) ? 0 : 1;
  int ck1 = -1, ck2 = -1, cs1 = 0, cs2 = 0, cgr = 0;   // chunk `lane`: top keys, scores, grams
  // the first 128 adds of chunk k + 1 are loaded while chunk k is scored: their
  // indices at the top of chunk k, their gathers at its end
  int pbs, pnB, pds, pnD, pxs, pnX, pxe;
  int ptot = chunk_plan(s, K, eb, 0, pbs, pnB, pds, pnD, pxs, pnX, pxe);
  uint64_t n0 = resolve_ref(T, chunk_ref(S, s, seed, rs, lane, 0, ptot, pbs, pnB, pds, pnD, pxs, pnX, pxe));
  uint64_t n1 = resolve_ref(T, chunk_ref(S, s, seed, rs, lane + 64, 0, ptot, pbs, pnB, pds, pnD, pxs, pnX, pxe));
  for (int k = 0; k < K; ++k) {
    const int bs = pbs, nB = pnB, ds = pds, nD = pnD, xs = pxs, nX = pnX, xe = pxe, tot = ptot;
    const uint64_t a0 = n0, a1 = n1;
    uint64_t r0 = 0, r1 = 0;
    if (k + 1 < K) {
      ptot = chunk_plan(s, K, eb, k + 1, pbs, pnB, pds, pnD, pxs, pnX, pxe);
      r0 = chunk_ref(S, s, seed, rs, lane, k + 1, ptot, pbs, pnB, pds, pnD, pxs, pnX, pxe);
      r1 = chunk_ref(S, s, seed, rs, lane + 64, k + 1, ptot, pbs, pnB, pds, pnD, pxs, pnX, pxe);
    }
    reinterpret_cast<uint4*>(s.tote)[lane] = make_uint4(0, 0, 0, 0);
    wsync();
    const int seedn = k == 0 ? 1 : 0;
    for (int t = lane; t < tot; t += 64) {
      const uint64_t a = t < 128 ? (t < 64 ? a0 : a1)
                                 : resolve_ref(T, chunk_ref(S, s, seed, rs, t, k, tot, bs, nB, ds, nD, xs, nX, xe));
      const uint32_t k1 = (uint32_t)a & 0xFF, k2 = (uint32_t)(a >> 16) & 0xFF, k3 = (uint32_t)(a >> 32) & 0xFF;
      // the low half sums the score (read with the reference's uint16 wrap), the
      // high half counts the adds: a group (the 4 keys of one lane) is in use
      // (Tote's in_use_mask_) iff one of its keys has a non-zero high half
      if (k1) atomicAdd(&s.tote[k1], ((uint32_t)(a >> 8) & 0xFF) | 0x10000u);
      if (k2) atomicAdd(&s.tote[k2], ((uint32_t)(a >> 24) & 0xFF) | 0x10000u);
      if (k3) atomicAdd(&s.tote[k3], ((uint32_t)(a >> 40) & 0xFF) | 0x10000u);
    }
    const int score_count = nB + seedn;
    if (k + 1 < K) {
      n0 = resolve_ref(T, r0);
      n1 = resolve_ref(T, r1);
    }
    wsync();
    if (s.has_pri) {                         // the prior whacks zero their key's score (ZeroPSLang :39-42)
      const int wk = lane < 4 ? s.pri_wk[rs][lane] : 0;
      if (wk) atomicAnd(&s.tote[wk], 0xFFFF0000u);
      wsync();
    }
    // top keys of the in-use groups: (uint16 score desc, key asc).  The
    // reference sorts three (CurrentTopThreeKeys) but SetChunkSummary reads
    // only the first two (scoreonescriptspan.cc:60-96), so two rounds.
    const uint4 v4 = reinterpret_cast<const uint4*>(s.tote)[lane];
    const bool inuse = ((v4.x | v4.y | v4.z | v4.w) >> 16) != 0;
    const uint32_t cand[4] = {v4.x & 0xFFFF, v4.y & 0xFFFF, v4.z & 0xFFFF, v4.w & 0xFFFF};
    int key3[2] = {-1, -1};
    uint32_t sc3[2] = {0, 0};
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      uint32_t best = 0;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int key = lane * 4 + i;
        const bool taken = key == key3[0];
        const uint32_t comp = (inuse && !taken) ? ((cand[i] + 1) << 8) | (uint32_t)(255 - key) : 0u;
        best = comp > best ? comp : best;
      }
      best = wave::wmax(best);
      if (best) {
        key3[r] = 255 - (int)(best & 0xFF);
        sc3[r] = (best >> 8) - 1;
      }
    }
    // lane k keeps chunk k's top two keys and scores; the summaries are made after the loop
    if (lane == k) {
      ck1 = key3[0]; ck2 = key3[1];
      cs1 = key3[0] >= 0 ? (int)sc3[0] : 0;
      cs2 = key3[1] >= 0 ? (int)sc3[1] : 0;
      cgr = score_count;
    }
    wsync();
  }
  if constexpr (D) mark_sub(s, lane, 3, t2);
  // SetChunkSummary (scoreonescriptspan.cc:60-96) for every chunk at once, one
  // lane per chunk (K <= kMaxCh = 64); the DocTote adds then run in chunk order on lane 0
  int lo = 0, hi = 0, lang1 = 0, lang2 = 0, rd = 0, rsc = 0;
  if (lane < K) {
    const uint32_t lo_k = s.lo[lane];
    lo = lo_k == kInf ? dummy_off : (int)lo_k;
    hi = dummy_off;
    if (lane + 1 < K && s.lo[lane + 1] != kInf) hi = (int)s.lo[lane + 1];
    const uint64_t* kt = T.keytab + 256 * (uint32_t)ulscript;
    const uint64_t i1 = gld(kt + (uint8_t)ck1), i2 = gld(kt + (uint8_t)ck2);
    lang1 = (int)(i1 & 0xFFFF); lang2 = (int)(i2 & 0xFFFF);
    const int len = hi - lo;
    int actual = 0;
    if (len > 0) actual = (int)((uint32_t)cs1 << 10) / len;
    const int expected = (int16_t)(uint16_t)(i1 >> 32);
    const uint16_t s1 = (uint16_t)cs1, s2 = (uint16_t)cs2, grams = (uint16_t)cgr;
    rd = (uint8_t)reliability_delta(s1, s2, grams);
    const int c1 = (int)((i1 >> 16) & 0xFFFF);
    if (c1 != 0 && c1 == (int)((i2 >> 16) & 0xFFFF)) rd = 100;
    rsc = (uint8_t)reliability_expected(actual, expected);
    cs1 = s1; cs2 = s2; cgr = grams;
  }
  const int Kv = K < kMaxSummaries ? K : kMaxSummaries;   // the summary buffer keeps this many
  if constexpr (VEC) {
    // linear[] of the round (LinearizeAll :856-975): the seed, then by offset
    // with delta < distinct < base on ties, each stream in its own order; the
    // dummy entry at the round end
    VecSlot* vs = V->vs;
    const int NL = 1 + eb + ed + ex;
    if (lane == 0) {
      vs->lin_off[0] = (uint32_t)lowest;
      vs->lin_add[0] = seed;
      vs->lin_off[NL] = (uint32_t)dummy_off;
      vs->lin_add[NL] = 0;
    }
    for (int t = lane; t < eb; t += 64) {
      const int o = S.be_off[t];
      const int r = 1 + t + count_upto(S.d_off, ed, o, true) + count_upto(S.x_off, ex, o, true);
      vs->lin_off[r] = (uint32_t)o;
      vs->lin_add[r] = adds_by_index(T, S.be_ai[t]);
    }
    for (int j = lane; j < ed; j += 64) {
      const int o = S.d_off[j];
      const int r = 1 + j + count_upto(S.x_off, ex, o, false) + count_upto(S.be_off, eb, o, false);
      vs->lin_off[r] = (uint32_t)o;
      vs->lin_add[r] = adds_by_index(T, S.d_ai[j]);
    }
    for (int j = lane; j < ex; j += 64) {
      const int o = S.x_off[j];
      const int r = 1 + j + count_upto(S.d_off, ed, o, true) + count_upto(S.be_off, eb, o, false);
      vs->lin_off[r] = (uint32_t)o;
      vs->lin_add[r] = adds_by_index(T, S.x_ai[j]);
    }
    gsync();
    // chunk k's first linear entry (chunk_start): the seed and every earlier
    // chunk's emissions come before it
    int cst = 0;
    if (lane > 0 && lane < K) cst = min(1 + (int)s.bst[lane] + (int)s.st[0][lane] + (int)s.st[1][lane], NL);
    // SharpenBoundaries (:780-845), chunk after chunk; chunk i's new start
    // moves its offset, and so the bytes of chunks i - 1 and i
    int prior_linear = 0, prior_lang = rdl(lang1, 0);
    for (int i = 1; i < Kv; ++i) {
      const int this_lang = rdl(lang1, i), this_linear = rdl(cst, i);
      if (this_lang == prior_lang) {
        prior_linear = this_linear;
        continue;
      }
      const int next_linear = i + 1 < Kv ? rdl(cst, i + 1) : NL;
      if (same_close_set(T, prior_lang, this_lang)) {
        prior_linear = this_linear;
        prior_lang = this_lang;
        continue;
      }
      const uint32_t ps0 = per_script_number(T, ulscript, prior_lang), ps1 = per_script_number(T, ulscript, this_lang);
      const int better = better_boundary_w(vs, ps0, ps1, prior_linear, this_linear, next_linear, lane);
      const int noff = (int)vs->lin_off[better];
      if (lane == i) {
        lo = noff;
        cst = better;
      }
      prior_linear = better;
      prior_lang = this_lang;
    }
    // bytes = the (sharpened) next start minus this one
    const int nlo = __shfl(lo, lane + 1 < 64 ? lane + 1 : lane, 64);
    if (lane < K) hi = lane + 1 < K ? nlo : dummy_off;
  }
  for (int k = 0; k < K; ++k) {
    const int l1 = rdl(lang1, k), l0 = rdl(lo, k), h0 = rdl(hi, k), sc = rdl(cs1, k);
    const int r1 = rdl(rd, k), r2 = rdl(rsc, k);
    if (lane == 0) {
      const uint16_t bytes = (uint16_t)(h0 - l0);
      if (k < kMaxSummaries) dt_add(s, (uint16_t)l1, bytes, sc, r1 < r2 ? r1 : r2);
      if (D && s.dbg) {
        const int bs = s.bst[k], be = k == K - 1 ? eb : s.bst[k + 1];
        const int ds = s.st[0][k], de = s.st[0][k + 1], xs = s.st[1][k], xe = s.st[1][k + 1];
        uint32_t* o = s.dbg + 1 + s.dbg_pos;
        const uint32_t v[18] = {'C', (uint32_t)l0, (uint32_t)h0, (uint32_t)l1, (uint32_t)rdl(lang2, k),
                                (uint32_t)sc, (uint32_t)rdl(cs2, k), (uint32_t)rdl(cgr, k), (uint32_t)r1,
                                (uint32_t)r2, (uint32_t)bs, (uint32_t)be, (uint32_t)ds,
                                (uint32_t)de, (uint32_t)xs, (uint32_t)xe, (uint32_t)s.theta[k], (uint32_t)(eb << 16 | K)};
        for (int i = 0; i < 18; ++i) o[i] = v[i];
        s.dbg_pos += 18;
        s.dbg[0] = s.dbg_pos;
      }
    }
  }
  wsync();
  if constexpr (VEC) {
    // SummaryBufferToVector (:389-509), chunk after chunk
    VecState& Vr = *V;
    const int unk = (int)T.unknown_lang;
    for (int i = 0; i < Kv; ++i) {
      const int uoff = rdl(lo, i), ulen = rdl(hi, i) - uoff;
      const int l1 = rdl(lang1, i), l2 = rdl(lang2, i), r1 = rdl(rd, i), r2 = rdl(rsc, i);
      int moff = vec_map_back(Vr, uoff);
      if (moff > 0) {
        // trim back to a word start in the original text: at most 12 bytes,
        // leaving 3 in the prior item; over bytes >= 0x41, plus one '"#@
        const int prior_size = Vr.n > 0 ? Vr.last_bytes : 0;
        int nlim = min(min(prior_size - 3, moff), 12);
        const bool in = lane < nlim;
        const uint8_t b = in ? gld(Vr.doc + moff - lane - 1) : (uint8_t)0;
        const uint64_t stop = __ballot(in && b < 0x41);
        int k = stop ? __builtin_ctzll(stop) : 0;
        if (k < nlim) {
          const uint32_t c = gld(Vr.doc + moff - k - 1);
          if (c == '\'' || c == '"' || c == '#' || c == '@') ++k;
        }
        if (k > 0) {
          Vr.last_bytes -= k;
          vec_store(Vr, lane);
          moff -= k;
        }
      }
      const int mlen = vec_map_back(Vr, uoff + ulen) - moff;
      int nl = l1;
      bool delta_bad = r1 < 75, score_bad = r2 < 75;         // kUnreliablePercentThreshold
      const int prior_lang = Vr.n > 0 ? Vr.last_lang : unk;
      if (prior_lang == l1) delta_bad = false;
      if (same_close_set(T, l1, prior_lang)) { nl = prior_lang; delta_bad = false; }
      if (same_close_set(T, l1, l2) && prior_lang == l2) { nl = prior_lang; delta_bad = false; }
      const int next_lang = i + 1 < Kv ? rdl(lang1, i + 1) : unk;   // NextChunkLang
      if (delta_bad && prior_lang == l2 && next_lang == l2) { nl = prior_lang; delta_bad = false; }
      if (delta_bad || score_bad) nl = unk;
      vec_item(Vr, nl, moff, mlen, lane);
    }
    gsync();
  }
  // the ring keeps the last four distinct langprobs
  if (lane == 0) {
    uint64_t r4[4];
    for (int i = 0; i < 4; ++i) {
      const int u = ex - kMaxBoosts + i;
      r4[i] = u < 0 ? s.ring[rs][u + kMaxBoosts] : adds_by_index(T, gld(&S.x_ai[u]));
    }
    for (int i = 0; i < 4; ++i) s.ring[rs][i] = r4[i];
  }
  wsync();
  if constexpr (D) mark_sub(s, lane, 4, t2);
}


template <class SM>
__device__ void dbg_round(const Slot& S, SM& s, int off, int next, int nb, int nd, int nx, bool octa, int lane) {
  if (!s.dbg) return;
  const uint32_t h[6] = {'R', (uint32_t)off, (uint32_t)next, (uint32_t)nb, (uint32_t)nd, (uint32_t)nx};
  dbg_words(s, lane, h, 6);
  uint32_t* o = s.dbg + 1 + s.dbg_pos;
  for (int i = lane; i < nb; i += 64) { o[2 * i] = S.b_off[i]; o[2 * i + 1] = S.b_ind[i]; }
  o += 2 * nb;
  for (int i = lane; i < nd; i += 64) { o[2 * i] = octa ? S.d_hoff[i] : S.d_off[i]; o[2 * i + 1] = S.d_ind[i]; }
  o += 2 * nd;
  for (int i = lane; i < nx; i += 64) { o[2 * i] = octa ? S.x_hoff[i] : S.x_off[i]; o[2 * i + 1] = S.x_ind[i]; }
  wave::wsync();
  if (lane == 0) {
    s.dbg_pos += 2 * (nb + nd + nx);
    s.dbg[0] = s.dbg_pos;
  }
  gsync();
}

// ScoreOneScriptSpan (scoreonescriptspan.cc:1302-1333) with the round loops
// of ScoreCJKScriptSpan / ScoreQuadScriptSpan (:1163-1277).
template <bool D, bool VEC = false, class SM = Smem, class WN = Win>
__device__ __forceinline__ bool score_span(const DevTables& T, Slot& S, SM& s, WN& win, int tb,
                                           int ulscript, int lane, uint32_t* tr, uint32_t doc, uint32_t cflags,
                                           VecState* V = nullptr) {
  int rt = rtype_of(T, ulscript);
  if ((cflags & kCLDFlagScoreAsQuads) && rt != RTypeCJK) rt = RTypeMany;   // scoreonescriptspan.cc:1318-1320
  if (rt == RTypeNone || rt == RTypeOne) {
    if (lane == 0) dt_add(s, (uint16_t)default_language(T, ulscript), tb, tb, 100);
    wsync();
    if constexpr (VEC) {
      // JustOneItemToVector (:513-548): the span after its leading space
      if (tb < 1 && !V->seq) return false;           // (a span of one cut character: the sequential spans)
      const int moff = vec_map_back(*V, 1);
      vec_item(*V, default_language(T, ulscript), moff, vec_map_back(*V, tb) - moff, lane);
    }
    return true;
  }
  if (tb <= 1) return true;
  int off = 1;
  long long t = (D && s.prof) ? (long long)clock64() : 0;
  if (rt == RTypeCJK) {
    while (off < tb) {
      int nb, nd, nx;
      if constexpr (D) trace(tr, lane, doc, 20, off);
      int eb, edm, exm;
      bool ok = true;
      const int next = cjk_round<D>(T, win, s, tb, S, off, nb, nd, nx, eb, edm, exm, ok, lane);
      if (!ok) return false;
      if constexpr (D) trace(tr, lane, doc, 21, next);
      if constexpr (D) dbg_round(S, s, off, next, nb, nd, nx, true, lane);
      if constexpr (D) mark(s, lane, 6, t);
      score_round<D, VEC>(T, S, s, ulscript, true, nb, nd, nx, off, next, lane, eb, edm, exm, V);
      if constexpr (D) mark(s, lane, 7, t);
      off = next;
    }
    return true;
  }
  bool ok = true;
  const int start = 1 + (ufl(win_text(win, s, 0, 2, ok, lane)[1]) == ' ' ? 1 : 0);
  int nws, nsp;
  if (!ok || !word_lists(win, s, tb, start, S, nws, nsp, lane)) return false;
  if constexpr (D) trace(tr, lane, doc, 10, nws);
  const int nch = build_chain(win, s, tb, S, nws, lane);
  if (nch < 0) return false;
  if constexpr (D) trace(tr, lane, doc, 11, nch);
  if constexpr (D) mark(s, lane, 4, t);
  int c0 = 0, j0 = 0;
  while (off < tb) {
    int nb, nd, nx;
    if constexpr (D) trace(tr, lane, doc, 12, off);
    int eb, edm, exm;
    const int next = quad_round<D>(T, win, s, tb, S, nch, c0, nb, eb, ok, lane);
    if (!ok) return false;
    if constexpr (D) trace(tr, lane, doc, 13, next);
    if constexpr (D) mark(s, lane, 5, t);
    octa_round<D>(T, win, s, S, nsp, j0, off, next, nd, nx, edm, exm, ok, lane);
    if (!ok) return false;
    if constexpr (D) trace(tr, lane, doc, 14, (uint32_t)(nd << 16 | nx));
    if constexpr (D) dbg_round(S, s, off, next, nb, nd, nx, true, lane);
    if constexpr (D) mark(s, lane, 6, t);
    score_round<D, VEC>(T, S, s, ulscript, false, nb, nd, nx, off, next, lane, eb, edm, exm, V);
    if constexpr (D) mark(s, lane, 7, t);
    off = next;
  }
  return true;
}

// DetectLanguageSummaryV2 (compact_lang_det_impl.cc:1707-2106) for one
// document: pass 1, and pass 2 with Repeats when pass 1 is not good enough.
// Returns the number of passes, or -reason (kWhy*) to re-queue.
enum { kWhyLength = 1, kWhyClassify = 2, kWhySpan = 3, kWhySqueeze = 4, kWhyCapacity = 5 };
// MoveLang1ToLang2's vector half (compact_lang_det_impl.cc:1122-1147), lane 0
// over the document's vector: relabel lang1 -> lang2, merge neighbours that
// now share a language.
__device__ __noinline__ void vec_move_lang(VecState* V, int from_lang, int to_lang, int unk) {
  int k = 0, prior = unk;
  for (int i = 0; i < V->n; ++i) {
    cld_chunk c = V->v[i];
    if (c.lang1 == (uint16_t)from_lang) c.lang1 = (uint16_t)to_lang;
    if ((int)c.lang1 == prior && k > 0) {
      V->v[k - 1].bytes += c.bytes;
    } else {
      V->v[k] = c;
      ++k;
    }
    prior = c.lang1;
  }
  V->n = k;
}

// Pass modes (k_long's speculation for the longest documents of a small
// batch): kPassesAll runs compact_lang_det_impl.cc:1848-2105's passes in
// order; kPassFirstOnly stops after a pass 1 that is not good enough and
// returns kNeedsRepeats (a Squeeze restart still runs its passes here);
// kPassRepeatsOnly starts at pass 2 = Repeats|Finish, what a pass 1 without
// the Squeeze restart is followed by.  Pass 2 reads nothing pass 1 computed
// (the DocTote, the boost ring and the predictor start fresh), so the two can
// run on two waves at once and the document costs the longer, not the sum.
constexpr int kPassesAll = 0, kPassFirstOnly = 1, kPassRepeatsOnly = 2;
constexpr int kNeedsRepeats = 4;
// SEQ: the sequential span source (cld_seq.hip) over page *seqd instead of
// classify() + next_span() over g (g / L are then that page); its own
// instantiation, so the parallel one carries none of its registers.
template <bool D, bool VEC = false, bool SEQ = false>
__device__ __forceinline__ int detect(const DevTables& T, const uint8_t* g, int L, Slot& S, Smem& s, int lane,
                      cld_result* __restrict__ out, uint32_t* tr, uint32_t doc, uint32_t cflags,
                      const uint32_t* __restrict__ pri, const uint8_t* __restrict__ hf, VecState* V = nullptr,
                      int mode = kPassesAll, const uint32_t* hp = nullptr, const uint32_t* hg = nullptr,
                      const SeqDoc* seqd = nullptr) {
  const int unk = (int)T.unknown_lang;
  // ApplyHints priors (ScoreBoosts, scoreonescriptspan.cc:125-152): boosts as tote adds, whacks as keys
  if (lane == 0) s.has_pri = pri != nullptr;
  if (lane < 16) {
    const uint32_t lp = pri ? gld(pri + lane) : 0u;
    if (lane < 8) s.pri_add[lane >> 2][lane & 3] = lp ? tote_adds(T, lp) : 0ull;
    else s.pri_wk[(lane - 8) >> 2][lane & 3] = (uint8_t)((lp >> 8) & 0xFF);
  }
  wsync();
  if (L == 0) {
    if (lane == 0) {
      Extract x;
      for (int i = 0; i < 3; ++i) { x.lang3[i] = unk; x.pct3[i] = 0; x.ns3[i] = 0.0; x.rp3[i] = 0; }
      x.text_bytes = 0;
      write_result(out, x, unk, false);
    }
    return 1;
  }
  if (!SEQ && L > kDocCap - 64) return -kWhyLength;
  const DocView dv{g, L, hf, hp, hg};
  if constexpr (D) trace(tr, lane, doc, 1, L);
  long long t = (D && s.prof) ? (long long)clock64() : 0;

  bool careful = true;                           // a cut last character: span text may be malformed
  if constexpr (!SEQ) {
    if (!classify(T, dv, S, careful, lane)) return -kWhyClassify;
  }
  if constexpr (D) mark(s, lane, 0, t);
  if constexpr (D) trace(tr, lane, doc, 2, 0);
  // Passes (compact_lang_det_impl.cc:1848-2105): 1 = flags 0; the Squeeze
  // trigger restarts the document as pass 2 = Squeeze; otherwise pass 2 =
  // Repeats|Finish.  After a Squeeze pass that is not good enough, pass 3 =
  // Squeeze|Repeats|Finish.  The Repeats predictor is document-wide (pred),
  // the Squeeze one is fresh per span (pred2).
  bool sq = false;
  int nsp = 0, cur = 0;                          // span cache (pass 1): spans recorded, bytes used
  bool cache_ok = !VEC && mode != kPassRepeatsOnly;   // (vec mode rebuilds pass 2's spans with their offset map)
  for (int pass = mode == kPassRepeatsOnly ? 2 : 1; pass <= 3; ++pass) {
    const bool rep = pass == 3 || (pass == 2 && !sq);    // Repeats always comes with Finish
    const bool from_cache = pass == 2 && rep && cache_ok;
    if constexpr (VEC) {                         // each pass starts a new vector (:1730-1732)
      V->n = 0;
      V->over = false;
    }
    if (lane == 0) s.dt.init();
    if (lane < 8) s.ring[lane >> 2][lane & 3] = 0;
    uint32_t hcarry = 0, ep = 0;
    if (from_cache) {
      // Repeats over every cached span first, predictor in LDS (the scoring
      // state it shares the LDS with is dead until the span loop below)
      for (int i = lane; i < kPredictionTableSize / 8; i += 64) reinterpret_cast<uint4*>(s.pred)[i] = make_uint4(0, 0, 0, 0);
      wsync();
      for (int i = 0; i < nsp; ++i) {
        bool okr;
        const int tb = rep_span_lds(s.pred, S.pred, S.lbd + ufl(S.sp_off[i]), ufl(S.sp_tb[i]), hcarry, careful, okr, lane);
        if (!okr) return -kWhySpan;
        if (lane == 0) S.sp_tb[i] = tb;
      }
      gsync();
      if constexpr (D) mark(s, lane, 3, t);
    } else if (rep) {
      ep = new_epoch(S.epoch, S.pred, lane);
    }
    const bool rep_inline = rep && !from_cache;
    wsync();
    int next = 0, total = 0, ci = 0, rlo = -1;
    bool restart = false;
    for (;;) {
      int ul = 0, st = 0, tb;
      uint8_t* lb = S.lb[0];
      if constexpr (D) trace(tr, lane, doc, 3, next);
      if (from_cache) {
        if (ci >= nsp) break;
        tb = ufl(S.sp_tb[ci]);
        ul = ufl(S.sp_ul[ci]);
        lb = S.lbd + ufl(S.sp_off[ci]);
        ++ci;
      } else {
        const bool rec = pass == 1 && cache_ok && cur + kLB <= kLbdCap && nsp < kMaxSpans;
        if (pass == 1 && !rec) cache_ok = false;
        if (rec) lb = S.lbd + cur;
        if constexpr (SEQ)
          tb = seq_span<VEC>(T, *seqd, S, lb, next, ul, st, VEC ? V->vs->omap : nullptr, lane);
        else
          tb = dv.hp ? next_span<VEC, true>(T, dv, S, lb, next, ul, st, lane, VEC ? V->vs->omap : nullptr,
                                            VEC ? V->hpos : nullptr, VEC ? V->hgap : nullptr, nullptr, &rlo)
                     : next_span<VEC>(T, dv, S, lb, next, ul, st, lane, VEC ? V->vs->omap : nullptr,
                                      VEC ? V->hpos : nullptr, VEC ? V->hgap : nullptr);
        if (st == 0) break;
        if (st < 0) return -kWhySpan;
        if (rec) {
          if (lane == 0) { S.sp_off[nsp] = cur; S.sp_tb[nsp] = tb; S.sp_ul[nsp] = ul; }
          ++nsp;
          cur += (tb + 64 + 15) & ~15;           // text, its pads and the hash read slack
        }
      }
      if constexpr (D) trace(tr, lane, doc, 4, tb);
      if constexpr (D) mark(s, lane, 1, t);
      if (pass == 1) {
        if (tb > 2048 && squeeze_trigger(S, lb, careful, lane)) {   // recursion with Squeeze (:1867-1900)
          restart = true;
          cache_ok = false;
          break;
        }
        if constexpr (D) mark(s, lane, 2, t);
      }
      bool ok;
      if (tb + 48 <= kLdsText) {
        // the span (and its pads) fits in LDS: 16 bytes per lane per step
        const int n16 = (tb + 48 + 15) >> 4;
        for (int i = lane; i < n16; i += 64)
          reinterpret_cast<uint4*>(s.text)[i] = reinterpret_cast<const uint4*>(lb)[i];
        wsync();
        if (sq) tb = squeeze_span<VEC>(S, s.text, tb, careful, lane);        // in place, as the reference does
        if (rep_inline) {
          bool okr;
          tb = rep_words<VEC>(S, s.text, s.text, tb, hcarry, ep, careful, okr, lane);   // in place, as the reference does
          if (!okr) return -kWhySpan;
          if constexpr (D) mark(s, lane, 3, t);
        }
        if constexpr (D) trace(tr, lane, doc, 5, tb);
        if constexpr (D) {
          const uint32_t v[4] = {'S', (uint32_t)ul, (uint32_t)tb, (uint32_t)pass};
          dbg_words(s, lane, v, 4);
          dbg_text(s, lane, s.text, tb);
        }
        WinOf<SEQ> win{nullptr, 0, 16 * n16, 16 * n16};                   // the whole span is in s.text
        ok = score_span<D, VEC>(T, S, s, win, tb, ul, lane, tr, doc, cflags, V);
      } else {
        const uint8_t* text = lb;
        if (sq) tb = squeeze_span<VEC>(S, lb, tb, careful, lane);
        if (rep_inline) {
          bool okr;
          tb = rep_words<VEC>(S, lb, S.lb[1], tb, hcarry, ep, careful, okr, lane);
          if (!okr) return -kWhySpan;
          text = S.lb[1];
          if constexpr (D) mark(s, lane, 3, t);
        }
        if constexpr (D) trace(tr, lane, doc, 5, tb);
        if constexpr (D) {
          const uint32_t v[4] = {'S', (uint32_t)ul, (uint32_t)tb, (uint32_t)pass};
          dbg_words(s, lane, v, 4);
          dbg_text(s, lane, text, tb);
        }
        WinOf<SEQ> win{text, 0, 0, (tb + 48 + 15) & ~15};                // windows of it go to s.text (SEQ: read in place)
        ok = score_span<D, VEC>(T, S, s, win, tb, ul, lane, tr, doc, cflags, V);
      }
      if (!ok) return -kWhyCapacity;
      t = (D && s.prof) ? (long long)clock64() : 0;
      total += tb;
    }
    if (restart) {
      sq = true;
      continue;
    }
    if constexpr (VEC) {
      auto mv = [&](int from_lang, int to_lang) {
        if (lane == 0) vec_move_lang(V, from_lang, to_lang, unk);
        V->n = rdl(V->n, 0);
      };
      if (wave::finish_document(T, s.dt, total, rep, out, lane, (cflags & kCLDFlagBestEffort) != 0, mv)) {
        // FinishResultVector(0, buffer_length) (:1688-1702): the first item
        // starts at 0, the last ends at the document end
        if (lane == 0 && V->n > 0 && !V->over) {
          cld_chunk f = V->v[0];
          if (f.offset > 0) {
            f.bytes += f.offset;
            f.offset = 0;
            V->v[0] = f;
          }
          cld_chunk e = V->v[V->n - 1];
          if (e.offset + e.bytes < L) {
            e.bytes += L - (e.offset + e.bytes);
            V->v[V->n - 1] = e;
          }
        }
        gsync();
        return pass;
      }
    } else {
      if (wave::finish_document(T, s.dt, total, rep, out, lane, (cflags & kCLDFlagBestEffort) != 0)) return pass;
      if (mode == kPassFirstOnly && pass == 1) return kNeedsRepeats;   // the speculative wave has pass 2
    }
  }
  return 0;
}

// ------------------------------------------------ staged long-document path
// k_long runs every stage of a document in one kernel, so the kernel carries
// the registers of its largest stage (128 VGPRs with spills: 4 waves/SIMD)
// and the LDS of the union of the text window and the Repeats predictor, and
// k_long's time follows its resident waves (round4d_waves.txt).  The staged
// path splits pass 1 and pass 2 into kernels of their own (cld_kernels.hip):
//   k_lspan   classify + GetOneScriptSpan/LowerScriptSpan + the Squeeze
//             trigger test: pass 1's lowered spans into the document's region
//             of a per-batch store (st_spans)
//   k_lscore  ScoreOneScriptSpan over the stored spans, DocTote, the document
//             level (st_score): pass 1, or pass 2 (Repeats|Finish)
//   k_lrep    CheapRepWordsInplace over the stored spans, in place, predictor
//             in LDS (st_rep): what pass 2 scores
// each with its own register and LDS budget.  The stages are the very
// functions detect() calls, in the same order, on the same span text (pass 2
// from the span cache), so results are the same.  A document the staged path
// does not take -- the Squeeze restart, a re-queued span, spans that outgrow
// the slot's span cache, no room left in the store -- goes to the fused k_long
// whole, from scratch.
//
// The stage functions are inlined into their kernels: an out-of-line call
// passes the LDS state as a generic pointer, and its FLAT accesses count
// against LGKM like the gathers.
//
// A document's region: StHdr, the spans back to back (each followed by its
// pads and NULs, 16-byte aligned), then the span table (one u64 per span:
// offset in the region | text_bytes << 32 | ulscript << 56).
#ifndef LNG_PAR_MIN
#define LNG_PAR_MIN 48
#endif
constexpr int kParMin = LNG_PAR_MIN, kParG = 16;   // span-parallel documents: > kParMin spans, kParG spans per group
// Batches of pages (long documents of 8 KB and more on average, k_lspan)
// split only documents of more than kParMinPages spans: scored whole, a
// 200-760-span 16 KB page costs less than its groups plus their boost-ring
// reconstruction, and the heavy-first lists keep it out of the tail (C3:
// 73.0 ms at 48, 64.7 at 400, 63.3 at 2000; C5, whose many-span documents
// stand out from the rest, keeps kParMin: 400 there took 44.1 -> 45.8 ms;
// profiles/round5_par_ab.txt).
#ifndef LNG_PAR_MIN_PAGES
#define LNG_PAR_MIN_PAGES 2000
#endif
constexpr int kParMinPages = LNG_PAR_MIN_PAGES;
struct StHdr {
  uint32_t nsp, careful, tab;
  uint32_t par;                                  // span-parallel documents: offset of the record arrays, else 0
};
constexpr uint64_t kStNone = ~0ull;
__device__ __forceinline__ int st_advance(int tb) { return (tb + 48 + 15) & ~15; }   // text + "   \0" + NULs

// Pass 1's spans of one document (detect()'s pass-1 span loop up to the
// scoring) into the slot's span cache, then, at their exact size, into a
// region of the store taken from *pool_units (16-byte units).  Returns the
// region's byte offset, or kStNone: the fused kernel takes the document.
__device__ __forceinline__ uint64_t st_spans(const DevTables& T, const DocView& dv, Slot& S, uint8_t* pool, uint64_t pool_units,
                             uint32_t* pool_ctr, int lane, int par_min = kParMin) {
  bool careful;
  if (!classify(T, dv, S, careful, lane)) return kStNone;
#if defined(LNG_LAB_STOP) && LNG_LAB_STOP == 1
  return kStNone;                                // (lab builds only: stage timing)
#endif
  int next = 0, nsp = 0, cur = 0, rlo = -1;
  SpanCursor sc;                                 // the span builder's pipeline, span to span
  for (;;) {
    if (cur + kLB > kLbdCap || nsp >= kMaxSpans) return kStNone;
    int ul = 0, st = 0;
    const int tb = dv.hp ? next_span<false, true>(T, dv, S, S.lbd + cur, next, ul, st, lane, nullptr, nullptr, nullptr,
                                                  nullptr, &rlo)
                         : next_span<false>(T, dv, S, S.lbd + cur, next, ul, st, lane, nullptr, nullptr, nullptr,
                                            nullptr, nullptr, &sc);
    if (st == 0) break;
    if (st < 0) return kStNone;
    if (tb > 2048 && squeeze_trigger(S, S.lbd + cur, careful, lane)) return kStNone;   // the Squeeze restart
    if (lane == 0) {
      S.sp_off[nsp] = cur;
      S.sp_tb[nsp] = tb;
      S.sp_ul[nsp] = ul;
    }
    ++nsp;
    cur += st_advance(tb);
  }
  gsync();
#if defined(LNG_LAB_STOP) && LNG_LAB_STOP == 2
  return kStNone;                                // (lab builds only: stage timing)
#endif
  // span-parallel documents (more than kParMin spans): after the span table,
  // roff[nsp + 1] (first record of span j), rcnt[nsp], then the records --
  // at most tb / 16 + 8 DocTote adds per span (a chunk holds >= 20 base hits
  // or 50 unigrams, a round <= 1000 hits: chunks <= tb / 40 + rounds)
  uint32_t par = 0, recs = 0;
  uint64_t bytes = sizeof(StHdr) + cur + 8ull * nsp;
  if (nsp > par_min) {
    par = (uint32_t)bytes;
    for (int j = 0; j < nsp; ++j) recs += (uint32_t)(ufl(S.sp_tb[j]) / 16 + 8);
    bytes += 4ull * (2 * nsp + 1);
    bytes = (bytes + 7) & ~7ull;
    bytes += 8ull * recs;
  }
  const uint32_t units = (uint32_t)((bytes + 15) >> 4);
  uint32_t got = 0;
  if (lane == 0) got = atomicAdd(pool_ctr, units);
  got = uflu(__shfl((int)got, 0, 64));
  if ((uint64_t)got + units > pool_units) return kStNone;
  uint8_t* region = pool + ((uint64_t)got << 4);
  const int n16 = cur >> 4;
  uint4* dst = reinterpret_cast<uint4*>(region + sizeof(StHdr));
  const uint4* src = reinterpret_cast<const uint4*>(S.lbd);
  for (int i = lane; i < n16; i += 64) dst[i] = src[i];
  uint64_t* tab = reinterpret_cast<uint64_t*>(region + sizeof(StHdr) + cur);
  for (int j = lane; j < nsp; j += 64)
    tab[j] = (uint64_t)(uint32_t)(S.sp_off[j] + (int)sizeof(StHdr)) | ((uint64_t)(uint32_t)S.sp_tb[j] << 32) |
             ((uint64_t)(uint32_t)S.sp_ul[j] << 56);
  if (par) {                                     // record offsets (lane 0: once per document)
    uint32_t* roff = reinterpret_cast<uint32_t*>(region + par);
    if (lane == 0) {
      uint32_t acc = 0;
      for (int j = 0; j < nsp; ++j) {
        roff[j] = acc;
        acc += (uint32_t)(S.sp_tb[j] / 16 + 8);
      }
      roff[nsp] = acc;
    }
  }
  if (lane == 0) {
    StHdr h{(uint32_t)nsp, careful ? 1u : 0u, (uint32_t)(sizeof(StHdr) + cur), par};
    *reinterpret_cast<StHdr*>(region) = h;
  }
  gsync();
  return (uint64_t)got << 4;
}

// Documents over kDocCap (round 5; they used to take the sequential kernel of earlier rounds):
// the span cache and the slot's letter-stop bitmap hold at most 512 KB of
// spans and 1 MB of text, so the region is reserved at its worst case and
// written directly -- the spans (at most 4 lowered bytes per raw byte plus
// 128 bytes per span), the span table and the span-parallel arrays at fixed
// places, then the bitmap -- the same layout the other kernels read.  Spans:
// up to one per 16 raw bytes (tweets run together make one per ~100 bytes;
// more, and the fused kernel hands the document on).
constexpr uint64_t kStBigMax = 64ull << 20;      // longest document taken here
__device__ __forceinline__ uint64_t st_big_spans(uint64_t L) { return L / 16 > kMaxSpans ? L / 16 : kMaxSpans; }
__device__ __forceinline__ uint64_t st_big_text(uint64_t L) { return 4 * L + 128ull * st_big_spans(L); }
__device__ __forceinline__ uint64_t st_big_bytes(uint64_t L) {
  const uint64_t tc = st_big_text(L), ns = st_big_spans(L);
  return sizeof(StHdr) + tc + 8ull * ns + 4ull * (2 * ns + 1) + 8 + 8 * (tc / 16 + 8ull * ns) + 8 * (L / 64 + 2) + 64;
}
__device__ __forceinline__ bool st_spans_big(const DevTables& T, const DocView& dv, Slot& S, uint8_t* region,
                                             int lane, int par_min = kParMin) {
  const uint64_t L = (uint64_t)dv.len, tc = st_big_text(L), tab_off = sizeof(StHdr) + tc, ns = st_big_spans(L);
  const uint64_t par_off = tab_off + 8ull * ns;
  uint64_t* lsm = reinterpret_cast<uint64_t*>(region + ((st_big_bytes(L) - 8 * (L / 64 + 2) - 64) & ~7ull));
  bool careful;
  if (!classify(T, dv, S, careful, lane, lsm)) return false;
  uint64_t* tab = reinterpret_cast<uint64_t*>(region + tab_off);
  int next = 0, nsp = 0, rlo = -1;
  uint64_t cur = sizeof(StHdr);
  for (;;) {
    if (cur + 4ull * (L - (uint64_t)next) + 128 > sizeof(StHdr) + tc || (uint64_t)nsp >= ns) return false;
    int ul = 0, st = 0;
    const int tb = dv.hp ? next_span<false, true>(T, dv, S, region + cur, next, ul, st, lane, nullptr, nullptr, nullptr,
                                                  lsm, &rlo)
                         : next_span<false>(T, dv, S, region + cur, next, ul, st, lane, nullptr, nullptr, nullptr, lsm);
    if (st == 0) break;
    if (st < 0) return false;
    if (tb > 2048 && squeeze_trigger(S, region + cur, careful, lane)) return false;   // the Squeeze restart
    if (lane == 0) tab[nsp] = cur | ((uint64_t)(uint32_t)tb << 32) | ((uint64_t)(uint32_t)ul << 56);
    ++nsp;
    cur += (uint64_t)st_advance(tb);
  }
  gsync();
  uint32_t par = 0;
  if (nsp > par_min) {
    par = (uint32_t)par_off;
    if (lane == 0) {
      uint32_t* roff = reinterpret_cast<uint32_t*>(region + par);
      uint32_t acc = 0;
      for (int j = 0; j < nsp; ++j) {
        roff[j] = acc;
        acc += (uint32_t)(((tab[j] >> 32) & 0xFFFFFF) / 16 + 8);
      }
      roff[nsp] = acc;
    }
  }
  if (lane == 0) {
    StHdr h{(uint32_t)nsp, careful ? 1u : 0u, (uint32_t)tab_off, par};
    *reinterpret_cast<StHdr*>(region) = h;
  }
  gsync();
  return true;
}

// One pass over a document's stored spans: detect()'s span loop (scoring
// part) and the document level.  rep: pass 2 (Repeats|Finish), the spans
// already through st_rep.  Returns 1 (result written), 0 (pass 1 not good
// enough: pass 2 follows) or -kWhyCapacity.
template <class SM>
__device__ __forceinline__ int st_score(const DevTables& T, Slot& S, SM& s, const uint8_t* region, bool rep, cld_result* out,
                        uint32_t cflags, const uint32_t* __restrict__ pri, int lane) {
  if (lane == 0) s.has_pri = pri != nullptr;
  if (lane < 16) {
    const uint32_t lp = pri ? gld(pri + lane) : 0u;
    if (lane < 8) s.pri_add[lane >> 2][lane & 3] = lp ? tote_adds(T, lp) : 0ull;
    else s.pri_wk[(lane - 8) >> 2][lane & 3] = (uint8_t)((lp >> 8) & 0xFF);
  }
  if (lane == 0) s.dt.init();
  if (lane < 8) s.ring[lane >> 2][lane & 3] = 0;
  wsync();
  const StHdr* h = reinterpret_cast<const StHdr*>(region);
  const int nsp = (int)uflu(gld(&h->nsp));
  const uint64_t* tab = reinterpret_cast<const uint64_t*>(region + uflu(gld(&h->tab)));
  int total = 0;
  for (int j = 0; j < nsp; ++j) {
    const uint64_t e = ufl64(gld(tab + j));
    const uint8_t* lb = region + (uint32_t)e;
    const int tb = (int)((e >> 32) & 0xFFFFFF), ul = (int)(e >> 56);
    bool ok;
    if (tb + 48 <= (int)sizeof(s.text)) {
      const int n16 = (tb + 48 + 15) >> 4;
      for (int i = lane; i < n16; i += 64)
        reinterpret_cast<uint4*>(s.text)[i] = gld4(reinterpret_cast<const uint32_t*>(lb) + 4 * i);
      wsync();
      Win win{nullptr, 0, 16 * n16, 16 * n16};
      ok = score_span<false, false>(T, S, s, win, tb, ul, lane, nullptr, 0, cflags, nullptr);
    } else {
      Win win{lb, 0, 0, (tb + 48 + 15) & ~15};
      ok = score_span<false, false>(T, S, s, win, tb, ul, lane, nullptr, 0, cflags, nullptr);
    }
    if (!ok) return -kWhyCapacity;
    total += tb;
  }
  return wave::finish_document(T, s.dt, total, rep, out, lane, (cflags & kCLDFlagBestEffort) != 0);
}

// CheapRepWordsInplace over a document's stored spans, in order, one
// predictor for the document (detect()'s from_cache pass 2).  False: a span
// the in-place formulation cannot take (the fused k_long redoes the document).
__device__ __forceinline__ bool st_rep(uint16_t* tbl, Slot& S, uint8_t* region, int lane) {
  StHdr* h = reinterpret_cast<StHdr*>(region);
  const int nsp = (int)uflu(gld(&h->nsp));
  const bool careful = uflu(gld(&h->careful)) != 0;
  uint64_t* tab = reinterpret_cast<uint64_t*>(region + uflu(gld(&h->tab)));
  for (int i = lane; i < kPredictionTableSize / 8; i += 64) reinterpret_cast<uint4*>(tbl)[i] = make_uint4(0, 0, 0, 0);
  wsync();
  uint32_t hcarry = 0;
  for (int j = 0; j < nsp; ++j) {
    const uint64_t e = ufl64(gld(tab + j));
    bool okr;
    const int tb = rep_span_lds(tbl, S.pred, region + (uint32_t)e, (int)((e >> 32) & 0xFFFFFF), hcarry, careful, okr,
                                lane);
    if (!okr) return false;
    if (lane == 0) tab[j] = (e & ~(0xFFFFFFull << 32)) | ((uint64_t)(uint32_t)tb << 32);
  }
  gsync();
  return true;
}

// ------------------------------------------------ span-parallel scoring
// A span costs a wave ~15 us per pass whatever its length (every stage is a
// chain of dependent steps), so a document of thousands of short spans --
// scripts alternating word by word -- takes one wave tens of milliseconds
// (a 64 KB page of 3,082 spans: 48 ms; profiles/round5_doc_latency.jsonl), and
// every launch holding one waits for it.  Within a pass the spans depend on
// each other only through the DocTote (adds in span order) and the boost ring
// of each script class (the last four distinct-hit langprobs,
// scoreonescriptspan.cc:112-152, 305-315).  So a document of more than
// kParMin spans is scored kParG spans per wave (k_lgroup, st_group):
//   * a group's entering ring, per class its spans use, is the last four
//     distinct emissions of the earlier spans of that class: they come from
//     re-running the hit rounds (no scoring) of those spans, newest first,
//     until four are found or the document start is reached (span_distinct);
//   * the group's spans are then scored as one wave would, the ring carried
//     from span to span, and their DocTote adds recorded in order (REC);
//   * k_lfinish replays every span's adds into the DocTote in span order and
//     runs the document level (st_par_finish).
// Scoring is a function of the span text, the entering ring and the priors,
// so the result is what one wave scoring the spans in order computes.

// The rtype a stored span is scored with (score_span).
__device__ __forceinline__ int span_rt(const DevTables& T, int ul, uint32_t cflags) {
  int rt = rtype_of(T, ul);
  if ((cflags & kCLDFlagScoreAsQuads) && rt != RTypeCJK) rt = RTypeMany;
  return rt;
}

// A round's last (up to) four distinct emissions into last[] (newest at [3]).
__device__ __forceinline__ void take_distinct(const Slot& S, int exm, uint32_t (&last)[4], int& cnt) {
  for (int i = exm - 4 < 0 ? 0 : exm - 4; i < exm; ++i) {
    last[0] = last[1];
    last[1] = last[2];
    last[2] = last[3];
    last[3] = uflu(gld(&S.x_ai[i]));
    ++cnt;
  }
}

// The distinct emissions of one stored span (its hit rounds, no scoring):
// the last four as tote adds into ring[idx-4 .. idx) going backwards -- the
// newest is written at ring[idx - 1] -- until idx reaches 0.
template <class SM>
__device__ __forceinline__ bool span_distinct(const DevTables& T, Slot& S, SM& s, const uint8_t* lb, int tb, int rt,
                                              uint64_t* ring, int& idx, int lane) {
  if (rt == RTypeNone || rt == RTypeOne || tb <= 1) return true;
  bool ok = true;
  Win win{lb, 0, 0, (tb + 48 + 15) & ~15};
  if (tb + 48 <= (int)sizeof(s.text)) {
    const int n16 = (tb + 48 + 15) >> 4;
    for (int i = lane; i < n16; i += 64)
      reinterpret_cast<uint4*>(s.text)[i] = gld4(reinterpret_cast<const uint32_t*>(lb) + 4 * i);
    wsync();
    win = Win{nullptr, 0, 16 * n16, 16 * n16};
  }
  // the rounds' distinct emissions, newest last; kept: the last four overall
  uint32_t last[4] = {0, 0, 0, 0};               // adds indices, newest at [3]
  int cnt = 0;
  int off = 1;
  if (rt == RTypeCJK) {
    while (off < tb) {
      int nb, nd, nx, eb, edm, exm;
      const int next = cjk_round<false>(T, win, s, tb, S, off, nb, nd, nx, eb, edm, exm, ok, lane);
      if (!ok) return false;
      take_distinct(S, exm, last, cnt);
      off = next;
    }
  } else {
    const int start = 1 + (ufl(win_text(win, s, 0, 2, ok, lane)[1]) == ' ' ? 1 : 0);
    int nws, nsp;
    if (!ok || !word_lists(win, s, tb, start, S, nws, nsp, lane)) return false;
    const int nch = build_chain(win, s, tb, S, nws, lane);
    if (nch < 0) return false;
    int c0 = 0, j0 = 0;
    while (off < tb) {
      int nb, nd, nx, eb, edm, exm;
      const int next = quad_round<false>(T, win, s, tb, S, nch, c0, nb, eb, ok, lane);
      if (!ok) return false;
      octa_round<false>(T, win, s, S, nsp, j0, off, next, nd, nx, edm, exm, ok, lane);
      if (!ok) return false;
      take_distinct(S, exm, last, cnt);
      off = next;
    }
  }
  const int n = cnt < 4 ? cnt : 4;
  for (int i = 0; i < n && idx > 0; ++i) {
    --idx;
    if (lane == 0) ring[idx] = adds_by_index(T, last[3 - i]);
  }
  return true;
}

// Group [j0, j1) of a span-parallel document: priors, the entering rings
// (lookback), then the spans scored in order with their DocTote adds
// recorded.  Returns 1, or -kWhyCapacity (the fused kernel redoes it).
template <class SM>
__device__ __forceinline__ int st_group(const DevTables& T, Slot& S, SM& s, uint8_t* region, int j0, int j1,
                                        uint32_t cflags, const uint32_t* __restrict__ pri, int lane) {
  if (lane == 0) s.has_pri = pri != nullptr;
  if (lane < 16) {
    const uint32_t lp = pri ? gld(pri + lane) : 0u;
    if (lane < 8) s.pri_add[lane >> 2][lane & 3] = lp ? tote_adds(T, lp) : 0ull;
    else s.pri_wk[(lane - 8) >> 2][lane & 3] = (uint8_t)((lp >> 8) & 0xFF);
  }
  if (lane < 8) s.ring[lane >> 2][lane & 3] = 0;
  wsync();
  const StHdr* h = reinterpret_cast<const StHdr*>(region);
  const uint64_t* tab = reinterpret_cast<const uint64_t*>(region + uflu(gld(&h->tab)));
  const uint32_t par = uflu(gld(&h->par));
  const uint32_t* roff = reinterpret_cast<const uint32_t*>(region + par);
  const int nsp = (int)uflu(gld(&h->nsp));
  uint32_t* rcnt = const_cast<uint32_t*>(roff) + nsp + 1;
  uint64_t* recs = reinterpret_cast<uint64_t*>(region + ((par + 4ull * (2 * nsp + 1) + 7) & ~7ull));
  // the classes the group's scored spans use
  bool need[2] = {false, false};
  for (int j = j0; j < j1; ++j) {
    const uint64_t e = ufl64(gld(tab + j));
    const int ul = (int)(e >> 56), rt = span_rt(T, ul, cflags);
    if (rt == RTypeMany || rt == RTypeCJK) need[((uint32_t)ul == T.latin) ? 0 : 1] = true;
  }
  int idx[2] = {need[0] ? 4 : 0, need[1] ? 4 : 0};
  for (int j = j0 - 1; j >= 0 && (idx[0] > 0 || idx[1] > 0); --j) {
    const uint64_t e = ufl64(gld(tab + j));
    const int ul = (int)(e >> 56), tb = (int)((e >> 32) & 0xFFFFFF), rt = span_rt(T, ul, cflags);
    const int rs = ((uint32_t)ul == T.latin) ? 0 : 1;
    if (idx[rs] == 0 || !(rt == RTypeMany || rt == RTypeCJK)) continue;
    if (!span_distinct(T, S, s, region + (uint32_t)e, tb, rt, s.ring[rs], idx[rs], lane)) {
      if (lane == 0) rcnt[j0] = 0xFFFFFFFFu;
      gsync();
      return -kWhyCapacity;
    }
  }
  wsync();
  for (int j = j0; j < j1; ++j) {
    const uint64_t e = ufl64(gld(tab + j));
    const uint8_t* lb = region + (uint32_t)e;
    const int tb = (int)((e >> 32) & 0xFFFFFF), ul = (int)(e >> 56);
    if (lane == 0) {
      const uint32_t r0 = gld(roff + j);
      s.rec = recs + r0;
      s.rec_cap = gld(roff + j + 1) - r0;
      s.rec_n = 0;
      s.rec_over = 0;
    }
    wsync();
    bool ok;
    if (tb + 48 <= (int)sizeof(s.text)) {
      const int n16 = (tb + 48 + 15) >> 4;
      for (int i = lane; i < n16; i += 64)
        reinterpret_cast<uint4*>(s.text)[i] = gld4(reinterpret_cast<const uint32_t*>(lb) + 4 * i);
      wsync();
      Win win{nullptr, 0, 16 * n16, 16 * n16};
      ok = score_span<false, false>(T, S, s, win, tb, ul, lane, nullptr, 0, cflags, nullptr);
    } else {
      Win win{lb, 0, 0, (tb + 48 + 15) & ~15};
      ok = score_span<false, false>(T, S, s, win, tb, ul, lane, nullptr, 0, cflags, nullptr);
    }
    if (!ok) {
      if (lane == 0) rcnt[j0] = 0xFFFFFFFFu;     // the document's finish hands it to the fused kernel
      gsync();
      return -kWhyCapacity;
    }
    if (lane == 0) rcnt[j] = s.rec_over ? 0xFFFFFFFFu : s.rec_n;
  }
  gsync();
  return 1;
}

// The document level of a span-parallel document: every span's recorded
// adds into the DocTote in span order, then finish_document.  Returns as
// st_score; -kWhyCapacity when a span's adds outgrew their room.
template <class SM>
__device__ __forceinline__ int st_par_finish(const DevTables& T, SM& s, const uint8_t* region, bool rep,
                                             cld_result* out, uint32_t cflags, int lane) {
  const StHdr* h = reinterpret_cast<const StHdr*>(region);
  const uint64_t* tab = reinterpret_cast<const uint64_t*>(region + uflu(gld(&h->tab)));
  const uint32_t par = uflu(gld(&h->par));
  const uint32_t* roff = reinterpret_cast<const uint32_t*>(region + par);
  const int nsp = (int)uflu(gld(&h->nsp));
  const uint32_t* rcnt = roff + nsp + 1;
  const uint64_t* recs = reinterpret_cast<const uint64_t*>(region + ((par + 4ull * (2 * nsp + 1) + 7) & ~7ull));
  int total = 0, bad = 0;
  for (int j0 = 0; j0 < nsp; j0 += 64) {
    const int j = j0 + lane;
    int tb = 0;
    if (j < nsp) {
      tb = (int)((gld(tab + j) >> 32) & 0xFFFFFF);
      bad |= gld(rcnt + j) == 0xFFFFFFFFu;
    }
    total += (int)wave::wsum((uint32_t)tb);
  }
  if (__ballot(bad != 0)) return -kWhyCapacity;
  if (lane == 0) {
    s.dt.init();
    for (int j = 0; j < nsp; ++j) {
      const uint32_t r0 = roff[j], n = rcnt[j];
      for (uint32_t k = 0; k < n; ++k) {
        const uint64_t r = recs[r0 + k];
        s.dt.add((uint16_t)(r & 0xFFFF), (int)((r >> 16) & 0xFFFF), (int)((r >> 32) & 0xFFFF), (int)((r >> 48) & 0xFF));
      }
    }
  }
  wsync();
  return wave::finish_document(T, s.dt, total, rep, out, lane, (cflags & kCLDFlagBestEffort) != 0);
}

// The fused span builder emits separators and pads as ' ' without lowering
// them; that is exact only if the lowercaser maps ' ' to itself.
__device__ bool space_lowers_to_space(const DevTables& T) {
  const uint8_t sp = ' ';
  uint64_t o = 0;
  int olen = 0;
  return lower_char(T, &sp, 1, o, olen) && olen == 1 && o == (uint64_t)' ';
}

}  // namespace lng
}  // namespace cld
