// cld_wave.hip -- one wavefront per document (documents of <= CAP bytes).
//
// The lane-per-document front end keeps ~8 KB of per-document state in
// private memory; on gfx950 that is scratch, and a launch over 1M tweets moved
// ~13 GB of scratch through HBM (profiles/round1a_c2_pmc_*.csv).  Here the 64
// lanes of a wavefront share one document, its state sits in LDS (~7 KB per
// wave), and every stage that is data-parallel in the reference runs across
// lanes:
//
//   stage                         reference                      across lanes
//   load + per-byte script/scan   getonescriptspan.cc:480-485,   bytes
//                                 utf8statetable.cc:362-554
//   span runs (GetOneScriptSpan)  getonescriptspan.cc:799-1027   64-bit ballot masks +
//                                                                scalar bit scans
//   LowerScriptSpan               utf8statetable.cc:608-867      characters + prefix sum
//   GetQuadHits chain             cldutil.cc:315-405             next[] per byte, scalar walk,
//                                                                hashes/probes per quad
//   GetOctaHits                   cldutil.cc:416-533             words (scalar repeat filter)
//   GetUniHits / GetBiHits        cldutil.cc:201-310             characters
//   LinearizeAll + ChunkAll       scoreonescriptspan.cc:856-1031 emissions: chunk id by
//                                                                rank arithmetic (no merge)
//   ScoreOneChunk / boosts        scoreonescriptspan.cc:208-302  LDS atomics into a u32 tote,
//                                                                3x wave argmax for top-3
//   DocTote / summary             tote.cc, compact_lang_det_impl lane 0 (a few dozen ops)
//
// A document the wave cannot reproduce exactly in this form (longer than CAP,
// a byte sequence whose scanner/lowercaser state crosses a character
// boundary, a bucket overflow, or a second pass) is appended to the re-queue
// list and redone from scratch by k_long, so results stay
// bit-identical to the sequential restatement in every case.

namespace cld {
namespace wave {


__device__ __forceinline__ int ufl(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint32_t uflu(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }
__device__ __forceinline__ uint64_t ufl64(uint64_t v) {
  return ((uint64_t)uflu((uint32_t)(v >> 32)) << 32) | uflu((uint32_t)v);
}
__device__ __forceinline__ int rdl(int v, int l) { return __builtin_amdgcn_readlane(v, l); }
__device__ __forceinline__ uint32_t rdlu(uint32_t v, int l) { return (uint32_t)__builtin_amdgcn_readlane((int)v, l); }
__device__ __forceinline__ uint64_t rdl64(uint64_t v, int l) {
  return ((uint64_t)rdlu((uint32_t)(v >> 32), l) << 32) | rdlu((uint32_t)v, l);
}


// Order LDS traffic between lanes of one wavefront (no workgroup barrier:
// the waves of a workgroup work on different documents).
__device__ __forceinline__ void wsync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ uint64_t lanemask_lt(int lane) { return lane ? (~0ull >> (64 - lane)) : 0ull; }
// The lane id recomputed where a stage starts (v_mbcnt, as volatile asm): the
// compiler would otherwise hoist the per-lane values derived from it out of
// the document's span loop and spill them to scratch (8 waves/SIMD leave 64
// VGPRs), a scratch write per lane and document.
__device__ __forceinline__ int lane_here() {
  int l;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
  return l;
}

// Register arrays indexed by a wave-uniform register number r (entry i of a
// 64*N list lives in lane i&63 of register i>>6).
template <int N, class V>
__device__ __forceinline__ V pick(const V (&a)[N], int r) {
  V v = a[0];
#pragma unroll
  for (int i = 1; i < N; ++i) if (r == i) v = a[i];
  return v;
}
template <int N, class V>
__device__ __forceinline__ void put_lane(V (&a)[N], int r, int l, V val) {
  const bool me = (int)__lane_id() == l;
#pragma unroll
  for (int i = 0; i < N; ++i)
    if (r == i && me) a[i] = val;
}
template <int N>
__device__ __forceinline__ void or_bit(uint64_t (&a)[N], int r, int l) {
#pragma unroll
  for (int i = 0; i < N; ++i) if (r == i) a[i] |= 1ull << l;
}

// Wavefront scans and reductions on DPP (no LDS round trip): Hillis-Steele
// inside each 16-lane row (row_shr 1, 2, 4, 8), then row 0's total into row 1
// and row 2's into row 3 (row_bcast:15), then lane 31 into rows 2-3
// (row_bcast:31).  Lanes without a source keep the identity (bound_ctrl off,
// old = identity).  Called with all 64 lanes active.
constexpr int kDppRowShr = 0x110, kDppRowBcast15 = 0x142, kDppRowBcast31 = 0x143;
template <class Op>
__device__ __forceinline__ uint32_t dpp_scan_incl(uint32_t x, uint32_t id, Op op) {
  const int xi = (int)x;
  x = op(x, (uint32_t)__builtin_amdgcn_update_dpp((int)id, xi, kDppRowShr | 1, 0xF, 0xF, false));
  x = op(x, (uint32_t)__builtin_amdgcn_update_dpp((int)id, (int)x, kDppRowShr | 2, 0xF, 0xF, false));
  x = op(x, (uint32_t)__builtin_amdgcn_update_dpp((int)id, (int)x, kDppRowShr | 4, 0xF, 0xF, false));
  x = op(x, (uint32_t)__builtin_amdgcn_update_dpp((int)id, (int)x, kDppRowShr | 8, 0xF, 0xF, false));
  x = op(x, (uint32_t)__builtin_amdgcn_update_dpp((int)id, (int)x, kDppRowBcast15, 0xA, 0xF, false));
  x = op(x, (uint32_t)__builtin_amdgcn_update_dpp((int)id, (int)x, kDppRowBcast31, 0xC, 0xF, false));
  return x;
}
struct OpAdd { __device__ uint32_t operator()(uint32_t a, uint32_t b) const { return a + b; } };
struct OpMax { __device__ uint32_t operator()(uint32_t a, uint32_t b) const { return a > b ? a : b; } };
struct OpMin { __device__ uint32_t operator()(uint32_t a, uint32_t b) const { return a < b ? a : b; } };
struct OpOr { __device__ uint32_t operator()(uint32_t a, uint32_t b) const { return a | b; } };

// Value of lane-1 (wave_shr:1); lane 0 gets `first`.
constexpr int kDppWaveShr1 = 0x138, kDppWaveShl1 = 0x130;
__device__ __forceinline__ uint32_t wshr1(uint32_t x, uint32_t first) {
  return (uint32_t)__builtin_amdgcn_update_dpp((int)first, (int)x, kDppWaveShr1, 0xF, 0xF, false);
}
__device__ __forceinline__ uint64_t wshr1_64(uint64_t x) {
  return ((uint64_t)wshr1((uint32_t)(x >> 32), (uint32_t)(x >> 32)) << 32) | wshr1((uint32_t)x, (uint32_t)x);
}

__device__ __forceinline__ int excl_scan(int v, int lane) {
  (void)lane;
  return (int)dpp_scan_incl((uint32_t)v, 0u, OpAdd()) - v;
}
__device__ __forceinline__ int wsum(int v) { return rdl((int)dpp_scan_incl((uint32_t)v, 0u, OpAdd()), 63); }
__device__ __forceinline__ uint32_t wmax(uint32_t v) { return rdlu(dpp_scan_incl(v, 0u, OpMax()), 63); }
__device__ __forceinline__ uint32_t wmin(uint32_t v) { return rdlu(dpp_scan_incl(v, 0xFFFFFFFFu, OpMin()), 63); }
__device__ __forceinline__ uint64_t wor64(uint64_t v) {
  const uint32_t lo = rdlu(dpp_scan_incl((uint32_t)v, 0u, OpOr()), 63);
  const uint32_t hi = rdlu(dpp_scan_incl((uint32_t)(v >> 32), 0u, OpOr()), 63);
  return ((uint64_t)hi << 32) | lo;
}

// Per-wave capacities for documents of at most CAP bytes.  Anything that
// would overflow them is re-queued, never truncated.
template <int CAP>
struct Cfg {
  static constexpr int DOC = CAP + 32;              // document + NUL padding (DocView semantics)
  static constexpr int NM = (CAP + 63) / 64;        // 64-bit mask words over document bytes
  static constexpr int SB = CAP + 72;               // span text: ' ' + letters/single spaces + "   \0"
  static constexpr int LB = (SB * 3) / 2 + 64;      // lowered span (max per-char growth 1.5x) + hash read pad
  static constexpr int NR = 2;                      // registers of 64 entries: quad chain, words
  static constexpr int NB = NR * 64;                // base hits / quad chain / words
  static constexpr int QM = ((LB + 63) / 64) * 2;   // u32 words of chain marks (whole u64 windows)
  static constexpr int NE = 160;                    // base emissions (<= 2 langprobs per hit; overflow requeues)
  static constexpr int ND = 96;
  static constexpr int NX = 160;
  static constexpr int MAXCH = NE / kChunksizeQuads + 3;
  static_assert(NB < kMaxScoringHits - 1, "a round must never reach the reference's hit cap");
  static_assert(CAP < 2048, "spans of a short document can never reach the squeeze test");
  // Packed tote (kToteNoCarry): a key's 16-bit half can neither wrap nor
  // carry into its neighbour when every add is <= kMaxLgProbScore (the host
  // checks the table at load) and a chunk holds at most NE + ND + NX + 1
  // emissions plus 4 distinct boosts and 4 prior boosts.
  static_assert((NE + ND + NX + 9) * kMaxLgProbScore < 65536, "tote headroom");
};

template <int CAP>
struct Smem {
  using C = Cfg<CAP>;
  uint8_t doc[C::DOC];
  uint8_t sn[C::DOC];                 // script number at each byte position (GetUTF8LetterScriptNum)
  uint64_t lsm[C::NM];                // letter stops: char start, scanner stops there, script != 0
  uint64_t ent[C::NM];                // rewritten HTML (cld_html.hip): lookaheads here see script 0
  union alignas(16) {                 // one span's life: raw text -> base hits -> chunk ids
    uint8_t sbuf[C::SB];              //   span text (raw); dead once lowered
    struct {                          //   quad chain (quad_hits, before its base hits are written)
      uint32_t qmark[C::QM];          //   chain entries as bits over lowered-text positions
      uint16_t qws[C::NB];            //   word starts
      uint16_t qchn[C::NB];           //   chain entries, in order
    };
    struct {                          //   base hits before expansion (hit streams -> scoring)
      uint32_t b_ind[C::NB];
      uint16_t b_off[C::NB];
    };
    struct {                          //   chunk plan, written after the base hits are expanded:
      int32_t theta[C::MAXCH];        //   chunk k takes delta/distinct emissions at offset <= theta_k
      uint16_t st[3][C::MAXCH + 1];   //   first base / delta / distinct emission of chunk k
    };
  };
  union alignas(16) {                 // scoring reads only hit offsets, never the span text:
    uint8_t lbuf[C::LB];              //   lowered span text
    uint32_t tote[128];               //   chunk tote: two 16-bit keys per word (see kToteNoCarry)
  };
  union alignas(16) {                 // stage-local arrays
    uint16_t nx[CAP];                 // load: p + ScanToLetterOrSpecial(p, L - p)
    uint16_t nxq[C::LB];              // quad hits: next quad start for a quad starting at p
    uint16_t wsp[C::NB + 1];          // octa hits: word-ending spaces
    struct {                          // scoring: base emissions (offset, langprob), linear order
      uint32_t be_lp[C::NE];
      uint16_t be_off[C::NE + 1];
    } e;
  } a;
  uint16_t d_off[C::ND]; uint32_t d_ind[C::ND];   // delta hits; compacted in place to emissions
  uint16_t x_off[C::NX]; uint32_t x_ind[C::NX];   // distinct hits; likewise
  uint16_t E[C::MAXCH];               // cumulative base-emission count closing each chunk
  uint32_t lo[C::MAXCH];
  uint32_t ring[2][4];                // distinct boosts, latn / othr, oldest first
  DocTote dt;
};

// -------------------------------------------------------------- bit scans
template <int NM>
__device__ __forceinline__ int find_first(const uint64_t* m, int from, int L) {
  if (from >= L) return L;
  int w = from >> 6;
  uint64_t x = ufl64(m[w]) & (~0ull << (from & 63));
  for (;;) {
    if (x) { int r = (w << 6) + __builtin_ctzll(x); return r < L ? r : L; }
    ++w;
    if (w >= NM || (w << 6) >= L) return L;
    x = ufl64(m[w]);
  }
}

// Index of a 1-3 byte sequence in the per-character property table T.cpt
// (built on device by k_build_cpt from lng::cpt_eval; layout in cld_long.hip):
// bits 0-7 script, 8-9 scan class (0 continue, 1 stop, 3 non-local), 10
// lowerable with <= 4 output bytes, 11-14 lowered length, 32-63 lowered bytes.
__device__ __forceinline__ int cpt_index(uint32_t b0, uint32_t b1, uint32_t b2, int n) {
  if (n == 1) return (int)b0;
  if (n == 2) return 128 + (int)((b0 & 0x1F) << 6 | (b1 & 0x3F));
  return 2176 + (int)((b0 & 0x0F) << 12 | (b1 & 0x3F) << 6 | (b2 & 0x3F));
}

// ------------------------------------------------------- stage 0: document
// Loads the document, computes script numbers and scanner stops per byte
// and checks that the per-character formulation below reproduces the
// sequential scanner: the document tiles into lead+continuation characters
// and a scan started at any character either stops on it or continues to the
// scan result of the next character.
template <int CAP>
__device__ bool load_document(const DevTables& T, const uint8_t* __restrict__ g, int L, Smem<CAP>& s, int lane,
                              const uint8_t* __restrict__ hf) {
  using C = Cfg<CAP>;
  static_assert(CAP == 256 && C::DOC == 288, "one aligned dword per lane covers the document");
  {
    // aligned dword loads of only the words that overlap [g, g+L) (never past
    // the buffer), realigned with the next lane's word, bytes >= L zeroed
    const uintptr_t ga = reinterpret_cast<uintptr_t>(g);
    const int sh = (int)(ga & 3);
    const uint32_t* gw = reinterpret_cast<const uint32_t*>(ga - (uintptr_t)sh);
    const int nw = (L + sh + 3) >> 2;                    // <= 65
    const uint32_t w0 = lane < nw ? gld(gw + lane) : 0u;     // (gld: global, not FLAT, loads)
    const uint32_t w64 = nw > 64 ? gld(gw + 64) : 0u;
    // lane + 1's word (DPP wave_shl:1); lane 63 keeps `old` = word 64
    const uint32_t nxt = (uint32_t)__builtin_amdgcn_update_dpp((int)w64, (int)w0, kDppWaveShl1, 0xF, 0xF, false);
    const uint32_t v = sh == 0 ? w0 : __builtin_amdgcn_alignbyte(nxt, w0, (uint32_t)sh);
    const int nb = L - 4 * lane;
    const uint32_t keep = nb >= 4 ? 0xFFFFFFFFu : nb <= 0 ? 0u : (1u << (8 * nb)) - 1u;
    reinterpret_cast<uint32_t*>(s.doc)[lane] = v & keep;
    if (lane < (C::DOC - 256) / 4) reinterpret_cast<uint32_t*>(s.doc)[64 + lane] = 0u;
    // a rewritten HTML page's lookahead marks (one byte per position), else none
    if (hf) {
      for (int w = 0; w < C::NM; ++w) {
        const uint64_t m = __ballot(w * 64 + lane < L && gld(hf + w * 64 + lane) != 0);
        if (lane == 0) s.ent[w] = m;
      }
    } else if (lane < C::NM) {
      s.ent[lane] = 0ull;
    }
  }
  wsync();
  DocView dv{s.doc, L};
  // Fast path: every character is a complete, well-formed 1-3 byte sequence
  // whose scanner class is local (continue or stop) -- then one property-table
  // lookup per character gives its script and whether the scan stops on it,
  // the same per-character formulation k_long's classify() uses.  Anything
  // else takes the state-machine path below, unchanged.
  {
    int slow = 0, conts = 0, need = 0;
    // every window's property gathers are issued before any is used: one L2
    // round trip for the document instead of one per 64-byte window
    int idx[C::NM];
#pragma unroll
    for (int w = 0; w < C::NM; ++w) idx[w] = -1;
#pragma unroll
    for (int w = 0; w < C::NM; ++w) {
      if (w * 64 >= L) break;                           // (uniform)
      // branch-free per byte: the document is zero-padded to DOC bytes
      const int p = w * 64 + lane;
      const uint32_t c = s.doc[p], b1 = s.doc[p + 1], b2 = s.doc[p + 2];
      const bool in = p < L;
      const bool cont = in && (c & 0xC0) == 0x80, lead = in && !cont;
      const int n = utf8_len((uint8_t)c);
      const bool bad = lead && (n > 3 || p + n > L || (n >= 2 && (b1 & 0xC0) != 0x80) || (n == 3 && (b2 & 0xC0) != 0x80));
      conts += cont ? 1 : 0;
      slow |= bad ? 1 : 0;
      const bool ok = lead && !bad;
      need += ok ? n - 1 : 0;
      idx[w] = ok ? cpt_index(c, b1, b2, n) : -1;
    }
    uint64_t ev[C::NM];
#pragma unroll
    for (int w = 0; w < C::NM; ++w) ev[w] = idx[w] >= 0 ? gld(T.cpt + idx[w]) : 0ull;
#pragma unroll
    for (int w = 0; w < C::NM; ++w) {
      // script number at every byte (0 off the lead bytes: only lead bytes are read)
      const int p = w * 64 + lane;
      const uint64_t e = ev[w];
      const int st = (int)((e >> 8) & 3);
      slow |= st == 3 ? 1 : 0;
      s.sn[p] = (uint8_t)e;
      const uint64_t m = __ballot(st == 1 && (e & 0xFF) != 0);
      if (lane == 0) s.lsm[w] = m;                      // (a lane-indexed register array would live in scratch)
    }
    slow |= wsum(conts - need) != 0 ? 1 : 0;               // every continuation byte is claimed
    if (__ballot(slow != 0) == 0) {
      if (lane < 4) s.sn[L + lane] = (uint8_t)script_num(T, dv, L + lane);
      wsync();
      return true;
    }
  }
  for (int p = lane; p < L + 4; p += 64) s.sn[p] = (uint8_t)script_num(T, dv, p);
  for (int p = lane; p < L; p += 64) s.a.nx[p] = (uint16_t)(p + scan_to_letter_or_special(T, dv, p, L - p));
  wsync();
  int bad = 0, conts = 0, need = 0;
  for (int p = lane; p < L; p += 64) {
    uint8_t c = s.doc[p];
    if ((c & 0xC0) == 0x80) { ++conts; continue; }
    int n = utf8_len(c);
    if (p + n > L) { bad = 1; continue; }
    for (int k = 1; k < n; ++k) bad |= ((s.doc[p + k] & 0xC0) != 0x80);
    need += n - 1;
    int np = s.a.nx[p];
    if (np != p) {
      int q = p + n;
      int want = q >= L ? L : (int)s.a.nx[q];
      bad |= (np != want);
    }
  }
  bad |= (wsum(conts) != wsum(need)) ? 1 : 0;
  if (__ballot(bad != 0)) return false;
  for (int w = 0; w < C::NM; ++w) {
    int p = w * 64 + lane;
    bool ls = false;
    if (p < L) ls = ((s.doc[p] & 0xC0) != 0x80) && s.a.nx[p] == p && s.sn[p] != 0;
    uint64_t m = __ballot(ls);
    if (lane == 0) s.lsm[w] = m;
  }
  wsync();
  return true;
}

// ------------------------------------------------ stage 1: one script span
// GetOneScriptSpan (getonescriptspan.cc:799-1027, plain text) as runs:
// ' ' + run1 + ' ' + run2 + ' ' ... + runK + ' ' + "   \0".  A run starts at
// a letter stop of the span script (or Inherited) and ends at the first
// character the letters loop would break on; the gap after it is skipped to
// the next letter stop, which either continues the span or starts the next.
// Returns text_bytes (0 = no further span); *next advances like next_byte_.
template <int CAP>
__device__ int next_span(const DevTables& T, Smem<CAP>& s, int L, int& next, int& ulscript, int lane) {
  lane = lane_here();
  using C = Cfg<CAP>;
  const int common = (int)T.common, inherited = (int)T.inherited;
  const int q = find_first<C::NM>(s.lsm, next, L);
  if (q >= L) { next = L; return 0; }
  const int spanscript = ufl(s.sn[q]);
  ulscript = spanscript;
  // All lanes at once, one 64-byte window at a time.  Events: B = a character
  // the letters loop breaks on, O = a letter stop of the span script (or
  // Inherited), F = a letter stop of another script.  In a run only B matters
  // (it ends the run: ' '), in a gap only letter stops (O starts the next run,
  // F ends the span), and B and O never coincide -- so a byte is in a run iff
  // the last B/O event at or before it is an O (the carried state if none).
  if (lane == 0) s.sbuf[0] = ' ';
  int put = 1, take = L;
  bool run = true;                                   // q is an O event
  for (int w = q >> 6; w < C::NM && w * 64 < L; ++w) {
    const int x = w * 64 + lane;
    const bool valid = x >= q && x < L;
    const uint32_t c = valid ? s.doc[x] : 0u;
    const bool lead = valid && (c & 0xC0) != 0x80;
    bool brk = false, ok = false, foreign = false;
    if (lead) {
      const int sc = s.sn[x];
      if (sc != spanscript && sc != inherited) {
        if (sc == common) {
          brk = true;
        } else {
          // (a lookahead onto a rewritten HTML entity sees the raw '&': script 0)
          const int xn = x + utf8_len((uint8_t)c);
          const int sc2 = (xn < 64 * C::NM && ((s.ent[xn >> 6] >> (xn & 63)) & 1)) ? 0 : s.sn[xn];
          brk = sc2 != common && sc2 != spanscript;
        }
      }
      if ((s.lsm[w] >> lane) & 1) {
        if (sc == spanscript || sc == inherited) ok = true;
        else foreign = true;
      }
    }
    const uint64_t Bm = __ballot(brk), Om = __ballot(ok);
    const uint64_t evm = Bm | Om;
    const uint64_t ev_le = evm & (lane == 63 ? ~0ull : ((2ull << lane) - 1)), ev_lt = evm & lanemask_lt(lane);
    const bool inrun = ev_le ? ((Om >> (63 - __builtin_clzll(ev_le))) & 1) : run;
    const bool prev_run = ev_lt ? ((Om >> (63 - __builtin_clzll(ev_lt))) & 1) : run;
    const uint64_t Em = __ballot(foreign && (brk || !prev_run));   // F while in a gap: the span ends here
    const int stop = Em ? __builtin_ctzll(Em) : 64;
    const bool cp = valid && inrun && lane < stop;
    const bool sep = brk && prev_run && lane <= stop;
    const int cnt = (cp ? 1 : 0) + (sep ? 1 : 0);
    const int pos = put + excl_scan(cnt, lane);
    if (cp) s.sbuf[pos] = (uint8_t)c;
    if (sep) s.sbuf[pos] = ' ';
    put = rdl(pos + cnt, 63);
    if (stop < 64) {
      take = w * 64 + stop;
      run = false;
      break;
    }
    if (evm) run = (Om >> (63 - __builtin_clzll(evm))) & 1;
  }
  if (run) {                                         // the document ended inside a run
    if (lane == 0) s.sbuf[put] = ' ';
    ++put;
  }
  if (lane < 4) s.sbuf[put + lane] = lane < 3 ? ' ' : 0;
  next = take;
  wsync();
  return put;
}

// ------------------------------------------------ stage 2: lowercase
// One character through the utf8repl_lettermarklower machine
// (utf8statetable.cc:645-760), starting and -- checked -- ending in state 0,
// so the characters of the span can be lowered independently.  Output bytes
// are packed little-endian into *out.
__device__ __forceinline__ void setb(uint64_t& o, int i, uint32_t v) {
  o = (o & ~(0xFFull << (8 * i))) | ((uint64_t)(v & 0xFF) << (8 * i));
}
__device__ bool lower_char_sm(const DevSM& sm, const uint8_t* src, int n, uint64_t& out, int& olen) {
  const int sh = (int)sm.shift;
  const int nE = 1 << sh;
  const int64_t tb0 = sm.state0;
  int64_t tb = tb0;
  out = 0; olen = 0;
  for (int i = 0; i < n; ++i) {
    const uint8_t c = src[i];
    const int e = sm8(sm, tb + c);
    if (olen >= 8) return false;
    out |= (uint64_t)c << (8 * olen);
    ++olen;
    if (e < kExitIllegalStructure) { tb = tb0 + ((int64_t)e << sh); continue; }
    switch (e) {
      case kExitReplace31:
        if (olen < 3) return false;
        olen -= 2; setb(out, olen - 1, sm8(sm, tb + c + nE * 1));
        out &= olen >= 8 ? ~0ull : ((1ull << (8 * olen)) - 1);
        break;
      case kExitReplace32:
        if (olen < 3) return false;
        olen -= 1; setb(out, olen - 2, sm8(sm, tb + c + nE * 2)); setb(out, olen - 1, sm8(sm, tb + c + nE * 1));
        out &= (1ull << (8 * olen)) - 1;
        break;
      case kExitReplace21:
        if (olen < 2) return false;
        olen -= 1; setb(out, olen - 1, sm8(sm, tb + c + nE * 1));
        out &= (1ull << (8 * olen)) - 1;
        break;
      case kExitReplace3:
        if (olen < 3) return false;
        setb(out, olen - 3, sm8(sm, tb + c + nE * 3)); setb(out, olen - 2, sm8(sm, tb + c + nE * 2));
        setb(out, olen - 1, sm8(sm, tb + c + nE * 1));
        break;
      case kExitReplace2:
        if (olen < 2) return false;
        setb(out, olen - 2, sm8(sm, tb + c + nE * 2)); setb(out, olen - 1, sm8(sm, tb + c + nE * 1));
        break;
      case kExitReplace1:
        setb(out, olen - 1, sm8(sm, tb + c + nE * 1));
        break;
      case kExitReplace1S0:
        setb(out, olen - 1, sm8(sm, tb + c + 256 * 1));
        break;
      case kExitReplaceOffset2:
      case kExitSpecial:
      case kExitReplaceOffset1: {
        bool z = (nE != 256) && in_state_zero(sm, tb);
        int offset = 0;
        if (e == kExitReplaceOffset2) offset += (uint8_t)sm8(sm, tb + c + (z ? 256 : nE) * 2) << 8;
        offset += (uint8_t)sm8(sm, tb + c + (z ? 256 : nE) * 1);
        if ((uint32_t)offset >= sm.n_remap) return false;
        const uint8_t* re = sm.remap + 4 * offset;
        const int del = re[0] & 0x7F, add = re[1] & 0x7F, soff = re[2] | (re[3] << 8);
        if ((re[0] & 0x80) || del > olen || olen - del + add > 8) return false;
        olen -= del;
        out &= olen ? ((1ull << (8 * olen)) - 1) : 0ull;
        for (int k = 0; k < add; ++k) {
          uint32_t v = ((uint32_t)(soff + k) < sm.n_rstr) ? sm.rstr[soff + k] : 0u;
          out |= (uint64_t)v << (8 * olen);
          ++olen;
        }
        break;
      }
      default:
        return false;
    }
    tb = tb0;
  }
  if (tb != tb0) return false;
  // the output must itself tile into characters (hit scanners step by lead byte)
  for (int i = 0; i < olen;) {
    uint32_t b = (uint32_t)(out >> (8 * i)) & 0xFF;
    if ((b & 0xC0) == 0x80) return false;
    int m = utf8_len((uint8_t)b);
    if (i + m > olen) return false;
    for (int k = 1; k < m; ++k)
      if ((((uint32_t)(out >> (8 * (i + k)))) & 0xC0) != 0x80) return false;
    i += m;
  }
  return true;
}
__device__ __forceinline__ bool lower_char(const DevTables& T, const uint8_t* src, int n, uint64_t& out, int& olen) {
  return lower_char_sm(T.lower, src, n, out, olen);
}

// LowerScriptSpan (getonescriptspan.cc:1033-1054): returns text_bytes, or -1.
template <int CAP>
__device__ int lower_span(const DevTables& T, Smem<CAP>& s, int text_bytes, int lane) {
  lane = lane_here();
  using C = Cfg<CAP>;
  const int ilen = text_bytes + 3;
  int obase = 0;
  int bad = 0;
  for (int w0 = 0; w0 < ilen; w0 += 64) {
    const int p = w0 + lane;
    uint64_t o = 0;
    int olen = 0;
    if (p < ilen && (s.sbuf[p] & 0xC0) != 0x80) {
      // one property-table lookup per 1-3 byte character (the table holds
      // lower_char's result when it is <= 4 bytes); the machine otherwise
      const int n = utf8_len(s.sbuf[p]);
      const uint32_t b1 = s.sbuf[p + 1], b2 = s.sbuf[p + 2];
      const bool wf = n <= 3 && (n < 2 || (b1 & 0xC0) == 0x80) && (n < 3 || (b2 & 0xC0) == 0x80);
      const uint64_t e = wf ? T.cpt[cpt_index(s.sbuf[p], b1, b2, n)] : 0ull;
      if ((e >> 10) & 1) {
        olen = (int)((e >> 11) & 15);
        o = e >> 32;
      } else if (!lower_char(T, &s.sbuf[p], n, o, olen)) {
        bad = 1;
        olen = 0;
      }
    }
    const int pre = excl_scan(olen, lane);
    const int tot = rdl(pre + olen, 63);
    if (obase + tot + 4 > C::LB - 16) bad = 1;
    else
      for (int k = 0; k < olen; ++k) s.lbuf[obase + pre + k] = (uint8_t)(o >> (8 * k));
    obase += tot;
  }
  if (__ballot(bad != 0)) return -1;
  for (int k = lane; k < 20; k += 64) s.lbuf[obase + k] = 0;
  wsync();
  return obase - 3;
}

// QuadHashV2 (cldutil_shared.cc:167-202, the same arithmetic as quad_hash_v2)
// of the n bytes at LDS text position p: the words at p, p+4, p+8 from four
// aligned dword reads, the bytes before and after from two byte reads.
__device__ __forceinline__ uint32_t quad_hash_lds(const uint8_t* text, int p, int n) {
  const uint32_t* tw = reinterpret_cast<const uint32_t*>(text);
  const int i0 = p >> 2;
  const uint32_t sh = (uint32_t)(p & 3);
  const uint32_t x0 = tw[i0], x1 = tw[i0 + 1], x2 = tw[i0 + 2], x3 = tw[i0 + 3];
  const uint32_t y0 = __builtin_amdgcn_alignbyte(x1, x0, sh), y1 = __builtin_amdgcn_alignbyte(x2, x1, sh),
                 y2 = __builtin_amdgcn_alignbyte(x3, x2, sh);
  const uint32_t pre = (text[p - 1] == ' ' ? 0x00004444u : 0u) | (text[p + n] == ' ' ? 0x44440000u : 0u);
  const uint32_t m = (n & 3) ? (1u << (8 * (n & 3))) - 1u : 0xFFFFFFFFu;   // kWordMask0[n & 3]
  const uint32_t a0 = n <= 4 ? (y0 & m) : y0;
  const uint32_t w0 = (a0 ^ (a0 >> 3)) ^ pre;
  const uint32_t a1 = n <= 8 ? (y1 & m) : y1;
  const uint32_t w1 = a1 ^ (a1 << 4);
  const uint32_t a2 = y2 & m;
  const uint32_t w2 = a2 ^ (a2 << 2);
  const uint32_t r = n <= 4 ? w0 : n <= 8 ? w0 + w1 : w0 + w1 + w2;
  return n == 0 ? 0u : r;
}

// ------------------------------------------------ stage 3: hit streams
// GetQuadHits (cldutil.cc:315-405).  The chain of quad starts is a pure
// function of position, so next[] is computed for every byte in parallel and
// walked by scalar code; hashes and bucket probes run per quad; the
// "not one of the last two hits" filter is a scalar pass over the results.
// Returns the end offset (reference `next`), or -1 on overflow.
template <int CAP>
__device__ int quad_hits(const DevTables& T, Smem<CAP>& s, int limit, int& nb, int lane) {
  lane = lane_here();
  using C = Cfg<CAP>;
  const uint8_t* text = s.lbuf;
  int start = 1;
  if (text[start] == ' ') ++start;
  // The chain never jumps over a space: it enters every word at its first
  // byte, and a word's entries depend on that word alone (k_long's
  // build_chain).  First, for every text position at once, GetQuadHits'
  // step from there (cldutil.cc:340-400): the quad [p, p4) of four characters
  // (stopping at a space), the next chain position and whether the word's
  // chain ends at p -- packed as (p4 - p) | (next - p) << 5 | end << 10 --
  // and the word starts.  Then one lane walks one word on those steps, one
  // LDS read per entry, marking its entries as bits over text positions: in
  // text order the marks are the chain.
  uint16_t* nfo = s.a.nxq;
  int nws = 0;
  for (int w0 = start; w0 < limit; w0 += 64) {
    const int p = w0 + lane;
    const bool in = p < limit;
    const int pc = in ? p : start;
    const int a1 = pc + adv_but_space(text[pc]);
    const int a2 = a1 + adv_but_space(text[a1]);
    const uint32_t c2 = text[a2];
    const int a3 = a2 + adv_but_space((uint8_t)c2);
    const int a4 = a3 + adv_but_space(text[a3]);
    const int nx = a2 + adv_space_vowel((uint8_t)c2);
    const bool fin = text[a4] == ' ' || a2 >= limit || nx >= limit;
    if (in) nfo[p] = (uint16_t)((a4 - p) | ((nx - p) << 5) | (fin ? 0x400 : 0));
    const bool isws = in && (p == start || text[p - 1] == ' ');
    const uint64_t m = __ballot(isws);
    if (isws) {
      const int k = nws + __popcll(m & lanemask_lt(lane));
      if (k < C::NB) s.qws[k] = (uint16_t)p;
    }
    nws += __popcll(m);
  }
  if (nws > C::NB) return -1;
  if (lane < C::QM) s.qmark[lane] = 0u;
  wsync();
#pragma unroll
  for (int r = 0; r < C::NR; ++r) {
    if (r * 64 >= nws) break;
    const int i = r * 64 + lane;
    if (i < nws) {
      int p = s.qws[i];
      for (;;) {
        atomicOr(&s.qmark[p >> 5], 1u << (p & 31));
        const uint32_t f = nfo[p];
        if (f & 0x400) break;
        p += (f >> 5) & 31;
      }
    }
  }
  wsync();
  int n = 0;
  for (int w = start >> 6; w * 64 < limit; ++w) {
    const uint64_t m = ufl64(*reinterpret_cast<const uint64_t*>(&s.qmark[2 * w]));
    if ((m >> lane) & 1) {
      const int k = n + __popcll(m & lanemask_lt(lane));
      if (k < C::NB) s.qchn[k] = (uint16_t)(w * 64 + lane);
    }
    n += __popcll(m);
  }
  if (n > C::NB) return -1;
  wsync();
  int cp[C::NR];
#pragma unroll
  for (int r = 0; r < C::NR; ++r) cp[r] = s.qchn[r * 64 + lane];
  wsync();                               // (the base hits below overwrite the chain lists)
  const int end = n == 0 ? start : limit;
  // per register of chain entries, in order: hashes and probes, the repeat
  // filter (drop a hit equal to either of the last two kept hits), and the
  // ordered compaction of the kept hits -- one register's values live at a
  // time (the filter's state A, B and the compaction base carry over)
  uint32_t A = 0, B = 0;                  // last two kept hashes (the reference's pq0/pq1 as a set)
  int base = 0;
#pragma unroll
  for (int r = 0; r < C::NR; ++r) {
    if (r * 64 >= n) break;                // (uniform: registers past the chain hold nothing)
    const int i = r * 64 + lane;
    uint32_t hv = 0, pr = 0;
    bool hit = false;
    if (i < n) {
      const int p = cp[r];
      hv = quad_hash_lds(text, p, (int)(nfo[p] & 31));
      uint32_t ind = 0;
      hit = quad_probe(T.quad, T.quad2, hv, ind) != 0;
      pr = ind;
    }
    // Assume every hit is kept: then a hit's two predecessors are the previous
    // hit lanes; from the first hit that equals one of them, resolve in order.
    const uint64_t hm = __ballot(hit);
    const uint64_t hb = hm & lanemask_lt(lane);
    const int q1 = hb ? 63 - __builtin_clzll(hb) : -1;
    const uint64_t hb2 = q1 > 0 ? (hb & lanemask_lt(q1)) : 0ull;
    const int q2 = hb2 ? 63 - __builtin_clzll(hb2) : -1;
    const uint32_t h1 = (uint32_t)__shfl((int)hv, q1 < 0 ? lane : q1, 64);
    const uint32_t h2 = (uint32_t)__shfl((int)hv, q2 < 0 ? lane : q2, 64);
    const uint32_t a = q1 < 0 ? A : h1;
    const uint32_t b = q1 < 0 ? B : (q2 < 0 ? A : h2);
    const uint64_t cm = __ballot(hit && (hv == a || hv == b));
    uint64_t k = hm;
    if (cm) {
      const int f = __builtin_ctzll(cm);
      k = hm & lanemask_lt(f);
      uint32_t xA = rdlu(a, f), xB = rdlu(b, f);
      for (uint64_t rest = hm & ~lanemask_lt(f); rest; rest &= rest - 1) {
        const int l = __builtin_ctzll(rest);
        const uint32_t v = rdlu(hv, l);
        if (v == xA || v == xB) continue;
        xB = xA;
        xA = v;
        k |= 1ull << l;
      }
      A = xA;
      B = xB;
    } else if (hm) {
      const int t1 = 63 - __builtin_clzll(hm);
      const uint64_t r2 = hm & ~(1ull << t1);
      B = r2 ? rdlu(hv, 63 - __builtin_clzll(r2)) : A;
      A = rdlu(hv, t1);
    }
    if ((k >> lane) & 1) {
      const int kk = base + __popcll(k & lanemask_lt(lane));
      s.b_off[kk] = (uint16_t)cp[r];
      s.b_ind[kk] = pr;
    }
    base += __popcll(k);
  }
  nb = base;
  wsync();
  return end;
}

// GetOctaHits (cldutil.cc:416-533): one lane per space-terminated word.
template <int CAP>
__device__ bool octa_hits(const DevTables& T, Smem<CAP>& s, int limit_next, int& nd, int& nx, int lane) {
  lane = lane_here();
  using C = Cfg<CAP>;
  const uint8_t* text = s.lbuf;
  int start = 1;
  if (text[start] == ' ') ++start;
  const int lim = limit_next + 1;
  // word-ending spaces, in order
  int nw = 0;
  for (int w0 = start; w0 < lim; w0 += 64) {
    const int p = w0 + lane;
    const bool sp = p < lim && text[p] == ' ';
    const uint64_t m = __ballot(sp);
    if (sp) {
      int k = nw + __popcll(m & lanemask_lt(lane));
      if (k < C::NB) s.a.wsp[k] = (uint16_t)p;
    }
    nw += __popcll(m);
  }
  if (nw > C::NB) return false;
  wsync();
  uint64_t wh[C::NR];
  int ws[C::NR], pws[C::NR];
#pragma unroll
  for (int r = 0; r < C::NR; ++r) { wh[r] = 0; ws[r] = 0; pws[r] = 0; }
#pragma unroll
  for (int r = 0; r < C::NR; ++r) {
    if (r * 64 >= nw) break;
    const int i = r * 64 + lane;
    if (i < nw) {
      const int a = i == 0 ? start : s.a.wsp[i - 1] + 1;
      const int e = s.a.wsp[i];
      ws[r] = a;
      pws[r] = i <= 1 ? start : s.a.wsp[i - 2] + 1;
      int we = a, q = a, cc = 0;
      while (q < e) {
        ++cc;
        q += utf8_len(text[q]);
        if (cc <= 8) we = q;
        else break;
      }
      wh[r] = octa_hash40(text + a, we - a);
    }
  }
  // repeat filter (updates the pair partner even when probes miss): every word
  // takes part; assume none repeats, so a word's two predecessors are the
  // previous two lanes; from the first repeat, resolve in order.
  uint64_t keep[C::NR];
  uint32_t tlo[C::NR], thi[C::NR];        // pair partner = the previous kept word
  uint64_t A = 0, B = 0;                  // last two kept word hashes (po0/po1 as a set)
#pragma unroll
  for (int r = 0; r < C::NR; ++r) {
    const int i = r * 64 + lane;
    const bool v = i < nw;
    const uint64_t vm = __ballot(v);
    keep[r] = 0; tlo[r] = 0; thi[r] = 0;
    if (!vm) continue;
    const int nv = __popcll(vm);
    const uint64_t w = wh[r];
    const uint64_t h1 = wshr1_64(w), h2 = wshr1_64(h1);   // lanes - 1, - 2 (used from lanes 1, 2 on)
    const uint64_t pa = lane >= 1 ? h1 : A;
    const uint64_t pb = lane >= 2 ? h2 : (lane == 1 ? A : B);
    const uint64_t cm = __ballot(v && (w == pa || w == pb));
    uint64_t k = vm;
    uint64_t tp = pa;
    if (cm) {
      const int f = __builtin_ctzll(cm);
      k = vm & lanemask_lt(f);
      uint64_t xA = rdl64(pa, f), xB = rdl64(pb, f);
      for (int l = f; l < nv; ++l) {
        const uint64_t hv = rdl64(w, l);
        if (hv == xA || hv == xB) continue;
        if (lane == l) tp = xA;
        xB = xA;
        xA = hv;
        k |= 1ull << l;
      }
      A = xA;
      B = xB;
    } else {
      B = nv >= 2 ? rdl64(w, nv - 2) : A;
      A = rdl64(w, nv - 1);
    }
    keep[r] = k;
    tlo[r] = (uint32_t)tp;
    thi[r] = (uint32_t)(tp >> 32);
  }
  // probes and ordered compaction: X gets (pair @ prior word, word @ word), D gets (word @ word)
  int xb = 0, db = 0;
  bool over = false;
#pragma unroll
  for (int r = 0; r < C::NR; ++r) {
    if (r * 64 >= nw) break;
    uint32_t pp = 0, xp = 0, dp = 0;
    const bool k = (keep[r] >> lane) & 1;
    if (k) {
      const uint64_t tph = ((uint64_t)thi[r] << 32) | tlo[r];
      if (tph != 0 && tph != wh[r]) pp = octa_lookup(T.distinctocta, pair_hash(tph, wh[r]));
      xp = octa_lookup(T.distinctocta, wh[r]);
      dp = octa_lookup(T.deltaocta, wh[r]);
    }
    const int cx = (pp != 0) + (xp != 0), cd = (dp != 0);
    const int ox = xb + excl_scan(cx, lane), od = db + excl_scan(cd, lane);
    const int tx = rdl(ox + cx, 63) - xb, td = rdl(od + cd, 63) - db;
    if (xb + tx > C::NX || db + td > C::ND) { over = true; break; }
    int o = ox;
    if (pp) { s.x_off[o] = (uint16_t)pws[r]; s.x_ind[o] = pp & ~T.distinctocta.key_mask; ++o; }
    if (xp) { s.x_off[o] = (uint16_t)ws[r]; s.x_ind[o] = xp & ~T.distinctocta.key_mask; }
    if (dp) { s.d_off[od] = (uint16_t)ws[r]; s.d_ind[od] = dp & ~T.deltaocta.key_mask; }
    xb += tx; db += td;
  }
  if (over) return false;
  nd = db; nx = xb;
  wsync();
  return true;
}

// GetUniHits + GetBiHits (cldutil.cc:201-310), one lane per character.
template <int CAP>
__device__ int cjk_hits(const DevTables& T, Smem<CAP>& s, int limit, int& nb, int& nd, int& nx, int lane) {
  lane = lane_here();
  using C = Cfg<CAP>;
  const uint8_t* text = s.lbuf;
  int start = 1;
  if (text[start] == ' ') ++start;
  int b = 0;
  uint32_t endmax = (uint32_t)start;
  for (int w0 = start; w0 < limit; w0 += 64) {
    const int p = w0 + lane;
    int prop = 0, len = 0;
    if (p < limit && (text[p] & 0xC0) != 0x80) {
      len = utf8_len(text[p]);
      prop = uni_prop(T, text + p, len);
      endmax = (uint32_t)(p + len) > endmax ? (uint32_t)(p + len) : endmax;
    }
    const uint64_t m = __ballot(prop > 0);
    if (prop > 0) {
      int k = b + __popcll(m & lanemask_lt(lane));
      if (k < C::NB) { s.b_off[k] = (uint16_t)(p + len); s.b_ind[k] = (uint32_t)prop; }
    }
    b += __popcll(m);
  }
  if (b > C::NB) return -1;
  const int next = (int)wmax(endmax);
  // bigrams from offset 1 (no leading-space skip) to next
  int dcount = 0, xcount = 0;
  for (int w0 = 1; w0 < next; w0 += 64) {
    const int p = w0 + lane;
    uint32_t dp = 0, xp = 0;
    if (p < next && (text[p] & 0xC0) != 0x80) {
      const int len = utf8_len(text[p]);
      const int len2 = utf8_len(text[p + len]) + len;
      if (6 <= len2) {
        const uint32_t bh = bi_hash_v2(text + p, len2);
        dp = quad_lookup(T.deltabi, bh);
        xp = quad_lookup(T.distinctbi, bh);
      }
    }
    const uint64_t md = __ballot(dp != 0), mx = __ballot(xp != 0);
    if (dp) {
      int k = dcount + __popcll(md & lanemask_lt(lane));
      if (k < C::ND) { s.d_off[k] = (uint16_t)p; s.d_ind[k] = dp & ~T.deltabi.key_mask; }
    }
    if (xp) {
      int k = xcount + __popcll(mx & lanemask_lt(lane));
      if (k < C::NX) { s.x_off[k] = (uint16_t)p; s.x_ind[k] = xp & ~T.distinctbi.key_mask; }
    }
    dcount += __popcll(md); xcount += __popcll(mx);
  }
  if (dcount > C::ND || xcount > C::NX) return -1;
  nb = b; nd = dcount; nx = xcount;
  wsync();
  return next;
}

// DocTote::Add (tote.cc:127-175) with the wave: lanes 0-23 read their slot's
// key, the reference's probe order (slot k&15, its partner ^8, then (k&7)+16;
// a free one in the same order; else the smallest value) is resolved on
// ballots and scalars, and lane 0 writes the one slot that changes.
__device__ __forceinline__ void dt_add_wave(DocTote& dt, int k, int bytes, int sc, int r, int lane) {
  const int s0 = k & 15, s1 = s0 ^ 8, s2 = (k & 7) + 16;
  const uint32_t key = lane < 24 ? dt.key[lane < 24 ? lane : 0] : (uint32_t)kUnusedKey;
  const uint64_t cand = (1ull << s0) | (1ull << s1) | (1ull << s2);
  const uint64_t same = __ballot(key == (uint32_t)k) & cand;
  const uint64_t fr = __ballot(key == (uint32_t)kUnusedKey) & cand;
  const uint64_t m = same ? same : fr;
  int a;
  if (m) {
    a = ((m >> s0) & 1) ? s0 : ((m >> s1) & 1) ? s1 : s2;
  } else {
    const int v0 = dt.value[s0], v1 = dt.value[s1], v2 = dt.value[s2];
    a = s0;
    int va = v0;
    if (v1 < va) { a = s1; va = v1; }
    if (v2 < va) a = s2;
  }
  if (lane == 0) {
    ++dt.incr_count;
    if (same) {
      dt.value[a] += bytes; dt.score[a] += sc; dt.rel[a] += r * bytes;
    } else {
      dt.key[a] = (uint16_t)k; dt.value[a] = bytes; dt.score[a] = sc; dt.rel[a] = r * bytes;
    }
  }
  wsync();
}

// ------------------------------------- stage 4: linearize + chunk + score
// LinearizeAll/ChunkAll/ScoreAllHits (scoreonescriptspan.cc:856-1031, 208-302)
// without materialising linear[]: every emitted langprob gets its chunk from
// rank arithmetic.  Linear order is the seed, then (offset, delta < distinct <
// base, index); chunk k closes after base-type emission E_k.
template <int CAP>
__device__ bool score_round(const DevTables& T, Smem<CAP>& s, int ulscript, bool cjk, int nb, int nd, int nx,
                            int dummy_off, int& ring_sel, int lane, const uint32_t* __restrict__ pri) {
  lane = lane_here();
  using C = Cfg<CAP>;
  const DevTbl& bo = cjk ? T.compat : T.quad;
  const DevTbl& bo2 = cjk ? T.compat : T.quad2;
  const DevTbl& dob = cjk ? T.deltabi : T.deltaocta;
  const DevTbl& xob = cjk ? T.distinctbi : T.distinctocta;
  const int chunksize = cjk ? kChunksizeUnis : kChunksizeQuads;

  // the first 64 delta/distinct langprob gathers are issued together with the
  // base ones, so the three table reads share one L2 round trip
  const uint32_t dpre = lane < nd ? ind_at(dob, s.d_ind[lane]) : 0u;
  const uint32_t xpre = lane < nx ? ind_at(xob, s.x_ind[lane]) : 0u;
  // base hits -> base emissions (1 or 2 langprobs each, zeros dropped), in order
  int eb = 0;
  for (int j0 = 0; j0 < nb; j0 += 64) {
    const int j = j0 + lane;
    uint32_t l1 = 0, l2 = 0;
    int off = 0;
    if (j < nb) {
      off = s.b_off[j];
      uint32_t ind = s.b_ind[j];
      const DevTbl* lb = &bo;
      if (ind & 0x80000000u) { lb = &bo2; ind &= ~0x80000000u; }
      if (ind < lb->size_one) {
        l1 = ind_at(*lb, ind);
      } else {
        ind += ind - lb->size_one;
        l1 = ind_at(*lb, ind); l2 = ind_at(*lb, ind + 1);
        if (l1 == 0) { l1 = l2; l2 = 0; }
      }
    }
    const int c = (l1 != 0) + (l2 != 0);
    const int o = eb + excl_scan(c, lane);
    eb = rdl(o + c, 63);
    if (eb > C::NE) return false;
    if (l1) { s.a.e.be_off[o] = (uint16_t)off; s.a.e.be_lp[o] = l1; }
    if (l2) { s.a.e.be_off[o + 1] = (uint16_t)off; s.a.e.be_lp[o + 1] = l2; }
  }
  // delta / distinct emissions
  int ed = 0, ex = 0;
  for (int j0 = 0; j0 < nd; j0 += 64) {
    const int j = j0 + lane;
    uint32_t lp = j0 == 0 ? dpre : j < nd ? ind_at(dob, s.d_ind[j]) : 0u;
    const int o = ed + excl_scan(lp != 0, lane);
    uint16_t off = j < nd ? s.d_off[j] : 0;
    if (lp) { s.d_off[o] = off; s.d_ind[o] = lp; }
    ed = rdl(o + (lp != 0), 63);
  }
  for (int j0 = 0; j0 < nx; j0 += 64) {
    const int j = j0 + lane;
    uint32_t lp = j0 == 0 ? xpre : j < nx ? ind_at(xob, s.x_ind[j]) : 0u;
    const int o = ex + excl_scan(lp != 0, lane);
    uint16_t off = j < nx ? s.x_off[j] : 0;
    if (lp) { s.x_off[o] = off; s.x_ind[o] = lp; }
    ex = rdl(o + (lp != 0), 63);
  }
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
  wsync();
  // Every chunk is one contiguous range of each stream (k_long's score_round):
  // base emission t has base number t+2 (the seed is #1), so chunk k holds base
  // emissions [E_{k-1} - 1, E_k - 1); a delta / distinct emission at offset o
  // follows 1 + #(base emissions with offset < o) base entries and lands in the
  // first chunk with that count < E_k, i.e. with o <= theta_k = be_off[E_k - 2].
  if (K == 1) {
    // one chunk (most short spans): it takes every stream whole and opens with
    // the seed at offset 1 (hit offsets are >= 1), so no chunk search is needed
    if (lane < 7) {
      const int v = lane == 0 ? 0x7FFFFFFF : lane == 2 ? eb : lane == 4 ? ed : lane == 6 ? ex : 0;
      if (lane == 0) s.theta[0] = v;
      else s.st[(lane - 1) >> 1][(lane - 1) & 1] = (uint16_t)v;
    }
    if (lane == 0) s.lo[0] = 1u;
  } else {
  if (lane <= K) {                                     // K <= MAXCH < 64
    const int k = lane;
    if (k < K) {
      int th = 0x7FFFFFFF;
      if (k < K - 1) {
        const int idx = (int)s.E[k] - 2;
        th = idx < 0 ? -1 : (idx < eb ? (int)s.a.e.be_off[idx] : 0x7FFFFFFF);
      }
      s.theta[k] = th;
      s.st[0][k] = (uint16_t)(k == 0 ? 0 : min(max((int)s.E[k - 1] - 1, 0), eb));
    } else {
      s.st[0][K] = (uint16_t)eb;
    }
    s.st[1][k] = (uint16_t)ed;
    s.st[2][k] = (uint16_t)ex;
  }
  wsync();
  for (int pass = 0; pass < 2; ++pass) {               // first delta / distinct emission of each chunk
    const int n = pass == 0 ? ed : ex;
    int pch = -1;
    for (int i0 = 0; i0 < n; i0 += 64) {
      const int i = i0 + lane;
      int ch = K - 1;
      if (i < n) {
        const int o = pass == 0 ? s.d_off[i] : s.x_off[i];
        int lo_c = 0, hi_c = K - 1;
        while (lo_c < hi_c) {
          const int mid = (lo_c + hi_c) >> 1;
          if (o <= s.theta[mid]) hi_c = mid;
          else lo_c = mid + 1;
        }
        ch = lo_c;
      }
      const int prev = (int)wshr1((uint32_t)ch, (uint32_t)pch);   // lane - 1's chunk
      if (i < n)
        for (int k = prev + 1; k <= ch; ++k) s.st[1 + pass][k] = (uint16_t)i;
      pch = rdl(ch, 63);
    }
  }
  wsync();
  // lo[k] = first (lowest) offset in chunk k; chunk 0 opens with the seed at `lowest` = 1
  if (lane < K) {
    const int k = lane;
    uint32_t m = k == 0 ? 1u : 0xFFFFFFFFu;
    const int bs = s.st[0][k], be = s.st[0][k + 1], ds = s.st[1][k], de = s.st[1][k + 1];
    const int xs = s.st[2][k], xe = s.st[2][k + 1];
    if (bs < be) m = min(m, (uint32_t)s.a.e.be_off[bs]);
    if (ds < de) m = min(m, (uint32_t)s.d_off[ds]);
    if (xs < xe) m = min(m, (uint32_t)s.x_off[xs]);
    s.lo[k] = m;
  }
  }
  // linear order starts with the seed at `lowest` (= 1 for the only round)
  const uint32_t seed = ((uint32_t)per_script_number_latin(T, default_language(T, ulscript)) << 8);
  const int rs = ((uint32_t)ulscript == T.latin) ? 0 : 1;
  ring_sel = rs;
  const int nboost = pri ? 2 * kMaxBoosts : kMaxBoosts;
  int ck1 = -1, ck2 = -1, cs1 = 0, cs2 = 0, cgr = 0;   // chunk `lane`: top keys, scores, grams
  wsync();
  for (int k = 0; k < K; ++k) {
    const int seedn = k == 0 ? 1 : 0;
    const int bs = s.st[0][k], nB = s.st[0][k + 1] - bs, ds = s.st[1][k], nD = s.st[1][k + 1] - ds;
    const int xs = s.st[2][k], xe = s.st[2][k + 1], nX = xe - xs;
    const int tot = seedn + nB + nD + nX + nboost;
    // chunk k's langprob t: the seed, its base, delta and distinct emissions,
    // then ScoreBoosts (scoreonescriptspan.cc:125-152): the last four distinct
    // langprobs up to the end of the chunk and, for a hinted document, the four
    // ApplyHints prior boosts of this script class (cld_detect_batch_ex: 16
    // langprobs per document, boost latn[4] othr[4], whack latn[4] othr[4])
    // (every candidate is read, with a clamped index, and one select chain
    // picks: no branch per stream)
    auto chunk_lp = [&](int t) -> uint32_t {
      const int u0 = t - seedn, u1 = u0 - nB, u2 = u1 - nD, u3 = u2 - nX, u4 = u3 - kMaxBoosts;
      const uint32_t vb = s.a.e.be_lp[min(max(bs + u0, 0), C::NE - 1)];
      const uint32_t vd = s.d_ind[min(max(ds + u1, 0), C::ND - 1)];
      const int v = xe - kMaxBoosts + u3;                  // boost u3: the v-th distinct emission
      const uint32_t vx = s.x_ind[min(max(u3 < 0 ? xs + u2 : v, 0), C::NX - 1)];
      const uint32_t vr = s.ring[rs][min(max(v + kMaxBoosts, 0), kMaxBoosts - 1)];
      const uint32_t vp = pri ? gld(pri + 4 * rs + min(max(u4, 0), kMaxBoosts - 1)) : 0u;
      const uint32_t r = u0 < 0 ? seed : u1 < 0 ? vb : u2 < 0 ? vd : u3 < 0 ? vx : u4 < 0 ? (v < 0 ? vr : vx) : vp;
      return t < tot ? r : 0u;
    };
    // ProcessProbV2Tote (cldutil.cc:128-138): bytes 5..7 of the kLgProbV2Tbl row,
    // gathered before the tote is cleared so the L2 round trip overlaps it
    uint32_t lp = chunk_lp(lane);
    uint32_t e = lp ? gld(reinterpret_cast<const uint32_t*>(T.lgprob + 8 * (lp & 0xFF) + 4)) : 0u;
    reinterpret_cast<uint2*>(s.tote)[lane] = make_uint2(0, 0);
    wsync();
    uint64_t gm = 0;
    for (int t = lane;;) {
      if (lp) {
        const uint32_t k1 = (lp >> 8) & 0xFF, k2 = (lp >> 16) & 0xFF, k3 = (lp >> 24) & 0xFF;
        if (k1) { atomicAdd(&s.tote[k1 >> 1], ((e >> 8) & 0xFF) << ((k1 & 1) * 16)); gm |= 1ull << (k1 >> 2); }
        if (k2) { atomicAdd(&s.tote[k2 >> 1], ((e >> 16) & 0xFF) << ((k2 & 1) * 16)); gm |= 1ull << (k2 >> 2); }
        if (k3) { atomicAdd(&s.tote[k3 >> 1], (e >> 24) << ((k3 & 1) * 16)); gm |= 1ull << (k3 >> 2); }
      }
      t += 64;
      if (t - lane >= tot) break;                      // (uniform)
      lp = chunk_lp(t);
      e = lp ? gld(reinterpret_cast<const uint32_t*>(T.lgprob + 8 * (lp & 0xFF) + 4)) : 0u;
    }
    gm = wor64(gm);
    const int score_count = nB + seedn;
    wsync();
    if (pri) {                           // then the whacks zero their top key's score (ZeroPSLang :39-42)
      const uint32_t wh = lane < 4 ? gld(pri + 8 + 4 * rs + lane) : 0u;
      if (wh > 0) {
        const uint32_t k1 = (wh >> 8) & 0xFF;
        atomicAnd(&s.tote[k1 >> 1], ~(0xFFFFu << ((k1 & 1) * 16)));
      }
      wsync();
    }
    // top keys of the in-use groups: (score desc, key asc).  The reference
    // sorts three (CurrentTopThreeKeys) but SetChunkSummary reads only the
    // first two (scoreonescriptspan.cc:60-96), so two rounds.
    const uint2 v2 = reinterpret_cast<const uint2*>(s.tote)[lane];
    const bool inuse = (gm >> lane) & 1;
    uint32_t cand[4] = {v2.x & 0xFFFF, v2.x >> 16, v2.y & 0xFFFF, v2.y >> 16};
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
      best = wmax(best);
      if (best) { key3[r] = 255 - (int)(best & 0xFF); sc3[r] = (best >> 8) - 1; }
    }
    // lane k keeps chunk k's top two; the summaries are made after the loop
    if (lane == k) {
      ck1 = key3[0]; ck2 = key3[1];
      cs1 = key3[0] >= 0 ? (int)sc3[0] : 0;
      cs2 = key3[1] >= 0 ? (int)sc3[1] : 0;
      cgr = score_count;
    }
    wsync();
  }
  // SetChunkSummary (scoreonescriptspan.cc:60-96) for every chunk at once, one
  // lane per chunk; the DocTote adds then run in chunk order on lane 0
  int sum_lang = 0, sum_bytes = 0, sum_rel = 0;
  if (lane < K) {
    const uint32_t lo_k = s.lo[lane];
    const int lo = lo_k == 0xFFFFFFFFu ? dummy_off : (int)lo_k;
    int hi = dummy_off;
    if (lane + 1 < K && s.lo[lane + 1] != 0xFFFFFFFFu) hi = (int)s.lo[lane + 1];
    // language, close set and expected score of both keys: one gather each
    // from the per-GPU key table (lng::keytab_eval: FromPerScriptNumber,
    // close sets, kAvgDeltaOctaScore)
    const uint64_t* kt = T.keytab + 256 * (uint32_t)ulscript;
    const uint64_t i1 = gld(kt + (uint8_t)ck1), i2 = gld(kt + (uint8_t)ck2);
    const int lang1 = (int)(i1 & 0xFFFF);
    const int len = hi - lo;
    int actual = 0;
    if (len > 0) actual = (int)((uint32_t)cs1 << 10) / len;
    const int expected = (int16_t)(uint16_t)(i1 >> 32);
    const uint16_t bytes = (uint16_t)len, grams = (uint16_t)cgr;
    const uint16_t s1 = (uint16_t)cs1, s2 = (uint16_t)cs2;
    int rd = (uint8_t)reliability_delta(s1, s2, grams);
    const int c1 = (int)((i1 >> 16) & 0xFFFF);
    if (c1 != 0 && c1 == (int)((i2 >> 16) & 0xFFFF)) rd = 100;
    const int rsc = (uint8_t)reliability_expected(actual, expected);
    sum_lang = (uint16_t)lang1; sum_bytes = bytes; sum_rel = rd < rsc ? rd : rsc;
    cs1 = s1;
  }
  const int nsum = K < kMaxSummaries ? K : kMaxSummaries;
  for (int k = 0; k < nsum; ++k) {
    const int l1 = rdl(sum_lang, k), by = rdl(sum_bytes, k), sc = rdl(cs1, k), rl = rdl(sum_rel, k);
    dt_add_wave(s.dt, l1, by, sc, rl, lane);
  }
  // the ring keeps the last four distinct langprobs
  if (lane == 0) {
    uint32_t r4[4];
    for (int i = 0; i < 4; ++i) {
      const int u = ex + i;
      r4[i] = u < 4 ? s.ring[rs][u] : s.x_ind[u - 4];
    }
    for (int i = 0; i < 4; ++i) s.ring[rs][i] = r4[i];
  }
  wsync();
  return true;
}

// The document level below keeps DocTote slot `lane` (lanes 0-23) in
// registers: the per-slot arithmetic (close sets, divisions) runs across lanes
// at once, the control (which slot merges, which pass) on wave-uniform scalars
// read back with readlane, so no branch on it costs an exec-mask round trip.
struct SlotRegs {
  uint32_t key;
  int val, sc, rl;
};
__device__ __forceinline__ SlotRegs load_slots(const DocTote& dt, int lane) {
  const bool in = lane < 24;
  const int j = in ? lane : 0;
  SlotRegs r;
  r.key = in ? dt.key[j] : kUnusedKey;
  r.val = in ? dt.value[j] : -1;
  r.sc = in ? dt.score[j] : 0;
  r.rl = in ? dt.rel[j] : 0;
  return r;
}

// DocTote::Sort(3) (tote.cc:221-250) across lanes 0-23, one lane per slot.
// Pass s of the reference's partial bubble sort swaps slot s with every later
// slot whose value beats the current holder (strictly): the holders are the
// running-maximum records r1 < ... < rm of slots s+1..23.  Afterwards slot s
// has rm's entry, r1 has s's, and rj has r(j-1)'s; nothing else moves.
// Unused slots count as value -1 (the reference sets that as it scans).
__device__ __forceinline__ void sort3_regs(SlotRegs& r, int lane) {
  const bool in = lane < 24;
  if (r.key == kUnusedKey) r.val = -1;
#pragma unroll
  for (int p = 0; p < 3; ++p) {
    // exclusive running max of slots p..lane-1 (values biased to unsigned)
    const uint32_t m = dpp_scan_incl((in && lane >= p) ? (uint32_t)r.val ^ 0x80000000u : 0u, 0u, OpMax());
    const int ex = (int)(wshr1(m, 0u) ^ 0x80000000u);
    const uint64_t R = __ballot(in && lane > p && r.val > ex);
    if (R) {
      const uint64_t below = R & lanemask_lt(lane);
      const int src = lane == p ? 63 - __builtin_clzll(R)
                    : ((R >> lane) & 1) ? (below ? 63 - __builtin_clzll(below) : p) : lane;
      r.key = (uint32_t)__shfl((int)r.key, src, 64);
      r.val = __shfl(r.val, src, 64);
      r.sc = __shfl(r.sc, src, 64);
      r.rl = __shfl(r.rl, src, 64);
    }
  }
}

// RefineScoredClosePairs (compact_lang_det_impl.cc:1105-1147): slot s, in
// order, merges into the first later slot of its close set.  The close sets
// are gathered for all slots at once; the slots that have one (a handful at
// most) are visited in order on scalars.
struct NoMove {
  __device__ __forceinline__ void operator()(int, int) const {}
};
// mv(from_lang, to_lang), wave-uniform, for every merge in order: vec mode
// relabels the chunk vector there (MoveLang1ToLang2, :1122-1147).
template <class Mv = NoMove>
__device__ __forceinline__ void refine_close_pairs_regs(const DevTables& T, SlotRegs& r, int lane, Mv&& mv = Mv{}) {
  int cs = lane < 24 ? close_set(T, (int)r.key) : 0;
  uint64_t todo = __ballot(cs != 0);
  while (todo) {
    const int s = __builtin_ctzll(todo);
    todo &= todo - 1;
    const int css = rdl(cs, s);
    if (css == 0) continue;                                    // emptied by an earlier merge
    const uint64_t mm = __ballot(lane > s && cs == css);
    if (!mm) continue;
    const int s2 = __builtin_ctzll(mm);
    const bool s_from = rdl(r.val, s) < rdl(r.val, s2);        // the smaller moves into the larger
    const int from = s_from ? s : s2, to = s_from ? s2 : s;
    const int fv = rdl(r.val, from), fs = rdl(r.sc, from), fr = rdl(r.rl, from);
    mv(rdl((int)r.key, from), rdl((int)r.key, to));
    if (lane == to) { r.val += fv; r.sc += fs; r.rl += fr; }
    if (lane == from) { r.key = kUnusedKey; r.sc = 0; r.rl = 0; cs = 0; }   // (value stays, as there)
  }
}

// RemoveUnreliableLanguages (compact_lang_det_impl.cc:997-1101) on the slot
// registers.  todo = the slots unreliable on entry: only they can act, since a
// merge leaves its target reliable (np >= 41 over at least its own bytes) and
// empties its source.  They are visited in slot order on scalars and rechecked
// as the reference does (an earlier merge may have emptied or fixed one); the
// second loop (drop what is still unreliable) runs across lanes.  The
// reference's Find on the sorted tote is a linear scan: the first slot whose
// key matches.  As there, a merge moves reliability and bytes into the score
// field and leaves value alone.
__device__ __forceinline__ void remove_unreliable_regs(const DevTables& T, SlotRegs& r, uint64_t todo, int lane) {
  const int unk = (int)T.unknown_lang;
  while (todo) {
    const int s = __builtin_ctzll(todo);
    todo &= todo - 1;
    const int lang = rdl((int)r.key, s);
    if (lang == kUnusedKey) continue;
    const int bytes = rdl(r.val, s), reli = rdl(r.rl, s);
    if (bytes == 0) continue;
    const int rp = reli / bytes;
    if (rp >= 41) continue;
    int alt = unk;
    if ((uint32_t)lang <= T.hawaiian && (uint32_t)lang < T.n_closest) alt = gld(T.closest + lang);
    if (alt == unk) continue;
    const uint64_t am = __ballot(lane < 24 && (int)r.key == alt);
    if (!am) continue;
    const int as = __builtin_ctzll(am);
    const int bytes2 = rdl(r.val, as), reli2 = rdl(r.rl, as);
    if (bytes2 == 0) continue;
    const int rp2 = reli2 / bytes2;
    int to = as, from = s;
    if (rp2 < rp || (rp2 == rp && lang < alt)) { to = s; from = as; }
    int np = rp > rp2 ? rp : rp2;
    if (np < 41) np = 41;
    const int nbytes = bytes + bytes2;
    if (lane == from) { r.key = kUnusedKey; r.sc = 0; r.rl = 0; }
    if (lane == to) { r.sc = nbytes; r.rl = np * nbytes; }
  }
  if (lane < 24 && r.key != kUnusedKey && r.val != 0 && r.rl / (r.val ? r.val : 1) < 41) {
    r.key = kUnusedKey;
    r.sc = 0;
    r.rl = 0;
  }
}

// ExtractLangEtc (compact_lang_det_impl.cc:1276-1384): slots 0-2 in lanes
// 0-2, their divisions in parallel; the results as wave-uniform scalars
// (normalized score of slot `lane` in ns).
struct DocSum {
  int lang[3], pct[3];
  int text_bytes;
  bool reliable;
};
__device__ __forceinline__ DocSum extract_regs(const DevTables& T, const SlotRegs& r, int total, int lane, double& ns) {
  const int unk = (int)T.unknown_lang;
  const bool valid = lane < 3 && r.key != kUnusedKey && (int)r.key != unk;
  const int bc = valid ? r.val : 0;
  const int rp = valid ? r.rl / (bc ? bc : 1) : 0;
  ns = (valid && bc > 0) ? (double)((int32_t)((uint32_t)r.sc << 10) / (bc > 0 ? bc : 1)) : 0.0;
  const int b0 = rdl(bc, 0), b1 = rdl(bc, 1), b2 = rdl(bc, 2);
  const int t12 = b0 + b1, t123 = t12 + b2;
  const int tot = total < t123 ? t123 : total;
  const int div = tot > 1 ? tot : 1;
  const int cum = lane == 0 ? b0 : lane == 1 ? t12 : t123;
  const int pc = (cum * 100) / div;
  int q0 = rdl(pc, 0), q1 = rdl(pc, 1), q2 = rdl(pc, 2);
  q2 -= q1;
  q1 -= q0;
  if (q1 < q2) { ++q1; --q2; }
  if (q0 < q1) { ++q0; --q1; }
  const int lg = valid ? (int)r.key : unk;
  DocSum d;
  d.lang[0] = rdl(lg, 0); d.lang[1] = rdl(lg, 1); d.lang[2] = rdl(lg, 2);
  d.pct[0] = q0; d.pct[1] = q1; d.pct[2] = q2;
  d.text_bytes = tot;
  d.reliable = rdl(valid ? 1 : 0, 0) && rdl(rp, 0) >= 41;
  if (100 - (q0 + q1 + q2) > 20) d.reliable = false;
  return d;
}

__device__ __forceinline__ double rdl_f64(double v, int l) {
  return __longlong_as_double((long long)rdl64((uint64_t)__double_as_longlong(v), l));
}

// Document level (compact_lang_det_impl.cc:1997-2065).  Returns 1 with the
// result written, or 0 when the first pass is not good enough and the Repeats
// pass must follow (never when `final`).  best_effort: kCLDFlagBestEffort
// (:1998-2000, :1493): no unreliable-language removal and no UNKNOWN for a
// small return percent.
template <class Mv = NoMove>
__device__ __forceinline__ int finish_document(const DevTables& T, DocTote& dt, int total, bool final, cld_result* __restrict__ out,
                               int lane, bool best_effort = false, Mv&& mv = Mv{}) {
  SlotRegs r = load_slots(dt, lane);
  refine_close_pairs_regs(T, r, lane, mv);
  sort3_regs(r, lane);
  double ns;
  DocSum x = extract_regs(T, r, total, lane, ns);
  const bool good = final || total <= 256 || (x.reliable && x.pct[0] >= 70) ||
                    (x.reliable && x.pct[0] + x.pct[1] >= 93);
  if (!good) return 0;
  if (!best_effort) {
    // RemoveUnreliableLanguages (:997-1101) only when some slot is unreliable
    const bool unrel = lane < 24 && r.key != kUnusedKey && r.val != 0 && r.rl / (r.val ? r.val : 1) < 41;
    if (const uint64_t todo = __ballot(unrel)) {
      remove_unreliable_regs(T, r, todo, lane);
      sort3_regs(r, lane);
      x = extract_regs(T, r, total, lane, ns);
    }
  }
  // CalcSummaryLang (:1414-1522) on the scalars
  Extract e;
#pragma unroll
  for (int i = 0; i < 3; ++i) { e.lang3[i] = x.lang[i]; e.pct3[i] = x.pct[i]; e.rp3[i] = 0; e.ns3[i] = 0.0; }
  e.text_bytes = x.text_bytes;
  e.reliable = x.reliable;
  bool rel;
  const int summary = calc_summary_lang(T, total, e, rel, best_effort);
  const double n0 = rdl_f64(ns, 0), n1 = rdl_f64(ns, 1), n2 = rdl_f64(ns, 2);
  if (lane == 0) {
    cld_result o;
    o.lang3[0] = (uint16_t)x.lang[0]; o.lang3[1] = (uint16_t)x.lang[1]; o.lang3[2] = (uint16_t)x.lang[2];
    o.summary_lang = (uint16_t)summary;
    o.percent3[0] = (int8_t)x.pct[0]; o.percent3[1] = (int8_t)x.pct[1]; o.percent3[2] = (int8_t)x.pct[2];
    o.is_reliable = rel ? 1 : 0;
    o.text_bytes = x.text_bytes;
    o.normalized3[0] = n0; o.normalized3[1] = n1; o.normalized3[2] = n2;
    *out = o;
  }
  return 1;
}

// ------------------------------------------------------ the document
template <int CAP>
__device__ bool detect(const DevTables& T, const uint8_t* __restrict__ g, int L, Smem<CAP>& s, int lane,
                       cld_result* __restrict__ out, unsigned long long* __restrict__ prof, uint32_t cflags,
                       const uint32_t* __restrict__ pri, const uint8_t* __restrict__ hf) {
  // optional per-stage cycle accounting (CLD_PROFILE_STAGES=1): 0 load, 1 span,
  // 2 lower, 3 quad/uni, 4 octa/bi, 5 score, 6 document level
  long long t_stage = prof ? (long long)clock64() : 0;
  auto mark = [&](int st) {
    if (prof) {
      long long t = (long long)clock64();
      if (lane == 0) atomicAdd(&prof[st], (unsigned long long)(t - t_stage));
      t_stage = t;
    }
  };

  const int unk = (int)T.unknown_lang;
  if (L == 0) {
    if (lane == 0) {
      Extract x;
      for (int i = 0; i < 3; ++i) { x.lang3[i] = unk; x.pct3[i] = 0; x.ns3[i] = 0.0; x.rp3[i] = 0; }
      x.text_bytes = 0;
      write_result(out, x, unk, false);
    }
    return true;
  }
  if (!load_document<CAP>(T, g, L, s, lane, hf)) return false;
  mark(0);
  if (lane == 0) s.dt.init();
  if (lane < 8) s.ring[lane >> 2][lane & 3] = 0;
  wsync();
  int next = 0, total = 0;
  for (;;) {
    int ulscript = 0;
    int tb = next_span<CAP>(T, s, L, next, ulscript, lane);
    mark(1);
    if (tb == 0) break;
    tb = lower_span<CAP>(T, s, tb, lane);
    mark(2);
    if (tb < 0) return false;
    int rt = rtype_of(T, ulscript);
    if ((cflags & kCLDFlagScoreAsQuads) && rt != RTypeCJK) rt = RTypeMany;   // scoreonescriptspan.cc:1318-1320
    if (rt == RTypeNone || rt == RTypeOne) {
      if (lane == 0) s.dt.add((uint16_t)default_language(T, ulscript), tb, tb, 100);
      wsync();
    } else {
      const bool cjk = rt == RTypeCJK;
      int nb = 0, nd = 0, nx = 0, endo;
      if (cjk) {
        endo = cjk_hits<CAP>(T, s, tb, nb, nd, nx, lane);
        mark(3);
        if (endo < 0) return false;
      } else {
        endo = quad_hits<CAP>(T, s, tb, nb, lane);
        mark(3);
        if (endo < 0) return false;
        if (!octa_hits<CAP>(T, s, endo, nd, nx, lane)) return false;
        mark(4);
      }
      if (endo < tb) return false;     // a second round would be needed (never for short documents)
      int rsel;
      if (1 < tb && !score_round<CAP>(T, s, ulscript, cjk, nb, nd, nx, endo, rsel, lane, pri)) return false;
      mark(5);
    }
    total += tb;
  }
  const int ok = finish_document(T, s.dt, total, false, out, lane, (cflags & kCLDFlagBestEffort) != 0);
  mark(6);
  return ok != 0;
}

}  // namespace wave
}  // namespace cld
