// cld_kernels.hip -- batch kernels over the device pipeline.
//
//  k_wave<CAP>   one wavefront per document of <= CAP bytes, state in LDS.
//  k_long        one wavefront per document of any length up to lng::kDocCap,
//                per-wave slot in HBM; persistent grid over the wave kernel's
//                re-queue list.
//                Documents the parallel span builder cannot formulate take
//                its sequential span source (cld_seq.hip) in the same wave.
#include "cld_kernels.h"
// The A/B knobs of earlier rounds that gave wrong results by design are gone;
// refuse a build that still asks for one.
#if defined(WAVE_STOP) || defined(LNG_EXP_NOADDS) || defined(HTML_EXP) || defined(LNG_INC)
#error "experiment knobs (WAVE_STOP, LNG_EXP_NOADDS, HTML_EXP, LNG_INC) are not part of the product build"
#endif
#include "cld_prims.hip"
#include "cld_wave.hip"
#include "cld_long.hip"
#include "cld_html.hip"

static_assert(kHtmlSoftMin == cld::kMaxScriptBytes, "kHtmlSoftMin is kMaxScriptBytes");
static_assert(kLongDocCap == (uint64_t)cld::lng::kDocCap, "kLongDocCap is lng::kDocCap");

namespace cld {

// Vec-mode routing: every document to k_long<VEC>'s list (one atomic per
// wavefront); k_long reads each one's routing bits itself.
__global__ __launch_bounds__(256) void k_route_vec(int n, uint32_t* __restrict__ counters,
                                                  uint32_t* __restrict__ long_list);

// Compaction of the per-document pool regions into document order.
__global__ __launch_bounds__(256) void k_vec_gather(const cld_chunk* __restrict__ pool,
                                                   const uint64_t* __restrict__ pool_off,
                                                   const int32_t* __restrict__ n_chunks,
                                                   const uint64_t* __restrict__ pos, int n,
                                                   cld_chunk* __restrict__ dst) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int m = n_chunks[i];
  for (int k = 0; k < m; ++k) dst[pos[i] + k] = pool[pool_off[i] + k];
}

// One wavefront per document of <= CAP bytes, WPB documents per workgroup.
// One wave (document) per workgroup (WAVE_WPB, cld_kernels.h): a block's LDS
// is released as soon as its own document is done, not when the slowest of
// four is (C2 139M -> 167M docs/s; profiles/round1q_ab_wpb/).  WAVE_WPS waves
// per SIMD: 8 blocks of 5088 B LDS per SIMD fit the CU's 160 KB (the chunk
// tote overlays the lowered span text; raw span text, base hits and chunk
// ids share one buffer) and 64 VGPRs hold without spills (7 -> 8 waves:
// C2 167M -> 169M, profiles/round1q_ab_wps8/).
#ifndef WAVE_WPS
#define WAVE_WPS 8
#endif
template <int CAP, int WPB>
__global__ __launch_bounds__(64 * WPB, WAVE_WPS) void k_wave(DevTables T, const uint8_t* __restrict__ buf,
                                                   const uint64_t* __restrict__ offs, int n,
                                                   cld_result* __restrict__ out,
                                                   uint32_t* __restrict__ requeue_list,
                                                   uint32_t* __restrict__ counters,
                                                   unsigned long long* __restrict__ prof,
                                                   const uint8_t* __restrict__ special,
                                                   uint32_t* __restrict__ special_list, int special_ctr,
                                                   uint32_t cflags, const uint32_t* __restrict__ priors,
                                                   const uint8_t* __restrict__ hbuf, const uint8_t* __restrict__ hflag) {
  __shared__ wave::Smem<CAP> smem[WPB];
  // wave index through readfirstlane: the document pointer, its length, the
  // result pointer and the LDS base are then scalars, not VGPRs live across
  // the whole document
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  // XCD-aware: workgroups go round-robin over the 8 XCDs, so block b's
  // documents come from slice b & 7 of the batch.  Neighbouring documents
  // then share an XCD (and its L2) for the lines they share.
  const int per = ((n + WPB - 1) / WPB + 7) >> 3;          // blocks per XCD slice
  const int i = ((int)(blockIdx.x & 7) * per + (int)(blockIdx.x >> 3)) * WPB + wv;
  if (i >= n) return;
  // k_route has already listed the HTML documents (for k_long) and those
  // longer than CAP (for k_long); hinted plain ones are scored here with their
  // ApplyHints priors
  const uint8_t sp = special ? special[i] : (uint8_t)0;
  if (sp & kSpecialHtml) return;
  const uint32_t* pri = (sp & kSpecialPriors) ? priors + 16ull * i : nullptr;
  const uint64_t a = offs[i], b = offs[i + 1];
  const int64_t len = (int64_t)(b - a);
  if (len > CAP) return;
  // stage cycles (CLD_PROFILE_STAGES=1) are sampled on one document in 64, so
  // the accounting atomics do not themselves become the bottleneck
  // a rewritten HTML page (cld_html.hip) is read from hbuf, with its lookahead marks
  const bool rw = (sp & kSpecialRewritten) != 0;
  const bool rq = !wave::detect<CAP>(T, (rw ? hbuf : buf) + a, (int)len, smem[wv], lane, &out[i],
                                     (i & 63) == 0 ? prof : nullptr, cflags, pri, rw ? hflag + a : nullptr);
  if (rq && lane == 0) {                       // rare (state-machine or capacity cases)
    if (requeue_list) {
      uint32_t k = atomicAdd(&counters[kCtrRequeue], 1u);
      requeue_list[k] = (uint32_t)i;
    } else {                                   // run_tiny: the mark travels with the results
      out[i].summary_lang = kWaveRequeued;
    }
  }
}

// Appends `val` of every lane with `pred` to list under *ctr with one atomic
// per wavefront (all 64 lanes call it).
__device__ __forceinline__ void wave_append(bool pred, uint32_t* ctr, uint32_t* list, uint32_t val, uint32_t* ctr2) {
  const uint64_t m = __ballot(pred);
  if (!m) return;
  const int leader = __builtin_ctzll(m), lane = (int)(threadIdx.x & 63);
  uint32_t base = 0;
  if (lane == leader) {
    base = atomicAdd(ctr, (uint32_t)__popcll(m));
    if (ctr2) atomicAdd(ctr2, (uint32_t)__popcll(m));
  }
  base = (uint32_t)__shfl((int)base, leader, 64);
  if (pred) list[base + __popcll(m & wave::lanemask_lt(lane))] = val;
}

__global__ __launch_bounds__(256) void k_route_vec(int n, uint32_t* __restrict__ counters,
                                                  uint32_t* __restrict__ long_list) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  wave_append(i < n, &counters[kCtrRequeue], long_list, (uint32_t)i, nullptr);
}

constexpr int kLenBuckets = 64;

// Routing before k_wave, one thread per document: HTML documents to
// k_long's list, documents longer than k_wave's CAP to k_long's, each with
// one atomic per wavefront instead of one per document (a batch of 100K pages
// used to queue every page through the same counter from k_wave).  Block 0
// also zeroes k_len_hist's histogram and cursors (hist2, nullable): one
// launch fewer per batch than a memset.
__global__ __launch_bounds__(256) void k_route(const uint64_t* __restrict__ offs, int n,
                                              const uint8_t* __restrict__ special, int cap,
                                              uint32_t* __restrict__ counters, uint32_t* __restrict__ requeue_list,
                                              uint32_t* __restrict__ special_list, int special_ctr,
                                              uint32_t* __restrict__ hist2) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (hist2 && blockIdx.x == 0 && threadIdx.x < 2 * kLenBuckets) hist2[threadIdx.x] = 0;
  bool html = false, lng = false;
  if (i < n) {
    html = special && (special[i] & kSpecialHtml);
    lng = !html && offs[i + 1] - offs[i] > (uint64_t)cap;
  }
  wave_append(html, &counters[special_ctr], special_list, (uint32_t)i, &counters[kCtrSpecial]);
  wave_append(lng, &counters[kCtrRequeue], requeue_list, (uint32_t)i, nullptr);
}

// One wavefront per long document, persistent: each wave owns slot
// blockIdx.x * WPB + wave and pulls documents from the wave kernel's re-queue
// list (one atomic per document) until the list is drained -- every wave
// reaches that exit.  Documents the parallel span builder cannot formulate
// are scored again from the sequential span source (cld_seq.hip).
// LNG_WPS waves per SIMD.  The kernel is latency-bound on its HBM slots:
// more resident waves beat the extra spills (C3, 30K pages: 4 -> 496K, 5 ->
// 538K, 6 -> 553K, 7 -> 578K, 8 -> 541K docs/s; profiles/round1e_*).  After
// round 1j's lane-parallel chunk summaries 8 wins (C3 100K pages: 6 -> 566K,
// 7 -> 738K, 8 -> 754K docs/s; profiles/round1j_ab_long/).  9 does not fit.
#ifndef LNG_WPS
#define LNG_WPS 4
#endif
// Speculation for small batches (k_long below): up to nwaves / kSpecShare of
// the longest documents get a second wave, when the batch has at most
// kSpecBatchWaves documents per resident wave (a full batch is throughput-
// bound and keeps one wave per document).
constexpr uint32_t kSpecShare = 8, kSpecBatchWaves = 4;
// SEQ: the instantiation that drains seq_list (the documents the parallel
// one hands on): their spans come from the sequential span source.
template <int WPB, bool DIAG, bool VEC, bool SEQ = false>
__global__ __launch_bounds__(64 * WPB, LNG_WPS) void k_long(const DevTables* __restrict__ Tp,
                                                  const uint8_t* __restrict__ buf,
                                                  const uint64_t* __restrict__ offs,
                                                  const uint32_t* __restrict__ list,
                                                  cld_result* __restrict__ out, uint8_t* __restrict__ slots,
                                                  uint32_t* __restrict__ seq_list,
                                                  uint32_t* __restrict__ counters, uint32_t* trace,
                                                  uint32_t* dbg, uint32_t dbg_doc,
                                                  unsigned long long* prof, uint32_t cflags,
                                                  const uint8_t* __restrict__ special,
                                                  const uint32_t* __restrict__ priors,
                                                  const uint8_t* __restrict__ hbuf, const uint8_t* __restrict__ hflag,
                                                  uint32_t fault_doc, uint8_t* __restrict__ vslots,
                                                  cld_chunk* __restrict__ pool, const uint64_t* __restrict__ pool_off,
                                                  int32_t* __restrict__ n_chunks, const uint32_t* __restrict__ hpos,
                                                  const uint32_t* __restrict__ hgap, cld_result* __restrict__ spec_out,
                                                  uint32_t* __restrict__ spec_take, int ctr_total, int ctr_deq) {
  __shared__ lng::Smem smem[WPB];
  const DevTables& T = *Tp;
  // wave index through readfirstlane: the slot pointer (and every S.field
  // address) is then scalar instead of a VGPR pair per field
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  uint32_t* tr = (DIAG && trace) ? trace + 4 * (blockIdx.x * WPB + wv) : nullptr;
  lng::Slot& S = *reinterpret_cast<lng::Slot*>(slots + (uint64_t)(blockIdx.x * WPB + wv) * sizeof(lng::Slot));
  const uint32_t total =
      wave::uflu(__hip_atomic_load(&counters[ctr_total], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  if (total == 0) return;                       // empty re-queue list: no dequeue atomics at all
  // Speculation (small batches only, so full batches keep their throughput):
  // the first nspec documents of the longest-first list -- the ones a small
  // launch waits for -- get two waves, one running pass 1 (kPassFirstOnly)
  // and one pass 2 (kPassRepeatsOnly, into spec_out).  Entries 2q / 2q + 1
  // are document q's two roles, entries from 2 * nspec on one document each.
  // The last wave to leave takes pass 2's result for every document whose
  // pass 1 was not good enough (spec_take).
  const uint32_t nwaves = gridDim.x * WPB;
  const uint32_t nspec =
      (!VEC && !SEQ && spec_out && total <= kSpecBatchWaves * nwaves) ? min(total, nwaves / kSpecShare) : 0u;
  const uint32_t entries = total + nspec;
  if constexpr (DIAG) lng::trace(tr, lane, 0xFFFFFFFFu, 97, 0);
  const bool exact = lng::space_lowers_to_space(T);
  if constexpr (DIAG) lng::trace(tr, lane, 0xFFFFFFFFu, 98, exact);
  for (;;) {
    // Whole-wave atomic (lane 0 adds 1, the others 0) read back from lane 0.
    // A lane-0-only atomic feeding readfirstlane at the loop head let the
    // compiler split the loop so the other lanes re-read k = 0 forever.
    const uint32_t e = wave::uflu(atomicAdd(&counters[ctr_deq], lane == 0 ? 1u : 0u));
    if (e >= entries) break;
    const uint32_t k = e < 2 * nspec ? e >> 1 : e - nspec;      // list position
    const int mode = e < 2 * nspec ? ((e & 1) ? lng::kPassRepeatsOnly : lng::kPassFirstOnly) : lng::kPassesAll;
    const uint32_t i = list[k];
    const uint64_t a = offs[i], b = offs[i + 1];
    const uint64_t len = b - a;
    int passes = 0;
    if (lane == 0) {
      smem[wv].dbg = (DIAG && dbg && i == dbg_doc) ? dbg : nullptr;
      smem[wv].dbg_pos = 0;
      smem[wv].prof = DIAG ? prof : nullptr;
    }
    wave::wsync();
    const uint8_t spi = special ? special[i] : (uint8_t)0;
    const bool rw = (spi & kSpecialRewritten) != 0;   // a rewritten HTML page (cld_html.hip)
    // its byte -> page offset maps, for the span soft limit of pages of
    // kMaxScriptBytes and more (cld_html.hip writes them for those)
    const bool hbig = rw && hpos && len >= (uint64_t)kMaxScriptBytes;
    const uint32_t* hp = hbig ? hpos + a : nullptr;
    const uint32_t* hg = hbig ? hgap + a : nullptr;
    const uint32_t* pri = (spi & kSpecialPriors) ? priors + 16ull * i : nullptr;
    // The sequential span source (cld_seq.hip) over the page as given: for a
    // page the HTML rewrite did not take (still kSpecialHtml), one whose
    // rewritten offsets vec mode cannot use (kSpecialNoVec), a document past
    // the slot's bitmap, a table set whose lowercaser does not keep ' ', and
    // -- after the parallel attempt -- any document that attempt could not
    // formulate.  Those go to seq_list, which the SEQ instantiation drains;
    // the span-level stages are the same either way.
    const bool html_raw = (spi & kSpecialHtml) != 0;
    const bool fault = i == fault_doc;               // fault injection (CLD_FAULT_DOC, tests only)
    const bool to_seq = !SEQ && !fault &&
                        (!exact || html_raw || (VEC && (spi & kSpecialNoVec)) || len > (uint64_t)lng::kDocCap);
    cld_result* o = (!VEC && mode == lng::kPassRepeatsOnly) ? spec_out + k : &out[i];
    lng::VecState V;
    if constexpr (VEC) {
      // ResultChunkVector mode (cld_detect_batch_vec): the vector goes to the
      // document's pool region; a vector that outgrows it reports -1 (the host
      // redoes the document with a larger region)
      V.vs = reinterpret_cast<lng::VecSlot*>(vslots + (uint64_t)(blockIdx.x * WPB + wv) * sizeof(lng::VecSlot));
      const uint64_t reg = pool_off[i + 1] - pool_off[i];
      V.v = pool + pool_off[i];
      V.cap = reg > 0x7FFFFFFFull ? 0x7FFFFFFF : (int)reg;
      V.n = 0;
      V.over = false;
      V.doc = buf + a;                           // (the page as given: the vector maps into it)
      V.L = (int)len;
      V.last_off = V.last_bytes = V.last_lang = 0;
      V.hpos = (rw && !SEQ) ? hpos + a : nullptr;   // a rewritten HTML page: rewritten byte -> page offset
      V.hgap = (rw && !SEQ) ? hgap + a : nullptr;
      V.seq = SEQ;
    }
    if (!fault && !to_seq) {
      if constexpr (SEQ) {
        const lng::SeqDoc sq{buf + a, (int)len, !(spi & (kSpecialHtml | kSpecialRewritten | kSpecialNoVec))};
        passes = lng::detect<DIAG, VEC, true>(T, buf + a, (int)len, S, smem[wv], lane, o, tr, i, cflags, pri, nullptr,
                                              VEC ? &V : nullptr, lng::kPassesAll, nullptr, nullptr, &sq);
        if (lane == 0) atomicAdd(&counters[kCtrSeq], 1u);
      } else {
        passes = lng::detect<DIAG, VEC>(T, (rw ? hbuf : buf) + a, (int)len, S, smem[wv], lane, o, tr, i, cflags,
                                        pri, rw ? hflag + a : nullptr, VEC ? &V : nullptr, VEC ? lng::kPassesAll : mode,
                                        hp, hg);
      }
    }
    if constexpr (DIAG) lng::trace(tr, lane, i, 99, passes);
    passes = wave::ufl(passes);
    const bool good = passes >= 1 && passes <= 3 && !fault;
    // handed on: the SEQ instantiation redoes the document whole (a pass-2
    // speculative wave's failure is handed on by its pass-1 wave's taker)
    const bool hand_on = !SEQ && !fault && !good && passes != lng::kNeedsRepeats;
    if constexpr (VEC) {
      if (lane == 0 && !hand_on) n_chunks[i] = (good && !V.over) ? V.n : -1;
    }
    if (!VEC && mode == lng::kPassRepeatsOnly) {   // pass 2 in spec_out[k]; taken or not by its pass-1 wave
      if (lane == 0 && !good) spec_out[k].summary_lang = CLD_LANG_FAILED;
      continue;
    }
    if (passes == lng::kNeedsRepeats && !fault) {
      if (lane == 0) spec_take[atomicAdd(&counters[kCtrSpecTake], 1u)] = k;
      continue;
    }
    if (lane == 0) {
      if (good) {
        atomicAdd(&counters[kCtrPass1 + passes - 1], 1u);
      } else if (hand_on) {
        seq_list[atomicAdd(&counters[kCtrRequeue2], 1u)] = i;
        if (!to_seq) atomicAdd(&counters[kCtrWhy + min(max(-passes, 0), 7)], 1u);
      } else {
        // No result for this document: it is marked (summary CLD_LANG_FAILED)
        // and counted; the host redoes it alone, the rest of the batch stands.
        atomicAdd(&counters[kCtrError], 1u);
        mark_failed(T, &out[i]);
      }
    }
  }
  if (nspec) {
    // the last wave out hands over the speculative pass-2 results (every
    // wave's stores released before its count, acquired by the last)
    __threadfence();
    const uint32_t done = wave::uflu(atomicAdd(&counters[kCtrSpecDone], lane == 0 ? 1u : 0u));
    if (done == nwaves - 1) {
      __threadfence();
      const uint32_t nt = __hip_atomic_load(&counters[kCtrSpecTake], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      for (uint32_t p = lane; p < nt; p += 64) {
        const uint32_t k = spec_take[p], i = list[k];
        const cld_result r = spec_out[k];
        if (r.summary_lang == CLD_LANG_FAILED) {      // pass 2 could not run here: the SEQ kernel redoes it
          seq_list[atomicAdd(&counters[kCtrRequeue2], 1u)] = i;
        } else {
          out[i] = r;
          atomicAdd(&counters[kCtrPass2], 1u);
        }
      }
    }
  }
  if constexpr (DIAG) lng::trace(tr, lane, 0xFFFFFFFFu, 100, total);
}

// ------------------------------------------------ staged long-document path
// (cld_long.hip, st_spans / st_score / st_rep).  Persistent grids, one wave
// per document at a time, each with its own occupancy: LNG_SPAN_WPS waves per
// SIMD for k_lspan (96 VGPRs, no LDS), LNG_ST_WPS for k_lscore (its LDS is the
// LNG_ST_TEXT text window without the Repeats predictor; a longer span is
// scored through windows of it), LNG_REP_WPS for k_lrep (one wave per
// workgroup, 8 KB of LDS predictor each).  C3, 100K 16 KB pages: fused k_long
// 86.1 ms; staged at 5/5/5 waves and a 5 KB window 77.0 ms, at 5/6/5 and 3 KB
// 73.6 ms (gpurun_out/r5j), at 6/7/5 and 2 KB ~72 ms (r5k).  A block of a span
// wider than the window (win_text) sends the document to the fused kernel,
// whose window is 6 KB (a 1 KB window sent 81% of C3 to the sequential kernel
// of earlier rounds).
#ifndef LNG_ST_WPS
#define LNG_ST_WPS 7
#endif
#ifndef LNG_SPAN_WPS
#define LNG_SPAN_WPS 6
#endif
#ifndef LNG_REP_WPS
#define LNG_REP_WPS 5
#endif
#ifndef LNG_ST_TEXT
#define LNG_ST_TEXT 2048
#endif
constexpr int kStWPB = 4;
using StSmem = lng::SmemT<LNG_ST_TEXT, false>;
static_assert(kStWPB * sizeof(StSmem) * (4 * LNG_ST_WPS / kStWPB) <= 160 * 1024, "k_lscore LDS per CU");

// The stored and pass-2 lists are two-ended: documents of more than
// kHeavySpans spans (a span costs a wave ~15 us per pass whatever its length)
// fill from the top, the others from the bottom, and the consumers take the
// heavy ones first -- longest work first, as the LPT list orders by bytes.
// Without it a 200-span page of a C3 batch (16 KB like the rest) or a C5
// batch's pass-2 list could come last and set the kernel's tail.
#ifndef LNG_HEAVY_SPANS
#define LNG_HEAVY_SPANS 32
#endif
constexpr uint32_t kHeavySpans = LNG_HEAVY_SPANS;
__device__ __forceinline__ void st_put(uint32_t* list, uint32_t* counters, int ctr_lo, int ctr_hi, uint32_t n,
                                       bool heavy, uint32_t v) {   // (one lane)
  if (heavy) list[n - 1 - atomicAdd(&counters[ctr_hi], 1u)] = v;
  else list[atomicAdd(&counters[ctr_lo], 1u)] = v;
}
__device__ __forceinline__ uint32_t st_get(const uint32_t* list, uint32_t nh, uint32_t n, uint32_t e) {
  return e < nh ? list[n - 1 - e] : list[e - nh];
}
__device__ __forceinline__ uint32_t st_count(uint32_t* counters, int ctr) {
  return wave::uflu(__hip_atomic_load(&counters[ctr], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}

__global__ __launch_bounds__(64 * kStWPB, LNG_SPAN_WPS) void k_lspan(
    const DevTables* __restrict__ Tp, const uint8_t* __restrict__ buf, const uint64_t* __restrict__ offs,
    const uint32_t* __restrict__ list, uint8_t* __restrict__ slots, uint8_t* __restrict__ pool, uint64_t pool_bytes,
    uint64_t* __restrict__ meta, uint32_t* __restrict__ ok_list, uint32_t* __restrict__ fall_list,
    uint32_t* __restrict__ counters, const uint8_t* __restrict__ special, const uint8_t* __restrict__ hbuf,
    const uint8_t* __restrict__ hflag, const uint32_t* __restrict__ hpos, const uint32_t* __restrict__ hgap,
    uint32_t fault_doc, uint32_t small_total, const uint32_t* __restrict__ hist, uint32_t* __restrict__ par_list,
    uint64_t* __restrict__ group_list, uint32_t gcap, uint32_t heavy_kb, uint32_t n) {
  const DevTables& T = *Tp;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  lng::Slot& S = *reinterpret_cast<lng::Slot*>(slots + (uint64_t)(blockIdx.x * kStWPB + wv) * sizeof(lng::Slot));
  const uint32_t total =
      wave::uflu(__hip_atomic_load(&counters[kCtrRequeue], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  if (total == 0) return;
  // Documents of heavy_kb and more (k_len_hist's length buckets, longest
  // first) take one wave tens of milliseconds (a 64 KB page ~40 ms): every
  // stage kernel would wait for them in turn, where the fused kernel waits
  // once while its other waves run the rest (C5: fused 51.6 ms, staged 91 ms;
  // C3's 16 KB pages: staged 77 ms, fused 86 ms).  A batch holding one goes
  // to the fused kernel whole.
  uint32_t heavy = 0;
  if (hist && heavy_kb && lane < kLenBuckets - (int)heavy_kb) heavy = hist[lane];   // buckets of (L >> 10) >= heavy_kb
  heavy = wave::wsum(heavy);
  // the fused kernel takes the batch, in list order (documents over kDocCap,
  // which it does not take, still come here)
  const bool fused = total <= small_total || heavy;
  // page batches (mean long document >= 8 KB; hist bucket b holds 63 - b KB)
  // split only their heaviest documents (lng::kParMinPages)
  int par_min = lng::kParMin;
  if (hist) {
    uint64_t cnt = 0, kb = 0;
    for (int b = 0; b < kLenBuckets; ++b) {
      const uint64_t c = wave::uflu(hist[b]);
      cnt += c;
      kb += c * (uint64_t)(kLenBuckets - 1 - b);
    }
    if (cnt && kb >= 8 * cnt) par_min = lng::kParMinPages;
  }
  const bool exact = lng::space_lowers_to_space(T);
  const uint64_t units = pool_bytes >> 4;
  for (;;) {
    const uint32_t k = wave::uflu(atomicAdd(&counters[kCtrStDqSpan], lane == 0 ? 1u : 0u));
    if (k >= total) break;                       // every wave reaches this exit
    const uint32_t i = list[k];
    const uint64_t a = offs[i], L = offs[i + 1] - a;
    if (fused && L <= (uint64_t)(lng::kDocCap - 64)) {
      if (lane == 0) fall_list[atomicAdd(&counters[kCtrStFall], 1u)] = i;
      continue;
    }
    const uint8_t spi = special ? special[i] : (uint8_t)0;
    const bool rw = (spi & kSpecialRewritten) != 0;
    const bool hbig = rw && hpos && L >= (uint64_t)kMaxScriptBytes;   // (the soft limit's page offsets)
    const uint32_t* hp = hbig ? hpos + a : nullptr;
    const uint32_t* hg = hbig ? hgap + a : nullptr;
    uint64_t at = lng::kStNone;
    // (pages the HTML rewrite did not take go to the fused kernel, whose
    // sequential span source scans them in HTML mode)
    const bool take = exact && !(spi & kSpecialHtml) && i != fault_doc;
    if (take && L <= (uint64_t)(lng::kDocCap - 64)) {
      const DocView dv{(rw ? hbuf : buf) + a, (int)L, rw ? hflag + a : nullptr, hp, hg};
      at = lng::st_spans(T, dv, S, pool, units, &counters[kCtrStPool], lane, par_min);
    } else if (take && L <= lng::kStBigMax) {   // over kDocCap: a worst-case region
      const uint64_t u = (lng::st_big_bytes(L) + 15) >> 4;
      uint32_t got = 0;
      if (lane == 0) got = atomicAdd(&counters[kCtrStPool], (uint32_t)u);
      got = wave::uflu(__shfl((int)got, 0, 64));
      if ((uint64_t)got + u <= units) {
        const DocView dv{(rw ? hbuf : buf) + a, (int)L, rw ? hflag + a : nullptr, hp, hg};
        if (lng::st_spans_big(T, dv, S, pool + ((uint64_t)got << 4), lane, par_min)) at = (uint64_t)got << 4;
      }
    }
    // a span-parallel document (more than kParMin spans): its groups to the group list
    uint32_t ng = 0, gb = 0, nsp = 0;
    if (at != lng::kStNone) {
      const lng::StHdr* h = reinterpret_cast<const lng::StHdr*>(pool + at);
      nsp = wave::uflu(gld(&h->nsp));
      if (wave::uflu(gld(&h->par))) {
        ng = (nsp + lng::kParG - 1) / lng::kParG;
        if (lane == 0) gb = atomicAdd(&counters[kCtrStG1], ng);
        gb = wave::uflu(__shfl((int)gb, 0, 64));
        const bool fits = (uint64_t)gb + ng <= gcap;
        for (uint32_t g = lane; g < ng && gb + g < gcap; g += 64)
          group_list[gb + g] = fits ? ((uint64_t)k | ((uint64_t)g << 32)) : ~0ull;   // (~0: a skipped entry)
        if (!fits) at = lng::kStNone;
      }
    }
    if (lane == 0) {
      if (at == lng::kStNone) {
        fall_list[atomicAdd(&counters[kCtrStFall], 1u)] = i;
      } else {
        meta[k] = at;
        if (ng) par_list[atomicAdd(&counters[kCtrStPar1], 1u)] = k;
        else st_put(ok_list, counters, kCtrStOk, kCtrStOkH, n, nsp > kHeavySpans, k);
      }
    }
  }
}

template <bool P2>
__global__ __launch_bounds__(64 * kStWPB, LNG_ST_WPS) void k_lscore(
    const DevTables* __restrict__ Tp, const uint32_t* __restrict__ list, cld_result* __restrict__ out,
    uint8_t* __restrict__ slots, uint8_t* __restrict__ pool, const uint64_t* __restrict__ meta,
    const uint32_t* __restrict__ in_list, uint32_t* __restrict__ p2_list, uint32_t* __restrict__ fall_list,
    uint32_t* __restrict__ counters, uint32_t cflags, const uint8_t* __restrict__ special,
    const uint32_t* __restrict__ priors, uint32_t n) {
  __shared__ StSmem smem[kStWPB];
  const DevTables& T = *Tp;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  lng::Slot& S = *reinterpret_cast<lng::Slot*>(slots + (uint64_t)(blockIdx.x * kStWPB + wv) * sizeof(lng::Slot));
  const uint32_t nh = st_count(counters, P2 ? kCtrStP2H : kCtrStOkH);
  const uint32_t total = nh + st_count(counters, P2 ? kCtrStP2 : kCtrStOk);
  if (total == 0) return;
  if (lane == 0) {
    smem[wv].dbg = nullptr;
    smem[wv].dbg_pos = 0;
    smem[wv].prof = nullptr;
  }
  for (;;) {
    const uint32_t e = wave::uflu(atomicAdd(&counters[P2 ? kCtrStDqS2 : kCtrStDqS1], lane == 0 ? 1u : 0u));
    if (e >= total) break;                       // every wave reaches this exit
    const uint32_t k = st_get(in_list, nh, n, e);
    if (P2 && (k & 0x80000000u)) continue;       // a span-parallel document: k_lgroup / k_lfinish
    const uint64_t at = meta[k];
    if (P2 && at == lng::kStNone) continue;      // k_lrep handed it to the fused k_long
    const uint32_t i = list[k];
    const uint8_t spi = special ? special[i] : (uint8_t)0;
    const int r = lng::st_score(T, S, smem[wv], pool + at, P2, &out[i], cflags,
                                (spi & kSpecialPriors) ? priors + 16ull * i : nullptr, lane);
    const uint32_t nsp = (!P2 && r == 0) ? wave::uflu(gld(&reinterpret_cast<const lng::StHdr*>(pool + at)->nsp)) : 0u;
    if (lane == 0) {
      if (r == 1) {
        atomicAdd(&counters[P2 ? kCtrPass2 : kCtrPass1], 1u);
      } else if (r == 0 && !P2) {
        st_put(p2_list, counters, kCtrStP2, kCtrStP2H, n, nsp > kHeavySpans, k);
      } else {                                   // capacity (the LDS window): the fused kernel redoes it
        fall_list[atomicAdd(&counters[kCtrStFall], 1u)] = i;
      }
    }
  }
}

// Span-parallel documents (cld_long.hip "span-parallel scoring"): kParG
// spans per wave (k_lgroup), then the document level per document
// (k_lfinish), for pass 1 and -- after k_lrep -- pass 2.
using ParSmem = lng::SmemT<LNG_ST_TEXT, false, true>;
using FinSmem = lng::SmemT<16, false>;

template <bool P2>
__global__ __launch_bounds__(64 * kStWPB, LNG_ST_WPS) void k_lgroup(
    const DevTables* __restrict__ Tp, const uint32_t* __restrict__ list, uint8_t* __restrict__ slots,
    uint8_t* __restrict__ pool, const uint64_t* __restrict__ meta, const uint64_t* __restrict__ group_list,
    uint32_t gcap, uint32_t* __restrict__ counters, uint32_t cflags, const uint8_t* __restrict__ special,
    const uint32_t* __restrict__ priors) {
  __shared__ ParSmem smem[kStWPB];
  const DevTables& T = *Tp;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  lng::Slot& S = *reinterpret_cast<lng::Slot*>(slots + (uint64_t)(blockIdx.x * kStWPB + wv) * sizeof(lng::Slot));
  uint32_t total = wave::uflu(
      __hip_atomic_load(&counters[P2 ? kCtrStG2 : kCtrStG1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  total = total < gcap ? total : gcap;
  if (total == 0) return;
  if (lane == 0) {
    smem[wv].dbg = nullptr;
    smem[wv].dbg_pos = 0;
    smem[wv].prof = nullptr;
  }
  for (;;) {
    const uint32_t e = wave::uflu(atomicAdd(&counters[P2 ? kCtrStDqG2 : kCtrStDqG1], lane == 0 ? 1u : 0u));
    if (e >= total) break;                       // every wave reaches this exit
    const uint64_t it = group_list[e];
    if (it == ~0ull) continue;
    const uint32_t k = (uint32_t)it, g = (uint32_t)(it >> 32);
    const uint64_t at = meta[k];
    if (at == lng::kStNone) continue;            // (pass 2: k_lrep handed it to the fused k_long)
    const uint32_t i = list[k];
    const uint8_t spi = special ? special[i] : (uint8_t)0;
    const int nsp = (int)wave::uflu(gld(&reinterpret_cast<const lng::StHdr*>(pool + at)->nsp));
    const int j0 = (int)g * lng::kParG, j1 = min(nsp, j0 + lng::kParG);
    (void)lng::st_group(T, S, smem[wv], pool + at, j0, j1, cflags,
                        (spi & kSpecialPriors) ? priors + 16ull * i : nullptr, lane);
  }
}

template <bool P2>
__global__ __launch_bounds__(64 * kStWPB, LNG_ST_WPS) void k_lfinish(
    const DevTables* __restrict__ Tp, const uint32_t* __restrict__ list, cld_result* __restrict__ out,
    uint8_t* __restrict__ pool, const uint64_t* __restrict__ meta, uint32_t* __restrict__ par_lists, uint32_t n,
    uint64_t* __restrict__ group_list2, uint32_t gcap, uint32_t* __restrict__ p2_list,
    uint32_t* __restrict__ fall_list, uint32_t* __restrict__ counters, uint32_t cflags) {
  __shared__ FinSmem smem[kStWPB];
  const DevTables& T = *Tp;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const uint32_t* in_list = par_lists + (P2 ? n : 0);
  const uint32_t total = wave::uflu(
      __hip_atomic_load(&counters[P2 ? kCtrStPar2 : kCtrStPar1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  if (total == 0) return;
  for (;;) {
    const uint32_t e = wave::uflu(atomicAdd(&counters[P2 ? kCtrStDqF2 : kCtrStDqF1], lane == 0 ? 1u : 0u));
    if (e >= total) break;                       // every wave reaches this exit
    const uint32_t k = in_list[e];
    const uint64_t at = meta[k];
    if (P2 && at == lng::kStNone) continue;      // k_lrep handed it to the fused k_long
    const uint32_t i = list[k];
    const int r = lng::st_par_finish(T, smem[wv], pool + at, P2, &out[i], cflags, lane);
    if (r == 0 && !P2) {                         // pass 2: Repeats (k_lrep), then its groups again
      const int nsp = (int)wave::uflu(gld(&reinterpret_cast<const lng::StHdr*>(pool + at)->nsp));
      const uint32_t ng = (uint32_t)(nsp + lng::kParG - 1) / lng::kParG;
      uint32_t gb = 0;
      if (lane == 0) gb = atomicAdd(&counters[kCtrStG2], ng);
      gb = wave::uflu(__shfl((int)gb, 0, 64));
      const bool fits = (uint64_t)gb + ng <= gcap;
      for (uint32_t g = lane; g < ng && gb + g < gcap; g += 64)
        group_list2[gb + g] = fits ? ((uint64_t)k | ((uint64_t)g << 32)) : ~0ull;
      if (lane == 0) {
        if (fits) {
          st_put(p2_list, counters, kCtrStP2, kCtrStP2H, n, true, k | 0x80000000u);
          par_lists[n + atomicAdd(&counters[kCtrStPar2], 1u)] = k;
        } else {
          fall_list[atomicAdd(&counters[kCtrStFall], 1u)] = i;
        }
      }
    } else if (lane == 0) {
      if (r == 1) atomicAdd(&counters[P2 ? kCtrPass2 : kCtrPass1], 1u);
      else fall_list[atomicAdd(&counters[kCtrStFall], 1u)] = i;   // (records outgrew their room, a group failed)
    }
  }
}

__global__ __launch_bounds__(64, LNG_REP_WPS) void k_lrep(const uint32_t* __restrict__ list,
                                                         uint8_t* __restrict__ slots, uint8_t* __restrict__ pool,
                                                         uint64_t* __restrict__ meta,
                                                         const uint32_t* __restrict__ p2_list,
                                                         uint32_t* __restrict__ fall_list,
                                                         uint32_t* __restrict__ counters, uint32_t n) {
  __shared__ __attribute__((aligned(16))) uint16_t pred[kPredictionTableSize];
  const int lane = threadIdx.x & 63;
  lng::Slot& S = *reinterpret_cast<lng::Slot*>(slots + (uint64_t)blockIdx.x * sizeof(lng::Slot));
  const uint32_t nh = st_count(counters, kCtrStP2H);
  const uint32_t total = nh + st_count(counters, kCtrStP2);
  if (total == 0) return;                        // (no dequeue atomics: 5,120 of them on one word took 80 us)
  for (;;) {
    const uint32_t e = wave::uflu(atomicAdd(&counters[kCtrStDqRep], lane == 0 ? 1u : 0u));
    if (e >= total) break;                       // every wave reaches this exit
    const uint32_t k = st_get(p2_list, nh, n, e) & 0x7FFFFFFFu;   // (bit 31: a span-parallel document)
    if (!lng::st_rep(pred, S, pool + meta[k], lane) && lane == 0) {   // (the fused kernel redoes it whole)
      meta[k] = lng::kStNone;
      fall_list[atomicAdd(&counters[kCtrStFall], 1u)] = list[k];
      atomicAdd(&counters[kCtrWhy + lng::kWhySpan], 1u);
    }
  }
}

// Longest-first order for k_long's persistent grid (LPT list scheduling):
// documents land in 1 KB length buckets, longest bucket first, so the last
// documents a wave picks up are short ones and the grid drains evenly.  The
// order inside a bucket is whatever the atomics give; a document's result
// never depends on which wave scored it or when.
__device__ __forceinline__ uint32_t len_bucket(uint64_t len) {
  const uint64_t b = len >> 10;
  return (uint32_t)(kLenBuckets - 1) - (uint32_t)(b < kLenBuckets - 1 ? b : kLenBuckets - 1);
}

__global__ __launch_bounds__(256) void k_len_hist(const uint64_t* __restrict__ offs,
                                                 const uint32_t* __restrict__ list,
                                                 const uint32_t* __restrict__ counters,
                                                 uint8_t* __restrict__ key, uint32_t* __restrict__ hist) {
  __shared__ uint32_t h[kLenBuckets];
  if (threadIdx.x < kLenBuckets) h[threadIdx.x] = 0;
  __syncthreads();
  const uint32_t total = counters[kCtrRequeue];
  for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < total; k += gridDim.x * blockDim.x) {
    const uint32_t i = list[k];
    const uint32_t b = len_bucket(offs[i + 1] - offs[i]);
    key[k] = (uint8_t)b;
    atomicAdd(&h[b], 1u);
  }
  __syncthreads();
  if (threadIdx.x < kLenBuckets && h[threadIdx.x]) atomicAdd(&hist[threadIdx.x], h[threadIdx.x]);
}

__global__ __launch_bounds__(256) void k_len_scatter(const uint32_t* __restrict__ list,
                                                    const uint32_t* __restrict__ counters,
                                                    const uint8_t* __restrict__ key,
                                                    const uint32_t* __restrict__ hist,
                                                    uint32_t* __restrict__ cursor, uint32_t* __restrict__ sorted) {
  __shared__ uint32_t base[kLenBuckets];
  if (threadIdx.x == 0) {
    uint32_t s = 0;
    for (int b = 0; b < kLenBuckets; ++b) { base[b] = s; s += hist[b]; }
  }
  __syncthreads();
  // block-aggregated: positions inside the block from LDS counters, one
  // global atomic per (block, bucket) present -- a batch whose documents all
  // share a bucket (C3's pages) used to serialise on one cursor
  __shared__ uint32_t lcnt[kLenBuckets], lbase[kLenBuckets];
  const uint32_t total = counters[kCtrRequeue];
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t k0 = blockIdx.x * blockDim.x; k0 < total; k0 += stride) {
    if (threadIdx.x < kLenBuckets) lcnt[threadIdx.x] = 0;
    __syncthreads();
    const uint32_t k = k0 + threadIdx.x;
    const uint32_t b = k < total ? key[k] : 0u;
    const uint32_t pos = k < total ? atomicAdd(&lcnt[b], 1u) : 0u;
    __syncthreads();
    if (threadIdx.x < kLenBuckets && lcnt[threadIdx.x])
      lbase[threadIdx.x] = atomicAdd(&cursor[threadIdx.x], lcnt[threadIdx.x]);
    __syncthreads();
    if (k < total) sorted[base[b] + lbase[b] + pos] = list[k];
    __syncthreads();
  }
}

// Per (script, key) language / close set / expected score table for k_long.
__global__ __launch_bounds__(256) void k_build_keytab(DevTables T, uint64_t* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= 256 * 256) return;
  out[i] = lng::keytab_eval(T, i >> 8, i & 255);
}

// Tote adds per indirect entry of one scoring table (k_long reads them with
// one gather instead of the indirect langprob and then its kLgProbV2Tbl row).
__global__ __launch_bounds__(256) void k_build_adds(DevTables T, DevTbl t, uint64_t* __restrict__ out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= t.n_ind) return;
  const uint32_t lp = t.ind[i];
  out[i] = lp ? (lng::tote_adds(T, lp) | (1ull << 63)) : 0ull;
}

// Character property table (lng::cpt_eval over every 1-3 byte sequence).
__global__ __launch_bounds__(256) void k_build_cpt(DevTables T, uint64_t* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= lng::kCptSize) return;
  uint8_t b[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  int n;
  if (i < 128) {
    b[0] = (uint8_t)i;
    n = 1;
  } else if (i < 2176) {
    const int j = i - 128;
    b[0] = (uint8_t)(0xC0 | (j >> 6));
    b[1] = (uint8_t)(0x80 | (j & 63));
    n = 2;
  } else {
    const int j = i - 2176;
    b[0] = (uint8_t)(0xE0 | (j >> 12));
    b[1] = (uint8_t)(0x80 | ((j >> 6) & 63));
    b[2] = (uint8_t)(0x80 | (j & 63));
    n = 3;
  }
  out[i] = lng::cpt_eval(T, b, n);
}

// The flags word after the property table (T.cpt[kCptSize]): bit 0 = some
// 4-byte sequence (lead F0-F7, three continuation bytes) lowers differently in
// HTML mode than in plain text (the HTML half of a remap pair,
// utf8statetable.cc:755-762).  The reference's tables have none, so HTML pages
// with 4-byte characters take the rewrite (cld_html.hip html_lower_same).
__global__ __launch_bounds__(256) void k_build_cpt4(DevTables T, uint64_t* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= 8 << 18) return;
  const uint8_t b[4] = {(uint8_t)(0xF0 | (i >> 18)), (uint8_t)(0x80 | ((i >> 12) & 63)),
                        (uint8_t)(0x80 | ((i >> 6) & 63)), (uint8_t)(0x80 | (i & 63))};
  uint8_t lp[16], lh[16];
  const int fp = lower_replace_sm(T.lower, b, 4, lp, 16, true), fh = lower_replace_sm(T.lower, b, 4, lh, 16, false);
  bool diff = fp != fh;
  for (int k = 0; k < fp && k < 16; ++k) diff |= lp[k] != lh[k];
  if (diff) atomicOr(reinterpret_cast<unsigned int*>(out + lng::kCptSize), 1u);
}

}  // namespace cld

extern "C" {
size_t cld_cpt_entries() { return cld::lng::kCptSize + 1; }   // + the flags word (k_build_cpt4)
hipError_t cld_build_cpt(const DevTables* T, uint64_t* out, hipStream_t s) {
  hipLaunchKernelGGL(cld::k_build_cpt, dim3((cld::lng::kCptSize + 255) / 256), dim3(256), 0, s, *T, out);
  hipError_t e = hipMemsetAsync(out + cld::lng::kCptSize, 0, sizeof(uint64_t), s);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(cld::k_build_cpt4, dim3((8 << 18) / 256), dim3(256), 0, s, *T, out);
  return hipGetLastError();
}
size_t cld_keytab_entries() { return 256 * 256; }
size_t cld_adds_entries(const DevTables* T) {
  return (size_t)T->compat.n_ind + T->deltabi.n_ind + T->distinctbi.n_ind + T->quad.n_ind + T->quad2.n_ind +
         T->deltaocta.n_ind + T->distinctocta.n_ind;
}
hipError_t cld_build_adds(DevTables* T, uint64_t* out, hipStream_t s) {
  for (DevTbl* t : {&T->compat, &T->deltabi, &T->distinctbi, &T->quad, &T->quad2, &T->deltaocta, &T->distinctocta}) {
    t->adds = out;
    if (t->n_ind) hipLaunchKernelGGL(cld::k_build_adds, dim3((t->n_ind + 255) / 256), dim3(256), 0, s, *T, *t, out);
    out += t->n_ind;
  }
  return hipGetLastError();
}
hipError_t cld_build_keytab(const DevTables* T, uint64_t* out, hipStream_t s) {
  hipLaunchKernelGGL(cld::k_build_keytab, dim3(256), dim3(256), 0, s, *T, out);
  return hipGetLastError();
}
hipError_t cld_launch_order_long(const uint64_t* offs, const uint32_t* list, const uint32_t* counters,
                                 uint8_t* key, uint32_t* hist2, uint32_t* sorted, bool zeroed, hipStream_t s) {
  // hist2: 2 * kLenBuckets u32 (histogram, then scatter cursors), zeroed here
  // unless k_route already did (zeroed)
  if (!zeroed) {
    hipError_t e = hipMemsetAsync(hist2, 0, 2 * cld::kLenBuckets * sizeof(uint32_t), s);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(cld::k_len_hist, dim3(512), dim3(256), 0, s, offs, list, counters, key, hist2);
  hipLaunchKernelGGL(cld::k_len_scatter, dim3(512), dim3(256), 0, s, list, counters, key, hist2,
                     hist2 + cld::kLenBuckets, sorted);
  return hipGetLastError();
}
size_t cld_long_slot_bytes() { return sizeof(cld::lng::Slot); }
int cld_long_waves_per_simd() { return LNG_WPS; }

hipError_t cld_launch_long(const DevTables* d_T, const uint8_t* buf, const uint64_t* offs, const uint32_t* list,
                           cld_result* out, uint8_t* slots, int n_slots, uint32_t* seq_list,
                           uint32_t* counters, uint32_t* trace, uint32_t* dbg, uint32_t dbg_doc,
                           unsigned long long* prof, uint32_t cflags, const uint8_t* special,
                           const uint32_t* priors, const uint8_t* hbuf, const uint8_t* hflag, const uint32_t* hpos,
                           const uint32_t* hgap, uint32_t fault_doc, cld_result* spec_out, uint32_t* spec_take,
                           int ctr_total, int ctr_deq, hipEvent_t mid, hipStream_t s) {
  if (n_slots < kLongWPB) return hipErrorInvalidValue;
  dim3 grid(n_slots / kLongWPB), block(64 * kLongWPB);
  // diagnostics (trace / debug dump / stage cycles) live in their own instantiation:
  // they cost the production kernel registers even when switched off.  Then
  // the documents it handed on (seq_list, counters[kCtrRequeue2]), on the
  // sequential span source; `mid` (nullable) is recorded between the two.
  if (trace || dbg || prof) {
    hipLaunchKernelGGL((cld::k_long<kLongWPB, true, false>), grid, block, 0, s, d_T, buf, offs, list, out, slots,
                       seq_list, counters, trace, dbg, dbg_doc, prof, cflags, special, priors, hbuf, hflag,
                       fault_doc, nullptr, nullptr, nullptr, nullptr, hpos, hgap, spec_out, spec_take, ctr_total,
                       ctr_deq);
    if (mid) (void)hipEventRecord(mid, s);
    hipLaunchKernelGGL((cld::k_long<kLongWPB, true, false, true>), grid, block, 0, s, d_T, buf, offs, seq_list, out,
                       slots, seq_list, counters, trace, dbg, dbg_doc, prof, cflags, special, priors, hbuf, hflag,
                       fault_doc, nullptr, nullptr, nullptr, nullptr, hpos, hgap, nullptr, nullptr, kCtrRequeue2,
                       kCtrDequeue2);
  } else {
    hipLaunchKernelGGL((cld::k_long<kLongWPB, false, false>), grid, block, 0, s, d_T, buf, offs, list, out, slots,
                       seq_list, counters, trace, dbg, dbg_doc, prof, cflags, special, priors, hbuf, hflag,
                       fault_doc, nullptr, nullptr, nullptr, nullptr, hpos, hgap, spec_out, spec_take, ctr_total,
                       ctr_deq);
    if (mid) (void)hipEventRecord(mid, s);
    hipLaunchKernelGGL((cld::k_long<kLongWPB, false, false, true>), grid, block, 0, s, d_T, buf, offs, seq_list, out,
                       slots, seq_list, counters, trace, dbg, dbg_doc, prof, cflags, special, priors, hbuf, hflag,
                       fault_doc, nullptr, nullptr, nullptr, nullptr, hpos, hgap, nullptr, nullptr, kCtrRequeue2,
                       kCtrDequeue2);
  }
  return hipGetLastError();
}

size_t cld_long_spec_docs(int n_slots) { return (size_t)n_slots / cld::kSpecShare; }

int cld_staged_waves_per_simd() {
  const int a = LNG_ST_WPS > LNG_REP_WPS ? LNG_ST_WPS : LNG_REP_WPS;
  return a > LNG_SPAN_WPS ? a : LNG_SPAN_WPS;
}

hipError_t cld_launch_staged(const DevTables* d_T, const uint8_t* buf, const uint64_t* offs, const uint32_t* list,
                             cld_result* out, uint8_t* slots, int n_waves, uint8_t* pool, uint64_t pool_bytes,
                             uint64_t* meta, uint32_t* ok_list, uint32_t* p2_list, uint32_t* fall_list,
                             uint32_t* counters, uint32_t cflags, const uint8_t* special,
                             const uint32_t* priors, const uint8_t* hbuf, const uint8_t* hflag, const uint32_t* hpos,
                             const uint32_t* hgap, uint32_t fault_doc, uint32_t small_total, const uint32_t* hist,
                             uint32_t heavy_kb, uint32_t* par_lists,
                             size_t n, size_t gcap, hipStream_t s) {
  // n_waves: the slots (resident waves) of the widest launch below
  const int per_simd = cld_staged_waves_per_simd();
  const int cus = n_waves / (4 * per_simd);
  if (cus < 1) return hipErrorInvalidValue;
  const dim3 gst(cus * 4 * LNG_ST_WPS / cld::kStWPB), gsp(cus * 4 * LNG_SPAN_WPS / cld::kStWPB), bst(64 * cld::kStWPB);
  uint64_t* gl1 = reinterpret_cast<uint64_t*>(par_lists + 2 * n);
  uint64_t* gl2 = gl1 + gcap;
  const uint32_t gc = (uint32_t)gcap, nn = (uint32_t)n;
  hipLaunchKernelGGL(cld::k_lspan, gsp, bst, 0, s, d_T, buf, offs, list, slots, pool, pool_bytes, meta, ok_list,
                     fall_list, counters, special, hbuf, hflag, hpos, hgap, fault_doc, small_total, hist, par_lists,
                     gl1, gc, heavy_kb, nn);
  hipLaunchKernelGGL(cld::k_lscore<false>, gst, bst, 0, s, d_T, list, out, slots, pool, meta, ok_list, p2_list,
                     fall_list, counters, cflags, special, priors, nn);
  hipLaunchKernelGGL(cld::k_lgroup<false>, gst, bst, 0, s, d_T, list, slots, pool, meta, gl1, gc, counters, cflags,
                     special, priors);
  hipLaunchKernelGGL(cld::k_lfinish<false>, gst, bst, 0, s, d_T, list, out, pool, meta, par_lists, nn, gl2, gc,
                     p2_list, fall_list, counters, cflags);
  hipLaunchKernelGGL(cld::k_lrep, dim3(cus * 4 * LNG_REP_WPS), dim3(64), 0, s, list, slots, pool, meta, p2_list,
                     fall_list, counters, nn);
  hipLaunchKernelGGL(cld::k_lscore<true>, gst, bst, 0, s, d_T, list, out, slots, pool, meta, p2_list, p2_list,
                     fall_list, counters, cflags, special, priors, nn);
  hipLaunchKernelGGL(cld::k_lgroup<true>, gst, bst, 0, s, d_T, list, slots, pool, meta, gl2, gc, counters, cflags,
                     special, priors);
  hipLaunchKernelGGL(cld::k_lfinish<true>, gst, bst, 0, s, d_T, list, out, pool, meta, par_lists, nn, gl2, gc,
                     p2_list, fall_list, counters, cflags);
  return hipGetLastError();
}

size_t cld_vec_slot_bytes() { return sizeof(cld::lng::VecSlot); }

hipError_t cld_launch_route_vec(int n, uint32_t* counters, uint32_t* long_list, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(cld::k_route_vec, dim3((n + 255) / 256), dim3(256), 0, s, n, counters, long_list);
  return hipGetLastError();
}

hipError_t cld_launch_long_vec(const DevTables* d_T, const uint8_t* buf, const uint64_t* offs, const uint32_t* list,
                               cld_result* out, uint8_t* slots, uint8_t* vslots, int n_slots, uint32_t* seq_list,
                               uint32_t* counters, uint32_t cflags, const uint8_t* special, const uint32_t* priors,
                               const uint8_t* hbuf, const uint8_t* hflag, const uint32_t* hpos, const uint32_t* hgap,
                               cld_chunk* pool, const uint64_t* pool_off, int32_t* n_chunks, hipStream_t s) {
  if (n_slots < kLongWPB) return hipErrorInvalidValue;
  dim3 grid(n_slots / kLongWPB), block(64 * kLongWPB);
  hipLaunchKernelGGL((cld::k_long<kLongWPB, false, true>), grid, block, 0, s, d_T, buf, offs, list, out, slots,
                     seq_list, counters, nullptr, nullptr, 0xFFFFFFFFu, nullptr, cflags, special, priors, hbuf,
                     hflag, 0xFFFFFFFFu, vslots, pool, pool_off, n_chunks, hpos, hgap, nullptr, nullptr, kCtrRequeue,
                     kCtrDequeue);
  hipLaunchKernelGGL((cld::k_long<kLongWPB, false, true, true>), grid, block, 0, s, d_T, buf, offs, seq_list, out,
                     slots, seq_list, counters, nullptr, nullptr, 0xFFFFFFFFu, nullptr, cflags, special, priors, hbuf,
                     hflag, 0xFFFFFFFFu, vslots, pool, pool_off, n_chunks, hpos, hgap, nullptr, nullptr, kCtrRequeue2,
                     kCtrDequeue2);
  return hipGetLastError();
}

hipError_t cld_launch_vec_gather(const cld_chunk* pool, const uint64_t* pool_off, const int32_t* n_chunks,
                                 const uint64_t* pos, int n, cld_chunk* dst, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(cld::k_vec_gather, dim3((n + 255) / 256), dim3(256), 0, s, pool, pool_off, n_chunks, pos, n, dst);
  return hipGetLastError();
}
size_t cld_wave_smem_bytes() { return sizeof(cld::wave::Smem<kWaveCap>); }

hipError_t cld_launch_wave(const DevTables* T, const uint8_t* buf, const uint64_t* offs, int n,
                           cld_result* out, uint32_t* requeue_list, uint32_t* counters,
                           unsigned long long* prof, const uint8_t* special, uint32_t* special_list,
                           int special_ctr, uint32_t cflags, const uint32_t* priors, const uint8_t* hbuf,
                           const uint8_t* hflag, uint32_t* hist2, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(cld::k_route, dim3((n + 255) / 256), dim3(256), 0, s, offs, n, special, kWaveCap, counters,
                     requeue_list, special_list, special_ctr, hist2);
  const int per = ((n + kWaveWPB - 1) / kWaveWPB + 7) / 8;   // k_wave's XCD slices
  dim3 grid(8 * per), block(64 * kWaveWPB);
  hipLaunchKernelGGL((cld::k_wave<kWaveCap, kWaveWPB>), grid, block, 0, s, *T, buf, offs, n, out,
                     requeue_list, counters, prof, special, special_list, special_ctr, cflags, priors, hbuf, hflag);
  return hipGetLastError();
}

hipError_t cld_launch_wave_only(const DevTables* T, const uint8_t* buf, const uint64_t* offs, int n, cld_result* out,
                                uint32_t* requeue_list, uint32_t* counters, uint32_t cflags, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  const int per = ((n + kWaveWPB - 1) / kWaveWPB + 7) / 8;
  hipLaunchKernelGGL((cld::k_wave<kWaveCap, kWaveWPB>), dim3(8 * per), dim3(64 * kWaveWPB), 0, s, *T, buf, offs, n,
                     out, requeue_list, counters, nullptr, nullptr, nullptr, 0, cflags, nullptr, nullptr, nullptr);
  return hipGetLastError();
}

hipError_t cld_launch_html_rewrite(const DevTables* d_T, const uint8_t* buf, const uint64_t* offs, int n,
                                   uint8_t* special, uint8_t* hbuf, uint8_t* hflag, uint32_t* hpos, uint32_t* hgap,
                                   int hpos_min, unsigned long long* prof, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  const int blocks = std::min((n + cld::kHtmlWPB - 1) / cld::kHtmlWPB, 2048);   // persistent: pages by stride
  hipLaunchKernelGGL(cld::k_html_rewrite, dim3(blocks), dim3(64 * cld::kHtmlWPB), 0, s, d_T, buf, offs, n, special,
                     hbuf, hflag, hpos, hgap, hpos_min, prof);
  return hipGetLastError();
}

}
