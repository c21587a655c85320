// cld_kernels.h -- launch interface between the host runtime and the kernels.
#ifndef CLD_KERNELS_H_
#define CLD_KERNELS_H_
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>
#include "cld_device.h"

// Wavefront-per-document bucket (cld_wave.hip)
constexpr int kWaveCap = 256;
#ifndef WAVE_WPB
#define WAVE_WPB 1
#endif
constexpr int kWaveWPB = WAVE_WPB;   // waves (documents) per workgroup
// Largest kLgProbV2Tbl score byte the packed wave tote accepts (runtime checks the blob)
constexpr int kMaxLgProbScore = 16;


// Device counter slots (three 64-byte lines, zeroed per batch)
// kCtrRequeue/kCtrDequeue: the k_long list (documents longer than k_wave takes,
// the ones it hands on, HTML pages the rewrite did not take);
// kCtrSpecial: those HTML pages.  (kCtrRequeue2 / kCtrDequeue2: unused.)
enum { kCtrRequeue = 0, kCtrDequeue = 1, kCtrPass1 = 2, kCtrPass2 = 3, kCtrPass3 = 4, kCtrError = 5,
       kCtrRequeue2 = 6, kCtrDequeue2 = 7, kCtrWhy = 8 /* 8 slots: k_long re-queue reasons */,
       kCtrSpecial = 16, kCtrSpecTake = 17 /* k_long: speculative pass-2 results taken */,
       kCtrSpecDone = 18 /* k_long: waves finished (speculating launches) */,
       // staged long-document path (k_lspan / k_lscore / k_lrep): list counts and dequeue cursors
       kCtrStFall = 19 /* to the fused k_long */, kCtrStDqSpan = 20, kCtrStOk = 21 /* spans stored */,
       kCtrStDqS1 = 22, kCtrStP2 = 23 /* pass 2 */, kCtrStDqRep = 24, kCtrStDqS2 = 25, kCtrStDqFall = 26,
       kCtrStPool = 27 /* store 16-byte units taken */,
       // span-parallel documents: group lists and document lists of passes 1 and 2
       kCtrStG1 = 28, kCtrStDqG1 = 29, kCtrStPar1 = 30, kCtrStDqF1 = 31,
       kCtrStG2 = 32, kCtrStDqG2 = 33, kCtrStPar2 = 34, kCtrStDqF2 = 35,
       // heavy (many-span) entries of the stored and pass-2 lists, filled from the top
       kCtrStOkH = 36, kCtrStP2H = 37,
       kCtrSeq = 38 /* k_long: documents scored on the sequential span source (cld_seq.hip) */, kCtrSlots = 48 };
// Per-document routing bits of cld_detect_batch_ex (special[i])
// kSpecialRewritten: an HTML document k_html_rewrite turned into plain text
// (hbuf / hflag); k_long scores the original page if it needs the sequential
// span source.  kSpecialNoVec (vec mode): a rewritten page whose offset map the
// parallel span builder cannot reproduce (cld_html.hip); k_long<VEC> scans the
// original page with the sequential span source.
enum : uint8_t { kSpecialHtml = 1, kSpecialPriors = 2, kSpecialRewritten = 4, kSpecialNoVec = 8 };
// k_long: waves per workgroup
constexpr int kLongWPB = 4;

extern "C" {
// ResultChunkVector mode: k_route_vec lists every document under
// counters[kCtrRequeue]; k_long<VEC> then scores them with one VecSlot per
// resident wave (vslots: n_slots * cld_vec_slot_bytes()); document i builds
// its vector in pool[pool_off[i] .. pool_off[i+1]) and writes its size (or
// -1: it outgrew its region, or has no result) to n_chunks[i].
size_t cld_vec_slot_bytes();
hipError_t cld_launch_route_vec(int n, uint32_t* counters, uint32_t* long_list, hipStream_t s);
hipError_t cld_launch_long_vec(const DevTables* d_T, const uint8_t* buf, const uint64_t* offs, const uint32_t* list,
                               cld_result* out, uint8_t* slots, uint8_t* vslots, int n_slots, uint32_t* seq_list,
                               uint32_t* counters, uint32_t cflags, const uint8_t* special, const uint32_t* priors,
                               const uint8_t* hbuf, const uint8_t* hflag, const uint32_t* hpos, const uint32_t* hgap,
                               cld_chunk* pool, const uint64_t* pool_off, int32_t* n_chunks, hipStream_t s);
hipError_t cld_launch_vec_gather(const cld_chunk* pool, const uint64_t* pool_off, const int32_t* n_chunks,
                                 const uint64_t* pos, int n, cld_chunk* dst, hipStream_t s);
// special (nullable): per-document kSpecial* bits; HTML documents are appended
// to special_list under counters[special_ctr] instead of being scored, hinted
// ones (kSpecialPriors) are scored with their 16 ApplyHints langprobs
// (priors + 16 * i; k_long reads the same two arrays).
// cflags (every launcher): the caller's public CLD2 flags, CLD_FLAG_SCORE_AS_QUADS /
// CLD_FLAG_BEST_EFFORT (compact_lang_det.h:343, :349), the same for every document.
hipError_t cld_launch_wave(const DevTables* T, const uint8_t* buf, const uint64_t* offs, int n,
                           cld_result* out, uint32_t* requeue_list, uint32_t* counters,
                           unsigned long long* prof, const uint8_t* special, uint32_t* special_list,
                           int special_ctr, uint32_t cflags, const uint32_t* priors, const uint8_t* hbuf,
                           const uint8_t* hflag, uint32_t* hist2, hipStream_t s);
// k_wave alone, without k_route: the caller guarantees every document is at
// most kWaveCap bytes (run_tiny's request-sized batches).  Documents the wave
// kernel cannot finish are listed under counters[kCtrRequeue], or, with
// requeue_list == nullptr (counters unused), marked in their result:
// summary_lang = kWaveRequeued.
constexpr uint16_t kWaveRequeued = 0xFFFE;
// kMaxScriptBytes (cld_prims.hip): rewritten HTML pages this long and
// longer carry page offsets (hpos / hgap) for the span soft limit
constexpr int kHtmlSoftMin = 40928;
// lng::kDocCap (cld_long.hip): the fused k_long takes documents up to this
// many bytes less 64; longer ones need the staged path's big-document regions
constexpr uint64_t kLongDocCap = 1u << 20;
hipError_t cld_launch_wave_only(const DevTables* T, const uint8_t* buf, const uint64_t* offs, int n, cld_result* out,
                                uint32_t* requeue_list, uint32_t* counters, uint32_t cflags, hipStream_t s);
// HTML documents of the batch (special & kSpecialHtml) rewritten into plain
// text (cld_html.hip): hbuf / hflag are indexed like buf (offs); special is
// updated in place (kSpecialHtml -> kSpecialRewritten for each rewritten page);
// prof (nullable, CLD_PROFILE_STAGES=1): cycles of step 2 summed into prof[0].
// hpos (nullable): per rewritten byte, its page offset (vec mode's MapBack;
// the span soft limit of pages of kMaxScriptBytes and more); hgap (with hpos):
// at a byte that follows dropped '&'s, where they began.  Written for pages of
// hpos_min bytes and more (vec mode 0, plain kMaxScriptBytes).
hipError_t cld_launch_html_rewrite(const DevTables* d_T, const uint8_t* buf, const uint64_t* offs, int n,
                                   uint8_t* special, uint8_t* hbuf, uint8_t* hflag, uint32_t* hpos, uint32_t* hgap,
                                   int hpos_min, unsigned long long* prof, hipStream_t s);
size_t cld_wave_smem_bytes();
// (hist2: zeroed by k_route when cld_launch_wave was given it: zeroed = true)
hipError_t cld_launch_order_long(const uint64_t* offs, const uint32_t* list, const uint32_t* counters,
                                 uint8_t* key, uint32_t* hist2, uint32_t* sorted, bool zeroed, hipStream_t s);
size_t cld_long_slot_bytes();
size_t cld_cpt_entries();
hipError_t cld_build_cpt(const DevTables* T, uint64_t* out, hipStream_t s);
size_t cld_keytab_entries();
hipError_t cld_build_keytab(const DevTables* T, uint64_t* out, hipStream_t s);
// ind -> tote adds for the seven scoring tables, back to back in `out`
// (compat, deltabi, distinctbi, quad, quad2, deltaocta, distinctocta order);
// sets each table's `adds` pointer in *T.
size_t cld_adds_entries(const DevTables* T);
hipError_t cld_build_adds(DevTables* T, uint64_t* out, hipStream_t s);
int cld_long_waves_per_simd();
size_t cld_strip_scratch_bytes(int n);
hipError_t cld_launch_strip_offsets(const uint8_t* buf, const uint64_t* offs, int n, uint32_t flags,
                                    uint64_t* out_offs, void* scratch, hipStream_t s);
hipError_t cld_launch_strip_write(const uint8_t* buf, const uint64_t* offs, int n, uint32_t flags,
                                  const uint64_t* out_offs, uint8_t* out, hipStream_t s);
// fault_doc (k_long): test hook, batch index of a document made to fail
// (0xFFFFFFFF: none): it gets no result (summary CLD_LANG_FAILED).
// seq_list (n entries, counters[kCtrRequeue2]): the documents k_long hands to
// its SEQ instantiation (the sequential span source, cld_seq.hip), which the
// launch runs right after it.
// d_T: the device's DevTables copy in HBM (k_long reads the table set through
// it: holding the by-value kernel argument in registers made the kernel spill
// it to scratch and reload table fields from there at every probe)
hipError_t cld_launch_long(const DevTables* d_T, const uint8_t* buf, const uint64_t* offs, const uint32_t* list,
                           cld_result* out, uint8_t* slots, int n_slots, uint32_t* seq_list,
                           uint32_t* counters, uint32_t* trace, uint32_t* dbg, uint32_t dbg_doc,
                           unsigned long long* prof, uint32_t cflags, const uint8_t* special,
                           const uint32_t* priors, const uint8_t* hbuf, const uint8_t* hflag, const uint32_t* hpos,
                           const uint32_t* hgap, uint32_t fault_doc, cld_result* spec_out, uint32_t* spec_take,
                           int ctr_total, int ctr_deq, hipEvent_t mid, hipStream_t s);
// spec_out / spec_take (nullable: no speculation): cld_long_spec_docs(n_slots)
// results and u32 entries, k_long's speculative pass-2 results for the
// longest documents of a small batch.
size_t cld_long_spec_docs(int n_slots);
// Staged long-document path (cld_long.hip, "staged long-document path"):
// k_lspan over `list` (counters[kCtrRequeue] documents) stores pass 1's spans
// in `pool` (meta[k]: the region of list entry k) and lists the entries it
// took (ok_list) and the documents it did not (fall_list, for the fused
// k_long: cld_launch_long with kCtrStFall / kCtrStDqFall); k_lscore scores
// pass 1 (to p2_list when not good enough), k_lrep runs Repeats over those,
// k_lscore<pass 2> finishes them.  small_total: a list this short goes whole
// to the fused kernel, in order (its speculation is for small batches), and
// so does a list holding a document of heavy_kb KB or more (hist: k_len_hist's
// length buckets; nullable; heavy_kb 0: no such rule).
// n_waves: resident waves the staged kernels may use (slots).
int cld_staged_waves_per_simd();
// par_lists (span-parallel documents): two u32 document lists of n entries
// each (passes 1, 2), then two u64 group lists of gcap entries each.
hipError_t cld_launch_staged(const DevTables* d_T, const uint8_t* buf, const uint64_t* offs, const uint32_t* list,
                             cld_result* out, uint8_t* slots, int n_waves, uint8_t* pool, uint64_t pool_bytes,
                             uint64_t* meta, uint32_t* ok_list, uint32_t* p2_list, uint32_t* fall_list,
                             uint32_t* counters, uint32_t cflags, const uint8_t* special,
                             const uint32_t* priors, const uint8_t* hbuf, const uint8_t* hflag, const uint32_t* hpos,
                             const uint32_t* hgap, uint32_t fault_doc, uint32_t small_total, const uint32_t* hist,
                             uint32_t heavy_kb, uint32_t* par_lists, size_t n, size_t gcap, hipStream_t s);
}
#endif
