/*
 * cld_mi355x.h -- C ABI of the MI355X-native CLD2-compatible language
 * detector (libcld_mi355x.so).  Plain C types only: no HIP or torch types.
 *
 * Drop-in for the reference's cgo boundary:
 *   detect_language()          replaces wrapper.h:8 / wrapper.cc:7-16
 *                              (called from main.go:77-81, handlers.go:151)
 * Batch boundary (new, same semantics per document):
 *   cld_detect_batch()         one DetectLanguageSummaryV2 per document
 *                              (compact_lang_det_impl.cc:1707-2106) with
 *                              plain text, no hints, flags 0 -- exactly what
 *                              wrapper.cc:9-12 asks CLD2 for.
 */
#ifndef CLD_MI355X_H_
#define CLD_MI355X_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Per-document result: the out-parameters of DetectLanguageSummaryV2
 * (compact_lang_det_impl.cc:1707-1720).  40 bytes, naturally aligned. */
typedef struct cld_result {
  uint16_t lang3[3];        /* top-3 Language enum values; UNKNOWN_LANGUAGE (26) if absent */
  uint16_t summary_lang;    /* V2 return value (UNKNOWN is NOT mapped to ENGLISH here)     */
  int8_t percent3[3];       /* percent of text bytes per language                          */
  uint8_t is_reliable;      /* 0/1                                                         */
  int32_t text_bytes;       /* letters-only text bytes scored                              */
  double normalized3[3];    /* (score << 10) / bytes per language                          */
} cld_result;

/* Error codes (negative errno style) */
#define CLD_OK 0
#define CLD_EINVAL (-22)
#define CLD_ENODEV (-19)
#define CLD_ENOMEM (-12)
#define CLD_EIO (-5)
#define CLD_EFAULT (-14)  /* a HIP runtime call failed (device error) */
#define CLD_ENOSPC (-28)  /* cld_detect_batch_vec: chunk_cap too small for the vectors */

/* summary_lang of a document the GPU could not score.  Such a document is
 * redone alone once; if it fails again the call returns CLD_EIO and every
 * other document's result is complete (lang3 = UNKNOWN, percent3 0,
 * text_bytes 0 for the failed one).  The kernels have no such case short of
 * a device fault: it exists so one bad document never costs a batch. */
#define CLD_LANG_FAILED 0xFFFF

/* cld_detect_batch flags: the service's text preparation, applied on the GPU
 * before detection (handlers.go:150-151).
 *   CLD_FLAG_STRIP_EXTRAS  StripExtras (handlers.go:198-210): keep the
 *                          strings.Fields words (unicode.IsSpace separators)
 *                          that start with neither "@" nor "http", each
 *                          followed by one ' '.
 *   CLD_FLAG_CSTRING       cut each document at its first NUL byte, as the
 *                          cgo hand-off does (main.go:77-81: C.CString, then
 *                          strlen in wrapper.cc:8).
 * STRIP_EXTRAS | CSTRING = exactly the text Detect_language() sees for one
 * request item of POST / (handlers.go:150-151). */
#define CLD_FLAG_STRIP_EXTRAS 1u
#define CLD_FLAG_CSTRING 2u
/* is_plain_text = false: the documents are HTML -- tags, comments, <script>
 * and <style> bodies are skipped and entities decoded by the span scanner
 * (getonescriptspan.cc:150-541, 592-1027), lang= attributes in the first 8 KB
 * become hints (compact_lang_det_impl.cc:1596-1611). */
#define CLD_FLAG_HTML 4u
/* The reference's public result-affecting flags, with the reference's values
 * (compact_lang_det.h:343-349), accepted in the `flags` word of every batch
 * entry point and applied to every document of the batch:
 *   CLD_FLAG_SCORE_AS_QUADS  kCLDFlagScoreAsQuads: scripts normally scored by
 *                            their script alone (RTypeOne/None: Greek, Thai,
 *                            ...) are quadgram-scored instead
 *                            (scoreonescriptspan.cc:1318-1320)
 *   CLD_FLAG_BEST_EFFORT     kCLDFlagBestEffort: no unreliable-language removal
 *                            and no UNKNOWN summary for a small top percent
 *                            (compact_lang_det_impl.cc:1998-2000, :1493)
 * The reference's debug-output flags (kCLDFlagHtml, Cr, Verbose, Quiet, Echo:
 * CLD_FLAG_DEBUG_MASK) only write diagnostics to stderr there; they are
 * accepted and ignored. */
#define CLD_FLAG_SCORE_AS_QUADS 0x0100u
#define CLD_FLAG_BEST_EFFORT 0x4000u
#define CLD_FLAG_DEBUG_MASK 0x3E00u

/* ResultChunk (compact_lang_det.h:147-153): one piece of a document in one
 * language; offset/bytes index the document as given; lang1 is a Language
 * enum, UNKNOWN_LANGUAGE (26) for unreliable or too-short pieces. */
typedef struct cld_chunk {
  int32_t offset;
  int32_t bytes;
  uint16_t lang1;
  uint16_t pad;
} cld_chunk;

/* CLDHints (compact_lang_det.h:134-139): per-document priors. */
typedef struct cld_hints {
  const char* content_language_hint;  /* "mi,en" boosts Maori and English; NULL / "" for none */
  const char* tld_hint;               /* "id" boosts Indonesian; NULL / "" for none */
  int32_t encoding_hint;              /* Encoding enum (encodings.h); CLD_UNKNOWN_ENCODING for none */
  int32_t language_hint;              /* Language enum; 26 (UNKNOWN_LANGUAGE) for none */
} cld_hints;
#define CLD_UNKNOWN_ENCODING 23

/* wrapper.h:8 -- returns a static ISO code; never NULL; UNKNOWN -> "en"
 * (compact_lang_det.cc:91-93).  Input is NUL-terminated, length = strlen
 * (wrapper.cc:8).  Thread-safe; concurrent callers are coalesced into GPU
 * micro-batches by the runtime. */
const char* detect_language(const char* text);

/* Optional explicit initialisation.  tables_path NULL -> $CLD_MI355X_TABLES or
 * the blob shipped next to the library.  n_devices <= 0 -> all visible GPUs.
 * Returns CLD_OK or a negative error.  Called implicitly by the entry points. */
int cld_init(const char* tables_path, int n_devices);
void cld_shutdown(void);

/* Initialise on exactly one GPU (HIP ordinal `device`); context index 0.
 * One process per GPU (torch.distributed / bench.py) uses this. */
int cld_init_device(const char* tables_path, int device);

/* Cost-balanced document shards: cuts[0..nshards] (cuts[0]=0, cuts[nshards]=n)
 * such that shard k = documents [cuts[k], cuts[k+1]), each holding about
 * 1/nshards of the estimated kernel cost (a document of <= 256 bytes: 480
 * units, a longer one: 41/8 units per byte + 2500; measured per-document
 * kernel times in units of 10 ps).  Host-only helper used by
 * cld_detect_batch's multi-GPU split and by multi-process callers. */
int cld_plan_shards(const uint64_t* offsets, size_t n, int nshards, size_t* cuts);

/* Sum of kernel durations (HIP events on the stream the kernels ran on) of
 * every batch enqueued on context `ctx` since the previous call; resets.
 * short_ms = wavefront kernel; general_ms = the long-document kernels (k_long, both instantiations). */
int cld_kernel_time(int ctx, double* short_ms, double* general_ms, int* launches);

/* Same accounting split per kernel stage: ms[0] the wavefront kernel (k_wave),
 * (with HTML pages: the GPU rewrite of the pages into plain text, k_html_rewrite,
 * is counted in ms[0]), ms[1] the long-document stage (length ordering + k_long on the
 * parallel span builder), ms[2] k_long's documents on the sequential span source (its SEQ
 * instantiation, cld_seq.hip).  Sums since the previous call of either
 * function; resets. */
int cld_kernel_times(int ctx, double* ms3, int* launches);

/* Diagnostics: per-stage shader-clock cycle sums on context `ctx` since the
 * previous call; 16 entries.  [0..7] short-document wavefront kernel (0 load,
 * 1 span, 2 lower, 3 quad/uni, 4 octa/bi, 5 score, 6 document level);
 * [8..15] long-document kernel (8 classify, 9 span+lowercase, 10 squeeze
 * test, 11 repeats, 12 word lists + quad chain, 13 quad hits, 14 octa/uni/bi
 * hits, 15 linearize/chunk/score).  All zero unless the runtime was started
 * with CLD_PROFILE_STAGES=1.  Resets. */
int cld_stage_cycles(int ctx, uint64_t* cycles16);

/* Batch detection.  Documents are [buf + offsets[i], buf + offsets[i+1]),
 * i < n (offsets has n+1 entries, non-decreasing).  Each document is scored
 * as if followed by NUL bytes, i.e. exactly like detect_language() on a
 * NUL-terminated copy of it (embedded NULs are kept, as with
 * CLD2::DetectLanguage(buffer, length, ...)).  `out` is caller-allocated
 * (n entries).  Host buffers; not retained after return.  Blocks until the
 * results are in `out`.  Documents are sharded across the initialised GPUs
 * by estimated cost; each shard streams through the GPU in chunks of <= 64 MB /
 * 512K documents (pinned staging, upload / kernels / download overlapped on
 * three streams).  A batch whose mean document is longer than 256 bytes goes
 * in chunks of <= 256 MB / 2M documents instead: each of a context's two chunk
 * slots then holds up to 256 MB of text plus 48 B per document in device
 * memory, and as much pinned host staging unless the caller's buffers are
 * pinned (CLD_CHUNK_MB scales both).  Request-sized calls (< 16 MB of text)
 * from concurrent callers are coalesced into one GPU batch; a batch of at
 * most 1024 documents of <= 256 bytes takes one upload, one kernel and one
 * download.  flags: 0 or CLD_FLAG_STRIP_EXTRAS / CLD_FLAG_CSTRING and
 * CLD_FLAG_SCORE_AS_QUADS / CLD_FLAG_BEST_EFFORT (above).  Thread-safe. */
int cld_detect_batch(const uint8_t* buf, const uint64_t* offsets, size_t n,
                     cld_result* out, uint32_t flags);

/* ExtDetectLanguageSummary (compact_lang_det.h:324-335 / impl.cc:1707) over a
 * batch: `hints` is NULL or one cld_hints per document (CLDHints); flags is
 * the reference's `flags` argument -- CLD_FLAG_SCORE_AS_QUADS,
 * CLD_FLAG_BEST_EFFORT, the ignored debug flags -- plus CLD_FLAG_HTML for
 * is_plain_text = false (all documents are HTML).  Results are the same
 * fields as cld_detect_batch.  Host buffers; blocks. */
int cld_detect_batch_ex(const uint8_t* buf, const uint64_t* offsets, size_t n, const cld_hints* hints,
                        uint32_t flags, cld_result* out);

/* ExtDetectLanguageSummary with a ResultChunkVector per document
 * (compact_lang_det.h:324-335): the same results as cld_detect_batch_ex plus
 * each document's chunk vector -- pieces of the document as given, in one
 * language each (SummaryBufferToVector / SharpenBoundaries / OffsetMap,
 * scoreonescriptspan.cc:389-548, 671-845; offsetmap.cc).  Vector mode changes
 * scoring the way the reference's does (SharpenBoundaries moves chunk bytes,
 * Squeeze/RepWords overwrite instead of cutting), so `out` can differ from
 * cld_detect_batch_ex's for the same document, exactly as there.
 * chunk_offsets[n+1] receives document i's chunks as
 * chunks[chunk_offsets[i] .. chunk_offsets[i+1]).  If chunk_cap is too small
 * the call returns CLD_ENOSPC with out and chunk_offsets complete and chunks
 * holding the first chunk_cap entries (CLD_ENOMEM: device memory ran out).  A document whose vector outgrows its
 * working region is redone alone with 8x the room; should that fail too, it
 * gets an empty vector and the call returns CLD_EIO with every other
 * document's result and vector complete.  Every document runs the sequential
 * kernel (not a high-throughput path, as in the reference). */
int cld_detect_batch_vec(const uint8_t* buf, const uint64_t* offsets, size_t n, const cld_hints* hints,
                         uint32_t flags, cld_result* out, cld_chunk* chunks, size_t chunk_cap,
                         uint64_t* chunk_offsets);

/* Host-only (no GPU): the ApplyHints result for one document.  priors: the
 * CLDLangPriors (OneCLDLangPrior = (weight << 10) + Language, at most 14)
 * after TrimCLDLangPriors(4); boosts16: prior boosts latn[4], othr[4] and
 * close-language whacks latn[4], othr[4] as langprobs.  Returns the prior
 * count, or a negative error.  doc may be NULL unless is_plain_text = 0. */
int cld_hint_priors(const uint8_t* doc, size_t len, int is_plain_text, const cld_hints* hints,
                    int16_t* priors14, uint32_t* boosts16);

/* Same, with every pointer in device memory of GPU `device` and work
 * enqueued on `stream` (a hipStream_t, NULL = the runtime's stream for that
 * device).  Asynchronous: returns once the kernels are enqueued.  Used by the
 * benchmark to time the path with inputs already resident in HBM. */
int cld_detect_batch_device(int device, const uint8_t* d_buf, const uint64_t* d_offsets,
                            size_t n, cld_result* d_out, void* stream);

/* cld_detect_batch_device with flags (preparation and CLD2 flags, as for
 * cld_detect_batch).  buf_bytes bounds
 * d_offsets[n] (the prepared copy is staged in a device buffer of
 * buf_bytes + n bytes).  Asynchronous like cld_detect_batch_device. */
int cld_detect_batch_device_ex(int device, const uint8_t* d_buf, const uint64_t* d_offsets, size_t n,
                               uint64_t buf_bytes, cld_result* d_out, uint32_t flags, void* stream);

/* The preparation step alone, on GPU 0 (host buffers): out_buf receives the
 * prepared documents back to back (capacity >= offsets[n]-offsets[0] + n
 * bytes), out_offsets[0..n] their offsets.  flags: CLD_FLAG_STRIP_EXTRAS and/or
 * CLD_FLAG_CSTRING.  Blocks until the result is on the host. */
int cld_prepare_batch(const uint8_t* buf, const uint64_t* offsets, size_t n, uint32_t flags,
                      uint8_t* out_buf, uint64_t* out_offsets);

/* Pinned host memory for callers of cld_detect_batch.  Documents, offsets and
 * results that live in such memory skip the runtime's staging copy: they are
 * DMA'd straight from/to it (the batch HTTP endpoint keeps its request and
 * response buffers here).  Any other host memory works too and is staged
 * through the runtime's own pinned chunk buffers.  NULL on failure. */
void* cld_host_alloc(size_t bytes);
void cld_host_free(void* p);

/* LanguageCode / LanguageName (lang_script.cc:212-217, :205-210). */
const char* cld_language_code(int lang);
const char* cld_language_name(int lang);

/* Counters of the most recent batch on this thread's last device call. */
typedef struct cld_batch_stats {
  uint64_t docs;
  uint64_t short_docs;       /* finished by the short-document (wavefront) kernel */
  uint64_t general_docs;     /* finished by the sequential any-length kernel      */
  uint64_t passes[4];        /* documents needing 1, 2, 3 passes; [3] = errors     */
  double short_ms, general_ms; /* kernel time from HIP events                     */
  uint64_t long_docs;        /* finished by the long-document wavefront kernel    */
  double long_ms;
  uint64_t long_requeue[8];  /* why k_long handed documents on: 1 length, 2 scanner
                                state, 3 span/lowercase, 4 Squeeze restart, 5 capacity */
} cld_batch_stats;
int cld_last_batch_stats(int device, cld_batch_stats* st);

/* ---- Run-time table loading (CLD2 dynamic data, cld2_dynamic_data.h:22-147).
 * A "cld2_data_file00" image carries the scoring tables of ScoringTables
 * (CJK unigram machine, kAvgDeltaOctaScore, compat/deltabi/distinctbi/quad/
 * quad2/deltaocta/distinctocta); the other tables stay the built-in ones.
 * Loading re-uploads the tables to every initialised GPU (after draining
 * in-flight work) and applies to every later call.  Not to be called
 * concurrently with detection calls (the reference's loaders are not either).
 *
 *   cld_load_data_from_file         replaces CLD2::loadDataFromFile
 *                                   (compact_lang_det.h:393, impl.cc:108-121)
 *   cld_load_data_from_raw_address  replaces CLD2::loadDataFromRawAddress
 *                                   (compact_lang_det.h:406, impl.cc:123-136)
 *   cld_unload_data                 replaces CLD2::unloadData (compact_lang_det.h:413);
 *                                   here it restores the built-in tables
 *   cld_is_data_dynamic             1 while data-file tables are in use
 *                                   (cf. CLD2::isDataDynamic, compact_lang_det.h:426)
 * They return CLD_OK or CLD_EINVAL (malformed file: bad marker, header or
 * file size mismatch as in cld2_dynamic_data_loader.cc:41-146, or a block /
 * indirect index outside the file); a failed load keeps the tables in use. */
int cld_load_data_from_file(const char* path);
int cld_load_data_from_raw_address(const void* raw, uint32_t length);
int cld_unload_data(void);
int cld_is_data_dynamic(void);

/* Host-only helpers (no GPU): write the tables in use as a CLDT blob, and
 * convert a cld2 data file over a base CLDT (NULL = the built-in one) into a
 * CLDT file -- the form the test oracle reads. */
int cld_export_tables(const char* out_cldt_path);
int cld_convert_data_file(const char* cld2_data_file, const char* base_cldt, const char* out_cldt_path);

/* Build / table identity string: "cld-mi355x <ver> tables=<path> quad=<q>
 * quad_build=<date>" where q says which quadgram table is live: "empty-Q0"
 * (the default: the reference's placeholder pattern, no quadgram scoring),
 * "synthetic-Q1" (the test/bench table, opted into via CLD_MI355X_TABLES) or
 * "other" (e.g. a real table from cld_load_data_from_file). */
const char* cld_version(void);

#ifdef __cplusplus
}
#endif
#endif /* CLD_MI355X_H_ */
