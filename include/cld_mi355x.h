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

/* Byte-balanced document shards: cuts[0..nshards] (cuts[0]=0, cuts[nshards]=n)
 * such that shard k = documents [cuts[k], cuts[k+1]).  Host-only helper used
 * by cld_detect_batch's multi-GPU split and by multi-process callers. */
int cld_plan_shards(const uint64_t* offsets, size_t n, int nshards, size_t* cuts);

/* Sum of kernel durations (HIP events on the stream the kernels ran on) of
 * every batch enqueued on context `ctx` since the previous call; resets.
 * short_ms = wavefront kernel; general_ms = long-document + sequential kernels. */
int cld_kernel_time(int ctx, double* short_ms, double* general_ms, int* launches);

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
 * by byte count.  flags must be 0 (reserved).  Thread-safe. */
int cld_detect_batch(const uint8_t* buf, const uint64_t* offsets, size_t n,
                     cld_result* out, uint32_t flags);

/* Same, with every pointer in device memory of GPU `device` and work
 * enqueued on `stream` (a hipStream_t, NULL = the runtime's stream for that
 * device).  Asynchronous: returns once the kernels are enqueued.  Used by the
 * benchmark to time the path with inputs already resident in HBM. */
int cld_detect_batch_device(int device, const uint8_t* d_buf, const uint64_t* d_offsets,
                            size_t n, cld_result* d_out, void* stream);

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

/* Build / table identity string ("cld-mi355x <ver> tables=<date> ..."). */
const char* cld_version(void);

#ifdef __cplusplus
}
#endif
#endif /* CLD_MI355X_H_ */
