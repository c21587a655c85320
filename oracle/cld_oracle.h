/* cld_oracle.h -- TEST INFRASTRUCTURE ONLY (see cld_oracle.c header). */
#ifndef CLD_ORACLE_H_
#define CLD_ORACLE_H_
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

/* Mirrors DetectLanguageSummaryV2's outputs (compact_lang_det_impl.cc:1707-1720) */
typedef struct {
  uint16_t lang3[3];
  uint16_t summary_lang;
  int32_t percent3[3];
  int32_t reliable_percent3[3];
  double normalized3[3];
  int32_t text_bytes;
  uint8_t is_reliable;
  uint8_t passes;
  uint8_t pad[2];
} cldo_result;

typedef struct {   /* ChunkSummary, scoreonescriptspan.h:240-252 */
  uint16_t offset, chunk_start, lang1, lang2, score1, score2, bytes, grams, ulscript;
  uint8_t rel_delta, rel_score;
} cldo_chunk;

typedef struct {   /* ResultChunk, compact_lang_det.h:147-153 */
  int32_t offset, bytes;
  uint16_t lang1, pad;
} cldo_rchunk;

typedef struct cldo_ctx cldo_ctx;
typedef void (*cldo_trace_fn)(void* arg, const char* line);

int cldo_load(const char* cldt_path);
cldo_ctx* cldo_ctx_new(void);
void cldo_ctx_free(cldo_ctx* c);
void cldo_set_trace(cldo_ctx* c, cldo_trace_fn fn, void* arg);
void cldo_set_trace_text(cldo_ctx* c, int on);   /* trace lines "lowered <flags> <hex>" per span */
int cldo_detect(cldo_ctx* c, const char* text, int len, cldo_result* r);
const char* cldo_detect_language(cldo_ctx* c, const char* text);
int cldo_detect_batch(const char* buf, const uint64_t* offsets, int n, cldo_result* out, int threads);
/* is_plain_text = 0: HTML mode (tags skipped, entities decoded).  priors: the
 * ApplyHints result as 16 langprobs (boost latn[4], othr[4], whack latn[4],
 * othr[4]), NULL for none; batch forms take one flag / 16 priors per document. */
int cldo_detect_ex(cldo_ctx* c, const char* text, int len, int is_plain_text, const uint32_t* priors,
                   cldo_result* r);
int cldo_detect_vec(cldo_ctx* c, const char* text, int len, int is_plain_text, const uint32_t* priors,
                    cldo_result* r, cldo_rchunk* out, int cap);
int cldo_detect_batch_ex(const char* buf, const uint64_t* offsets, int n, const uint8_t* plain,
                         const uint32_t* priors, cldo_result* out, int threads);
/* The caller's ExtDetectLanguageSummary flags (compact_lang_det.h:343-349):
 * 0x0100 kCLDFlagScoreAsQuads, 0x4000 kCLDFlagBestEffort; others ignored. */
void cldo_set_flags(cldo_ctx* c, int flags);
int cldo_detect_batch_flags(const char* buf, const uint64_t* offsets, int n, const uint8_t* plain,
                            const uint32_t* priors, cldo_result* out, int threads, int flags);
/* handlers.go:150-151 text preparation: flags 1 = StripExtras, 2 = C-string cut.
 * out capacity: offsets[n]-offsets[0] + n bytes. */
int cldo_prepare_batch(const char* buf, const uint64_t* offsets, int n, int flags, char* out,
                       uint64_t* out_offsets);
const char* cldo_language_code(int lang);
const char* cldo_language_name(int lang);
int cldo_meta(int which);
int cldo_score_linear(int ulscript, int score_cjk, int next_base, const uint16_t* offsets,
                      const uint8_t* types, const uint32_t* langprobs, int n_linear,
                      int dummy_offset, uint32_t* ring, cldo_chunk* out, int max_out);

int cldo_score_chunks(int ulscript, const uint16_t* offsets, const uint8_t* types,
                      const uint32_t* langprobs, int n_linear, const int* chunk_starts,
                      int n_chunks, uint32_t* ring, cldo_chunk* out);

int cldo_lower(const char* in, int len, char* out, int olen);
uint64_t cldo_gram_hash(int kind, const char* w, int n);   /* 0 quad, 1 bi, 2 octa */
int cldo_scan_spans(const char* text, int len, int is_plain_text, cldo_trace_fn fn, void* arg);
int cldo_scan_tag(const char* text, int len);
int cldo_read_entity(const char* text, int len, int* consumed);
uint64_t cldo_pair_hash(uint64_t a, uint64_t b);
uint32_t cldo_probe(int cldt_section, uint64_t hash);
int cldo_script_num(const char* s);

#ifdef __cplusplus
}
#endif
#endif
