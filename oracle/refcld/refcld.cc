// refcld.cc -- TEST INFRASTRUCTURE ONLY.  A C ABI over the reference CLD2
// itself, built in the reference's own dynamic-data mode (-DCLD2_DYNAMIC_MODE,
// the configuration cld2/internal/compile_dynamic.sh documents): the scoring
// tables are not linked in but loaded at run time from a cld2_data_file00
// through the reference's loader (CLD2::loadDataFromFile,
// compact_lang_det_impl.cc:108-136).  No generated table code and no stand-in
// is compiled: the data files come from tools/cld2_data_file.py over the same
// CLDT blob the product and the oracle read.
//
// It is the checker of last resort: tests compare the oracle (and through it
// the GPU path) with the reference's own DetectLanguageSummaryV2 /
// ExtDetectLanguageSummary on identical tables, documents, is_plain_text
// flags, hints and ResultChunkVector requests.  bench.py may time it as the
// "reference" CPU baseline.
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#include "compact_lang_det.h"

using namespace CLD2;

extern "C" {

typedef struct {              // per-document result (mirrors cldo_result's fields)
  int32_t lang3[3];
  int32_t percent3[3];
  double normalized3[3];
  int32_t text_bytes;
  int32_t summary_lang;
  int32_t is_reliable;
  int32_t n_chunks;           // ResultChunkVector size (vector mode), else 0
} refcld_result;

typedef struct {              // CLDHints (compact_lang_det.h:134-139)
  const char* content_language_hint;
  const char* tld_hint;
  int32_t encoding_hint;
  int32_t language_hint;
} refcld_hints;

typedef struct {              // ResultChunk (compact_lang_det.h:147-153)
  int32_t offset;
  int32_t bytes;
  uint16_t lang1;
  uint16_t pad;
} refcld_chunk;

int refcld_load(const char* data_file) {
  loadDataFromFile(data_file);
  return isDataLoaded() ? 0 : -1;
}

// One document.  hints == NULL: DetectLanguage's empty hints (compact_lang_det.cc:66-71).
// chunks != NULL: ExtDetectLanguageSummary with a ResultChunkVector, at most cap entries copied.
// flags: ExtDetectLanguageSummary's `flags` (compact_lang_det.h:329, :343-349).
static void detect_one(const char* text, int len, int plain, const refcld_hints* h, refcld_result* r,
                       refcld_chunk* chunks, int cap, std::string* scratch, int flags) {
  scratch->assign(text, (size_t)len);
  scratch->append(16, '\0');                    // NUL-terminated, as the wrapper hands it over
  CLDHints hints = {NULL, "", 23 /* UNKNOWN_ENCODING (encodings.h) */, UNKNOWN_LANGUAGE};
  if (h) {
    hints.content_language_hint = h->content_language_hint;
    hints.tld_hint = h->tld_hint ? h->tld_hint : "";
    hints.encoding_hint = h->encoding_hint;
    hints.language_hint = (Language)h->language_hint;
  }
  Language l3[3];
  int p3[3], tb = 0;
  double n3[3];
  bool rel = false;
  ResultChunkVector vec;
  Language s = ExtDetectLanguageSummary(scratch->data(), len, plain != 0, &hints, flags, l3, p3, n3,
                                        chunks ? &vec : NULL, &tb, &rel);
  for (int i = 0; i < 3; ++i) { r->lang3[i] = l3[i]; r->percent3[i] = p3[i]; r->normalized3[i] = n3[i]; }
  r->text_bytes = tb;
  r->summary_lang = s;
  r->is_reliable = rel ? 1 : 0;
  r->n_chunks = chunks ? (int)vec.size() : 0;
  if (chunks)
    for (int i = 0; i < (int)vec.size() && i < cap; ++i) {
      chunks[i].offset = vec[i].offset;
      chunks[i].bytes = vec[i].bytes;
      chunks[i].lang1 = vec[i].lang1;
      chunks[i].pad = 0;
    }
}

int refcld_detect_flags(const char* text, int len, int plain, const refcld_hints* h, refcld_result* r,
                        refcld_chunk* chunks, int cap, int flags) {
  if (!isDataLoaded()) return -1;
  std::string s;
  detect_one(text, len, plain, h, r, chunks, cap, &s, flags);
  return 0;
}

int refcld_detect(const char* text, int len, int plain, const refcld_hints* h, refcld_result* r,
                  refcld_chunk* chunks, int cap) {
  return refcld_detect_flags(text, len, plain, h, r, chunks, cap, 0);
}

typedef struct {
  const char* buf; const uint64_t* offs; int lo, hi;
  const uint8_t* plain; const refcld_hints* hints; refcld_result* out; int flags;
} job_t;

static void* run(void* a) {
  job_t* j = (job_t*)a;
  std::string s;
  for (int i = j->lo; i < j->hi; ++i)
    detect_one(j->buf + j->offs[i], (int)(j->offs[i + 1] - j->offs[i]), j->plain ? j->plain[i] : 1,
               j->hints ? j->hints + i : NULL, &j->out[i], NULL, 0, &s, j->flags);
  return NULL;
}

// n documents over `threads` pthreads; plain / hints per document or NULL;
// flags as ExtDetectLanguageSummary's, for every document.
int refcld_detect_batch_flags(const char* buf, const uint64_t* offs, int n, const uint8_t* plain,
                              const refcld_hints* hints, refcld_result* out, int threads, int flags) {
  if (!isDataLoaded()) return -1;
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  std::vector<pthread_t> th(threads);
  std::vector<job_t> jobs(threads);
  for (int t = 0; t < threads; ++t) {
    jobs[t] = job_t{buf, offs, (int)((int64_t)n * t / threads), (int)((int64_t)n * (t + 1) / threads), plain,
                    hints, out, flags};
    pthread_create(&th[t], NULL, run, &jobs[t]);
  }
  for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
  return 0;
}

int refcld_detect_batch(const char* buf, const uint64_t* offs, int n, const uint8_t* plain,
                        const refcld_hints* hints, refcld_result* out, int threads) {
  return refcld_detect_batch_flags(buf, offs, n, plain, hints, out, threads, 0);
}

// Vector mode over `threads` pthreads: document i's chunks go to
// chunks[chunk_base[i] ..], at most chunk_base[i + 1] - chunk_base[i] of them
// (out[i].n_chunks is the full count).
typedef struct {
  const char* buf; const uint64_t* offs; int lo, hi; const uint8_t* plain; refcld_result* out;
  refcld_chunk* chunks; const uint64_t* base; int flags;
} vjob_t;

static void* run_vec(void* a) {
  vjob_t* j = (vjob_t*)a;
  std::string s;
  for (int i = j->lo; i < j->hi; ++i)
    detect_one(j->buf + j->offs[i], (int)(j->offs[i + 1] - j->offs[i]), j->plain ? j->plain[i] : 1, NULL, &j->out[i],
               j->chunks + j->base[i], (int)(j->base[i + 1] - j->base[i]), &s, j->flags);
  return NULL;
}

int refcld_detect_batch_vec(const char* buf, const uint64_t* offs, int n, const uint8_t* plain, refcld_result* out,
                            refcld_chunk* chunks, const uint64_t* chunk_base, int threads, int flags) {
  if (!isDataLoaded()) return -1;
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  std::vector<pthread_t> th(threads);
  std::vector<vjob_t> jobs(threads);
  for (int t = 0; t < threads; ++t) {
    jobs[t] = vjob_t{buf, offs, (int)((int64_t)n * t / threads), (int)((int64_t)n * (t + 1) / threads), plain, out,
                     chunks, chunk_base, flags};
    pthread_create(&th[t], NULL, run_vec, &jobs[t]);
  }
  for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
  return 0;
}

}  // extern "C"
