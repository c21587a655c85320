/* dl_bench.c -- per-call cost of the zero-change drop-in, wrapper.h's
 * detect_language, timed from C.
 *
 * The reference service calls Detect_language once per document, serially
 * within a request, with requests on concurrent goroutines
 * (handlers.go:132-151, main.go:77-81 -> wrapper.cc:7-16).  This harness
 * replays that: `callers` threads each loop over single documents (NUL-
 * terminated copies, as C.CString hands them over) and time every call.
 *
 *   dl_bench gpu <corpus.bin> <offsets.bin> <callers> <calls_per_caller>
 *       detect_language from libcld_mi355x.so
 *   dl_bench ref <librefcld2.so> <cld2_data_file> <corpus.bin> <offsets.bin> <callers> <calls_per_caller>
 *       the reference CLD2 itself (oracle/_ref, its DetectLanguage path through
 *       refcld_detect) -- test infrastructure, loaded only in this mode
 *
 * One JSON line: latency p50 / p99 / max per call, calls and documents per
 * second over the timed region (all callers start together after warm-up).
 */
#include <dlfcn.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/resource.h>
#include <time.h>

#include "wrapper.h"

static double now_s(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

static double cpu_s(void) {           /* user + system CPU of the process so far */
  struct rusage r;
  getrusage(RUSAGE_SELF, &r);
  return (double)r.ru_utime.tv_sec + 1e-6 * (double)r.ru_utime.tv_usec + (double)r.ru_stime.tv_sec +
         1e-6 * (double)r.ru_stime.tv_usec;
}

/* cgroup v2 CPU throttling so far (microseconds), or -1 where not readable */
static long long throttled_us(void) {
  FILE* f = fopen("/sys/fs/cgroup/cpu.stat", "r");
  if (!f) return -1;
  char k[64];
  long long v, t = -1;
  while (fscanf(f, "%63s %lld", k, &v) == 2)
    if (!strcmp(k, "throttled_usec")) t = v;
  fclose(f);
  return t;
}

static void* slurp(const char* path, size_t* n) {
  FILE* f = fopen(path, "rb");
  if (!f) { perror(path); exit(2); }
  fseek(f, 0, SEEK_END);
  long len = ftell(f);
  fseek(f, 0, SEEK_SET);
  void* p = malloc(len > 0 ? (size_t)len : 1);
  if (fread(p, 1, (size_t)len, f) != (size_t)len) { perror(path); exit(2); }
  fclose(f);
  *n = (size_t)len;
  return p;
}

/* refcld_detect (oracle/refcld/refcld.cc): one document, the reference's own
 * ExtDetectLanguageSummary with DetectLanguage's empty hints */
typedef struct { int32_t lang3[3], percent3[3]; double normalized3[3]; int32_t text_bytes, summary_lang, is_reliable, n_chunks; } ref_result;
typedef int (*ref_detect_fn)(const char*, int, int, const void*, ref_result*, void*, int);
static ref_detect_fn ref_detect;

typedef struct {
  char** docs;
  size_t n_docs;
  int caller, callers, calls, warm;
  double* lat;
  pthread_barrier_t* bar;
  unsigned long long sink;
} job_t;

static void one(job_t* j, size_t i) {
  if (ref_detect) {
    ref_result r;
    ref_detect(j->docs[i], (int)strlen(j->docs[i]), 1, NULL, &r, NULL, 0);
    j->sink += (unsigned)r.summary_lang;
  } else {
    j->sink += (unsigned char)detect_language(j->docs[i])[0];
  }
}

static void* run(void* a) {
  job_t* j = (job_t*)a;
  size_t i = (size_t)j->caller % j->n_docs;
  for (int k = 0; k < j->warm; ++k, i = (i + (size_t)j->callers) % j->n_docs) one(j, i);
  pthread_barrier_wait(j->bar);
  for (int k = 0; k < j->calls; ++k, i = (i + (size_t)j->callers) % j->n_docs) {
    const double t0 = now_s();
    one(j, i);
    j->lat[k] = now_s() - t0;
  }
  pthread_barrier_wait(j->bar);
  return NULL;
}

static int cmp_d(const void* a, const void* b) {
  const double x = *(const double*)a, y = *(const double*)b;
  return x < y ? -1 : x > y;
}

int main(int argc, char** argv) {
  const int ref = argc > 1 && strcmp(argv[1], "ref") == 0;
  if (argc < (ref ? 8 : 6)) {
    fprintf(stderr, "usage: %s gpu corpus.bin offsets.bin callers calls\n"
                    "       %s ref librefcld2.so data_file corpus.bin offsets.bin callers calls\n", argv[0], argv[0]);
    return 2;
  }
  const int a0 = ref ? 4 : 2;
  if (ref) {
    void* h = dlopen(argv[2], RTLD_NOW);
    if (!h) { fprintf(stderr, "%s\n", dlerror()); return 2; }
    int (*load)(const char*) = (int (*)(const char*))dlsym(h, "refcld_load");
    ref_detect = (ref_detect_fn)dlsym(h, "refcld_detect");
    if (!load || !ref_detect || load(argv[3]) != 0) { fprintf(stderr, "reference load failed\n"); return 2; }
  }
  size_t nb, no;
  const char* buf = (const char*)slurp(argv[a0], &nb);
  const uint64_t* offs = (const uint64_t*)slurp(argv[a0 + 1], &no);
  const size_t n = no / 8 - 1;
  const int callers = atoi(argv[a0 + 2]);
  const int calls = atoi(argv[a0 + 3]);
  char** docs = (char**)malloc(sizeof(char*) * n);
  for (size_t i = 0; i < n; ++i) {
    const size_t len = (size_t)(offs[i + 1] - offs[i]);
    docs[i] = (char*)malloc(len + 1);
    memcpy(docs[i], buf + offs[i], len);
    docs[i][len] = 0;
  }
  if (!ref) (void)detect_language("warm up the runtime");
  pthread_barrier_t bar;
  pthread_barrier_init(&bar, NULL, (unsigned)callers + 1);
  job_t* jobs = (job_t*)calloc((size_t)callers, sizeof(job_t));
  pthread_t* th = (pthread_t*)calloc((size_t)callers, sizeof(pthread_t));
  for (int c = 0; c < callers; ++c) {
    jobs[c] = (job_t){docs, n, c, callers, calls, 20, (double*)malloc(sizeof(double) * (size_t)calls), &bar, 0};
    pthread_create(&th[c], NULL, run, &jobs[c]);
  }
  pthread_barrier_wait(&bar);          /* everyone warmed up */
  const double t0 = now_s(), c0 = cpu_s();
  const long long th0 = throttled_us();
  pthread_barrier_wait(&bar);          /* everyone done */
  const double wall = now_s() - t0, cpu = cpu_s() - c0;
  const long long th1 = throttled_us();
  for (int c = 0; c < callers; ++c) pthread_join(th[c], NULL);
  const size_t nl = (size_t)callers * (size_t)calls;
  double* all = (double*)malloc(sizeof(double) * nl);
  size_t k = 0;
  unsigned long long sink = 0;
  for (int c = 0; c < callers; ++c) {
    for (int i = 0; i < calls; ++i) all[k++] = jobs[c].lat[i];
    sink += jobs[c].sink;
  }
  qsort(all, nl, sizeof(double), cmp_d);
  printf("{\"mode\": \"%s\", \"callers\": %d, \"calls\": %zu, \"latency_us_p50\": %.1f, \"latency_us_p99\": %.1f, "
         "\"latency_us_max\": %.1f, \"docs_per_s\": %.0f, \"seconds\": %.3f, \"cpu_us_per_call\": %.2f, "
         "\"throttled_ms\": %.1f, \"sink\": %llu}\n",
         ref ? "reference" : "gpu", callers, nl, 1e6 * all[nl / 2], 1e6 * all[(size_t)(0.99 * (double)(nl - 1))],
         1e6 * all[nl - 1], (double)nl / wall, wall, 1e6 * cpu / (double)nl,
         (th0 >= 0 && th1 >= 0) ? 1e-3 * (double)(th1 - th0) : -1.0, sink);
  return 0;
}
