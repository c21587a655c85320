/* req_bench.c -- request-sized calls of the batch C ABI, timed from C.
 *
 * The reference service takes request bodies of at most 1 MiB
 * (handlers.go:33-68) and scores each item (handlers.go:105-186); a Go batch
 * route over this library would make one cld_detect_batch call per request.
 * This harness replays that: documents (a packed corpus written by
 * tools/req_rate.py) are cut into requests of at most REQ_BYTES of text, and
 * `callers` threads issue them concurrently, each call blocking like the
 * cgo call would.  Reported: per-call latency p50 / p99 and whole-run
 * documents per second.  No Python anywhere in the timed region.
 *
 *   req_bench <corpus.bin> <offsets.bin> <callers> [req_bytes] [reps]
 */
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "cld_mi355x.h"

static double now_s(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
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

typedef struct {
  const uint8_t* buf;
  const uint64_t* offs;
  const size_t* req;      /* request r = documents [req[r], req[r+1]) */
  size_t n_req;
  int caller, callers, reps;
  double* lat;            /* per call (seconds), indexed like the calls this thread makes */
  size_t n_lat;
  cld_result* out;
  int rc;
} job_t;

static void* run(void* a) {
  job_t* j = (job_t*)a;
  j->n_lat = 0;
  for (int rep = 0; rep < j->reps; ++rep)
    for (size_t r = (size_t)j->caller; r < j->n_req; r += (size_t)j->callers) {
      const size_t lo = j->req[r], hi = j->req[r + 1];
      const double t0 = now_s();
      const int rc = cld_detect_batch(j->buf, j->offs + lo, hi - lo, j->out, 0);
      j->lat[j->n_lat++] = now_s() - t0;
      if (rc != CLD_OK) { j->rc = rc; return NULL; }
    }
  return NULL;
}

static int cmp_d(const void* a, const void* b) {
  const double x = *(const double*)a, y = *(const double*)b;
  return x < y ? -1 : x > y;
}

int main(int argc, char** argv) {
  if (argc < 4) {
    fprintf(stderr, "usage: %s corpus.bin offsets.bin callers [req_bytes] [reps]\n", argv[0]);
    return 2;
  }
  size_t nb, no;
  const uint8_t* buf = (const uint8_t*)slurp(argv[1], &nb);
  const uint64_t* offs = (const uint64_t*)slurp(argv[2], &no);
  const size_t n = no / 8 - 1;
  const int callers = atoi(argv[3]);
  const uint64_t req_bytes = argc > 4 ? strtoull(argv[4], NULL, 10) : (1u << 20);
  const int reps = argc > 5 ? atoi(argv[5]) : 3;
  /* requests: consecutive documents up to req_bytes of text (at least one) */
  size_t* req = (size_t*)malloc(sizeof(size_t) * (n + 2));
  size_t n_req = 0;
  req[0] = 0;
  for (size_t i = 0; i < n;) {
    size_t k = i + 1;
    while (k < n && offs[k + 1] - offs[i] <= req_bytes) ++k;
    req[++n_req] = k;
    i = k;
  }
  if (cld_init(NULL, 0) != CLD_OK) { fprintf(stderr, "cld_init failed\n"); return 1; }
  /* warm-up: every caller's first calls allocate its chunk slots and staging */
  {
    cld_result* w = (cld_result*)malloc(sizeof(cld_result) * (req[1] - req[0]));
    for (int k = 0; k < 3; ++k) cld_detect_batch(buf, offs, req[1] - req[0], w, 0);
    free(w);
  }
  job_t* jobs = (job_t*)calloc((size_t)callers, sizeof(job_t));
  pthread_t* th = (pthread_t*)calloc((size_t)callers, sizeof(pthread_t));
  size_t maxreq = 0;
  for (size_t r = 0; r < n_req; ++r)
    if (req[r + 1] - req[r] > maxreq) maxreq = req[r + 1] - req[r];
  for (int c = 0; c < callers; ++c) {
    jobs[c] = (job_t){buf, offs, req, n_req, c, callers, reps, NULL, 0, NULL, CLD_OK};
    jobs[c].lat = (double*)malloc(sizeof(double) * (n_req / (size_t)callers + 2) * (size_t)reps);
    jobs[c].out = (cld_result*)malloc(sizeof(cld_result) * maxreq);
  }
  const double t0 = now_s();
  for (int c = 0; c < callers; ++c) pthread_create(&th[c], NULL, run, &jobs[c]);
  for (int c = 0; c < callers; ++c) pthread_join(th[c], NULL);
  const double wall = now_s() - t0;
  size_t nl = 0;
  for (int c = 0; c < callers; ++c) {
    if (jobs[c].rc != CLD_OK) { fprintf(stderr, "caller %d: rc %d\n", c, jobs[c].rc); return 1; }
    nl += jobs[c].n_lat;
  }
  double* all = (double*)malloc(sizeof(double) * (nl + 1));
  size_t k = 0;
  for (int c = 0; c < callers; ++c)
    for (size_t i = 0; i < jobs[c].n_lat; ++i) all[k++] = jobs[c].lat[i];
  qsort(all, nl, sizeof(double), cmp_d);
  const double docs = (double)n * reps;
  printf("{\"callers\": %d, \"requests\": %zu, \"req_bytes_max\": %llu, \"docs_per_request\": %.1f, "
         "\"calls\": %zu, \"latency_ms_p50\": %.3f, \"latency_ms_p99\": %.3f, \"latency_ms_max\": %.3f, "
         "\"docs_per_s\": %.0f, \"bytes_per_s\": %.0f, \"seconds\": %.3f}\n",
         callers, n_req, (unsigned long long)req_bytes, (double)n / (double)n_req, nl, 1e3 * all[nl / 2],
         1e3 * all[(size_t)(0.99 * (double)(nl - 1))], 1e3 * all[nl - 1], docs / wall,
         (double)(offs[n] - offs[0]) * reps / wall, wall);
  return 0;
}
