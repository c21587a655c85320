// dlqueue_sim.cpp -- detect_language's per-call queue (language-detector_amd/
// csrc/cld_dlqueue.h) under many callers, with a mock dispatch instead of the
// GPU.  Host-only: it measures the queue's own CPU cost per call and checks
// that every caller gets exactly its own result, with no lost wake-up.
//
//   dlqueue_sim <callers> <calls_per_caller> <dispatchers> <gpu_us> [caller_spin_us] [dispatcher_spin_us]
//
// The mock dispatch waits gpu_us (+ 20 ns per document), spinning like a
// busy-waiting stream synchronise, then writes each request's result (its
// document pointer and length).  Every request is a heap object freed the
// moment wait() returns, so a dispatcher still touching it afterwards is a
// use-after-free for the sanitizer builds (build/dlqueue_sim_asan / _tsan).
// One JSON line.
#include <stdio.h>
#include <stdlib.h>
#include <sys/resource.h>
#include <time.h>

#include <algorithm>
#include <atomic>
#include <thread>
#include <vector>

#include "cld_dlqueue.h"

static double now_s() {
  timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}
static double cpu_s() {
  rusage r;
  getrusage(RUSAGE_SELF, &r);
  return (double)r.ru_utime.tv_sec + 1e-6 * (double)r.ru_utime.tv_usec + (double)r.ru_stime.tv_sec +
         1e-6 * (double)r.ru_stime.tv_usec;
}

struct Res {
  uintptr_t p;
  size_t len;
};

static cld::DlQueue g_q;
static std::atomic<long> g_batches{0}, g_docs{0};
static const size_t kStop = ~(size_t)0;

static void dispatcher(double gpu_us, int spin_us) {
  std::vector<cld::DlReq*> v;
  for (;;) {
    v.clear();
    for (cld::DlReq* r = g_q.take(spin_us); r; r = r->next) v.push_back(r);
    bool stop = false;
    const double t0 = now_s(), wait = 1e-6 * gpu_us + 2e-8 * (double)v.size();
    while (now_s() - t0 < wait) {}
    for (cld::DlReq* r : v) {
      if (r->len == kStop) stop = true;
      *static_cast<Res*>(r->res) = Res{reinterpret_cast<uintptr_t>(r->p), r->len};
      r->rc = 0;
      g_q.done_one();
    }
    cld::finish_batch(v.data(), v.size());
    g_batches.fetch_add(1);
    g_docs.fetch_add((long)v.size());
    if (stop) return;
  }
}

int main(int argc, char** argv) {
  if (argc < 5) {
    fprintf(stderr, "usage: %s callers calls dispatchers gpu_us [caller_spin_us] [dispatcher_spin_us]\n", argv[0]);
    return 2;
  }
  const int callers = atoi(argv[1]), calls = atoi(argv[2]), nd = atoi(argv[3]);
  const double gpu_us = atof(argv[4]);
  const int cspin = argc > 5 ? atoi(argv[5]) : 20, dspin = argc > 6 ? atoi(argv[6]) : 50;
  std::vector<std::thread> ds;
  for (int k = 0; k < nd; ++k) ds.emplace_back(dispatcher, gpu_us, dspin);
  std::atomic<long> wrong{0};
  std::vector<std::vector<double>> lat(callers);
  const double t0 = now_s(), c0 = cpu_s();
  std::vector<std::thread> cs;
  for (int c = 0; c < callers; ++c)
    cs.emplace_back([&, c] {
      lat[c].reserve(calls);
      for (int i = 0; i < calls; ++i) {
        const uint8_t* p = reinterpret_cast<const uint8_t*>((uintptr_t)(c * 100000 + i + 1));
        const size_t len = (size_t)(c + i) % 256;
        Res* res = new Res{0, 0};
        cld::DlReq* r = new cld::DlReq(p, len, res);
        const double a = now_s();
        const int before = g_q.enter();
        g_q.push(r);
        r->wait(before < 16 ? cspin : 0);
        lat[c].push_back(now_s() - a);
        if (r->rc != 0 || res->p != reinterpret_cast<uintptr_t>(p) || res->len != len) wrong.fetch_add(1);
        delete r;
        delete res;
      }
    });
  for (auto& t : cs) t.join();
  const double wall = now_s() - t0, cpu = cpu_s() - c0;
  for (int k = 0; k < nd; ++k) {                 // one stop request per dispatcher, each waited for
    Res res{0, 0};
    cld::DlReq r(nullptr, kStop, &res);
    g_q.enter();
    g_q.push(&r);
    r.wait(0);
  }
  for (auto& t : ds) t.join();
  std::vector<double> all;
  for (auto& l : lat) all.insert(all.end(), l.begin(), l.end());
  std::sort(all.begin(), all.end());
  const size_t n = all.size();
  printf("{\"callers\": %d, \"calls\": %zu, \"wrong\": %ld, \"dispatchers\": %d, \"batches\": %ld, "
         "\"docs_per_batch\": %.1f, \"latency_us_p50\": %.1f, \"latency_us_p99\": %.1f, \"calls_per_s\": %.0f, "
         "\"cpu_us_per_call\": %.2f}\n",
         callers, n, wrong.load(), nd, g_batches.load(), (double)g_docs.load() / (double)std::max(1L, g_batches.load()),
         1e6 * all[n / 2], 1e6 * all[(size_t)(0.99 * (double)(n - 1))], (double)n / wall, 1e6 * cpu / (double)n);
  return wrong.load() ? 1 : 0;
}
