// coalesce_sim.cpp -- the request coalescer (language-detector_amd/csrc/
// cld_coalesce.h) under many callers, with a mock dispatch instead of the GPU.
// Host-only: it measures the coalescer's own cost (queueing, parking,
// wake-ups) and checks that every caller gets exactly its own results.
//
//   coalesce_sim <callers> <calls_per_caller> <gpu_us> [sleep|spin] [slots_any] [slots_tiny] [spin_us]
//                [tree|direct] [mixed]
//
// The mock dispatch waits gpu_us (+ 20 ns per document) -- sleeping, or
// spinning like a busy-waiting stream synchronise -- then writes each
// document's result (its first byte and length).  One JSON line.
//
// Every request is a heap object freed as soon as submit() returns, so a
// poster still touching it afterwards is a use-after-free that the sanitizer
// builds (build/coalesce_sim_asan, build/coalesce_sim_tsan) report.  "mixed":
// every fourth caller submits non-tiny requests of 64 documents, every eighth
// with other flags; their latency is reported apart (non-tiny p99).
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <algorithm>
#include <atomic>
#include <thread>
#include <vector>

#include "cld_coalesce.h"

static double now_s() {
  timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

static double g_gpu_us = 30;
static bool g_spin = false;
static std::atomic<long> g_groups{0}, g_docs{0};

static void mock_run(const std::vector<cld::CoReq*>& grp, void*) {
  size_t docs = 0;
  for (auto* r : grp) docs += r->n;
  const double wait = 1e-6 * g_gpu_us + 2e-8 * (double)docs;
  if (g_spin) {
    const double t0 = now_s();
    while (now_s() - t0 < wait) {
    }
  } else {
    timespec ts{0, (long)(wait * 1e9)};
    nanosleep(&ts, nullptr);
  }
  for (auto* r : grp) {
    uint64_t* o = (uint64_t*)r->out;
    for (size_t i = 0; i < r->n; ++i) {
      const uint64_t a = r->offs[i], b = r->offs[i + 1];
      o[i] = ((b - a) << 8) | (b > a ? r->buf[a] : 0);
    }
    r->rc = 0;
  }
  g_groups.fetch_add(1);
  g_docs.fetch_add((long)docs);
}

int main(int argc, char** argv) {
  if (argc < 4) {
    fprintf(stderr, "usage: %s callers calls gpu_us [sleep|spin] [slots_any] [slots_tiny]\n", argv[0]);
    return 2;
  }
  const int callers = atoi(argv[1]), calls = atoi(argv[2]);
  g_gpu_us = atof(argv[3]);
  g_spin = argc > 4 && strcmp(argv[4], "spin") == 0;
  cld::Coalescer co;
  co.run = mock_run;
  co.slots_any = argc > 5 ? atoi(argv[5]) : 1;
  co.slots_tiny = argc > 6 ? atoi(argv[6]) : 2;
  co.spin_us = argc > 7 ? atoi(argv[7]) : 0;
  co.tree_wake = !(argc > 8 && strcmp(argv[8], "direct") == 0);
  const bool mixed = argc > 9 && strcmp(argv[9], "mixed") == 0;
  // documents: 4096 strings of 20..199 bytes
  std::vector<uint8_t> buf;
  std::vector<uint64_t> offs{0};
  unsigned s = 12345;
  for (int i = 0; i < 4096; ++i) {
    const int len = 20 + (int)((s = s * 1103515245u + 12345u) >> 16) % 180;
    for (int k = 0; k < len; ++k) buf.push_back((uint8_t)('a' + ((s >> (k % 16)) + k) % 26));
    offs.push_back(buf.size());
  }
  std::vector<std::vector<double>> lat(callers), lat_big(callers);
  std::atomic<long> bad{0};
  pthread_barrier_t bar;
  pthread_barrier_init(&bar, nullptr, (unsigned)callers + 1);
  std::vector<std::thread> th;
  for (int c = 0; c < callers; ++c)
    th.emplace_back([&, c] {
      lat[c].reserve(calls);
      pthread_barrier_wait(&bar);
      const bool big = mixed && c % 4 == 3;
      const size_t nd = big ? 64 : 1;
      const uint32_t flags = mixed && c % 8 == 7 ? 1u : 0u;
      std::vector<uint64_t> res(nd);
      for (int k = 0; k < calls; ++k) {
        const size_t i = ((size_t)c * 7919 + (size_t)k * 31) % (4096 - nd);
        auto* r = new cld::CoReq(buf.data(), offs.data() + i, nd, res.data(), flags, !big);
        const double t0 = now_s();
        const int rc = co.submit(r);
        delete r;
        (big ? lat_big : lat)[c].push_back(now_s() - t0);
        bool ok = rc == 0;
        for (size_t j = 0; j < nd; ++j)
          ok = ok && res[j] == (((offs[i + j + 1] - offs[i + j]) << 8) | buf[offs[i + j]]);
        if (!ok) bad.fetch_add(1);
      }
      pthread_barrier_wait(&bar);
    });
  pthread_barrier_wait(&bar);
  const double t0 = now_s();
  pthread_barrier_wait(&bar);
  const double wall = now_s() - t0;
  for (auto& t : th) t.join();
  std::vector<double> all, big;
  for (auto& v : lat) all.insert(all.end(), v.begin(), v.end());
  for (auto& v : lat_big) big.insert(big.end(), v.begin(), v.end());
  std::sort(all.begin(), all.end());
  std::sort(big.begin(), big.end());
  const size_t n = all.size();
  const double big_p99 = big.empty() ? 0.0 : 1e6 * big[(size_t)(0.99 * (double)(big.size() - 1))];
  printf("{\"callers\": %d, \"calls\": %zu, \"gpu_us\": %.1f, \"wait\": \"%s\", \"slots\": [%d, %d], "
         "\"latency_us_p50\": %.1f, \"latency_us_p99\": %.1f, \"latency_us_max\": %.1f, \"docs_per_s\": %.0f, "
         "\"docs_per_group\": %.1f, \"spin_us\": %d, \"wake\": \"%s\", \"non_tiny_calls\": %zu, "
         "\"non_tiny_latency_us_p99\": %.1f, \"wrong\": %ld}\n",
         callers, n + big.size(), g_gpu_us, g_spin ? "spin" : "sleep", co.slots_any.load(), co.slots_tiny.load(), 1e6 * all[n / 2],
         1e6 * all[(size_t)(0.99 * (double)(n - 1))], 1e6 * all[n - 1], (double)g_docs.load() / wall,
         (double)g_docs.load() / (double)std::max(1L, g_groups.load()), co.spin_us, co.tree_wake ? "tree" : "direct",
         big.size(), big_p99, bad.load());
  return bad.load() ? 1 : 0;
}
