// copy_rate.cpp -- host memcpy throughput from pageable memory into pinned
// (hipHostMalloc) memory with 1..16 threads, and the cost of hipHostRegister /
// hipHostUnregister of the same range: the two ways run_host_shard can feed
// the upload DMA from a pageable caller buffer.
//   copy_rate [MB]
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
  const size_t n = (argc > 1 ? strtoull(argv[1], nullptr, 10) : 137) << 20;
  std::vector<unsigned char> src(n, 7);
  unsigned char* dst = nullptr;
  if (hipHostMalloc((void**)&dst, n, hipHostMallocDefault) != hipSuccess) return 1;
  memset(dst, 0, n);
  for (int t : {1, 2, 4, 8, 12, 16, 24}) {
    double best = 1e9;
    for (int rep = 0; rep < 5; ++rep) {
      const double t0 = now();
      std::vector<std::thread> th;
      const size_t per = (n + t - 1) / t;
      for (int i = 0; i < t; ++i) {
        const size_t a = per * i, b = std::min(n, a + per);
        th.emplace_back([=, &src] { memcpy(dst + a, src.data() + a, b - a); });
      }
      for (auto& x : th) x.join();
      best = std::min(best, now() - t0);
    }
    printf("{\"threads\": %d, \"MB\": %zu, \"ms\": %.3f, \"GB_per_s\": %.1f}\n", t, n >> 20, 1e3 * best, n / best / 1e9);
  }
  for (int rep = 0; rep < 3; ++rep) {
    const double t0 = now();
    if (hipHostRegister(src.data(), n, hipHostRegisterDefault) != hipSuccess) return 1;
    const double t1 = now();
    (void)hipHostUnregister(src.data());
    const double t2 = now();
    printf("{\"register_ms\": %.3f, \"unregister_ms\": %.3f}\n", 1e3 * (t1 - t0), 1e3 * (t2 - t1));
  }
  return 0;
}
