// cld_kernels.hip -- batch kernels over the device pipeline.
//
//  k_short<CAP>  one lane per document of <= CAP bytes, all state in private
//                memory, pass 1 only.  Anything it cannot finish (longer
//                document, Squeeze restart, Repeats pass, capacity) is
//                appended to the re-queue list.
//  k_general     any document, all passes, per-lane state in a global arena;
//                persistent grid pulling documents from the re-queue list
//                with one atomic dequeue per document.
#include "cld_kernels.h"
#include "cld_pipeline.hip"
#include "cld_wave.hip"

namespace cld {

using ShortWork = Work<kShortSB, kShortLB, kShortHB, false>;
using GeneralWork = Work<kMaxScriptBuffer, kMaxScriptLowerBuffer, kMaxScoringHits + 8, true>;

__global__ __launch_bounds__(256) void k_short(DevTables T, const uint8_t* __restrict__ buf,
                                              const uint64_t* __restrict__ offs, int n,
                                              cld_result* __restrict__ out,
                                              uint32_t* __restrict__ requeue_list,
                                              uint32_t* __restrict__ counters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t a = offs[i], b = offs[i + 1];
  const int64_t len = (int64_t)(b - a);
  bool rq = len > kShortCap;
  if (!rq) {
    ShortWork w;
    Status st{false};
    DocView d{buf + a, (int)len};
    detect_doc(T, d, w, &out[i], st);
    rq = st.requeue;
  }
  if (rq) {
    uint32_t k = atomicAdd(&counters[kCtrRequeue], 1u);
    requeue_list[k] = (uint32_t)i;
  }
}

__global__ __launch_bounds__(64) void k_general(DevTables T, const uint8_t* __restrict__ buf,
                                               const uint64_t* __restrict__ offs,
                                               const uint32_t* __restrict__ list,
                                               cld_result* __restrict__ out,
                                               uint8_t* __restrict__ arena, uint64_t stride,
                                               uint32_t* __restrict__ counters) {
  const int lane = blockIdx.x * blockDim.x + threadIdx.x;
  GeneralWork& w = *reinterpret_cast<GeneralWork*>(arena + (uint64_t)lane * stride);
  const uint32_t total = __hip_atomic_load(&counters[kCtrRequeue], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  for (;;) {
    uint32_t k = atomicAdd(&counters[kCtrDequeue], 1u);
    if (k >= total) break;                       // every lane reaches this exit
    const uint32_t i = list[k];
    const uint64_t a = offs[i], b = offs[i + 1];
    Status st{false};
    DocView d{buf + a, (int)(b - a)};
    int passes = detect_doc(T, d, w, &out[i], st);
    if (passes >= 1 && passes <= 3) atomicAdd(&counters[kCtrPass1 + passes - 1], 1u);
    else atomicAdd(&counters[kCtrError], 1u);
  }
}

// One wavefront per document of <= CAP bytes, WPB documents per workgroup.
template <int CAP, int WPB>
__global__ __launch_bounds__(64 * WPB, 6) void k_wave(DevTables T, const uint8_t* __restrict__ buf,
                                                   const uint64_t* __restrict__ offs, int n,
                                                   cld_result* __restrict__ out,
                                                   uint32_t* __restrict__ requeue_list,
                                                   uint32_t* __restrict__ counters,
                                                   unsigned long long* __restrict__ prof) {
  __shared__ wave::Smem<CAP> smem[WPB];
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int i = blockIdx.x * WPB + wv;
  if (i >= n) return;
  const uint64_t a = offs[i], b = offs[i + 1];
  const int64_t len = (int64_t)(b - a);
  bool rq = len > CAP;
  if (!rq) rq = !wave::detect<CAP>(T, buf + a, (int)len, smem[wv], lane, &out[i], prof);
  if (rq && lane == 0) {
    uint32_t k = atomicAdd(&counters[kCtrRequeue], 1u);
    requeue_list[k] = (uint32_t)i;
  }
}

}  // namespace cld

extern "C" {
size_t cld_general_work_bytes() { return sizeof(cld::GeneralWork); }
size_t cld_short_work_bytes() { return sizeof(cld::ShortWork); }
size_t cld_wave_smem_bytes() { return sizeof(cld::wave::Smem<kWaveCap>); }

hipError_t cld_launch_wave(const DevTables* T, const uint8_t* buf, const uint64_t* offs, int n,
                           cld_result* out, uint32_t* requeue_list, uint32_t* counters,
                           unsigned long long* prof, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  dim3 grid((n + kWaveWPB - 1) / kWaveWPB), block(64 * kWaveWPB);
  hipLaunchKernelGGL((cld::k_wave<kWaveCap, kWaveWPB>), grid, block, 0, s, *T, buf, offs, n, out,
                     requeue_list, counters, prof);
  return hipGetLastError();
}

hipError_t cld_launch_short(const DevTables* T, const uint8_t* buf, const uint64_t* offs, int n,
                            cld_result* out, uint32_t* requeue_list, uint32_t* counters,
                            hipStream_t s) {
  if (n <= 0) return hipSuccess;
  dim3 grid((n + 255) / 256), block(256);
  hipLaunchKernelGGL(cld::k_short, grid, block, 0, s, *T, buf, offs, n, out, requeue_list, counters);
  return hipGetLastError();
}

hipError_t cld_launch_general(const DevTables* T, const uint8_t* buf, const uint64_t* offs,
                              const uint32_t* list, cld_result* out, uint8_t* arena,
                              uint64_t stride, int lanes, uint32_t* counters, hipStream_t s) {
  dim3 grid(lanes / 64), block(64);
  hipLaunchKernelGGL(cld::k_general, grid, block, 0, s, *T, buf, offs, list, out, arena, stride,
                     counters);
  return hipGetLastError();
}
}
