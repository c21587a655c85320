// cld_strip.hip -- the service's per-document text preparation, on the GPU.
//
// handlers.go:150-151 prepares each request text before detection:
//   textStr = StripExtras(textStr)          handlers.go:198-210
//   code := Detect_language(textStr)        main.go:77-81: C.CString -> strlen
// StripExtras keeps the strings.Fields words that do not start with "@" or
// "http" and appends one ' ' after each kept word; the cgo hand-off then cuts
// the text at its first NUL byte.  cld_detect_batch applies these steps on
// the device when asked (CLD_FLAG_STRIP_EXTRAS / CLD_FLAG_CSTRING), so a
// batch of raw request texts is prepared and scored without a host pass.
//
// strings.Fields splits on unicode.IsSpace runes: \t \n \v \f \r ' ', U+0085,
// U+00A0, U+1680, U+2000-U+200A, U+2028, U+2029, U+202F, U+205F, U+3000.
// Every one of them is a valid UTF-8 sequence starting with an ASCII or a lead
// byte, and Go's decoder starts a rune at every such byte (a valid sequence
// only ever covers continuation bytes; an invalid one advances one byte), so
// "a space rune starts at byte p" depends only on bytes p..p+2 and the word
// structure is byte-local -- one byte per lane, 64 bytes per step.
//
// Two kernels and a scan: k_strip_len (stripped length per document) ->
// exclusive scan -> k_strip_write (bytes at their output positions).
// Algorithmic bytes: the text is read once per kernel and written once.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "cld_kernels.h"

namespace cld {
namespace strip {

constexpr int kWPB = 4;          // documents (waves) per workgroup
constexpr int kScanBlock = 1024; // scan tile

__device__ __forceinline__ uint32_t ldb(const uint8_t* p, int64_t i, int64_t n) {
  return (i >= 0 && i < n) ? (uint32_t)p[i] : 0x100u;   // 0x100: outside the document
}

// Length (1-3) of the unicode.IsSpace rune starting at p[i], 0 if none.
__device__ __forceinline__ int space_len(const uint8_t* p, int64_t i, int64_t n) {
  const uint32_t c = ldb(p, i, n);
  if (c == 0x20 || (c >= 0x09 && c <= 0x0D)) return 1;
  if (c == 0xC2) {
    const uint32_t c1 = ldb(p, i + 1, n);
    return (c1 == 0x85 || c1 == 0xA0) ? 2 : 0;
  }
  if (c == 0xE1) return (ldb(p, i + 1, n) == 0x9A && ldb(p, i + 2, n) == 0x80) ? 3 : 0;
  if (c == 0xE2) {
    const uint32_t c1 = ldb(p, i + 1, n), c2 = ldb(p, i + 2, n);
    if (c1 == 0x80) return (c2 <= 0x8A || c2 == 0xA8 || c2 == 0xA9 || c2 == 0xAF) && c2 >= 0x80 ? 3 : 0;
    return (c1 == 0x81 && c2 == 0x9F) ? 3 : 0;
  }
  if (c == 0xE3) return (ldb(p, i + 1, n) == 0x80 && ldb(p, i + 2, n) == 0x80) ? 3 : 0;
  return 0;
}

// Byte i lies inside a space rune.
__device__ __forceinline__ bool in_space(const uint8_t* p, int64_t i, int64_t n) {
  if (i < 0 || i >= n) return true;                      // document edges act as separators
  if (space_len(p, i, n)) return true;
  if (i >= 1 && space_len(p, i - 1, n) >= 2) return true;
  return i >= 2 && space_len(p, i - 2, n) == 3;
}

// A word starting at p[i] is dropped: HasPrefix(word, "@") || HasPrefix(word, "http")
// (the four bytes of "http" are non-space ASCII, so they are inside the word).
__device__ __forceinline__ bool dropped(const uint8_t* p, int64_t i, int64_t n) {
  if (ldb(p, i, n) == '@') return true;
  return ldb(p, i, n) == 'h' && ldb(p, i + 1, n) == 't' && ldb(p, i + 2, n) == 't' && ldb(p, i + 3, n) == 'p';
}

// One document, 64 bytes per step.  WRITE = false: returns the prepared
// length; WRITE = true: stores the first `limit` prepared bytes at dst.
template <bool WRITE>
__device__ int64_t prepare(const uint8_t* __restrict__ p, int64_t n, bool strip, bool cstr, uint8_t* __restrict__ dst,
                           int64_t limit, int lane) {
  int64_t out = 0;                 // prepared bytes before this step (wave-uniform)
  int64_t first_nul = INT64_MAX;   // output position of the first NUL (wave-uniform)
  bool carry_keep = true;          // keep flag of a word running into this step
  const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
  for (int64_t base = 0; base < n; base += 64) {
    const int64_t i = base + lane;
    const bool valid = i < n;
    const uint32_t c = valid ? p[i] : 0u;
    bool keep_byte, word_end;
    if (strip) {
      const bool ws = !valid || in_space(p, i, n);
      const bool ws_prev = in_space(p, i - 1, n);
      const bool ws_next = in_space(p, i + 1, n);
      const bool start = !ws && ws_prev;
      const uint64_t starts = __ballot(start);
      const uint64_t keeps = __ballot(start && !dropped(p, i, n));
      // keep flag of this byte's word: its start in this step, else the carried one
      const uint64_t mine = starts & (lt | (1ull << lane));
      const bool keep = mine ? ((keeps >> (63 - __clzll(mine))) & 1ull) != 0 : carry_keep;
      keep_byte = !ws && keep;
      word_end = keep_byte && ws_next;
      const uint64_t last = __ballot(lane == 63 ? keep : false);
      carry_keep = last != 0;
    } else {
      keep_byte = valid;
      word_end = false;
    }
    const uint64_t kb = __ballot(keep_byte), we = __ballot(word_end);
    const int64_t pos = out + __popcll(kb & lt) + __popcll(we & lt);
    if (cstr) {
      const uint64_t nul = __ballot(keep_byte && c == 0);
      if (nul && first_nul == INT64_MAX) {
        const int l = __ffsll((long long)nul) - 1;
        first_nul = out + __popcll(kb & (l ? (~0ull >> (64 - l)) : 0ull)) + __popcll(we & (l ? (~0ull >> (64 - l)) : 0ull));
      }
    }
    if constexpr (WRITE) {
      if (keep_byte && pos < limit) dst[pos] = (uint8_t)c;
      if (word_end && pos + 1 < limit) dst[pos + 1] = ' ';
    }
    out += __popcll(kb) + __popcll(we);
    if (cstr && first_nul != INT64_MAX) break;   // nothing after the first NUL survives
  }
  return out < first_nul ? out : first_nul;
}

__global__ __launch_bounds__(64 * kWPB) void k_strip_len(const uint8_t* __restrict__ buf,
                                                         const uint64_t* __restrict__ offs, int n, uint32_t flags,
                                                         uint64_t* __restrict__ len) {
  const int d = blockIdx.x * kWPB + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (d >= n) return;
  const uint64_t a = offs[d], b = offs[d + 1];
  const int64_t l = prepare<false>(buf + a, (int64_t)(b - a), flags & 1u, flags & 2u, nullptr, 0, lane);
  if (lane == 0) len[d] = (uint64_t)l;
}

__global__ __launch_bounds__(64 * kWPB) void k_strip_write(const uint8_t* __restrict__ buf,
                                                           const uint64_t* __restrict__ offs, int n,
                                                           uint32_t flags, const uint64_t* __restrict__ out_offs,
                                                           uint8_t* __restrict__ out) {
  const int d = blockIdx.x * kWPB + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (d >= n) return;
  const uint64_t a = offs[d], b = offs[d + 1];
  const uint64_t o = out_offs[d], lim = out_offs[d + 1] - o;
  prepare<true>(buf + a, (int64_t)(b - a), flags & 1u, flags & 2u, out + o, (int64_t)lim, lane);
}

// Exclusive scan of n lengths into offs[0..n] (offs[n] = total), 3 phases.
__device__ __forceinline__ uint64_t block_incl_scan(uint64_t v, uint64_t* sm) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint64_t y = __shfl_up(v, d, 64);
    if (lane >= d) v += y;
  }
  if (lane == 63) sm[w] = v;
  __syncthreads();
  if (w == 0) {
    uint64_t s = lane < (kScanBlock / 64) ? sm[lane] : 0;
#pragma unroll
    for (int d = 1; d < 16; d <<= 1) {
      const uint64_t y = __shfl_up(s, d, 64);
      if (lane >= d) s += y;
    }
    if (lane < kScanBlock / 64) sm[lane] = s;
  }
  __syncthreads();
  if (w > 0) v += sm[w - 1];
  return v;
}

__global__ __launch_bounds__(kScanBlock) void k_scan_tiles(const uint64_t* __restrict__ len, int n,
                                                           uint64_t* __restrict__ offs, uint64_t* __restrict__ tile) {
  __shared__ uint64_t sm[kScanBlock / 64];
  const int i = blockIdx.x * kScanBlock + threadIdx.x;
  const uint64_t v = i < n ? len[i] : 0;
  const uint64_t inc = block_incl_scan(v, sm);
  if (i < n) offs[i + 1] = inc;             // tile-local inclusive sums
  if (threadIdx.x == kScanBlock - 1) tile[blockIdx.x] = inc;
}

__global__ __launch_bounds__(kScanBlock) void k_scan_carry(uint64_t* __restrict__ tile, int ntiles) {
  __shared__ uint64_t sm[kScanBlock / 64];
  __shared__ uint64_t carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (int b = 0; b < ntiles; b += kScanBlock) {    // exclusive, in place, any tile count
    const int i = b + threadIdx.x;
    const uint64_t v = i < ntiles ? tile[i] : 0;
    const uint64_t inc = block_incl_scan(v, sm);
    const uint64_t c = carry;
    __syncthreads();
    if (i < ntiles) tile[i] = c + inc - v;
    if (threadIdx.x == kScanBlock - 1) carry = c + inc;
    __syncthreads();
  }
}

__global__ __launch_bounds__(kScanBlock) void k_scan_add(uint64_t* __restrict__ offs, int n,
                                                         const uint64_t* __restrict__ tile) {
  const int i = blockIdx.x * kScanBlock + threadIdx.x;
  if (i < n) offs[i + 1] += tile[blockIdx.x];
  if (i == 0) offs[0] = 0;
}

}  // namespace strip
}  // namespace cld

extern "C" {
size_t cld_strip_scratch_bytes(int n) {
  const size_t tiles = ((size_t)n + cld::strip::kScanBlock - 1) / cld::strip::kScanBlock;
  return ((size_t)n + tiles + 1) * sizeof(uint64_t);
}

// Prepared-text offsets for n documents: out_offs[0..n].  scratch: cld_strip_scratch_bytes(n).
hipError_t cld_launch_strip_offsets(const uint8_t* buf, const uint64_t* offs, int n, uint32_t flags,
                                    uint64_t* out_offs, void* scratch, hipStream_t s) {
  using namespace cld::strip;
  if (n <= 0) return hipMemsetAsync(out_offs, 0, sizeof(uint64_t), s);
  uint64_t* len = (uint64_t*)scratch;
  uint64_t* tile = len + n;
  const int ntiles = (n + kScanBlock - 1) / kScanBlock;
  hipLaunchKernelGGL(k_strip_len, dim3((n + kWPB - 1) / kWPB), dim3(64 * kWPB), 0, s, buf, offs, n, flags, len);
  hipLaunchKernelGGL(k_scan_tiles, dim3(ntiles), dim3(kScanBlock), 0, s, len, n, out_offs, tile);
  hipLaunchKernelGGL(k_scan_carry, dim3(1), dim3(kScanBlock), 0, s, tile, ntiles);
  hipLaunchKernelGGL(k_scan_add, dim3(ntiles), dim3(kScanBlock), 0, s, out_offs, n, tile);
  return hipGetLastError();
}

hipError_t cld_launch_strip_write(const uint8_t* buf, const uint64_t* offs, int n, uint32_t flags,
                                  const uint64_t* out_offs, uint8_t* out, hipStream_t s) {
  using namespace cld::strip;
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_strip_write, dim3((n + kWPB - 1) / kWPB), dim3(64 * kWPB), 0, s, buf, offs, n, flags,
                     out_offs, out);
  return hipGetLastError();
}
}
