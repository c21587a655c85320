// cld_dlqueue.h -- the per-call path of detect_language (wrapper.h:8), the
// zero-change drop-in: many threads each asking for one short document.
//
// Round 5 ran these calls through the request coalescer (cld_coalesce.h): the
// first caller to find a dispatch slot free led a group.  At 256 callers the
// process spent 112 us of CPU per call (4.6 us for the reference CLD2 itself;
// tools/dl_bench.c cpu_us_per_call) on a shared queue lock, group scans of the
// whole queue and condition-variable handoffs, and the box's 16-CPU cgroup
// quota then throttled it for tens of milliseconds at a time.  Here:
//
//  * a caller with no other call in flight runs its call itself (no handoff:
//    a lone caller's round trip stays what it was); otherwise it pushes a
//    request onto a lock-free stack (one CAS) and waits on a word of its own
//    request, spinning briefly while few calls are in flight, else sleeping
//    on a futex at once;
//  * dispatcher threads (a few per GPU, one tiny slot each) take the whole
//    stack with one exchange -- everything that arrived while they were busy
//    becomes the next launch -- run it, write each request's result and wake
//    the batch as a binary tree (finish_batch);
//  * an idle dispatcher spins a little before it sleeps; a push wakes a
//    sleeping one with one futex call.
//
// Host-only and GPU-free: tools/dlqueue_sim.cpp drives it with a mock
// dispatch under ASan and TSan (tests/test_coalesce.py).
#ifndef CLD_DLQUEUE_H_
#define CLD_DLQUEUE_H_
#include <linux/futex.h>
#include <stddef.h>
#include <stdint.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <atomic>
#include <chrono>

namespace cld {

inline void futex_wait(std::atomic<uint32_t>* a, uint32_t v) {
  syscall(SYS_futex, reinterpret_cast<uint32_t*>(a), FUTEX_WAIT_PRIVATE, v, nullptr, nullptr, 0);
}
inline void futex_wake(std::atomic<uint32_t>* a) {
  syscall(SYS_futex, reinterpret_cast<uint32_t*>(a), FUTEX_WAKE_PRIVATE, 1, nullptr, nullptr, 0);
}
inline void cpu_relax() { __builtin_ia32_pause(); }

struct DlReq {
  const uint8_t* p = nullptr;
  size_t len = 0;
  void* res = nullptr;           // where the dispatcher writes the result (its type)
  int rc = 0;
  DlReq* next = nullptr;         // the queue's link (the dispatcher's after take())
  DlReq* kid[2] = {nullptr, nullptr};   // finished by this caller once it is done (wake-up tree)
  // kWaiting -> kDone, or kWaiting -> kSleeping -> kDone.  The dispatcher
  // touches the request only up to its exchange to kDone (rc and the result
  // are written before it), so the caller may return the moment it sees kDone.
  enum : uint32_t { kWaiting = 0, kSleeping = 1, kDone = 2 };
  std::atomic<uint32_t> state{kWaiting};
  DlReq(const uint8_t* p_, size_t len_, void* res_) : p(p_), len(len_), res(res_) {}

  // Caller: waits for kDone, then finishes its kids; spins up to spin_us
  // first (0: sleep at once).
  void wait(int spin_us) {
    if (spin_us > 0) {
      const auto t0 = std::chrono::steady_clock::now();
      for (int k = 0; state.load(std::memory_order_acquire) == kWaiting; ++k) {
        cpu_relax();
        if ((k & 255) == 255 && std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(spin_us)) break;
      }
    }
    uint32_t s = kWaiting;
    if (state.compare_exchange_strong(s, kSleeping))
      s = kSleeping;
    while (s != kDone) {
      futex_wait(&state, kSleeping);
      s = state.load(std::memory_order_acquire);
    }
    DlReq* k0 = kid[0];
    DlReq* k1 = kid[1];
    if (k0) k0->finish();
    if (k1) k1->finish();
  }
  // Publishes rc / the result (written before) and wakes a sleeper.
  void finish() {
    if (state.exchange(kDone) == kSleeping) futex_wake(&state);
  }
};

// Dispatcher: hands a finished batch (results and rc written) back to its
// callers.  One futex wake-up costs ~1.5 us; woken one by one a 48-request
// batch kept the dispatcher 70 us from its next launch (tools/dlqueue_sim), so
// the batch is woken as a binary tree: the dispatcher finishes the first two,
// each caller the two below it before it returns.  The kids are set before
// any request is finished (a finished caller may return at once).
inline void finish_batch(DlReq* const* v, size_t n) {
  for (size_t j = 0; j < n; ++j)
    for (int c = 0; c < 2; ++c) {
      const size_t k = 2 * j + 2 + (size_t)c;
      v[j]->kid[c] = k < n ? v[k] : nullptr;
    }
  for (size_t j = 0; j < 2 && j < n; ++j) v[j]->finish();
}

class DlQueue {
 public:
  // Caller: counts itself in (returns the calls in flight before it); then
  // either runs its call itself (nothing else in flight) and leave()s, or
  // push()es it.
  int enter() { return inflight_.fetch_add(1); }
  void leave() { inflight_.fetch_sub(1); }
  // Caller (entered): enqueue.
  void push(DlReq* r) {
    DlReq* h = head_.load();
    do r->next = h; while (!head_.compare_exchange_weak(h, r));
    if (sleepers_.load() > 0) {
      seq_.fetch_add(1);
      futex_wake(&seq_);
    }
  }
  // Dispatcher: blocks until a request is queued, then takes every queued
  // one, oldest first (linked through next).  Spins up to spin_us before
  // sleeping.
  DlReq* take(int spin_us) {
    for (;;) {
      DlReq* l = head_.exchange(nullptr);
      if (!l && spin_us > 0) {
        const auto t0 = std::chrono::steady_clock::now();
        for (int k = 0; !head_.load(std::memory_order_relaxed); ++k) {
          cpu_relax();
          if ((k & 255) == 255 && std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(spin_us)) break;
        }
        l = head_.exchange(nullptr);
      }
      if (!l) {
        // announce the sleep, then look once more: a push either sees the
        // announcement (and bumps seq_, so the wait returns at once) or
        // happened before it (and the exchange below takes it)
        const uint32_t s = seq_.load();
        sleepers_.fetch_add(1);
        l = head_.exchange(nullptr);
        if (!l) futex_wait(&seq_, s);
        sleepers_.fetch_sub(1);
        if (!l) continue;
      }
      DlReq* f = nullptr;                      // LIFO -> FIFO
      while (l) {
        DlReq* n = l->next;
        l->next = f;
        f = l;
        l = n;
      }
      return f;
    }
  }
  // Dispatcher: one request is finished (before its finish()).
  void done_one() { inflight_.fetch_sub(1); }

 private:
  std::atomic<DlReq*> head_{nullptr};
  std::atomic<uint32_t> seq_{0};
  std::atomic<int> sleepers_{0};
  std::atomic<int> inflight_{0};
};

}  // namespace cld
#endif
