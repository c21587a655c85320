// cld_coalesce.h -- request coalescing for request-sized batch calls.
//
// A launch lasts as long as its longest document (one wavefront scores it
// start to end), and a GPU round trip has a fixed cost of tens of
// microseconds, so request-sized calls queued one after another pay both
// each; run together they pay them once.  Callers submit a request and block;
// the first caller to find a dispatch slot free takes the queued requests with
// its flags (within the group limits), runs them as one batch through `run`
// and hands every caller its results and return code.
//
// Slots: `slots_any` groups of any kind in flight, and up to `slots_tiny`
// while the extra ones carry tiny groups (requests marked `tiny`; a group
// whose first request is tiny takes only tiny requests, up to `tiny_docs`
// documents).
//
// Parking.  A queued caller sleeps on its own condition variable until its
// group is done (kDone) or it is promoted to form the next group (kLead).  A
// finished dispatcher wakes its group's members as a binary tree -- each woken
// member wakes two more before it returns -- so no thread issues more than a
// few wake-ups, and promotes the next queued caller to lead.  (One shared
// condition variable woke every waiter at every dispatch; re-acquiring the
// queue lock one by one cost ~1 ms per dispatch at 256 callers.)
//
// Host-only and GPU-free: tools/coalesce_sim.cpp drives it with a mock
// dispatch (tests/test_coalesce.py).
#ifndef CLD_COALESCE_H_
#define CLD_COALESCE_H_
#include <stddef.h>
#include <stdint.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <thread>
#include <mutex>
#include <vector>

namespace cld {

struct CoReq {
  const uint8_t* buf;
  const uint64_t* offs;          // n + 1 offsets into buf
  size_t n;
  void* out;                     // n results (the dispatcher's type)
  uint32_t flags;
  bool tiny;
  int rc = 0;
  enum { kWaiting = 0, kDone = 1, kLead = 2 };
  std::atomic<int> state{kWaiting};
  std::mutex m;
  std::condition_variable cv;
  bool promoted = false;         // under the queue lock: already asked to lead
  CoReq* kid[2] = {nullptr, nullptr};
  CoReq(const uint8_t* b, const uint64_t* o, size_t n_, void* r, uint32_t f, bool t)
      : buf(b), offs(o), n(n_), out(r), flags(f), tiny(t) {}
  // Lifetime rule: a CoReq lives on its caller's stack and dies when park()
  // (or settle()) returns kDone, so the poster must be finished with the
  // object by then.  post() stores the state and notifies while holding m,
  // and the waiter always takes m once after it sees a new state (in cv.wait,
  // or in settle() when the spin saw it), so it cannot return while a poster
  // is still inside post().
  void post(int st) {
    std::lock_guard<std::mutex> l(m);
    state.store(st);
    cv.notify_one();
  }
  // Waits for a poster that may still hold m (see above).
  void settle() { std::lock_guard<std::mutex> l(m); }
  // Spins up to spin_us first (a GPU round trip is tens of microseconds: most
  // waits end before a sleep and a wake-up would), then sleeps.
  int park(int spin_us) {
    int st = state.load();
    if (st == kWaiting && spin_us > 0) {
      const auto t0 = std::chrono::steady_clock::now();
      for (int k = 0; (st = state.load()) == kWaiting; ++k) {
        if ((k & 63) == 63) {
          if (std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(spin_us)) break;
          std::this_thread::yield();
        }
      }
    }
    {
      std::unique_lock<std::mutex> l(m);
      cv.wait(l, [&] { return (st = state.load()) != kWaiting; });
    }
    // a lead request is consumed here; if a dispatcher ran the request in the
    // meantime its kDone stays (a plain store would lose it)
    if (st == kLead) {
      int expect = kLead;
      if (!state.compare_exchange_strong(expect, kWaiting)) {
        st = expect;
        if (st == kDone) settle();
      }
    }
    return st;
  }
  bool done() const { return state.load() == kDone; }
  void wake_kids() {
    for (CoReq* k : kid)
      if (k) k->post(kDone);
  }
};

class Coalescer {
 public:
  using RunFn = void (*)(const std::vector<CoReq*>& grp, void* ctx);
  RunFn run = nullptr;
  void* ctx = nullptr;
  std::atomic<int> slots_any{1}, slots_tiny{1};   // (set by callers that know the device set)
  size_t tiny_docs = 1024;
  uint64_t max_bytes = 64ull << 20;
  size_t max_docs = 256 * 1024;
  int spin_us = 0;               // waiters spin this long before sleeping
  bool tree_wake = true;         // members wake each other (else the dispatcher wakes every one)

  // Blocks until the request has run (as part of some group); returns me->rc.
  int submit(CoReq* me) {
    std::vector<CoReq*> grp;
    std::unique_lock<std::mutex> lk(mu_);
    q_.push_back(me);
    for (;;) {
      if (me->done()) {                        // a promoted caller whose request another dispatcher ran
        lk.unlock();
        me->settle();
        me->wake_kids();
        return me->rc;
      }
      if (!form_group(&grp)) {
        lk.unlock();
        if (me->park(spin_us) == CoReq::kDone) {
          me->wake_kids();
          return me->rc;
        }
        lk.lock();                             // promoted: form the next group
        me->promoted = false;
        continue;
      }
      lk.unlock();
      run(grp, ctx);
      // wake-up tree over the other members, set before any wake-up (a woken
      // member returns, and its request with it)
      std::vector<CoReq*> others;
      others.reserve(grp.size());
      bool mine = false;
      for (CoReq* r : grp) {
        if (r == me) mine = true;
        else others.push_back(r);
      }
      if (tree_wake)
        for (size_t j = 0; j < others.size(); ++j)
          for (int c = 0; c < 2; ++c) {
            const size_t k = 2 * j + 2 + c;
            others[j]->kid[c] = k < others.size() ? others[k] : nullptr;
          }
      lk.lock();
      --active_;
      for (CoReq* r : q_)                      // the next group's dispatcher
        if (!r->promoted && r != me) {
          r->promoted = true;
          r->post(CoReq::kLead);
          break;
        }
      lk.unlock();
      for (size_t j = 0; j < (tree_wake ? 2 : others.size()) && j < others.size(); ++j) others[j]->post(CoReq::kDone);
      if (mine) return me->rc;
      lk.lock();
    }
  }

 private:
  // Caller holds mu_.
  bool form_group(std::vector<CoReq*>* grp) {
    const bool any_slot = active_ < slots_any.load(std::memory_order_relaxed);
    if (q_.empty() || !(any_slot || active_ < slots_tiny.load(std::memory_order_relaxed))) return false;
    // Only tiny slots free and a non-tiny request at the head of the queue
    // (the oldest): keep the slot, so that request takes the next free 'any'
    // slot instead of waiting behind a stream of tiny groups.
    if (!any_slot && !q_.front()->tiny) return false;
    const CoReq* first = nullptr;
    for (CoReq* r : q_)
      if (any_slot || r->tiny) {
        first = r;
        break;
      }
    if (!first) return false;
    const uint32_t f = first->flags;
    const bool tiny = first->tiny;
    uint64_t bytes = 0;
    size_t docs = 0;
    grp->clear();
    for (auto it = q_.begin(); it != q_.end();) {
      CoReq* r = *it;
      const uint64_t nb = r->offs[r->n] - r->offs[0];
      const bool fits = tiny ? r->tiny && docs + r->n <= tiny_docs
                             : grp->empty() || (bytes + nb <= max_bytes && docs + r->n <= max_docs);
      if (r->flags != f || !fits) {
        ++it;
        continue;
      }
      grp->push_back(r);
      bytes += nb;
      docs += r->n;
      it = q_.erase(it);
    }
    ++active_;
    return true;
  }
  std::mutex mu_;
  std::deque<CoReq*> q_;
  int active_ = 0;
};

}  // namespace cld
#endif
