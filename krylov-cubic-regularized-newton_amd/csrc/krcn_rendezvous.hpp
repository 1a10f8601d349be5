// krcn_rendezvous.hpp — the rendezvous of a virtual communicator's rank
// threads (host-only; krcn_comm_create_virtual in krcn_plan.hip, and the
// sanitizer stress test tests/native/rendezvous_stress.cpp).
//
// Every rank thread of the group calls arrive() once per all-reduce, in the
// same order on every rank.  The last to arrive runs the sum over all ranks'
// buffers (a device kernel in the library, a host loop in the stress test)
// WITHOUT holding the lock, then bumps the generation and releases the
// others.  A rank that never arrives (it failed, the caller drives fewer
// threads than ranks, or its sequence of collectives differs) breaks the
// group after timeout_s, and the failure text names every rank's progress.
#pragma once
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <mutex>
#include <string>

#include "krcn.h"

namespace krcn {

constexpr int kRvMaxRanks = 16;

struct Rendezvous {
  int P = 0;
  int timeout_s = 90;
  std::mutex mu;
  std::condition_variable cv;
  int arrived = 0, alive = 0;
  uint64_t gen = 0;                    // completed all-reduces of the group
  int64_t count = -1;
  int dtype = KRCN_F64;
  bool broken = false;                 // a rank's call was inconsistent or timed out
  int result = KRCN_OK;                // of the last completed all-reduce
  void* bufs[kRvMaxRanks] = {};
  // per rank, for the failure report: all-reduces entered, the count of the
  // last one, and whether the rank waits in the current one
  uint64_t seq[kRvMaxRanks] = {};
  int64_t last_count[kRvMaxRanks] = {};
  bool here[kRvMaxRanks] = {};

  // "gen 57, 7 of 8 arrived (count 2000000 f64); rank 4: 56 entered, last count 1, absent; ..."
  // (the caller holds mu)
  std::string state() const {
    char buf[160];
    snprintf(buf, sizeof(buf), "gen %llu, %d of %d arrived (count %lld %s)", (unsigned long long)gen, arrived, P,
             (long long)count, dtype == KRCN_F64 ? "f64" : "f32");
    std::string out = buf;
    for (int r = 0; r < P; ++r) {
      snprintf(buf, sizeof(buf), "; rank %d: %llu entered, last count %lld, %s", r, (unsigned long long)seq[r],
               (long long)last_count[r], here[r] ? "waiting" : "absent");
      out += buf;
    }
    return out;
  }

  // Rank `me` (its all-reduce counter *my_seq) arrives with buf[count].  The
  // last arrival calls sum(bufs, P, count, dtype) -> krcn_status.  Returns the
  // status; on failure *msg holds the text.
  template <class Sum>
  int arrive(int me, uint64_t* my_seq, void* buf, int64_t cnt, int dt, Sum&& sum, std::string* msg) {
    std::unique_lock<std::mutex> lk(mu);
    seq[me] = ++*my_seq;
    last_count[me] = cnt;
    if (broken) {
      *msg = "virtual all-reduce: the group is broken (an earlier rank failed): " + state();
      return KRCN_ERR_RCCL;
    }
    if (arrived == 0) {
      count = cnt;
      dtype = dt;
    } else if (count != cnt || dtype != dt) {
      broken = true;
      cv.notify_all();
      char b[160];
      snprintf(b, sizeof(b), "virtual all-reduce: rank %d passed %lld values, rank(s) before it %lld: ", me,
               (long long)cnt, (long long)count);
      *msg = b + state();
      return KRCN_ERR_RCCL;
    }
    bufs[me] = buf;
    here[me] = true;
    const uint64_t my = gen;
    if (++arrived == P) {
      // every other rank's buffer is final (each drained its stream before
      // arriving): sum without the lock, the others wait for gen to move
      void* b[kRvMaxRanks];
      for (int r = 0; r < P; ++r) b[r] = bufs[r];
      const int np = P;
      lk.unlock();
      const int st = sum(static_cast<void* const*>(b), np, cnt, dt);
      lk.lock();
      result = st;
      arrived = 0;
      for (int r = 0; r < P; ++r) here[r] = false;
      ++gen;
      cv.notify_all();
      if (st != KRCN_OK) *msg = "virtual all-reduce: the sum failed";
      return st;
    }
    // system_clock: wait_until on it is pthread_cond_timedwait, which TSan
    // intercepts (libstdc++'s steady-clock wait_for is pthread_cond_clockwait,
    // which GCC 11's TSan does not, and then reports every wait as a race)
    const auto until = std::chrono::system_clock::now() + std::chrono::seconds(timeout_s);
    const bool ok = cv.wait_until(lk, until, [&] { return gen != my || broken; });
    if (!ok || broken) {
      const bool timed_out = !ok && !broken;
      broken = true;
      cv.notify_all();
      char b[160];
      if (timed_out)
        snprintf(b, sizeof(b), "virtual all-reduce: rank %d timed out after %d s in its all-reduce #%llu: ", me,
                 timeout_s, (unsigned long long)*my_seq);
      else
        snprintf(b, sizeof(b), "virtual all-reduce: rank %d saw the group break in its all-reduce #%llu: ", me,
                 (unsigned long long)*my_seq);
      *msg = b + state();
      return KRCN_ERR_RCCL;
    }
    if (result != KRCN_OK) {
      *msg = "virtual all-reduce: the summing rank failed";
      return result;
    }
    return KRCN_OK;
  }
};

}  // namespace krcn
