// Stress test of the virtual communicator's rendezvous (krcn_rendezvous.hpp)
// under the host sanitizers (Makefile targets asan / tsan; run by
// tests/test_sanitizers.py).  P threads issue N all-reduces of varying
// length over host buffers with a host sum in rank order (the library's
// k_virtual_sum does the same on the device); every rank checks every result.
// Then the two failure paths: a missing rank (the others time out with the
// group's state in the message) and a rank passing a different count.
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "krcn_rendezvous.hpp"

using krcn::Rendezvous;

static int host_sum(void* const* bufs, int P, int64_t n, int) {
  for (int64_t i = 0; i < n; ++i) {
    double s = static_cast<const double*>(bufs[0])[i];
    for (int r = 1; r < P; ++r) s += static_cast<const double*>(bufs[r])[i];
    for (int r = 0; r < P; ++r) static_cast<double*>(bufs[r])[i] = s;
  }
  return KRCN_OK;
}

static int stress(int P, int N) {
  Rendezvous g;
  g.P = P;
  g.alive = P;
  g.timeout_s = 30;
  std::vector<int> bad(P, 0);
  std::vector<std::thread> th;
  for (int me = 0; me < P; ++me)
    th.emplace_back([&, me] {
      uint64_t seq = 0;
      std::vector<double> buf(257);
      for (int k = 0; k < N; ++k) {
        const int64_t n = 1 + (k * 37) % 257;
        for (int64_t i = 0; i < n; ++i) buf[size_t(i)] = double(me + 1) * double(k + i);
        std::string msg;
        if (g.arrive(me, &seq, buf.data(), n, KRCN_F64, host_sum, &msg) != KRCN_OK) {
          std::fprintf(stderr, "rank %d: %s\n", me, msg.c_str());
          bad[size_t(me)] = 1;
          return;
        }
        const double tri = double(P) * double(P + 1) / 2.0;
        for (int64_t i = 0; i < n; ++i)
          if (buf[size_t(i)] != tri * double(k + i)) {
            bad[size_t(me)] = 1;
            return;
          }
      }
    });
  for (auto& t : th) t.join();
  for (int b : bad)
    if (b) return 1;
  return 0;
}

// P - 1 ranks arrive, one never does: all of them fail, naming the absent rank
static int missing_rank(int P) {
  Rendezvous g;
  g.P = P;
  g.alive = P;
  g.timeout_s = 1;
  std::vector<std::string> msgs(P - 1);
  std::vector<int> st(P - 1, 0);
  std::vector<std::thread> th;
  for (int me = 0; me < P - 1; ++me)
    th.emplace_back([&, me] {
      uint64_t seq = 0;
      double x = 1.0;
      st[size_t(me)] = g.arrive(me, &seq, &x, 1, KRCN_F64, host_sum, &msgs[size_t(me)]);
    });
  for (auto& t : th) t.join();
  char absent[64];
  std::snprintf(absent, sizeof(absent), "rank %d: 0 entered, last count 0, absent", P - 1);
  for (int me = 0; me < P - 1; ++me)
    if (st[size_t(me)] != KRCN_ERR_RCCL || msgs[size_t(me)].find(absent) == std::string::npos) {
      std::fprintf(stderr, "missing-rank case, rank %d: status %d, message '%s'\n", me, st[size_t(me)],
                   msgs[size_t(me)].c_str());
      return 1;
    }
  return 0;
}

// ranks disagree on the count: the group breaks, every rank fails
static int mismatch(int P) {
  Rendezvous g;
  g.P = P;
  g.alive = P;
  g.timeout_s = 5;
  std::vector<int> st(P, 0);
  std::vector<std::thread> th;
  for (int me = 0; me < P; ++me)
    th.emplace_back([&, me] {
      uint64_t seq = 0;
      double x[2] = {1.0, 2.0};
      std::string msg;
      st[size_t(me)] = g.arrive(me, &seq, x, me == P / 2 ? 2 : 1, KRCN_F64, host_sum, &msg);
    });
  for (auto& t : th) t.join();
  int failed = 0;
  for (int s : st) failed += s != KRCN_OK;
  if (failed != P) {
    std::fprintf(stderr, "mismatch case: %d of %d ranks failed\n", failed, P);
    return 1;
  }
  return 0;
}

int main(int argc, char** argv) {
  const int N = argc > 1 ? std::atoi(argv[1]) : 2000;
  int rc = 0;
  for (int P : {2, 3, 8, 16}) rc |= stress(P, N);
  rc |= missing_rank(8);
  rc |= mismatch(8);
  std::printf("rendezvous stress %s\n", rc ? "FAILED" : "ok");
  return rc;
}
