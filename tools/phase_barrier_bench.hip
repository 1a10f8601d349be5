// Kernel boundary vs grid barrier on the rcv1 Lanczos step's shape (round-3
// verdict item 4: "the guide's barrier price is a claim until measured on
// this kernel").  One Lanczos step of rcv1 is three dependent phases:
//   1. pass 1  — stream X's plan (12.3 MB), write the 8 slice partials
//                (8 x n = 1.3 MB)
//   2. combine — every row's 8 partials -> u (n = 20,242)
//   3. pass 2  — every block loads ALL of u (its LDS window) and streams
//                X^T's plan (13.0 MB), writing its share of the d-vector
// The phases here move those bytes with plain streaming loads (no gathers),
// so what differs between the variants is only how the phases are joined:
//   eager: three launches per step on one stream (the product's schedule)
//   coop : one cooperative launch per step (hipLaunchCooperativeKernel: the
//          grid is co-resident), phases joined by two grid barriers (agent
//          release fence, ticket on a counter, the last arrival bumps a
//          generation word, the others poll it relaxed with s_sleep, then an
//          agent acquire fence; bounded spin with an error flag)
//   persist: one cooperative launch for all steps, three barriers per step
//   sc1  : both cooperative forms with the guide's cheaper hand-off: the
//          handed-off partials and u stored write-through (sc1) and read
//          with sc1 loads, a barrier with no fences (drain, ticket, poll)
//   xcd  : the sc1 forms with an XCD-hierarchical barrier (per-XCD tickets and
//          generations under one top counter), and that barrier alone
// Both grids are one 256-thread block per CU (256 blocks).  Per-step time is
// the median of 5 runs of 200 steps (HIP events).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/phase_barrier_bench.hip -o tools/phase_barrier_bench
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                   \
  do {                                                                                          \
    hipError_t e_ = (x);                                                                        \
    if (e_ != hipSuccess) {                                                                     \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));            \
      std::exit(1);                                                                             \
    }                                                                                           \
  } while (0)

constexpr int NT = 256;
constexpr int G = 256;           // blocks: one per CU
constexpr int N = 20242;         // rcv1 rows
constexpr int S = 8;             // slices of pass 1
constexpr int D = 47236;         // rcv1 columns
constexpr int64_t A_DBL = 12261532 / 8;   // pass-1 stream (bytes of the bench's byte model)
constexpr int64_t B_DBL = 13017308 / 8;   // pass-2 stream
constexpr int RPB = (N + G - 1) / G;      // combine rows per block
constexpr int DPB = (D + G - 1) / G;      // pass-2 outputs per block

struct Bufs {
  const double* A;
  const double* B;
  double* P;     // S x N partials
  double* U;     // N
  double* O;     // D
  unsigned* cnt;
  unsigned* gen;
  int* err;
};

__device__ __forceinline__ double block_sum(double v, double* sm) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  if ((threadIdx.x & 63) == 0) sm[threadIdx.x >> 6] = v;
  __syncthreads();
  const double r = (sm[0] + sm[1]) + (sm[2] + sm[3]);
  __syncthreads();
  return r;
}

template <bool SC1>
__device__ __forceinline__ void st(double* p, double v) {
  if constexpr (SC1) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else *p = v;
}
template <bool SC1>
__device__ __forceinline__ double ld(const double* p) {
  if constexpr (SC1) return __hip_atomic_load(const_cast<double*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else return *p;
}

// u (handed off) summed by the block with 8-byte sc1 loads, 8 in flight
__device__ __forceinline__ double stream_sum_sc1(const double* x, int64_t n) {
  double acc = 0.0;
  for (int64_t i = threadIdx.x; i < n; i += 8 * NT) {
    double a[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int64_t j = i + int64_t(u) * NT;
      a[u] = ld<true>(x + (j < n ? j : n - 1));
    }
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (i + int64_t(u) * NT < n) acc += a[u];
  }
  return acc;
}

// streaming sum of x[lo, hi) by the block, 16-byte loads, 8 in flight
__device__ __forceinline__ double stream_sum(const double* x, int64_t lo, int64_t hi) {
  double acc = 0.0;
  const double2* v = reinterpret_cast<const double2*>(x);
  for (int64_t i = lo / 2 + threadIdx.x; i < hi / 2; i += 8 * NT) {
    double2 a[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int64_t j = i + int64_t(u) * NT;
      a[u] = v[j < hi / 2 ? j : hi / 2 - 1];
    }
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (i + int64_t(u) * NT < hi / 2) acc += a[u].x + a[u].y;
  }
  return acc;
}

template <bool SC1 = false>
__device__ void phase1(const Bufs& b, int blk, double* sm) {
  const int64_t per = (A_DBL + G - 1) / G;
  const int64_t lo = (int64_t(blk) * per) & ~int64_t(1), hi = (lo + per < A_DBL ? lo + per : A_DBL) & ~int64_t(1);
  const double s = block_sum(stream_sum(b.A, lo, hi), sm);
  // this block's share of the slice partials
  const int pp = (S * N + G - 1) / G;
  for (int i = threadIdx.x; i < pp; i += NT) {
    const int q = blk * pp + i;
    if (q < S * N) st<SC1>(b.P + q, s * 1e-9 + double(q));
  }
}

template <bool SC1 = false>
__device__ void phase2(const Bufs& b, int blk) {
  for (int i = threadIdx.x; i < RPB; i += NT) {
    const int r = blk * RPB + i;
    if (r < N) {
      double t = 0.0;
#pragma unroll
      for (int s = 0; s < S; ++s) t += ld<SC1>(b.P + s * N + r);
      st<SC1>(b.U + r, t * 0.5);
    }
  }
}

template <bool SC1 = false>
__device__ void phase3(const Bufs& b, int blk, double* sm) {
  // the window: all of u, every block
  const double su = block_sum(SC1 ? stream_sum_sc1(b.U, N & ~1) : stream_sum(b.U, 0, N & ~1), sm);
  const int64_t per = (B_DBL + G - 1) / G;
  const int64_t lo = (int64_t(blk) * per) & ~int64_t(1), hi = (lo + per < B_DBL ? lo + per : B_DBL) & ~int64_t(1);
  const double s = block_sum(stream_sum(b.B, lo, hi), sm);
  for (int i = threadIdx.x; i < DPB; i += NT) {
    const int c = blk * DPB + i;
    if (c < D) b.O[c] = s + su * 1e-12 + double(c);
  }
}

__device__ void grid_barrier(const Bufs& b) {
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned g = __hip_atomic_load(b.gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned old = __hip_atomic_fetch_add(b.cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (old == gridDim.x - 1) {
      __hip_atomic_store(b.cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(b.gen, g + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      int spins = 0;
      while (__hip_atomic_load(b.gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == g) {
        __builtin_amdgcn_s_sleep(1);
        if (++spins > (1 << 22)) {   // bounded: every wave leaves
          __hip_atomic_store(b.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  }
  __syncthreads();
}

// the sc1 hand-off's barrier: every wave drains its write-through stores, one
// ticket per block, no fences (the consumers read the handed-off data sc1)
__device__ void grid_barrier_sc1(const Bufs& b) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned g = __hip_atomic_load(b.gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned old = __hip_atomic_fetch_add(b.cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (old == gridDim.x - 1) {
      __hip_atomic_store(b.cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(b.gen, g + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      int spins = 0;
      while (__hip_atomic_load(b.gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == g) {
        __builtin_amdgcn_s_sleep(1);
        if (++spins > (1 << 22)) {
          __hip_atomic_store(b.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
      }
    }
  }
  __syncthreads();
}

// XCD-hierarchical form of the same (the guide's barrier-xcd shape): a
// ticket on the block's XCD counter (blockIdx % 8: the dispatch's XCD
// round-robin), the XCD's last arrival takes a ticket on the top counter, the
// last of the 8 bumps the top generation; XCD leaders poll that and bump
// their XCD's generation, every other block polls its XCD's generation.
// Words sit 128 B apart: cnt[0] top (also the flat barriers' counter), cnt[32] top gen, cnt[64 + 32 x] XCD x
// counter, cnt[64 + 32 x + 16] XCD x gen.
__device__ __forceinline__ void poll_until_changed(unsigned* w, unsigned g, int* err) {
  int spins = 0;
  while (__hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == g) {
    __builtin_amdgcn_s_sleep(1);
    if (++spins > (1 << 22)) {
      __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      break;
    }
  }
}
__device__ void grid_barrier_xcd(const Bufs& b) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const int x = blockIdx.x % 8;
    const unsigned per = gridDim.x / 8;
    unsigned* xc = b.cnt + 64 + 32 * x;
    unsigned* xg = xc + 16;
    unsigned* top = b.cnt;
    unsigned* tg = b.cnt + 32;
    const unsigned g = __hip_atomic_load(xg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned old = __hip_atomic_fetch_add(xc, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (old == per - 1) {   // XCD leader
      __hip_atomic_store(xc, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned gt = __hip_atomic_load(tg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const unsigned ot = __hip_atomic_fetch_add(top, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (ot == 7) {
        __hip_atomic_store(top, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_store(tg, gt + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      } else {
        poll_until_changed(tg, gt, b.err);
      }
      __hip_atomic_store(xg, g + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      poll_until_changed(xg, g, b.err);
    }
  }
  __syncthreads();
}

__global__ __launch_bounds__(NT) void k_p1(Bufs b) {
  __shared__ double sm[4];
  phase1(b, blockIdx.x, sm);
}
__global__ __launch_bounds__(NT) void k_p2(Bufs b) { phase2(b, blockIdx.x); }
__global__ __launch_bounds__(NT) void k_p3(Bufs b) {
  __shared__ double sm[4];
  phase3(b, blockIdx.x, sm);
}
__global__ __launch_bounds__(NT) void k_coop(Bufs b, int steps) {
  __shared__ double sm[4];
  for (int it = 0; it < steps; ++it) {
    if (it > 0) grid_barrier(b);
    phase1(b, blockIdx.x, sm);
    grid_barrier(b);
    phase2(b, blockIdx.x);
    grid_barrier(b);
    phase3(b, blockIdx.x, sm);
  }
}

__global__ __launch_bounds__(NT) void k_coop_sc1(Bufs b, int steps) {
  __shared__ double sm[4];
  for (int it = 0; it < steps; ++it) {
    if (it > 0) grid_barrier_sc1(b);
    phase1<true>(b, blockIdx.x, sm);
    grid_barrier_sc1(b);
    phase2<true>(b, blockIdx.x);
    grid_barrier_sc1(b);
    phase3<true>(b, blockIdx.x, sm);
  }
}

__global__ __launch_bounds__(NT) void k_coop_xcd(Bufs b, int steps) {
  __shared__ double sm[4];
  for (int it = 0; it < steps; ++it) {
    if (it > 0) grid_barrier_xcd(b);
    phase1<true>(b, blockIdx.x, sm);
    grid_barrier_xcd(b);
    phase2<true>(b, blockIdx.x);
    grid_barrier_xcd(b);
    phase3<true>(b, blockIdx.x, sm);
  }
}
// the barrier alone, n times (nothing published)
__global__ __launch_bounds__(NT) void k_bar_xcd(Bufs b, int n) {
  for (int i = 0; i < n; ++i) grid_barrier_xcd(b);
}

template <class F>
static float median_us_per_step(F&& f, int steps) {
  hipEvent_t a, e;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&e));
  std::vector<float> t;
  for (int r = 0; r < 6; ++r) {
    CK(hipEventRecord(a, 0));
    f();
    CK(hipEventRecord(e, 0));
    CK(hipEventSynchronize(e));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, a, e));
    if (r > 0) t.push_back(ms * 1e3f / steps);
  }
  std::sort(t.begin(), t.end());
  return t[t.size() / 2];
}

int main() {
  int dev = 0, cus = 0, coop = 0, occ = 0;
  CK(hipGetDevice(&dev));
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  CK(hipDeviceGetAttribute(&coop, hipDeviceAttributeCooperativeLaunch, dev));
  CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_coop, NT, 0));
  std::printf("CUs %d, cooperative launch %d, k_coop blocks/CU %d\n", cus, coop, occ);
  if (!coop || occ * cus < G) {
    std::printf("grid of %d blocks cannot be co-resident: no cooperative run\n", G);
    return 1;
  }
  Bufs b{};
  double *A, *B, *P, *U, *O;
  CK(hipMalloc(&A, sizeof(double) * A_DBL));
  CK(hipMalloc(&B, sizeof(double) * B_DBL));
  CK(hipMalloc(&P, sizeof(double) * S * N));
  CK(hipMalloc(&U, sizeof(double) * N));
  CK(hipMalloc(&O, sizeof(double) * D));
  CK(hipMalloc(&b.cnt, sizeof(unsigned) * 512));
  CK(hipMalloc(&b.err, sizeof(int)));
  CK(hipMemset(A, 0, sizeof(double) * A_DBL));
  CK(hipMemset(B, 0, sizeof(double) * B_DBL));
  CK(hipMemset(b.cnt, 0, sizeof(unsigned) * 512));
  CK(hipMemset(b.err, 0, sizeof(int)));
  b.A = A; b.B = B; b.P = P; b.U = U; b.O = O; b.gen = b.cnt + 448;   // past the XCD words (cnt[64 .. 320))
  const int steps = 200;
  std::vector<double> o1(D), o2(D);
  const float te = median_us_per_step([&] {
    for (int i = 0; i < steps; ++i) {
      hipLaunchKernelGGL(k_p1, dim3(G), dim3(NT), 0, 0, b);
      hipLaunchKernelGGL(k_p2, dim3(G), dim3(NT), 0, 0, b);
      hipLaunchKernelGGL(k_p3, dim3(G), dim3(NT), 0, 0, b);
    }
  }, steps);
  CK(hipMemcpy(o1.data(), O, sizeof(double) * D, hipMemcpyDeviceToHost));
  int one = 1;
  void* args1[] = {&b, &one};
  const float tc = median_us_per_step([&] {
    for (int i = 0; i < steps; ++i)
      CK(hipLaunchCooperativeKernel(reinterpret_cast<const void*>(k_coop), dim3(G), dim3(NT), args1, 0, 0));
  }, steps);
  int st = steps;
  void* argsN[] = {&b, &st};
  const float tp = median_us_per_step([&] {
    CK(hipLaunchCooperativeKernel(reinterpret_cast<const void*>(k_coop), dim3(G), dim3(NT), argsN, 0, 0));
  }, steps);
  CK(hipMemcpy(o2.data(), O, sizeof(double) * D, hipMemcpyDeviceToHost));
  std::vector<double> o3(D);
  const float ts = median_us_per_step([&] {
    for (int i = 0; i < steps; ++i)
      CK(hipLaunchCooperativeKernel(reinterpret_cast<const void*>(k_coop_sc1), dim3(G), dim3(NT), args1, 0, 0));
  }, steps);
  const float tsp = median_us_per_step([&] {
    CK(hipLaunchCooperativeKernel(reinterpret_cast<const void*>(k_coop_sc1), dim3(G), dim3(NT), argsN, 0, 0));
  }, steps);
  CK(hipMemcpy(o3.data(), O, sizeof(double) * D, hipMemcpyDeviceToHost));
  std::vector<double> o4(D);
  const float tx = median_us_per_step([&] {
    for (int i = 0; i < steps; ++i)
      CK(hipLaunchCooperativeKernel(reinterpret_cast<const void*>(k_coop_xcd), dim3(G), dim3(NT), args1, 0, 0));
  }, steps);
  const float txp = median_us_per_step([&] {
    CK(hipLaunchCooperativeKernel(reinterpret_cast<const void*>(k_coop_xcd), dim3(G), dim3(NT), argsN, 0, 0));
  }, steps);
  CK(hipMemcpy(o4.data(), O, sizeof(double) * D, hipMemcpyDeviceToHost));
  const float tb = median_us_per_step([&] {
    CK(hipLaunchCooperativeKernel(reinterpret_cast<const void*>(k_bar_xcd), dim3(G), dim3(NT), argsN, 0, 0));
  }, steps);
  int err = 0;
  CK(hipMemcpy(&err, b.err, sizeof(int), hipMemcpyDeviceToHost));
  const bool same = o1 == o2 && o1 == o3 && o1 == o4;
  // each phase alone (launch cost included), for the boundary's share
  const float t1 = median_us_per_step([&] {
    for (int i = 0; i < steps; ++i) hipLaunchKernelGGL(k_p1, dim3(G), dim3(NT), 0, 0, b);
  }, steps);
  const float t2 = median_us_per_step([&] {
    for (int i = 0; i < steps; ++i) hipLaunchKernelGGL(k_p2, dim3(G), dim3(NT), 0, 0, b);
  }, steps);
  const float t3 = median_us_per_step([&] {
    for (int i = 0; i < steps; ++i) hipLaunchKernelGGL(k_p3, dim3(G), dim3(NT), 0, 0, b);
  }, steps);
  std::printf("per step (us): eager 3 launches %.2f | coop 1 launch + 2 barriers %.2f | persistent 3 barriers %.2f\n",
              te, tc, tp);
  std::printf("sc1 hand-off (write-through stores, sc1 loads, fence-free barrier): coop %.2f | persistent %.2f\n", ts, tsp);
  std::printf("XCD-hierarchical barrier, sc1 hand-off: coop %.2f | persistent %.2f | the barrier alone %.2f us\n", tx,
              txp, tb);
  std::printf("phases alone (us per launch, back to back): pass-1 stand-in %.2f, combine %.2f, pass-2 stand-in %.2f\n",
              t1, t2, t3);
  std::printf("outputs equal: %s, barrier timeouts: %d\n", same ? "yes" : "NO", err);
  return (same && !err) ? 0 : 2;
}
