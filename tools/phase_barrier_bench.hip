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

__device__ void phase1(const Bufs& b, int blk, double* sm) {
  const int64_t per = (A_DBL + G - 1) / G;
  const int64_t lo = (int64_t(blk) * per) & ~int64_t(1), hi = (lo + per < A_DBL ? lo + per : A_DBL) & ~int64_t(1);
  const double s = block_sum(stream_sum(b.A, lo, hi), sm);
  // this block's share of the slice partials
  const int pp = (S * N + G - 1) / G;
  for (int i = threadIdx.x; i < pp; i += NT) {
    const int q = blk * pp + i;
    if (q < S * N) b.P[q] = s * 1e-9 + double(q);
  }
}

__device__ void phase2(const Bufs& b, int blk) {
  for (int i = threadIdx.x; i < RPB; i += NT) {
    const int r = blk * RPB + i;
    if (r < N) {
      double t = 0.0;
#pragma unroll
      for (int s = 0; s < S; ++s) t += b.P[s * N + r];
      b.U[r] = t * 0.5;
    }
  }
}

__device__ void phase3(const Bufs& b, int blk, double* sm) {
  const double su = block_sum(stream_sum(b.U, 0, N & ~1), sm);   // the window: all of u, every block
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
  CK(hipMalloc(&b.cnt, sizeof(unsigned) * 2));
  CK(hipMalloc(&b.err, sizeof(int)));
  CK(hipMemset(A, 0, sizeof(double) * A_DBL));
  CK(hipMemset(B, 0, sizeof(double) * B_DBL));
  CK(hipMemset(b.cnt, 0, sizeof(unsigned) * 2));
  CK(hipMemset(b.err, 0, sizeof(int)));
  b.A = A; b.B = B; b.P = P; b.U = U; b.O = O; b.gen = b.cnt + 1;
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
  int err = 0;
  CK(hipMemcpy(&err, b.err, sizeof(int), hipMemcpyDeviceToHost));
  const bool same = o1 == o2;
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
  std::printf("phases alone (us per launch, back to back): pass-1 stand-in %.2f, combine %.2f, pass-2 stand-in %.2f\n",
              t1, t2, t3);
  std::printf("outputs equal: %s, barrier timeouts: %d\n", same ? "yes" : "NO", err);
  return (same && !err) ? 0 : 2;
}
