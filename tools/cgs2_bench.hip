// Microbenchmark of the CGS2 reorthogonalisation kernels (krcn_cgs2.hpp) at
// fixed basis sizes: per-kernel time (HIP events, median of 20) and the
// effective bandwidth over the V bytes each sweep streams.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I include \
//         -I krylov-cubic-regularized-newton_amd/csrc tools/cgs2_bench.hip -o tools/cgs2_bench
//   tools/cgs2_bench [d] [k ...]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "krcn_cgs2.hpp"

using namespace krcn;

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e = (x);                                                        \
    if (e != hipSuccess) {                                                     \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      std::exit(1);                                                            \
    }                                                                          \
  } while (0)

template <class F>
static float time_us(F&& f, int reps = 20) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  std::vector<float> t;
  for (int i = 0; i < reps + 3; ++i) {
    CK(hipEventRecord(a, 0));
    f();
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    if (i >= 3) t.push_back(ms * 1e3f);
  }
  std::sort(t.begin(), t.end());
  return t[t.size() / 2];
}

int main(int argc, char** argv) {
  using T = float;
  const int64_t d = argc > 1 ? std::atoll(argv[1]) : 47236;
  std::vector<int> ks;
  for (int i = 2; i < argc; ++i) ks.push_back(std::atoi(argv[i]));
  if (ks.empty()) ks = {64, 250, 500};
  const int kmax = *std::max_element(ks.begin(), ks.end());
  T *V, *z;
  double *h, *part, *pn;
  LanczosState* st;
  CK(hipMalloc(&V, sizeof(T) * d * kmax));
  CK(hipMalloc(&z, sizeof(T) * d));
  CK(hipMalloc(&h, sizeof(double) * (kmax + kCgsHPad)));
  CK(hipMalloc(&part, sizeof(double) * ((d + kCgsUpdCols - 1) / kCgsUpdCols) * kmax));
  CK(hipMalloc(&pn, sizeof(double) * 1024));
  CK(hipMalloc(&st, sizeof(LanczosState)));
  CK(hipMemset(st, 0, sizeof(LanczosState)));
  CK(hipMemset(V, 0, sizeof(T) * d * kmax));
  CK(hipMemset(z, 0, sizeof(T) * d));
  CK(hipMemset(h, 0, sizeof(double) * (kmax + kCgsHPad)));
  for (int k : ks) {
    const double vbytes = double(k) * double(d) * sizeof(T);
    const int n1 = int((d + cgs_dot_cols<T>() - 1) / cgs_dot_cols<T>());
    const int n3 = int((d + kCgsUpdCols - 1) / kCgsUpdCols);
    const int cached = int64_t(k) * kCgsSlabLd * int64_t(sizeof(T)) <= kCgsCacheBytes;
    const float t1 = time_us([&] {
      hipLaunchKernelGGL((k_cgs_dots<T>), dim3(n1, (k + kCgsDotRows - 1) / kCgsDotRows), dim3(kNT), 0, 0, d, k,
                         V, z, part, st);
    });
    const float tc = time_us([&] {
      hipLaunchKernelGGL(k_cgs_coeffs, dim3((k + kCgsHPad + kCgsCoefRows - 1) / kCgsCoefRows), dim3(kCgsCoefNT), 0, 0, part, n3, k, h, st);
    });
    const float t3 = time_us([&] {
      hipLaunchKernelGGL((k_cgs_update_dots<T>), dim3(n3), dim3(kCgsUpdNT), 0, 0, d, k, V, h, z, part, cached, st);
    });
    const float t5 = time_us([&] {
      hipLaunchKernelGGL((k_cgs_update_norm<T>), dim3(std::min(n3, 1024)), dim3(kCgsUpdNT), 0, 0, d, k, V, h, z,
                         pn, st);
    });
    const float all = time_us([&] {
      hipLaunchKernelGGL((k_cgs_dots<T>), dim3(n1, (k + kCgsDotRows - 1) / kCgsDotRows), dim3(kNT), 0, 0, d, k,
                         V, z, part, st);
      hipLaunchKernelGGL(k_cgs_coeffs, dim3((k + kCgsHPad + kCgsCoefRows - 1) / kCgsCoefRows), dim3(kCgsCoefNT), 0, 0, part, n1, k, h, st);
      hipLaunchKernelGGL((k_cgs_update_dots<T>), dim3(n3), dim3(kCgsUpdNT), 0, 0, d, k, V, h, z, part, cached, st);
      hipLaunchKernelGGL(k_cgs_coeffs, dim3((k + kCgsHPad + kCgsCoefRows - 1) / kCgsCoefRows), dim3(kCgsCoefNT), 0, 0, part, n3, k, h, st);
      hipLaunchKernelGGL((k_cgs_update_norm<T>), dim3(std::min(n3, 1024)), dim3(kCgsUpdNT), 0, 0, d, k, V, h, z,
                         pn, st);
    });
    std::printf("d %lld k %4d | dots %7.2f us (%5.0f GB/s) | coeffs %6.2f | update_dots %7.2f us (%5.0f GB/s) | "
                "update_norm %7.2f us (%5.0f GB/s) | step %7.2f us\n",
                (long long)d, k, t1, vbytes / t1 / 1e3, tc, t3, vbytes / t3 / 1e3, t5, vbytes / t5 / 1e3, all);
  }
  return 0;
}
