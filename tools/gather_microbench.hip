// Microbenchmark: streaming vs random-gather throughput on gfx950 (evidence for DESIGN.md §5).
// Build: hipcc --offload-arch=gfx950 -O3 tools/gather_microbench.hip -o gather_microbench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <random>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
typedef int i4 __attribute__((ext_vector_type(4)));
typedef double d2 __attribute__((ext_vector_type(2)));

// mode 0: stream idx+val only; 1: gather x[idx] only (idx streamed); 2: both (spmv core)
template <int MODE>
__global__ __launch_bounds__(256) void k(long nnz, const int* __restrict__ idx, const double* __restrict__ val,
                                         const double* __restrict__ x, double* __restrict__ out) {
  double acc = 0;
  long nq = nnz / 4;
  for (long q = blockIdx.x * 256L + threadIdx.x; q < nq; q += gridDim.x * 256L) {
    i4 c = *(const i4*)(idx + 4 * q);
    if (MODE == 0) {
      d2 a = *(const d2*)(val + 4 * q), b = *(const d2*)(val + 4 * q + 2);
      acc += a.x + a.y + b.x + b.y + c.x + c.y + c.z + c.w;
    } else if (MODE == 1) {
      acc += x[c.x] + x[c.y] + x[c.z] + x[c.w];
    } else {
      d2 a = *(const d2*)(val + 4 * q), b = *(const d2*)(val + 4 * q + 2);
      acc += a.x * x[c.x] + a.y * x[c.y] + b.x * x[c.z] + b.y * x[c.w];
    }
  }
  out[blockIdx.x * 256 + threadIdx.x] = acc;
}

// gather from an LDS copy of x (W <= 8192 doubles)
__global__ __launch_bounds__(256) void k_lds(long nnz, const int* __restrict__ idx, const double* __restrict__ val,
                                             const double* __restrict__ x, int W, double* __restrict__ out) {
  __shared__ double xs[8192];
  for (int i = threadIdx.x; i < W; i += 256) xs[i] = x[i];
  __syncthreads();
  double acc = 0;
  long nq = nnz / 4;
  for (long q = blockIdx.x * 256L + threadIdx.x; q < nq; q += gridDim.x * 256L) {
    i4 c = *(const i4*)(idx + 4 * q);
    d2 a = *(const d2*)(val + 4 * q), b = *(const d2*)(val + 4 * q + 2);
    acc += a.x * xs[c.x] + a.y * xs[c.y] + b.x * xs[c.z] + b.y * xs[c.w];
  }
  out[blockIdx.x * 256 + threadIdx.x] = acc;
}

int main() {
  const long nnz = 9097916 / 4 * 4;
  int *idx; double *val, *x, *out;
  CK(hipMalloc(&idx, nnz * 4)); CK(hipMalloc(&val, nnz * 8)); CK(hipMalloc(&x, 2000000 * 8));
  CK(hipMalloc(&out, 4096 * 256 * 8));
  std::vector<double> hv(nnz, 0.5); CK(hipMemcpy(val, hv.data(), nnz * 8, hipMemcpyHostToDevice));
  std::vector<double> hx(2000000, 1.0); CK(hipMemcpy(x, hx.data(), 2000000 * 8, hipMemcpyHostToDevice));
  std::mt19937 rng(1);
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  int Ws[] = {8192, 20000, 169000, 1355191};
  int grids[] = {1024, 2048, 4096};
  for (int W : Ws) {
    std::vector<int> hi(nnz);
    for (long i = 0; i < nnz; ++i) hi[i] = rng() % W;
    CK(hipMemcpy(idx, hi.data(), nnz * 4, hipMemcpyHostToDevice));
    for (int grid : grids) {
      for (int mode = 0; mode < 4; ++mode) {
        if (mode == 3 && W > 8192) continue;
        auto launch = [&]() {
          if (mode == 0) hipLaunchKernelGGL(k<0>, dim3(grid), dim3(256), 0, 0, nnz, idx, val, x, out);
          if (mode == 1) hipLaunchKernelGGL(k<1>, dim3(grid), dim3(256), 0, 0, nnz, idx, val, x, out);
          if (mode == 2) hipLaunchKernelGGL(k<2>, dim3(grid), dim3(256), 0, 0, nnz, idx, val, x, out);
          if (mode == 3) hipLaunchKernelGGL(k_lds, dim3(grid), dim3(256), 0, 0, nnz, idx, val, x, W, out);
        };
        for (int i = 0; i < 3; ++i) launch();
        CK(hipEventRecord(e0));
        const int R = 20;
        for (int i = 0; i < R; ++i) launch();
        CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        double us = ms * 1e3 / R;
        double bytes = mode == 1 ? nnz * 4.0 : nnz * 12.0;
        printf("W=%8d grid=%5d mode=%d  %8.1f us  stream %7.0f GB/s  gathers %6.1f G/s\n", W, grid, mode, us,
               bytes / us / 1e3, mode == 0 ? 0.0 : nnz / us / 1e3);
      }
    }
  }
  return 0;
}
