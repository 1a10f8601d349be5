// FETCH_SIZE calibration for the access widths the sorted passes use (MI355X_MICROARCH.md:
// "other access widths are uncalibrated: calibrate on a known byte count").
// Each kernel reads a 512 MiB buffer (twice the Infinity Cache) exactly once, coalesced,
// with 4-, 8- or 16-byte loads per lane; run under `rocprofv3 --pmc FETCH_SIZE` and divide.
// Build: hipcc --offload-arch=gfx950 -O3 tools/fetch_calib.hip -o fetch_calib
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
typedef int i4 __attribute__((ext_vector_type(4)));

template <typename V>
__global__ __launch_bounds__(256) void k_read(const V* __restrict__ a, long n, int* __restrict__ out) {
  int acc = 0;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += gridDim.x * 256L) {
    const V v = a[i];
    acc ^= reinterpret_cast<const int*>(&v)[0];
  }
  if (acc == 0x7fffffff) out[0] = acc;
}

int main() {
  const long bytes = 512L << 20;
  void* a;
  int* out;
  CK(hipMalloc(&a, bytes));
  CK(hipMalloc(&out, 64));
  CK(hipMemset(a, 1, bytes));
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL(k_read<int>, dim3(4096), dim3(256), 0, 0, (const int*)a, bytes / 4, out);
    hipLaunchKernelGGL(k_read<long>, dim3(4096), dim3(256), 0, 0, (const long*)a, bytes / 8, out);
    hipLaunchKernelGGL(k_read<i4>, dim3(4096), dim3(256), 0, 0, (const i4*)a, bytes / 16, out);
  }
  CK(hipDeviceSynchronize());
  printf("each launch reads %ld bytes (dword / dwordx2 / dwordx4 loads)\n", bytes);
  return 0;
}
