// Wave dispatch ramp on MI355X: how long after the first wave of a launch do
// the last waves start, by block size and LDS footprint?  Each wave stamps
// s_memrealtime (100 MHz) at entry; the kernel then spins ~20 us so that no
// CU frees up during the measurement.
// build: hipcc --offload-arch=gfx950 -O3 tools/dispatch_microbench.hip -o tools/dispatch_microbench
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

template <int NT, int LDS>
__global__ __launch_bounds__(NT) void k_stamp(unsigned long long* out, int spin) {
  __shared__ double pad[LDS / 8 > 0 ? LDS / 8 : 1];
  const unsigned long long t = __builtin_amdgcn_s_memrealtime();
  if ((threadIdx.x & 63) == 0) out[blockIdx.x * (NT / 64) + (threadIdx.x >> 6)] = t;
  pad[threadIdx.x % (LDS / 8 > 0 ? LDS / 8 : 1)] = double(t);
  unsigned long long e = t;
  while (e - t < (unsigned long long)spin) e = __builtin_amdgcn_s_memrealtime();
  if (pad[(threadIdx.x + 1) % (LDS / 8 > 0 ? LDS / 8 : 1)] == -1.0) out[0] = 0;
}

template <int NT, int LDS>
void run(int blocks, const char* name) {
  const int waves = blocks * (NT / 64);
  unsigned long long* d;
  hipMalloc(&d, sizeof(unsigned long long) * waves);
  std::vector<unsigned long long> h(waves);
  double sp[5];
  for (int it = 0; it < 5; ++it) {
    hipLaunchKernelGGL((k_stamp<NT, LDS>), dim3(blocks), dim3(NT), 0, 0, d, 2000);
    hipDeviceSynchronize();
    hipMemcpy(h.data(), d, sizeof(unsigned long long) * waves, hipMemcpyDeviceToHost);
    const auto mn = *std::min_element(h.begin(), h.end()), mx = *std::max_element(h.begin(), h.end());
    sp[it] = (mx - mn) / 100.0;
  }
  // per-block spread of the last run
  double bmax = 0;
  for (int b = 0; b < blocks; ++b) {
    const auto* p = h.data() + size_t(b) * (NT / 64);
    const auto mn = *std::min_element(p, p + NT / 64), mx = *std::max_element(p, p + NT / 64);
    bmax = std::max(bmax, (mx - mn) / 100.0);
  }
  // per-XCD (blocks b % 8 share one): first entry offset and spread
  double xoff[8], xsp[8];
  unsigned long long gmin = *std::min_element(h.begin(), h.end());
  for (int x = 0; x < 8; ++x) {
    unsigned long long mn = ~0ull, mx = 0;
    for (int b = x; b < blocks; b += 8)
      for (int w = 0; w < NT / 64; ++w) {
        mn = std::min(mn, h[size_t(b) * (NT / 64) + w]);
        mx = std::max(mx, h[size_t(b) * (NT / 64) + w]);
      }
    xoff[x] = (mn - gmin) / 100.0;
    xsp[x] = (mx - mn) / 100.0;
  }
  std::sort(sp, sp + 5);
  printf("%-34s blocks %5d waves %6d  first->last wave entry: median %6.2f us (min %6.2f)  max in-block spread %5.2f us\n",
         name, blocks, waves, sp[2], sp[0], bmax);
  printf("    per-XCD first-entry offset:");
  for (int x = 0; x < 8; ++x) printf(" %5.2f", xoff[x]);
  printf("   per-XCD spread:");
  for (int x = 0; x < 8; ++x) printf(" %5.2f", xsp[x]);
  printf("\n");
  hipFree(d);
}

int main() {
  run<1024, 159744>(256, "1024 thr, 156 KB LDS (1/CU)");
  run<1024, 0>(256, "1024 thr, no LDS");
  run<1024, 73728>(512, "1024 thr, 72 KB LDS (2/CU)");
  run<512, 0>(512, "512 thr, no LDS");
  run<256, 0>(1024, "256 thr, no LDS");
  run<256, 0>(2048, "256 thr, no LDS, 2048");
  run<64, 0>(4096, "64 thr, no LDS");
  run<256, 36864>(1024, "256 thr, 36 KB LDS (4/CU)");
  return 0;
}
