// krcn_cgs2.hpp — full reorthogonalisation of the Lanczos basis, CGS2
// (build-only extension: the reference has none, cubic.py:92-103).
//
// After step B, z = z_{j+1} is orthogonalised against V_{0..j} (k = j + 1 rows
// of the row-major basis, length d each) twice:
//   h1 = V z;  z1 = z - V^T h1;  h2 = V z1;  z2 = z1 - V^T h2
// V is tall-skinny and streamed (rcv1_stress: up to 500 x 47,236 fp32 = 94 MB
// per sweep), so the cost is the number of sweeps over V and how many bytes
// each CU keeps in flight.  The second pass's dot sweep is fused into the
// first pass's update sweep: a block caches its 32-column slab of V in LDS
// while it applies h1, then forms the partial dots of z1 from LDS — three
// sweeps over V per step instead of four, five launches, no d-length partial
// buffer:
//   k_cgs_dots        h1 partials per (column slab, row)        V read 1
//   k_cgs_coeffs      h1 = sum over slabs (fixed order)
//   k_cgs_update_dots z1 = z - V^T h1 in place, h2 partials     V read 2
//   k_cgs_coeffs      h2
//   k_cgs_update_norm z2 = z1 - V^T h2 in place, ||z2||^2 partials (the next
//                     step's beta)                              V read 3
// Every load instruction reads whole 128-B lines of rows (lanes on consecutive
// columns), from clamped addresses without branches, 16-32 loads in flight
// per lane.
// Sums are fixed-order: dots are products in double added per lane, then an
// xor butterfly over the wave; slab partials are added in slab order; each
// column's update adds 16 row-group sums in a fixed tree.  Deterministic.
#pragma once
#include "krcn_kernels.hpp"

namespace krcn {

constexpr int kCgsDotRows = 32;      // k_cgs_dots: rows per block (8 per wave)
constexpr int kCgsUpdCols = 32;      // update kernels: columns per block (a 128-B line of fp32 per row)
constexpr int kCgsUpdNT = 512;       //   threads: 32 columns x 16 row groups
constexpr int kCgsRowGroups = kCgsUpdNT / kCgsUpdCols;
constexpr int kCgsSlabLd = kCgsUpdCols + 4;   // padded LDS slab row (16-B aligned, spreads banks)
constexpr int kCgsCacheBytes = 73728;    // LDS slab cache of k_cgs_update_dots (2 blocks per CU)
constexpr int kCgsUnroll = 16;       // row loads in flight per thread in the update sweeps
constexpr int kCgsHPad = kCgsRowGroups * kCgsUnroll;   // zeros after h's k entries

// columns per k_cgs_dots block: 16 bytes per lane, lanes contiguous per load
template <typename T> constexpr int cgs_dot_cols() { return 64 * (16 / int(sizeof(T))); }

// h partials: part[b * k + r] = sum over slab b's columns of V[r, c] z[c].
// Grid: (column slabs, row blocks of kCgsDotRows); each wave holds its rows'
// loads (8 rows x 16 B per lane) in flight before reducing.
template <typename T>
__global__ __launch_bounds__(kNT) void k_cgs_dots(int64_t d, int k, const T* __restrict__ V,
                                                  const T* __restrict__ z, double* __restrict__ part,
                                                  const LanczosState* st) {
  if (st->done) return;
  constexpr int VW = 16 / int(sizeof(T));
  constexpr int RW = kCgsDotRows / (kNT / 64);   // rows per wave
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t c0 = int64_t(blockIdx.x) * cgs_dot_cols<T>() + lane;
  double zc[VW];
#pragma unroll
  for (int i = 0; i < VW; ++i) {
    const int64_t c = c0 + 64 * i;
    zc[i] = c < d ? double(z[c]) : 0.0;
  }
  const int rbase = blockIdx.y * kCgsDotRows + wave * RW;
  T v[RW][VW];
#pragma unroll
  for (int u = 0; u < RW; ++u) {
    const int r = rbase + u < k ? rbase + u : k - 1;
    const T* vr = V + int64_t(r) * d;
#pragma unroll
    for (int i = 0; i < VW; ++i) {   // clamped address, unconditional load (see cgs_col_sum)
      const int64_t c = c0 + 64 * i;
      const T x = vr[c < d ? c : d - 1];
      v[u][i] = c < d ? x : T(0);
    }
  }
#pragma unroll
  for (int u = 0; u < RW; ++u) {
    double acc = 0.0;
#pragma unroll
    for (int i = 0; i < VW; ++i) acc += double(v[u][i]) * zc[i];
    const double s = wave_sum(acc);
    if (lane == 0 && rbase + u < k) part[int64_t(blockIdx.x) * k + rbase + u] = s;
  }
}

// h[r] = sum over slabs b of part[b * k + r], for 16 rows per block: thread
// (row lane & 15, slab group sg = 4 wave + (lane >> 4)) adds slabs
// b = sg, sg + 64, ... in order (16 loads in flight, branch-free), and the 64
// group sums of a row are combined in a fixed tree; h[k .. k + kCgsHPad) = 0.
// Grid: ceil((k + kCgsHPad) / 16) blocks of 1024 threads.
constexpr int kCgsCoefRows = 16;
constexpr int kCgsCoefNT = 1024;
[[maybe_unused]] static __global__ __launch_bounds__(kCgsCoefNT) void k_cgs_coeffs(
    const double* __restrict__ part, int nslabs, int k, double* __restrict__ h, const LanczosState* st) {
  if (st->done) return;
  constexpr int SG = kCgsCoefNT / kCgsCoefRows;   // 64 slab groups
  __shared__ double sm[SG][kCgsCoefRows];
  const int ri = threadIdx.x % kCgsCoefRows, sg = threadIdx.x / kCgsCoefRows;
  const int r = blockIdx.x * kCgsCoefRows + ri;
  const int rc = r < k ? r : k - 1;
  constexpr int U = 16;
  double s = 0.0;
  for (int b0 = 0; b0 < nslabs; b0 += SG * U) {
    double a[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int b = b0 + sg + u * SG;
      a[u] = part[int64_t(b < nslabs ? b : nslabs - 1) * k + rc];
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (b0 + sg + u * SG < nslabs) s += a[u];
  }
  sm[sg][ri] = s;
  __syncthreads();
  if (sg == 0) {
    double t[SG];
#pragma unroll
    for (int i = 0; i < SG; ++i) t[i] = sm[i][ri];
#pragma unroll
    for (int w = SG / 2; w > 0; w >>= 1)
#pragma unroll
      for (int i = 0; i < w; ++i) t[i] = t[2 * i] + t[2 * i + 1];
    if (r < k) h[r] = t[0];
    else if (r < k + kCgsHPad) h[r] = 0.0;   // the update sweeps read h past k unconditionally
  }
}

// One column's share of V^T h over the thread's row group (rows g, g + 16, ...),
// kCgsUnroll row loads in flight; optionally keeps the loaded values in the
// LDS slab (row-major, 32 columns).
template <typename T, bool kCache>
__device__ __forceinline__ double cgs_col_sum(const T* __restrict__ V, int64_t d, int k, int64_t c, bool in, int g,
                                              const double* __restrict__ h, T* slab, int l) {
  constexpr int G = kCgsRowGroups, U = kCgsUnroll;
  // No branch in the body: loads from clamped addresses.  A load under a
  // condition is waited for before the branch joins (s_waitcnt vmcnt(0) each),
  // which serialises the U loads this loop keeps in flight.  The trip count
  // is uniform over the block.
  // h carries zeros in [k, k + G U) (k_cgs_coeffs), so rows past k weigh 0;
  // a column past d reads column d - 1 and is never stored.
  (void)in;
  const int64_t cc = c < d ? c : d - 1;
  double acc = 0.0;
  for (int r0 = 0; r0 < k; r0 += G * U) {
    T v[U];
    double hv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int r = r0 + g + u * G;
      v[u] = V[int64_t(r < k ? r : k - 1) * d + cc];
      hv[u] = h[r];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if constexpr (kCache) {   // rows past k rewrite row k - 1 with its own value
        const int r = r0 + g + u * G;
        slab[(r < k ? r : k - 1) * kCgsSlabLd + l] = v[u];
      }
      acc += hv[u] * double(v[u]);
    }
  }
  return acc;
}

// Combine the 16 row-group sums of the block's columns (fixed tree) and
// return z[c] - sum for the thread's column (row group 0 only).
__device__ __forceinline__ double cgs_combine(double acc, double (*red)[kCgsUpdCols], int g, int l) {
  constexpr int G = kCgsRowGroups;
  red[g][l] = acc;
  __syncthreads();
  double t[G];
  if (g == 0) {
#pragma unroll
    for (int i = 0; i < G; ++i) t[i] = red[i][l];
#pragma unroll
    for (int w = G / 2; w > 0; w >>= 1)
#pragma unroll
      for (int i = 0; i < w; ++i) t[i] = t[2 * i] + t[2 * i + 1];
  }
  return g == 0 ? t[0] : 0.0;
}

// z1 = z - V^T h (in place) over the block's 32 columns, then the partial dots
// of z1 with every row: part[b * k + r].  The slab V[0..k), [c0, c0 + 32)) is
// kept in LDS for the dots when it fits (cached), else re-read (L2-served).
template <typename T>
__global__ __launch_bounds__(kCgsUpdNT) void k_cgs_update_dots(int64_t d, int k, const T* __restrict__ V,
                                                               const double* __restrict__ h, T* __restrict__ z,
                                                               double* __restrict__ part, int cached,
                                                               const LanczosState* st) {
  if (st->done) return;
  __shared__ T slab[kCgsCacheBytes / sizeof(T)];
  __shared__ double red[kCgsRowGroups][kCgsUpdCols];
  __shared__ double zl[kCgsUpdCols];
  const int l = threadIdx.x % kCgsUpdCols, g = threadIdx.x / kCgsUpdCols;
  const int64_t c = int64_t(blockIdx.x) * kCgsUpdCols + l;
  const bool in = c < d;
  const double acc = cached ? cgs_col_sum<T, true>(V, d, k, c, in, g, h, slab, l)
                            : cgs_col_sum<T, false>(V, d, k, c, in, g, h, slab, l);
  const double sum = cgs_combine(acc, red, g, l);
  if (g == 0) {
    const T zn = in ? T(double(z[c]) - sum) : T(0);
    if (in) z[c] = zn;
    zl[l] = double(zn);
  }
  __syncthreads();
  // dots of z1 with every row over the block's 32 columns, one row per
  // thread, columns added in order (cached: 16-byte LDS reads of the slab row)
  for (int r = threadIdx.x; r < k; r += kCgsUpdNT) {
    double p = 0.0;
    if (cached) {
      const T* row = slab + r * kCgsSlabLd;
#pragma unroll
      for (int q = 0; q < kCgsUpdCols; ++q) p += double(row[q]) * zl[q];
    } else {
      const int64_t c0 = int64_t(blockIdx.x) * kCgsUpdCols;
      const T* row = V + int64_t(r) * d;
#pragma unroll 8
      for (int q = 0; q < kCgsUpdCols; ++q) {
        const T x = row[c0 + q < d ? c0 + q : d - 1];
        p += double(x) * zl[q];   // zl is 0 past d
      }
    }
    part[int64_t(blockIdx.x) * k + r] = p;
  }
}

// z2 = z1 - V^T h in place and the partials of ||z2||^2, one per block;
// grid-stride over 32-column slabs.
template <typename T>
__global__ __launch_bounds__(kCgsUpdNT) void k_cgs_update_norm(int64_t d, int k, const T* __restrict__ V,
                                                               const double* __restrict__ h, T* __restrict__ z,
                                                               double* __restrict__ pnorm,
                                                               const LanczosState* st) {
  if (st->done) return;
  __shared__ double red[kCgsRowGroups][kCgsUpdCols];
  __shared__ double sm[kCgsUpdNT / 64];
  const int l = threadIdx.x % kCgsUpdCols, g = threadIdx.x / kCgsUpdCols;
  double nrm = 0.0;
  const int64_t nslab = (d + kCgsUpdCols - 1) / kCgsUpdCols;
  for (int64_t b = blockIdx.x; b < nslab; b += gridDim.x) {
    const int64_t c = b * kCgsUpdCols + l;
    const bool in = c < d;
    const double acc = cgs_col_sum<T, false>(V, d, k, c, in, g, h, nullptr, l);
    const double sum = cgs_combine(acc, red, g, l);
    if (g == 0 && in) {
      const T zn = T(double(z[c]) - sum);
      z[c] = zn;
      nrm += double(zn) * double(zn);
    }
    __syncthreads();   // red is reused by the next slab
  }
  const double t = block_sum_nt<kCgsUpdNT>(nrm, sm);
  if (threadIdx.x == 0) pnorm[blockIdx.x] = t;
}

}  // namespace krcn
