// krcn_cgs2.hpp — full reorthogonalisation of the Lanczos basis, CGS2
// (build-only extension: the reference has none, cubic.py:92-103).
//
// After step B, z = z_{j+1} is orthogonalised against V_{0..j} (k = j + 1 rows
// of the row-major basis, length d each) twice:
//   h1 = V z;  z1 = z - V^T h1;  h2 = V z1;  z2 = z1 - V^T h2
// V is tall-skinny and streamed (rcv1_stress: up to 500 x 47,236 fp32 = 94 MB
// per sweep), so at large k the cost is the number of sweeps over V; at small
// k (half of a m = 500 run has k < 250) it is the fixed cost of each launch.
// Three sweeps, four launches:
//   k_cgs_rowdots     h1 partials per (column chunk, row): C chunks with
//                     C k <= kCgsRdParts, so the consumer reduces them itself
//                                                               V read 1
//   k_cgs_update_dots h1 = sum over chunks (prologue, into LDS);
//                     z1 = z - V^T h1 in place; the block caches its 32-column
//                     slab of V in LDS while applying h1 and forms the
//                     partial dots of z1 from LDS: h2 partials per slab
//                                                               V read 2
//   k_cgs_coeffs      h2 = sum over slabs (fixed order)
//   k_cgs_update_norm z2 = z1 - V^T h2 in place, ||z2||^2 partials (the next
//                     step's beta)                              V read 3
// The update sweeps keep U row loads in flight per thread with U sized to k
// (U = 1 at k <= 16 ... 16 at k > 128), so a small k issues no redundant
// loads.  Every load reads whole lines of rows (lanes on consecutive columns),
// from clamped addresses without branches.
// Sums are fixed-order: dots are products in double added per thread over its
// columns in order, then an xor butterfly over the wave and the waves in
// order; chunk and slab partials are added in chunk / slab order; each
// column's update adds 16 row-group sums in a fixed tree.  Deterministic.
#pragma once
#include "krcn_kernels.hpp"

namespace krcn {

constexpr int kCgsUpdCols = 32;      // update kernels: columns per block (a 128-B line of fp32 per row)
constexpr int kCgsUpdNT = 512;       //   threads: 32 columns x 16 row groups
constexpr int kCgsRowGroups = kCgsUpdNT / kCgsUpdCols;
constexpr int kCgsSlabLd = kCgsUpdCols + 4;   // padded LDS slab row (16-B aligned, spreads banks)
constexpr int kCgsCacheBytes = 73728;    // LDS slab cache of k_cgs_update_dots (2 blocks per CU)
constexpr int kCgsMaxU = 16;         // row loads in flight per thread in the update sweeps (k > 128)
constexpr int kCgsHPad = kCgsRowGroups * kCgsMaxU;   // zeros after h's k entries
constexpr int kCgsKMax = 2048;       // krcn_lanczos: m <= 2044

constexpr int kCgsRdNT = 256;        // k_cgs_rowdots: threads per block
constexpr int kCgsRdRows = 4;        //   rows per block (z loaded once for all four)
constexpr int kCgsRdU = 8;           //   column steps in flight per thread
constexpr int kCgsRdParts = 1024;    //   C k bound: the partials k_cgs_update_dots reduces
constexpr int kCgsRdPartsV = 4096;   //   (partials buffer floor, krcn_plan.hip reserve_reorth)

// column chunks of k_cgs_rowdots for k rows: C = min(kCgsRdParts / k, chunks
// of >= 2 x 1024 columns), at least 1
inline int cgs_rd_chunks(int64_t d, int k) {
  int64_t c = kCgsRdParts / k;
  const int64_t cmax = d / (2 * kCgsRdNT * kCgsRdU);
  if (c > cmax) c = cmax;
  return c < 1 ? 1 : int(c);
}

// update-sweep unroll for k rows: 16 row groups x U >= k where possible
inline int cgs_unroll(int k) {
  int u = 1;
  while (u < kCgsMaxU && kCgsRowGroups * u < k) u *= 2;
  return u;
}

// h1 partials: part[c * k + r] = sum over chunk c's columns of V[r, col] z[col].
// Grid: (C chunks, ceil(k / 4) row quads); chunk width cw.  A thread adds its
// columns t, t + 256, ... of the chunk in order, U steps in flight (4 rows +
// z each); rows past k recompute row k - 1 and are not stored.
template <typename T>
__global__ __launch_bounds__(kCgsRdNT) void k_cgs_rowdots(int64_t d, int k, int64_t cw, const T* __restrict__ V,
                                                          const T* __restrict__ z, double* __restrict__ part,
                                                          const LanczosState* st) {
  const int done = st->done;   // waited for after the sweep: its latency overlaps the loads
  constexpr int R = kCgsRdRows, U = kCgsRdU, NT = kCgsRdNT;
  __shared__ double sm[R][NT / 64];
  const int64_t cb = int64_t(blockIdx.x) * cw;
  const int64_t ce = cb + cw < d ? cb + cw : d;
  const int rb = blockIdx.y * R;
  const T* vr[R];
#pragma unroll
  for (int q = 0; q < R; ++q) vr[q] = V + int64_t(rb + q < k ? rb + q : k - 1) * d;
  double acc[R];
#pragma unroll
  for (int q = 0; q < R; ++q) acc[q] = 0.0;
  for (int64_t b = cb; b < ce; b += NT * U) {   // uniform trip count
    T zv[U], vv[R][U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t c = b + threadIdx.x + int64_t(NT) * u;
      const int64_t cc = c < ce ? c : ce - 1;
      zv[u] = z[cc];
#pragma unroll
      for (int q = 0; q < R; ++q) vv[q][u] = vr[q][cc];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const bool in = b + threadIdx.x + int64_t(NT) * u < ce;
      const double zu = in ? double(zv[u]) : 0.0;
#pragma unroll
      for (int q = 0; q < R; ++q) acc[q] += double(vv[q][u]) * zu;
    }
  }
  if (done) return;
  const int w = threadIdx.x >> 6;
#pragma unroll
  for (int q = 0; q < R; ++q) {
    const double s = wave_sum(acc[q]);
    if ((threadIdx.x & 63) == 0) sm[q][w] = s;
  }
  __syncthreads();
  if (threadIdx.x < R && rb + int(threadIdx.x) < k) {
    const int q = threadIdx.x;
    double t = sm[q][0];
#pragma unroll
    for (int i = 1; i < NT / 64; ++i) t += sm[q][i];
    part[int64_t(blockIdx.x) * k + rb + q] = t;
  }
}

// hs[r] = sum over c < C of part[c * k + r] (chunk order) for r < k, zeros in
// [k, HL); C > 1 stages the C k <= kCgsRdParts partials in LDS first (one
// round of global loads).  Ends with a barrier.
template <int NT>
__device__ __forceinline__ void cgs_load_h(const double* __restrict__ part, int C, int k, int HL, double* hs,
                                           double* stage) {
  if (C == 1) {
    for (int r0 = 0; r0 < HL; r0 += 4 * NT) {
      double a[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = r0 + threadIdx.x + i * NT;
        a[i] = part[r < k ? r : k - 1];
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = r0 + threadIdx.x + i * NT;
        if (r < HL) hs[r] = r < k ? a[i] : 0.0;
      }
    }
  } else {
    constexpr int PT = (kCgsRdParts + NT - 1) / NT;   // partials per thread (C k <= kCgsRdParts)
    const int P = C * k;
    double a[PT];
#pragma unroll
    for (int i = 0; i < PT; ++i) {
      const int q = threadIdx.x + i * NT;
      a[i] = part[q < P ? q : P - 1];
    }
#pragma unroll
    for (int i = 0; i < PT; ++i) {
      const int q = threadIdx.x + i * NT;
      if (q < P) stage[q] = a[i];
    }
    for (int r = k + threadIdx.x; r < HL; r += NT) hs[r] = 0.0;
    __syncthreads();
    for (int r = threadIdx.x; r < k; r += NT) {
      double t = stage[r];
      for (int c = 1; c < C; ++c) t += stage[c * k + r];
      hs[r] = t;
    }
  }
  __syncthreads();
}

// LDS of k_cgs_update_dots (dynamic): hs[HL] | zl[32] | slab of k rows (T) or
// the chunk partials (C > 1), whichever is larger.
__host__ __device__ inline int cgs_hlen(int k, int U) {
  const int h = k + kCgsRowGroups * U;
  const int r = kCgsRowGroups * kCgsUpdCols;   // the combine's sums reuse hs
  return h > r ? h : r;
}
template <typename T>
inline size_t cgs_upd_lds(int k, int U, int C, bool cached) {
  const size_t slab = cached ? size_t(k) * kCgsSlabLd * sizeof(T) : 0;
  const size_t stage = C > 1 ? size_t(C) * k * sizeof(double) : 0;
  return size_t(cgs_hlen(k, U) + kCgsUpdCols) * sizeof(double) + (slab > stage ? slab : stage);
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
  const int done = st->done;
  constexpr int SG = kCgsCoefNT / kCgsCoefRows;   // 64 slab groups
  __shared__ double sm[SG][kCgsCoefRows];
  const int ri = threadIdx.x % kCgsCoefRows, sg = threadIdx.x / kCgsCoefRows;
  const int r = blockIdx.x * kCgsCoefRows + ri;
  if (int(blockIdx.x) * kCgsCoefRows >= k) {   // a block of pad rows: zeros, no loads
    if (!done && sg == 0 && r < k + kCgsHPad) h[r] = 0.0;
    return;
  }
  const int rc = r < k ? r : k - 1;
  constexpr int U = 32;   // 2,048 slabs per round of loads
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
  if (done) return;
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
// U row loads in flight; optionally keeps the loaded values in the LDS slab
// (row-major, 32 columns).  h (global or LDS) carries zeros in [k, k + 16 U).
template <typename T, bool kCache, int U, int G = kCgsRowGroups>
__device__ __forceinline__ double cgs_col_sum(const T* __restrict__ V, int64_t d, int k, int64_t c, int g,
                                              const double* __restrict__ h, T* slab, int l) {
  // No branch in the body: loads from clamped addresses.  A load under a
  // condition is waited for before the branch joins (s_waitcnt vmcnt(0) each),
  // which serialises the U loads this loop keeps in flight.  The trip count
  // is uniform over the block.  Rows past k weigh 0; a column past d reads
  // column d - 1 and is never stored.
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

// Combine the G row-group sums of the block's CO columns (fixed tree) and
// return the sum for the thread's column (row group 0 only).
template <int G = kCgsRowGroups, int CO = kCgsUpdCols>
__device__ __forceinline__ double cgs_combine(double acc, double (*red)[CO], int g, int l) {
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

// h1 from the C chunk partials of k_cgs_rowdots (prologue, into LDS), then
// z1 = z - V^T h1 (in place) over the block's 32 columns, then the partial dots
// of z1 with every row: part2[b * k + r].  The slab V[0..k), [c0, c0 + 32)) is
// kept in LDS for the dots when it fits (kCache), else re-read (L2-served).
// The first U row loads, z and the state flag are issued before the prologue
// waits for the partials, so one memory latency covers all of them.  LDS is
// dynamic (cgs_upd_lds): a small k leaves room for more blocks per CU.
template <typename T, bool kCache, int U>
__global__ __launch_bounds__(kCgsUpdNT) void k_cgs_update_dots(int64_t d, int k, const T* __restrict__ V,
                                                               const double* __restrict__ part1, int C,
                                                               T* __restrict__ z, double* __restrict__ part2,
                                                               const LanczosState* st) {
  constexpr int G = kCgsRowGroups;
  extern __shared__ double dyn[];
  const int HL = cgs_hlen(k, U);
  double* hs = dyn;
  double* zl = dyn + HL;
  double* area = zl + kCgsUpdCols;
  T* slab = reinterpret_cast<T*>(area);
  const int l = threadIdx.x % kCgsUpdCols, g = threadIdx.x / kCgsUpdCols;
  const int64_t c = int64_t(blockIdx.x) * kCgsUpdCols + l;
  const bool in = c < d;
  const int64_t cc = in ? c : d - 1;
  T v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int r = g + u * G;
    v[u] = V[int64_t(r < k ? r : k - 1) * d + cc];
  }
  const T zc = z[cc];
  const int done = st->done;
  cgs_load_h<kCgsUpdNT>(part1, C, k, HL, hs, area);
  if (done) return;
  double acc = 0.0;
  for (int r0 = 0;;) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int r = r0 + g + u * G;
      if constexpr (kCache) slab[(r < k ? r : k - 1) * kCgsSlabLd + l] = v[u];   // rows past k rewrite row k - 1
      acc += hs[r] * double(v[u]);
    }
    r0 += G * U;
    if (r0 >= k) break;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int r = r0 + g + u * G;
      v[u] = V[int64_t(r < k ? r : k - 1) * d + cc];
    }
  }
  __syncthreads();   // every thread is done with hs before it holds the row-group sums
  const double sum = cgs_combine(acc, reinterpret_cast<double(*)[kCgsUpdCols]>(hs), g, l);
  if (g == 0) {
    const T zn = in ? T(double(zc) - sum) : T(0);
    if (in) z[c] = zn;
    zl[l] = double(zn);
  }
  __syncthreads();
  // dots of z1 with every row over the block's 32 columns, one row per
  // thread, columns added in order (cached: LDS reads of the slab row)
  for (int r = threadIdx.x; r < k; r += kCgsUpdNT) {
    double p = 0.0;
    if constexpr (kCache) {
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
    part2[int64_t(blockIdx.x) * k + r] = p;
  }
}

// z2 = z1 - V^T h in place (h from k_cgs_coeffs, zero-padded) and the
// partials of ||z2||^2, one per block; grid-stride over slabs of
// kCgsNormCols columns (a wave reads 256 contiguous bytes of a fp32 row; the
// 8 row groups are the block's waves).
constexpr int kCgsNormCols = 64;
constexpr int kCgsNormGroups = kCgsUpdNT / kCgsNormCols;
inline int cgs_norm_unroll(int k) {
  int u = 1;
  while (u < kCgsMaxU && kCgsNormGroups * u < k) u *= 2;
  return u;
}
template <typename T, int U>
__global__ __launch_bounds__(kCgsUpdNT) void k_cgs_update_norm(int64_t d, int k, const T* __restrict__ V,
                                                               const double* __restrict__ h, T* __restrict__ z,
                                                               double* __restrict__ pnorm,
                                                               const LanczosState* st) {
  constexpr int CO = kCgsNormCols, G = kCgsNormGroups;
  const int done = st->done;
  __shared__ double red[G][CO];
  __shared__ double sm[kCgsUpdNT / 64];
  const int l = threadIdx.x % CO, g = threadIdx.x / CO;
  double nrm = 0.0;
  const int64_t nslab = (d + CO - 1) / CO;
  for (int64_t b = blockIdx.x; b < nslab; b += gridDim.x) {
    const int64_t c = b * CO + l;
    const bool in = c < d;
    const double acc = cgs_col_sum<T, false, U, G>(V, d, k, c, g, h, nullptr, l);
    if (done) return;
    const double sum = cgs_combine<G, CO>(acc, red, g, l);
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

// ------------------------------------------------------ 1 KiB row pieces
// Round 4.  The batched sweeps above read V in 128-256 B row pieces (a
// column slab per block) and reach 3-3.5 TB/s on a cache-resident V; the
// row-contiguous dot sweep reaches 5.9.  The path below reads only whole
// 1 KiB pieces of rows (one 16-byte vector per lane) in every sweep, with all
// of a thread's loads issued at once (one round trip per block):
//   k_cgs_rowdots_v  h = V z as C chunk partials, one row per block
//                    (C <= kCgsRdChunksV)                      V read 1 / 3
//   k_cgs_colsweep   z' = z - V^T h over (column group x row range) blocks,
//                    h summed from the chunk partials in the prologue; the
//                    row ranges of a column group are combined in the
//                    launch by the last arrival              V read 2 / 4
// run as rowdots_v(z), colsweep(h1) -> z1, rowdots_v(z1), colsweep(h2) -> z2
// and the ||z2||^2 partials: four sweeps at the row-contiguous rate instead
// of three at the slab rate, four launches, and no coefficient reduction
// launch.  Rejected on the way (profiles/r04_cgs2_trace.txt): keeping the
// slab blocks but holding all k <= 512 rows of a thread in registers (one
// round trip, dots by a transposing butterfly) ran the update sweeps slower
// than the batched forms (128-B pieces, 1,477 blocks).
// Fixed order everywhere; the sums differ from the batched forms' order, not
// their definition (CGS2 is a build-only extension, tested at 1e-10).
template <typename T> struct Vec16;
template <> struct Vec16<float> { using type = float4; static constexpr int E = 4; };
template <> struct Vec16<double> { using type = double2; static constexpr int E = 2; };

template <typename T>
__device__ __forceinline__ double dot16(const typename Vec16<T>::type& a, const typename Vec16<T>::type& b) {
  if constexpr (Vec16<T>::E == 4) {
    double s = double(a.x) * double(b.x);
    s += double(a.y) * double(b.y);
    s += double(a.z) * double(b.z);
    s += double(a.w) * double(b.w);
    return s;
  } else {
    double s = double(a.x) * double(b.x);
    s += double(a.y) * double(b.y);
    return s;
  }
}

// part[c * k + r] = V[r, chunk c] . z[chunk c]; grid (C, k); chunk c covers
// vectors [c S kNT, (c + 1) S kNT) of the d / E per row.  Needs d E-aligned
// rows (d % E == 0) and 16-byte aligned V and z (checked by the launcher).
template <typename T, int S>
__global__ __launch_bounds__(kNT) void k_cgs_rowdots_v(int64_t d, int k, const T* __restrict__ V,
                                                       const T* __restrict__ z, double* __restrict__ part,
                                                       const LanczosState* st) {
  using V16 = typename Vec16<T>::type;
  constexpr int E = Vec16<T>::E;
  __shared__ double sm[kNT / 64];
  const int64_t nv = d / E;
  const int64_t vb = int64_t(blockIdx.x) * S * kNT + threadIdx.x;
  const int r = blockIdx.y;
  const V16* __restrict__ vr = reinterpret_cast<const V16*>(V + int64_t(r) * d);
  const V16* __restrict__ zv = reinterpret_cast<const V16*>(z);
  V16 a[S], b[S];
#pragma unroll
  for (int s = 0; s < S; ++s) {
    const int64_t i = vb + int64_t(s) * kNT;
    const int64_t ic = i < nv ? i : nv - 1;
    a[s] = vr[ic];
    b[s] = zv[ic];
  }
  const int done = st->done;
  double acc = 0.0;
#pragma unroll
  for (int s = 0; s < S; ++s)
    if (vb + int64_t(s) * kNT < nv) acc += dot16<T>(a[s], b[s]);
  if (done) return;
  const double t = block_sum(acc, sm);
  if (threadIdx.x == 0) part[int64_t(blockIdx.x) * k + r] = t;
}

// k_cgs_rowdots_v with the Lanczos step B fused (the first sweep of a
// reorthogonalised step): z = W - alpha v_j is formed per element from W and
// v_j = V[k - 1] exactly as k_lz_step_b forms it (alpha = the sum of step A's
// partials, every block, the same order as sum_partials), the blocks of row 0
// store it to V[k] (= z_{j+1}, unnormalised), block (0, 0) records alphas[k-1].
// Nothing is written once the recurrence is done (as k_lz_step_b).  The
// ||z||^2 partials of step B are not formed: k_cgs_colsweep's replace them.
template <typename T, int S>
__global__ __launch_bounds__(kNT) void k_cgs_rowdots_vb(int64_t d, int k, T* __restrict__ V,
                                                        const T* __restrict__ W, const double* __restrict__ pa,
                                                        int Pa, double* __restrict__ alphas, double* __restrict__ part,
                                                        const LanczosState* st) {
  using V16 = typename Vec16<T>::type;
  constexpr int E = Vec16<T>::E;
  __shared__ double sm[kNT / 64];
  const int64_t nv = d / E;
  const int64_t vb = int64_t(blockIdx.x) * S * kNT + threadIdx.x;
  const int r = blockIdx.y;
  const V16* __restrict__ vr = reinterpret_cast<const V16*>(V + int64_t(r) * d);
  const V16* __restrict__ vj = reinterpret_cast<const V16*>(V + int64_t(k - 1) * d);
  const V16* __restrict__ wv = reinterpret_cast<const V16*>(W);
  V16 a[S], wa[S], va[S];
#pragma unroll
  for (int s = 0; s < S; ++s) {
    const int64_t i = vb + int64_t(s) * kNT;
    const int64_t ic = i < nv ? i : nv - 1;
    a[s] = vr[ic];
    wa[s] = wv[ic];
    va[s] = vj[ic];
  }
  const int done = st->done;
  const double alpha = sum_partials(pa, Pa, sm);
  if (done) return;
  const T ta = T(alpha);
  V16* __restrict__ zo = reinterpret_cast<V16*>(V + int64_t(k) * d);
  double acc = 0.0;
#pragma unroll
  for (int s = 0; s < S; ++s) {
    const int64_t i = vb + int64_t(s) * kNT;
    V16 z;
    const T* w1 = reinterpret_cast<const T*>(&wa[s]);
    const T* v1 = reinterpret_cast<const T*>(&va[s]);
    T* z1 = reinterpret_cast<T*>(&z);
#pragma unroll
    for (int e = 0; e < E; ++e) z1[e] = w1[e] - ta * v1[e];   // the expression of k_lz_step_b
    if (i < nv) {
      acc += dot16<T>(a[s], z);
      if (r == 0) zo[i] = z;
    }
  }
  const double t = block_sum(acc, sm);
  if (threadIdx.x == 0) {
    part[int64_t(blockIdx.x) * k + r] = t;
    if (blockIdx.x == 0 && r == 0) alphas[k - 1] = alpha;
  }
}

// steps of k_cgs_rowdots_v: the fewest S in {1, 2, 4, 8, 16} whose chunks
// number C <= kCgsRdChunksV (C = chunks of S kNT vectors); the colsweep
// prologue sums a row's C partials in rounds of 8 loads.  (The C k bound of
// the batched path does not apply: no kernel stages all C k partials.)
constexpr int kCgsRdChunksV = 16;
inline int cgs_rdv_steps(int64_t nv, int /*k*/) {
  int s = 1;
  while (s < 16 && int64_t(s) * kNT * kCgsRdChunksV < nv) s *= 2;
  return s;
}
inline int cgs_rdv_chunks(int64_t nv, int s) { return int((nv + int64_t(s) * kNT - 1) / (int64_t(s) * kNT)); }

// z' = z - V^T h with 1 KiB row pieces (round 4): a block is a column group
// of CW = 64 E columns (one 16-byte vector per lane: a wave reads 1 KiB of a
// row per load) x a row range of NB batches of RB = 4 U rows (wave w takes
// rows w, w + 4, ... of a batch, U loads in flight per lane; the next batch
// is loaded when the previous one is added).  h for the block's rows is the
// sum of the C chunk partials of k_cgs_rowdots_v (chunk order).  The block's
// four waves are added in LDS (wave order); with Q > 1 row ranges each block
// stores its CW sums sc1 into y[q], drains, and draws a ticket from its
// column group's counter; the Q-th arrival adds the Q partials in range
// order, writes z' and resets the counter (the guide's sc1 split-K hand-off:
// cdna_hip_programming.md, projection GEMM item 2; MI355X_MICROARCH.md,
// inter-workgroup visibility: every handed-off byte stored sc1 by relaxed
// agent-scope atomic stores, every storing wave drained, the ticket drawn
// after a barrier, every read an sc1 load).  No release fence on the ticket:
// on gfx950 an agent release is buffer_wbl2 (an L2 write-back, ~1.7 us) on
// the last-arrival path of every column group, and the sc1 form needs none.
// Measured and not kept (round 5, profiles/r05i_cgs2_trace.txt): the next
// batch's loads issued before the current one is added (two batches in
// flight, 5.76 -> 5.79 ms of colsweep per m = 500 step) and rowdots blocks of
// up to 4 rows sharing their z loads (4.52 -> 4.87 ms: the registers of four
// rows cost more occupancy than the L2 re-reads of z they save), and blocks of
// 16 waves (U = 8, NB = 2: the same 256-row ranges with four times the waves
// a CU; 5.76 + 5.76 -> 5.37 + 5.53 ms at large k, slower at small k, the
// bench's reorth figure 20.95-21.01 -> 20.94-20.99 ms, profiles/r05n_cgs2_trace.txt),
// and rowdots blocks of 8 rows streaming past a z (or step-B z) held in
// registers, two rows in flight (plain sweep 4.5 -> 5.1 ms per step, reorth
// 21.0 -> 22.1 ms: fewer, longer blocks hide less latency than one row a
// block; profiles/r05u_cgs2_rowdots8_trace.txt).
// kNorm: the last arrival also stores the group's ||z'||^2 partial,
// pnorm[group].  Default shape
// (the launcher): U = 8, NB = 8, 256-row ranges — fewer ranges (fewer blocks,
// fewer partials and arrivals) beat one round trip per block: rcv1 stress
// 15.3-15.5 k (64-row ranges, U = 16) -> 16.0-16.1 k HVP/s.
template <typename T, int U, bool kNorm, int NB = 1>
__global__ __launch_bounds__(kNT) void k_cgs_colsweep(int64_t d, int k, const T* __restrict__ V,
                                                      const double* __restrict__ hp, int C, T* __restrict__ z,
                                                      double* __restrict__ y, int* __restrict__ cnt,
                                                      double* __restrict__ pnorm, const LanczosState* st) {
  using V16 = typename Vec16<T>::type;
  constexpr int E = Vec16<T>::E;
  constexpr int W = kNT / 64;
  constexpr int RB = W * U;
  constexpr int CW = 64 * E;
  __shared__ double hs[RB * NB];
  __shared__ double red[W][CW];
  __shared__ double smn[W];
  __shared__ int role;
  const int lane = threadIdx.x & 63, t = threadIdx.x;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // wave-uniform: row bases in SGPRs
  const int cg = blockIdx.x, q = blockIdx.y, Q = gridDim.y;
  const int64_t nv = d / E;
  const int64_t vi = int64_t(cg) * 64 + lane;
  const int64_t vic = vi < nv ? vi : nv - 1;
  const int r0 = q * RB * NB;   // the block's range: NB batches of RB rows
  // row bases are wave-uniform (SGPRs) and share one 32-bit lane offset: the
  // loads take the saddr form instead of a 64-bit address per load
  const uint32_t voff = uint32_t(vic) * uint32_t(sizeof(V16));
  V16 a[U];
  auto load = [&](int rb) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int r = rb + w + u * W;
      const char* rp = reinterpret_cast<const char*>(V + int64_t(r < k ? r : k - 1) * d);
      a[u] = *reinterpret_cast<const V16*>(rp + voff);
    }
  };
  load(r0);
  const int64_t c = int64_t(cg) * CW + t;
  const bool cin = t < CW && c < d;
  const T zc = z[c < d ? c : d - 1];
  const int done = st->done;
  for (int i = t; i < RB * NB; i += kNT) {   // C <= kCgsRdChunksV partials of a row
    const int r = r0 + i;
    const int rc = r < k ? r : k - 1;
    double hv = 0.0;
    for (int j0 = 0; j0 < C; j0 += 8) {   // rounds of 8 loads, chunk order
      double b[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) b[j] = hp[int64_t(j0 + j < C ? j0 + j : C - 1) * k + rc];
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (j0 + j < C) hv += b[j];
    }
    if (r >= k) hv = 0.0;
    hs[i] = hv;
  }
  __syncthreads();
  if (done) return;
  double acc[E];
#pragma unroll
  for (int e = 0; e < E; ++e) acc[e] = 0.0;
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) {   // batch nb's rows in order, then the next batch's loads
    if (nb > 0) {
      if (r0 + nb * RB >= k) break;
      load(r0 + nb * RB);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const double hv = hs[nb * RB + w + u * W];
      const T* av = reinterpret_cast<const T*>(&a[u]);
#pragma unroll
      for (int e = 0; e < E; ++e) acc[e] += hv * double(av[e]);
    }
  }
#pragma unroll
  for (int e = 0; e < E; ++e) red[w][lane * E + e] = acc[e];
  __syncthreads();
  double ys = 0.0;
  if (t < CW) {
    ys = red[0][t];
#pragma unroll
    for (int i = 1; i < W; ++i) ys += red[i][t];
  }
  if (Q > 1) {
    // The hand-off between the Q blocks of a column group.  Each partial is
    // an agent-scope atomic store (sc1: written through to the coherence
    // point); every wave waits for its own store to complete (vmcnt), the
    // block barrier orders that before thread 0's ticket (an agent-scope
    // fetch_add), and the last arrival reads the partials with agent-scope
    // atomic loads.  Only sc1 data is handed over, so no L2 write-back is
    // needed: the HIP memory model's agent-scope RELEASE on the ticket
    //  emits one (buffer_wbl2) and was measured — rcv1-stress
    // reorth 21.2 -> 26.5 ms per m = 500 step with a release fetch_add and an
    // acquire fence on the last arrival (profiles/r06e_cgs2_release_ab.txt),
    // 21.4 -> 43.0 ms with a release fence in every wave
    // (profiles/r06d_cgs2_fence_ab.txt) — so the hand-off stays at this
    // ISA-level protocol (DESIGN.md §5 *CGS2*).
    if (cin) __hip_atomic_store(y + int64_t(q) * d + c, ys, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __builtin_amdgcn_s_waitcnt(0x0f70);   // vmcnt(0) (gfx9 encoding; expcnt, lgkmcnt unconstrained)
    __syncthreads();
    if (t == 0) {
      const int old = __hip_atomic_fetch_add(cnt + cg, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      role = old == Q - 1;
      if (old == Q - 1) __hip_atomic_store(cnt + cg, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (!role) return;
    ys = 0.0;
    if (cin) {
      int qq = 0;
      for (; qq + 8 <= Q; qq += 8) {
        double b[8];
#pragma unroll
        for (int i = 0; i < 8; ++i)
          b[i] = __hip_atomic_load(y + int64_t(qq + i) * d + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
        for (int i = 0; i < 8; ++i) ys += b[i];
      }
      for (; qq < Q; ++qq) ys += __hip_atomic_load(y + int64_t(qq) * d + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  const T zn = T(double(zc) - ys);
  if (cin) z[c] = zn;
  if constexpr (kNorm) {
    const double s = block_sum(cin ? double(zn) * double(zn) : 0.0, smn);
    if (t == 0) pnorm[cg] = s;
  }
}

// rows per wave and batch of k_cgs_colsweep: U = umax past k = 4 umax, else
// the smallest power of two with 4 U >= k
inline int cgs_col_unroll(int k, int umax = 16) {
  int u = 1;
  while (u < umax && 4 * u < k) u *= 2;
  return u;
}


}  // namespace krcn
