// krcn_tiled.hpp — LDS-staged, XCD-sliced CSR passes (the HVP's two SpMVs).
//
// A pass computes, for every row r of a CSR matrix M (X for pass 1, X^T for
// pass 2), s_r = sum_k M_rk x_k and hands s_r to an epilogue.  Work layout:
//
//  * Tiles.  Rows are grouped into tiles of contiguous rows holding at most
//    kWaveTileNnz nonzeros (a longer row is a tile of its own, walked in
//    chunks).  Every wave works its own tiles: it streams the index/value
//    arrays with 16-byte loads, gathers x for the whole tile, writes the
//    products M_rk * x_k into its LDS slab and reduces the tile's rows out of
//    LDS with groups of L lanes.
//  * Slices.  When the gathered vector x is larger than what one XCD's 4 MiB L2
//    can keep hot next to the matrix stream, M is cut into S column slices
//    (S a multiple of 8) stored as S CSR blocks, and the tiles of slice s run on
//    blocks with blockIdx % 8 == s % 8 — the blocks the dispatcher deals to one
//    XCD — so each XCD gathers from a 1-2 MiB window of x that stays in its L2.
//    Slices write per-slice partial row sums; a combine pass adds them in slice
//    order and runs the epilogue.  Placement only affects speed, never results.
//
// Row-sum order (deterministic, independent of tiling and dispatch): lane l of
// the row's L-lane group sums elements l, l+L, l+2L, ... left to right, the L
// lane sums are combined by an xor butterfly, and slice partials are added in
// slice order.  L = 1 with S = 1 is exactly scipy's csr_matvec order.
#pragma once
#include "krcn_kernels.hpp"

namespace krcn {

// One tile: rows [row0, row1) of slice `slice`, nonzeros [p0, p1) of the
// pass's CSR arrays; long_row != 0 marks a single row with more than
// kWaveTileNnz nonzeros.  32 bytes: one scalar load per tile.
struct __attribute__((aligned(32))) TileDesc {
  int slice, long_row, row0, row1, p0, p1, pad0, pad1;
};

// Source of the gathered vector x for a pass: begin(sm) runs once per block
// (it may reduce partials and return true to skip the launch), get() the vector.
template <typename T> struct SrcPlain {
  const T* x;
  __device__ __forceinline__ bool begin(double*) { return false; }
  __device__ __forceinline__ const T* get() const { return x; }
};

// First launch of Lanczos loop step j: settles beta / breakdown (see
// lz_step_prologue) and gathers the unnormalised z_j.
template <typename T> struct SrcLzStep {
  LzCtl<T> c; LzVec<T> v;
  __device__ __forceinline__ bool begin(double* sm) { return lz_step_prologue(c, sm, v); }
  __device__ __forceinline__ const T* get() const { return v.z; }
};

// Later launches of a Lanczos step (state settled by an earlier launch).
template <typename T> struct SrcLzState {
  LzCtl<T> c; LzVec<T> v;
  __device__ __forceinline__ bool begin(double*) {
    if (c.mode == 0 && c.st->done) return true;
    v = lz_vec_from_state(c);
    return false;
  }
  __device__ __forceinline__ const T* get() const { return v.z; }
};

// An explicit vector, skipped once the recurrence has ended.
template <typename T> struct SrcGuard {
  const T* x; const LanczosState* st; int mode;
  __device__ __forceinline__ bool begin(double*) { return mode == 0 && st->done; }
  __device__ __forceinline__ const T* get() const { return x; }
};

// Per-slice partial store (sliced passes).
template <typename T> struct EpiSlicePart {
  T* part; int64_t ld;
  static constexpr bool kReduce = false;
  struct Pre {};
  template <class S> __device__ __forceinline__ void init(const S&) {}
  __device__ __forceinline__ Pre pre(int) const { return Pre{}; }
  __device__ __forceinline__ double row(int r, T s, int slice, const Pre&) const {
    part[int64_t(slice) * ld + r] = s;
    return 0.0;
  }
};

// ------------------------------------------------------------ wave tiles
// Each wave of a block owns its own tile (no block-wide barrier inside the
// tile loop): it streams the tile's column indices and values with 16-byte
// loads (int4 / double2 / float4), issues every gather of x before it touches
// LDS, stores the products in its private LDS slab, stages the tile's row
// pointers next to them, and reduces its rows out of LDS.
constexpr int kWaveTileNnz = 512;                    // nonzeros per wave tile
constexpr int kWaveTileRows = 128;                   // rows per wave tile (cap)
constexpr int kProdSlots = kWaveTileNnz + 8;         // 4-aligned window (+ pad)
constexpr int kWavesPerBlock = kNT / 64;
#ifndef KRCN_TILE_WAVES
#define KRCN_TILE_WAVES 1
#endif

__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Matrix streams use plain loads: between two HVPs a news20-sized matrix pair
// (218 MB) stays resident in the 256 MiB Infinity Cache, which nontemporal
// loads give up (measured: HVP 113 us plain vs 135 us nt on news20).
// -DKRCN_NT_STREAM_LOADS switches to nontemporal loads for A/B runs.
#ifdef KRCN_NT_STREAM_LOADS
#define KRCN_STREAM_LOAD(p) __builtin_nontemporal_load(p)
#else
#define KRCN_STREAM_LOAD(p) (*(p))
#endif

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef double f64x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <typename T> struct Vec4;
template <> struct Vec4<double> {
  __device__ __forceinline__ static void load(const double* p, double (&v)[4]) {
    const f64x2 a = KRCN_STREAM_LOAD(reinterpret_cast<const f64x2*>(p));
    const f64x2 b = KRCN_STREAM_LOAD(reinterpret_cast<const f64x2*>(p) + 1);
    v[0] = a.x; v[1] = a.y; v[2] = b.x; v[3] = b.y;
  }
};
template <> struct Vec4<float> {
  __device__ __forceinline__ static void load(const float* p, float (&v)[4]) {
    const f32x4 a = KRCN_STREAM_LOAD(reinterpret_cast<const f32x4*>(p));
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
  }
};

// prod[e - base] = val[e] * x[idx[e]] for e in [base, hi) (entries below the
// caller's first nonzero are staged too and never read), base a multiple of 4,
// hi - base <= kWaveTileNnz.  Lane chunks of 4 consecutive nonzeros; a chunk
// wholly inside [base, hi) uses 16-byte loads, the tail chunk scalar ones.
template <typename T>
__device__ __forceinline__ void wave_stage(T* prod, int64_t base, int64_t hi, const int* __restrict__ idx,
                                           const T* __restrict__ val, const T* __restrict__ x, int lane) {
  constexpr int kRounds = kWaveTileNnz / 256;
  int c[kRounds][4];
  T a[kRounds][4];
#pragma unroll
  for (int k = 0; k < kRounds; ++k) {
    const int64_t e = base + 4 * (lane + 64 * k);
    if (e + 3 < hi) {
      const i32x4 q = KRCN_STREAM_LOAD(reinterpret_cast<const i32x4*>(idx + e));
      c[k][0] = q.x; c[k][1] = q.y; c[k][2] = q.z; c[k][3] = q.w;
      Vec4<T>::load(val + e, a[k]);
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const bool ok = e + i < hi;
        c[k][i] = ok ? idx[e + i] : 0;
        a[k][i] = ok ? val[e + i] : T(0);
      }
    }
  }
  T gx[kRounds][4];
#pragma unroll
  for (int k = 0; k < kRounds; ++k) {
    const int64_t e = base + 4 * (lane + 64 * k);
#pragma unroll
    for (int i = 0; i < 4; ++i) gx[k][i] = (e + i < hi) ? x[c[k][i]] : T(0);
  }
#pragma unroll
  for (int k = 0; k < kRounds; ++k) {
    const int o = 4 * (lane + 64 * k);
    if (base + o < hi) {
#pragma unroll
      for (int i = 0; i < 4; ++i) prod[o + i] = a[k][i] * gx[k][i];
    }
  }
}

// The tiled pass.  ptr is the flattened slice-major row-pointer array
// (slice s, row r begins at ptr[s * rows + r]); tiles of XCD group g are
// tiles[tbeg[g] .. tbeg[g+1]), walked wave by wave.  groups = 8 when sliced.
template <typename T, int L, class Src, class Epi>
__global__ __launch_bounds__(kNT, KRCN_TILE_WAVES) void k_tiled_pass(int rows, int groups, const int* __restrict__ ptr,
                                                    const int* __restrict__ idx,
                                                    const T* __restrict__ val,
                                                    const TileDesc* __restrict__ tiles,
                                                    const int* __restrict__ tbeg, Src src, Epi epi,
                                                    double* __restrict__ partials) {
  __shared__ double sm[kNT / 64];
  if (src.begin(sm)) return;
  __shared__ T prod_all[kWavesPerBlock][kProdSlots];
  __shared__ int rp_all[kWavesPerBlock][kWaveTileRows + 1];
  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  T* prod = prod_all[wave];
  int* rpl = rp_all[wave];
  const T* x = src.get();
  epi.init(src);
  const int g = blockIdx.x % groups;
  const int j = (blockIdx.x / groups) * kWavesPerBlock + wave;
  const int stride = (gridDim.x / groups) * kWavesPerBlock;
  const int sub = lane & (L - 1);
  const int grp = lane / L;
  constexpr int kGroups = 64 / L;
  double acc = 0.0;
  for (int t = tbeg[g] + j; t < tbeg[g + 1]; t += stride) {
    const TileDesc td = tiles[t];
    const int* rp = ptr + int64_t(td.slice) * rows;
    if (!td.long_row) {
      const int64_t p0 = td.p0, p1 = td.p1;
      const int64_t base = p0 & ~int64_t(3);
      const int nr = td.row1 - td.row0;
      for (int i = lane; i <= nr; i += 64) rpl[i] = int(rp[td.row0 + i] - base);
      // epilogue operands of the first two row rounds, loaded under the stream
      typename Epi::Pre pf0{}, pf1{};
      if (sub == 0 && grp < nr) pf0 = epi.pre(td.row0 + grp);
      if (sub == 0 && grp + kGroups < nr) pf1 = epi.pre(td.row0 + grp + kGroups);
      wave_stage<T>(prod, base, p1, idx, val, x, lane);
      wave_lds_sync();
      int k = 0;
      for (int r = grp; r < nr; r += kGroups, ++k) {
        const int beg = rpl[r], end = rpl[r + 1];
        T s = T(0);
        for (int p = beg + sub; p < end; p += L) s += prod[p];
        if constexpr (L > 1) {
#pragma unroll
          for (int off = L / 2; off > 0; off >>= 1) s += __shfl_xor(s, off, L);
        }
        if (sub == 0) {
          const typename Epi::Pre pr = k == 0 ? pf0 : (k == 1 ? pf1 : epi.pre(td.row0 + r));
          acc += epi.row(td.row0 + r, s, td.slice, pr);
        }
      }
      wave_lds_sync();
    } else {
      // one long row, chunks of kWaveTileNnz; the first group keeps its
      // lane-strided running sums across chunks (element p goes to lane
      // (p - p0) % L, as in a short row).
      const int64_t p0 = td.p0, p1 = td.p1;
      T s = T(0);
      int64_t c0 = p0;
      while (c0 < p1) {
        const int64_t base = c0 & ~int64_t(3);
        const int64_t c1 = base + kWaveTileNnz < p1 ? base + kWaveTileNnz : p1;
        wave_stage<T>(prod, base, c1, idx, val, x, lane);
        wave_lds_sync();
        if (grp == 0) {
          const int64_t first = c0 + (((sub - (c0 - p0)) % L) + L) % L;
          for (int64_t p = first; p < c1; p += L) s += prod[p - base];
        }
        wave_lds_sync();
        c0 = c1;
      }
      if (grp == 0) {
        if constexpr (L > 1) {
#pragma unroll
          for (int off = L / 2; off > 0; off >>= 1) s += __shfl_xor(s, off, L);
        }
        if (sub == 0) acc += epi.row(td.row0, s, td.slice, epi.pre(td.row0));
      }
    }
  }
  if constexpr (Epi::kReduce) {
    const double tsum = block_sum(acc, sm);
    if (threadIdx.x == 0) partials[blockIdx.x] = tsum;
  }
}

// Combine pass of a sliced SpMV.  A block owns 64 rows; wave q sums slices
// q, q+4, q+8, ... in order (coalesced 64-row loads, S/4 per wave instead of
// S per thread), then s_r = (s_0 + s_1) + (s_2 + s_3) and the epilogue.
constexpr int kCombineRows = 64;
template <typename T, class Src, class Epi>
__global__ __launch_bounds__(kNT) void k_slice_combine(int rows, int S, const T* __restrict__ part,
                                                       Src src, Epi epi, double* __restrict__ partials) {
  __shared__ double sm[kNT / 64];
  if (src.begin(sm)) return;
  __shared__ T qs[kNT / 64][kCombineRows];
  epi.init(src);
  const int lane = threadIdx.x & 63, q = threadIdx.x >> 6;
  const int nchunks = (rows + kCombineRows - 1) / kCombineRows;
  double acc = 0.0;
  for (int ch = blockIdx.x; ch < nchunks; ch += gridDim.x) {
    const int r = ch * kCombineRows + lane;
    typename Epi::Pre p{};
    if (q == 0 && r < rows) p = epi.pre(r);
    T sq = T(0);
    if (r < rows)
      for (int k = q; k < S; k += kNT / 64) sq += part[int64_t(k) * rows + r];
    qs[q][lane] = sq;
    __syncthreads();
    if (q == 0 && r < rows) {
      const T sr = (qs[0][lane] + qs[1][lane]) + (qs[2][lane] + qs[3][lane]);
      acc += epi.row(r, sr, 0, p);
    }
    __syncthreads();
  }
  if constexpr (Epi::kReduce) {
    const double tsum = block_sum(acc, sm);
    if (threadIdx.x == 0) partials[blockIdx.x] = tsum;
  }
}

// Elementwise run of an epilogue over rows with precomputed sums (sharded
// modes: after the all-reduce of raw partial row sums).
template <typename T, class Src, class Epi>
__global__ __launch_bounds__(kNT) void k_rows_apply(int rows, const T* __restrict__ sums, Src src, Epi epi,
                                                    double* __restrict__ partials) {
  __shared__ double sm[kNT / 64];
  if (src.begin(sm)) return;
  epi.init(src);
  double acc = 0.0;
  for (int r = blockIdx.x * kNT + threadIdx.x; r < rows; r += gridDim.x * kNT)
    acc += epi.row(r, sums[r], 0, epi.pre(r));
  if constexpr (Epi::kReduce) {
    const double tsum = block_sum(acc, sm);
    if (threadIdx.x == 0) partials[blockIdx.x] = tsum;
  }
}

// ---------------------------------------------------------- slice builder
// slice id of every nonzero: largest s with bounds[s] <= col.
__global__ __launch_bounds__(kNT) void k_slice_of(int64_t nnz, const int* __restrict__ idx,
                                                  const int* __restrict__ bounds, int S,
                                                  int* __restrict__ sid) {
  for (int64_t e = int64_t(blockIdx.x) * kNT + threadIdx.x; e < nnz; e += int64_t(gridDim.x) * kNT) {
    const int c = idx[e];
    int lo = 0, hi = S;  // bounds[0] = 0 <= c < bounds[S]
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (bounds[mid] <= c) lo = mid; else hi = mid;
    }
    sid[e] = lo;
  }
}

// counts[s * rows + r + 1] += 1 for every nonzero (integer atomics: exact).
__global__ __launch_bounds__(kNT) void k_slice_counts(int rows, const int* __restrict__ ptr,
                                                      const int* __restrict__ sid,
                                                      int* __restrict__ counts) {
  const int lane = threadIdx.x & 63;
  const int wv = (blockIdx.x * kNT + threadIdx.x) >> 6;
  const int W = (gridDim.x * kNT) >> 6;
  for (int r = wv; r < rows; r += W)
    for (int p = ptr[r] + lane; p < ptr[r + 1]; p += 64)
      atomicAdd(&counts[int64_t(sid[p]) * rows + r + 1], 1);
}

template <typename T>
__global__ __launch_bounds__(kNT) void k_slice_gather(int64_t nnz, const int* __restrict__ perm,
                                                      const int* __restrict__ idx,
                                                      const T* __restrict__ val,
                                                      int* __restrict__ sidx, T* __restrict__ sval) {
  for (int64_t p = int64_t(blockIdx.x) * kNT + threadIdx.x; p < nnz; p += int64_t(gridDim.x) * kNT) {
    const int e = perm[p];
    sidx[p] = idx[e];
    sval[p] = val[e];
  }
}

}  // namespace krcn

namespace krcn {

// ------------------------------------------------------------ sorted tiles
// Gather coalescing.  The L1 tag path serves about one cache line per clock,
// so a gather wave-instruction costs about one clock per DISTINCT line its 64
// lanes touch.  In a sorted tile the nonzeros of a block tile (8 per thread)
// are stored ordered by gather index, packed with their slot in the tile's
// row-major order; consecutive lanes then gather neighbouring entries of x
// (profiles/r01_gather_microbench.txt), and the products are scattered back
// to their row-major slots in LDS, so the row sums — and every result — are
// bit-identical to the wave-tile layout with the same lanes and slices.
constexpr int kSortPerThread = 8;
// Occupancy the sorted pass is built for: 8 waves per SIMD (2 blocks of 1024,
// 4 of 512 or 8 of 256 threads per CU, matching the LDS footprint), so the
// register allocator keeps to 64 VGPRs.
#ifndef KRCN_SORT_WAVES
#define KRCN_SORT_WAVES 8
#endif
template <int NT> struct SortGeom {
  static constexpr int kTile = NT * kSortPerThread;   // nonzeros per block tile / sort segment
  static constexpr int kRows = kTile / 4;             // rows per block tile (cap)
  static constexpr int kSlotBits = NT == 256 ? 11 : NT == 512 ? 12 : 13;
  static_assert((1 << kSlotBits) == kTile, "slot field must address a whole tile");
  // packed word: (column - tile's column base) << kSlotBits | slot
  static constexpr int64_t kMaxWindow = int64_t(1) << (32 - kSlotBits);
};

// Block-wide sum over NT threads in a fixed order (pairwise over waves).
template <int NT>
__device__ __forceinline__ double block_sum_nt(double v, double* sm) {
  if constexpr (NT == kNT) {
    return block_sum(v, sm);
  } else {
    v = wave_sum(v);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) sm[w] = v;
    __syncthreads();
    double r[NT / 64];
#pragma unroll
    for (int i = 0; i < NT / 64; ++i) r[i] = sm[i];
#pragma unroll
    for (int h = NT / 128; h > 0; h >>= 1)
#pragma unroll
      for (int i = 0; i < h; ++i) r[i] = r[2 * i] + r[2 * i + 1];
    __syncthreads();
    return r[0];
  }
}

template <typename T, int L, int NT, class Src, class Epi>
__global__ __launch_bounds__(NT, KRCN_SORT_WAVES) void k_sorted_pass(int rows, int groups, const int* __restrict__ ptr,
                                                    const unsigned* __restrict__ gword,
                                                    const T* __restrict__ gval,
                                                    const TileDesc* __restrict__ tiles,
                                                    const int* __restrict__ tbeg, Src src, Epi epi,
                                                    double* __restrict__ partials) {
  using G = SortGeom<NT>;
  constexpr int kTile = G::kTile, kBits = G::kSlotBits;
  // Src::begin reduces over the first kNT threads only (sum_partials), so
  // every block size derives the same beta bits
  __shared__ double sm[NT / 64];
  if (src.begin(sm)) return;
  __shared__ T prod[kTile];
  __shared__ int rpl[G::kRows + 1];
  const T* x = src.get();
  epi.init(src);
  const int g = blockIdx.x % groups;
  const int j = blockIdx.x / groups;
  const int stride = gridDim.x / groups;
  const int t = threadIdx.x;
  const int sub = t & (L - 1);
  const int grp = t / L;
  constexpr int kGroups = NT / L;
  double acc = 0.0;
  for (int ti = tbeg[g] + j; ti < tbeg[g + 1]; ti += stride) {
    const TileDesc td = tiles[ti];
    const int* rp = ptr + int64_t(td.slice) * rows;
    const T* xb = x + td.pad0;
    if (!td.long_row) {
      const int p0 = td.p0, p1 = td.p1, nr = td.row1 - td.row0;
      unsigned wd[kSortPerThread];
      T a[kSortPerThread];
#pragma unroll
      for (int k = 0; k < kSortPerThread; ++k) {
        const int e = p0 + t + NT * k;
        const bool ok = e < p1;
        wd[k] = ok ? gword[e] : ~0u;
        a[k] = ok ? gval[e] : T(0);
      }
      T gx[kSortPerThread];
#pragma unroll
      for (int k = 0; k < kSortPerThread; ++k) {
#if KRCN_SORT_VARIANT == 1 || KRCN_SORT_VARIANT == 4
        gx[k] = T(wd[k] & 1);
#else
        gx[k] = wd[k] != ~0u ? xb[wd[k] >> kBits] : T(0);
#endif
      }
      for (int i = t; i <= nr; i += NT) rpl[i] = rp[td.row0 + i] - p0;
      typename Epi::Pre pf0{}, pf1{};
      if (sub == 0 && grp < nr) pf0 = epi.pre(td.row0 + grp);
      if (sub == 0 && grp + kGroups < nr) pf1 = epi.pre(td.row0 + grp + kGroups);
#pragma unroll
      for (int k = 0; k < kSortPerThread; ++k)
#if KRCN_SORT_VARIANT >= 2
        acc += double(a[k] * gx[k]);
#else
        if (wd[k] != ~0u) prod[wd[k] & (kTile - 1)] = a[k] * gx[k];
#endif
      __syncthreads();
      int kk = 0;
      for (int r = grp; r < nr; r += kGroups, ++kk) {
        const int beg = rpl[r], end = rpl[r + 1];
        T s = T(0);
#if KRCN_SORT_VARIANT != 3 && KRCN_SORT_VARIANT != 4
        for (int p = beg + sub; p < end; p += L) s += prod[p];
#else
        s = T(end - beg);
#endif
        if constexpr (L > 1) {
#pragma unroll
          for (int off = L / 2; off > 0; off >>= 1) s += __shfl_xor(s, off, L);
        }
        if (sub == 0) {
          const typename Epi::Pre pr = kk == 0 ? pf0 : (kk == 1 ? pf1 : epi.pre(td.row0 + r));
          acc += epi.row(td.row0 + r, s, td.slice, pr);
        }
      }
      __syncthreads();
    } else {
      // one long row in sort segments of kTile (a multiple of L): row element
      // q sits in segment q / kTile, slot q % kTile; the first group keeps
      // its lane-strided sums across segments.
      const int p0 = td.p0, p1 = td.p1;
      T s = T(0);
      for (int c0 = p0; c0 < p1; c0 += kTile) {
        const int c1 = c0 + kTile < p1 ? c0 + kTile : p1;
#pragma unroll
        for (int k = 0; k < kSortPerThread; ++k) {
          const int e = c0 + t + NT * k;
          if (e < c1) {
            const unsigned wv = gword[e];
            prod[wv & (kTile - 1)] = gval[e] * xb[wv >> kBits];
          }
        }
        __syncthreads();
        if (grp == 0)
          for (int p = sub; p < c1 - c0; p += L) s += prod[p];
        __syncthreads();
      }
      if (grp == 0) {
        if constexpr (L > 1) {
#pragma unroll
          for (int off = L / 2; off > 0; off >>= 1) s += __shfl_xor(s, off, L);
        }
        if (sub == 0) acc += epi.row(td.row0, s, td.slice, epi.pre(td.row0));
      }
    }
  }
  if constexpr (Epi::kReduce) {
    const double tsum = block_sum_nt<NT>(acc, sm);
    if (t == 0) partials[blockIdx.x] = tsum;
  }
}

// ------------------------------------------------- sorted-tile builder
// key[e] = (segment of e) << 32 | column of e, for the segments [segs[s], segs[s+1]).
__global__ __launch_bounds__(kNT) void k_seg_keys(int nseg, const int* __restrict__ segs,
                                                  const int* __restrict__ idx,
                                                  unsigned long long* __restrict__ key) {
  for (int s = blockIdx.x; s < nseg; s += gridDim.x)
    for (int e = segs[s] + threadIdx.x; e < segs[s + 1]; e += kNT)
      key[e] = (static_cast<unsigned long long>(s) << 32) | static_cast<unsigned int>(idx[e]);
}

template <typename T>
__global__ __launch_bounds__(kNT) void k_sorted_gather(int64_t nnz, const int* __restrict__ perm,
                                                       const unsigned long long* __restrict__ skey,
                                                       const int* __restrict__ segs,
                                                       const int* __restrict__ segbase,
                                                       const T* __restrict__ val, int slot_bits,
                                                       unsigned* __restrict__ gword, T* __restrict__ gval) {
  for (int64_t p = int64_t(blockIdx.x) * kNT + threadIdx.x; p < nnz; p += int64_t(gridDim.x) * kNT) {
    const int e = perm[p];
    const unsigned long long k = skey[p];
    const int s = int(k >> 32);
    const unsigned col = static_cast<unsigned>(k & 0xffffffffull) - static_cast<unsigned>(segbase[s]);
    gword[p] = (col << slot_bits) | static_cast<unsigned>(e - segs[s]);
    gval[p] = val[e];
  }
}

}  // namespace krcn
