// krcn_window.hpp — LDS-window CSR passes (the HVP's two SpMVs, short rows).
//
// Why: a sparse pass is limited by its gather, not its stream.  Gathering x
// through the vector cache costs about one clock per DISTINCT cache line a
// wave-instruction touches (profiles/r01_gather_microbench.txt); the sorted
// tiles of krcn_tiled.hpp coalesce that gather but pay a block-wide LDS
// scatter and two barriers per tile.  Here the gathered vector itself sits in
// LDS instead: a slice of W = 124 KiB / sizeof(T) consecutive entries of x is
// copied into LDS once per block, and every gather is a ds_read.
//
// Format (built by krcn_api.hip build_window_plan):
//  * S slices of W columns; slice s holds columns [s W, (s+1) W) as a CSR
//    block with slice-major flattened row pointers (row r of slice s begins at
//    ptr[s * rows + r]), 16-bit slice-local column offsets and the values —
//    10 bytes per nonzero instead of 12.
//  * Tiles of R consecutive rows (R = 16/32/64, from the mean row length per
//    slice); lane l of a wave owns row R t + l of tile t and sums its
//    elements left to right (1 lane per row — these formats are chosen for
//    short rows only).
//  * Segments {slice, t0, t1, flags}: block b runs segments sbeg[b] ..
//    sbeg[b+1]) in order; wave w takes tiles t0 + w, t0 + w + 16, ... (at most
//    kWinTMax each); kSegLoad loads the slice's window first, kSegFlush hands
//    the row sums to the epilogue afterwards and clears them.
//  Two ways to use it:
//  * accumulate (pass over X^T, few slices): every block owns one tile range
//    and walks all S slices over it (one segment per slice, flush on the
//    last); the per-lane running sum carries across slices, so row r is summed
//    strictly left to right over its whole CSR row — scipy's csc_matvec
//    order, bit for bit.
//  * slices (pass over X, many slices): the (slice, tile) work of each XCD
//    group is cut into equal pieces, one per block; every segment flushes to
//    per-slice partials, combined in slice order by k_slice_combine.
//
// Per tile and slice a wave stages up to kWinChunk nonzeros at a time: each
// lane loads 4 consecutive (offset, value) pairs with one 8-byte and two
// 16-byte loads (unconditional: indices past the chunk are clamped), gathers
// x from the LDS window, writes the products to its private LDS slab, and
// then every lane adds its row's products out of the slab in order.  No
// block-wide barrier outside the window loads.
#pragma once
#include "krcn_tiled.hpp"

namespace krcn {

struct __attribute__((aligned(16))) WinSeg {
  int slice, t0, t1, flags;
};
enum { kSegLoad = 1, kSegFlush = 2 };

constexpr int kWinNT = 1024;                 // one block per CU (the window takes the LDS)
constexpr int kWinWaves = kWinNT / 64;
constexpr int kWinChunk = 256;               // nonzeros per staging step (4 per lane)
constexpr int kWinBytes = 124 * 1024;        // LDS window
constexpr int kWinTMax = 6;                  // tiles per wave per segment (register sums)
constexpr int kWinPad = kWinChunk + 8;       // array padding: unconditional chunk loads stay in bounds
template <typename T> struct WinGeom {
  static constexpr int kW = kWinBytes / int(sizeof(T));   // window entries (fp64 15,872; fp32 31,744)
  static_assert(kW <= 65536, "16-bit slice-local offsets");
};

typedef unsigned short u16x4 __attribute__((ext_vector_type(4)));

template <typename T> struct Quad;
template <> struct Quad<double> {
  __device__ __forceinline__ static void load(const double* p, double (&v)[4]) {
    const f64x2 a = *reinterpret_cast<const f64x2*>(p);
    const f64x2 b = *(reinterpret_cast<const f64x2*>(p) + 1);
    v[0] = a.x; v[1] = a.y; v[2] = b.x; v[3] = b.y;
  }
};
template <> struct Quad<float> {
  __device__ __forceinline__ static void load(const float* p, float (&v)[4]) {
    const f32x4 a = *reinterpret_cast<const f32x4*>(p);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
  }
};

// One staged chunk: lane l holds nonzeros base + 4 l .. + 3 of [c0, hi).
template <typename T> struct WinChunk {
  u16x4 q;
  T v[4];
  int c0, base, hi;
};

// Issue the loads of the chunk starting at c0 of a tile ending at e1.
// Unconditional (the arrays carry kWinPad entries of padding): a branch
// around a load would make the compiler drain every outstanding load where
// the value is used, and the pipeline below relies on a younger chunk
// staying in flight while an older one is consumed.
template <typename T>
__device__ __forceinline__ void win_load(WinChunk<T>& c, int c0, int e1, const unsigned short* __restrict__ widx,
                                         const T* __restrict__ wval, int lane) {
  c.c0 = c0;
  c.base = c0 & ~3;
  c.hi = c.base + kWinChunk < e1 ? c.base + kWinChunk : e1;
  const int e = c.base + 4 * lane;
  c.q = *reinterpret_cast<const u16x4*>(widx + e);
  Quad<T>::load(wval + e, c.v);
}

// Gather x from the window, stage the products in the wave's slab, and add
// this lane's row elements [beg, end) that fall in the chunk, in order.
template <typename T>
__device__ __forceinline__ T win_consume(const WinChunk<T>& c, int beg, int end, const T* win, T* slab, int lane,
                                         T s) {
  const int e = c.base + 4 * lane;
  const unsigned short qi[4] = {c.q.x, c.q.y, c.q.z, c.q.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) slab[4 * lane + i] = c.v[i] * win[e + i < c.hi ? qi[i] : 0];
  wave_lds_sync();
  const int pb = beg > c.c0 ? beg : c.c0;
  const int pe = end < c.hi ? end : c.hi;
  for (int p = pb; p < pe; ++p) s += slab[p - c.base];
  wave_lds_sync();
  return s;
}

// Block barrier that orders LDS only (the window), leaving global loads of
// the next chunks in flight.
__device__ __forceinline__ void lds_block_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

template <typename T, int R, class Src, class Epi>
__global__ __launch_bounds__(kWinNT, 1) void k_window_pass(int rows, int64_t cols, const int* __restrict__ ptr,
                                                           const unsigned short* __restrict__ widx,
                                                           const T* __restrict__ wval,
                                                           const WinSeg* __restrict__ segs,
                                                           const int* __restrict__ sbeg, Src src, Epi epi,
                                                           double* __restrict__ partials) {
  constexpr int W = WinGeom<T>::kW;
  constexpr int kPer = (W + kWinNT - 1) / kWinNT;
  constexpr int K = kWinTMax;
  __shared__ double sm[kWinNT / 64];
  if (src.begin(sm)) return;
  __shared__ T win[W];
  __shared__ T slab_all[kWinWaves][kWinChunk];
  // wave index made explicitly uniform: tile bounds then live in SGPRs
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  T* slab = slab_all[wave];
  const T* x = src.get();
  epi.init(src);
  T acc[K];
#pragma unroll
  for (int k = 0; k < K; ++k) acc[k] = T(0);
  double red = 0.0;
  const int s0 = sbeg[blockIdx.x], s1 = sbeg[blockIdx.x + 1];
  for (int si = s0; si < s1; ++si) {
    const WinSeg sg = segs[si];
    const int* rp = ptr + int64_t(sg.slice) * rows;
    const int nt = sg.t1 - sg.t0 - wave > 0 ? (sg.t1 - sg.t0 - wave + kWinWaves - 1) / kWinWaves : 0;
    // wave-uniform bounds of this wave's tiles (clamped to a real tile when absent)
    int e0[K], e1[K], r0[K], nr[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      int t = sg.t0 + wave + k * kWinWaves;
      t = t < sg.t1 ? t : sg.t1 - 1;
      r0[k] = t * R;
      nr[k] = rows - r0[k] < R ? rows - r0[k] : R;
      e0[k] = rp[r0[k]];
      e1[k] = rp[r0[k] + nr[k]];
    }
    // order: window loads (to registers), first chunk, then the window
    // store; per-lane row bounds and epilogue operands after the window's
    // registers are free again
    constexpr int kPerW = kPer;
    T tmp[kPerW];
    const bool load_win = (sg.flags & kSegLoad) != 0;
    const int64_t wbase = int64_t(sg.slice) * W;
    const int wlen = cols - wbase < W ? int(cols - wbase) : W;
    if (load_win) {
#pragma unroll
      for (int k = 0; k < kPerW; ++k) {
        const int i = threadIdx.x + kWinNT * k;
        tmp[k] = x[wbase + (i < wlen ? i : wlen - 1)];
      }
    }
    WinChunk<T> ca, cb;
    win_load(ca, e0[0], e1[0], widx, wval, lane);
    if (load_win) {
      lds_block_barrier();   // every wave is done with the previous window
#pragma unroll
      for (int k = 0; k < kPerW; ++k) {
        const int i = threadIdx.x + kWinNT * k;
        if (i < wlen) win[i] = tmp[k];
      }
    }
    int bg[K], en[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int li = lane < nr[k] ? lane : nr[k];
      bg[k] = rp[r0[k] + li];
      en[k] = rp[r0[k] + li + (lane < nr[k] ? 1 : 0)];
    }
    typename Epi::Pre pre[K];
    if (sg.flags & kSegFlush) {
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const int r = r0[k] + lane;
        pre[k] = epi.pre(r < rows ? r : rows - 1);
      }
    }
    if (load_win) lds_block_barrier();
#pragma unroll
    for (int k = 0; k < K; ++k) {
      if (k >= nt) break;
      WinChunk<T>& cur = (k & 1) ? cb : ca;
      WinChunk<T>& nxt = (k & 1) ? ca : cb;
      if (k + 1 < K) win_load(nxt, e0[k + 1], e1[k + 1], widx, wval, lane);
      T s = win_consume(cur, bg[k], en[k], win, slab, lane, acc[k]);
      for (int c = cur.hi; c < e1[k];) {          // tiles longer than one chunk
        WinChunk<T> cx;
        win_load(cx, c, e1[k], widx, wval, lane);
        s = win_consume(cx, bg[k], en[k], win, slab, lane, s);
        c = cx.hi;
      }
      acc[k] = s;
    }
    if (sg.flags & kSegFlush) {
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const int t = sg.t0 + wave + k * kWinWaves;
        const int r = t * R + lane;
        if (k < nt && lane < R && r < rows) red += epi.row(r, acc[k], sg.slice, pre[k]);
        acc[k] = T(0);
      }
    }
  }
  if constexpr (Epi::kReduce) {
    const double tsum = block_sum_nt<kWinNT>(red, sm);
    if (threadIdx.x == 0) partials[blockIdx.x] = tsum;
  }
}

// 16-bit slice-local offsets of a uniformly sliced CSR (slice width W).
__global__ __launch_bounds__(kNT) void k_local_u16(int64_t nnz, const int* __restrict__ idx, int W,
                                                   unsigned short* __restrict__ out) {
  for (int64_t e = int64_t(blockIdx.x) * kNT + threadIdx.x; e < nnz; e += int64_t(gridDim.x) * kNT)
    out[e] = static_cast<unsigned short>(idx[e] % W);
}

}  // namespace krcn
