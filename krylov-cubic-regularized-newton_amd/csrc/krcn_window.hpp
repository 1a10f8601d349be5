// krcn_window.hpp — LDS-window CSR passes (the HVP's two SpMVs, short rows).
//
// Why: a sparse pass is limited by its gather, not its stream.  Gathering x
// through the vector cache costs about one clock per DISTINCT cache line a
// wave-instruction touches (profiles/r01_gather_microbench.txt); the sorted
// tiles of krcn_tiled.hpp coalesce that gather but pay a block-wide LDS
// scatter and two barriers per tile.  Here the gathered vector itself sits in
// LDS instead: a slice of up to WinGeom<T>::kW consecutive entries of x is
// copied into LDS once per block, and every gather is a ds_read.
//
// Format (built by krcn_api.hip build_window):
//  * S slices of W columns; slice s holds columns [s W, (s+1) W) as a CSR
//    block in slice-major order with 16-bit slice-local column offsets and
//    the values — 10 bytes per nonzero instead of 12 — and compact row
//    pointers: a 32-bit base per (slice, tile) plus 16-bit row ends relative
//    to it.
//  * Tiles of R consecutive rows (R = 16/32/64, from the mean row length per
//    slice); lane l of a wave owns row R t + l of tile t and sums its
//    elements left to right (1 lane per row — these formats are chosen for
//    short rows only).
//  * Segments {slice, t0, t1, flags}: block b runs segs[b * stride + i]
//    (the first entry carries the count); wave w takes tiles t0 + w,
//    t0 + w + 16, ...; kSegLoad loads the slice's window first, kSegFlush
//    hands the row sums to the epilogue.
//  Two ways to use it:
//  * accumulate (pass over X^T, few slices): every block owns one tile range
//    and walks all S slices over it (one segment per slice, flush on the
//    last); the per-lane running sum carries across slices, so row r is summed
//    strictly left to right over its whole CSR row — scipy's csc_matvec
//    order.
//  * slices (pass over X, many slices): block s + S c owns row chunk c of
//    slice s (one window per block, the slice's blocks on one XCD); every
//    tile flushes to per-slice partials, combined in slice order by
//    k_slice_combine.  SrcLzZ fuses the previous Lanczos step B into the
//    window load (z = w - alpha v).
//
// Per tile and slice a wave stages up to kWinChunk nonzeros at a time: each
// lane loads 4 consecutive (offset, value) pairs with one 8-byte and two
// 16-byte loads (unconditional: indices past the chunk are clamped), gathers
// x from the LDS window, writes the products to its private LDS slab, and
// then every lane adds its row's products out of the slab in order; chunk
// loads run two tiles ahead (a ring of three slots).  No block-wide barrier
// outside the window loads.
#pragma once
#include <type_traits>
#include <utility>

#include "krcn_tiled.hpp"

namespace krcn {

struct __attribute__((aligned(16))) WinSeg {
  int slice, t0, t1, flags;   // flags: kSegLoad | kSegFlush | (segments of the block << 8, first entry only)
};
enum { kSegLoad = 1, kSegFlush = 2 };

constexpr int kWinNT = 1024;                 // one block per CU (the window takes the LDS)
constexpr int kWinWaves = kWinNT / 64;
constexpr int kWinChunk = 256;               // nonzeros per staging step (4 per lane)
constexpr int kWinTMax = 6;                  // accumulate mode: tiles per wave (register sums)
constexpr int kWinPad = kWinChunk + 8;       // array padding: unconditional chunk loads stay in bounds
constexpr int kWinRing = 3;                  // chunk slots in flight per wave (slices mode)
constexpr int kWinBatch = 58;                // slices mode: tiles per batch of tile bases (64 - the look-ahead)
#ifndef KRCN_WIN_RING_ACCUM
#define KRCN_WIN_RING_ACCUM 2
#endif
constexpr int kWinRingAccum = KRCN_WIN_RING_ACCUM;   // (accumulate mode, register-bound)
#ifndef KRCN_WIN_SUMU
#define KRCN_WIN_SUMU 8   // long rows: slab reads batched per lane (same add order: the same bits)
#endif
#ifndef KRCN_WIN_COOP
#define KRCN_WIN_COOP 1   // very long runs of a slices-mode chunk summed by the whole wave (0: A/B, round 6)
#endif
constexpr int kWinCoopLen = 64;              // (KRCN_WIN_COOP) run length past which the wave sums it
#ifndef KRCN_WIN_FIRST
#define KRCN_WIN_FIRST 1   // window stored before the first chunk loads go out
#endif
// LDS: window + 16 slabs of kWinChunk + the reduction scratch must fit 160 KiB
template <typename T> struct WinGeom {
  static constexpr int kSlabBytes = kWinWaves * kWinChunk * int(sizeof(T));
  static constexpr int kBytes = 163840 - kSlabBytes - 256;
  static constexpr int kW = kBytes / int(sizeof(T));      // max window (fp64 16,352; fp32 32,704)
  static constexpr int kPer = (kW + kWinNT - 1) / kWinNT;  // window entries per thread
  static_assert(kW <= 65536, "16-bit slice-local offsets");
};

struct WinArgs {
  int rows, W, stride, S;
  int dbg;                       // diagnostic builds: stamp table (0 slices, 1 accumulate, 2 fused Lanczos)
  int ntiles;                    // tiles of R rows per slice
  int64_t cols;
  const int* tb;                 // tile bases: slice s, tile t begins at tb[s * (ntiles + 1) + t]
  const unsigned short* ro;      // row ends relative to their tile base: row r of slice s at ro[s * rows + r]
  const unsigned short* widx;    // slice-local column offsets
  const void* wval;
  const WinSeg* segs;            // block b: segs[b * stride + i]
  int kpb = 0;                   // slices mode: win_block_slice's mapping (0: block = slice + S chunk)
};

// Slices mode: block b's slice and row chunk.  kpb == 0: b = slice + S chunk
// (S a multiple of 8 and kpb a power of two: the slice's blocks share an XCD,
// b % 8).  Else (round 5: 85 slices x 3 blocks) the blocks of XCD b % 8 take
// consecutive slots of a slice-major numbering (slot = kpb slice + chunk):
// slot = (slots of the XCDs before b's) + b / 8, so a slice's blocks share
// an XCD except where its slots straddle two XCDs.  G = the grid.
__host__ __device__ inline void win_block_slice(int b, int G, int S, int kpb, int& slice, int& chunk) {
  if (kpb == 0) {
    slice = b % S;
    chunk = b / S;
    return;
  }
  const int x = b % 8, q = G / 8, r = G % 8;
  const int slot = x * q + (x < r ? x : r) + b / 8;
  slice = slot / kpb;
  chunk = slot % kpb;
}

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

#ifdef KRCN_WIN_TIMING
// Diagnostic builds only (-DKRCN_WIN_TIMING): s_memrealtime (100 MHz; a fixed
// offset per XCD, see tools/win_timeline.py) stamps per block: [0] entry,
// [1] after the source prologue, per segment i < 4: [2+2i] window ready,
// [3+2i] tiles done; [10] end; [16+w] wave w done with its last segment.
// Three tables (WinArgs::dbg): slices mode, accumulate mode, fused Lanczos pass 1.
constexpr int kWinDbgSlots = 32;
// one table per translation unit (separate code objects): each unit exports a
// reader, krcn_debug_win_stamps merges them
static __device__ unsigned long long krcn_win_dbg[3 * 2048 * kWinDbgSlots];
[[maybe_unused]] static int win_stamps_read(unsigned long long* out, int n, int reset) {
  if (hipDeviceSynchronize() != hipSuccess) return 1;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(krcn_win_dbg), sizeof(unsigned long long) * n) != hipSuccess) return 1;
  if (reset) {
    static unsigned long long z[3 * 2048 * kWinDbgSlots];
    if (hipMemcpyToSymbol(HIP_SYMBOL(krcn_win_dbg), z, sizeof(z)) != hipSuccess) return 1;
  }
  return 0;
}
#define KRCN_WIN_STAMP(slot)                                                                          \
  do {                                                                                                \
    if (threadIdx.x == 0 && blockIdx.x < 2048)                                                        \
      krcn_win_dbg[a.dbg * 2048 * kWinDbgSlots + blockIdx.x * kWinDbgSlots + (slot)] =   \
          __builtin_amdgcn_s_memrealtime();                                                           \
  } while (0)
#define KRCN_WIN_WAVE_STAMP(slot)                                                                     \
  do {                                                                                                \
    if ((threadIdx.x & 63) == 0 && blockIdx.x < 2048)                                                 \
      krcn_win_dbg[a.dbg * 2048 * kWinDbgSlots + blockIdx.x * kWinDbgSlots + (slot)] =   \
          __builtin_amdgcn_s_memrealtime();                                                           \
  } while (0)
#else
#define KRCN_WIN_STAMP(slot) do {} while (0)
#define KRCN_WIN_WAVE_STAMP(slot) do {} while (0)
#endif

// One staged chunk: lane l holds nonzeros base + 4 l .. + 3 of [c0, hi).
template <typename T> struct WinChunk {
  u16x4 q;
  T v[4];
  int c0, base, hi;
};

// Issue the loads of the chunk starting at c0 of a tile ending at e1.
// Unconditional (the arrays carry kWinPad entries of padding): a branch
// around a load would make the compiler drain every outstanding load where
// the value is used, and the pipeline relies on younger chunks staying in
// flight while an older one is consumed.
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
                                         T s, bool coop = false) {
  const int e = c.base + 4 * lane;
  const unsigned short qi[4] = {c.q.x, c.q.y, c.q.z, c.q.w};
#if defined(KRCN_WIN_ABL_NOSUM)        // ablation (timing only): no slab, no row walk
#pragma unroll
  for (int i = 0; i < 4; ++i) s += c.v[i] * win[e + i < c.hi ? qi[i] : 0];
  (void)beg; (void)end; (void)slab;
  return s;
#else
#pragma unroll
  for (int i = 0; i < 4; ++i) slab[4 * lane + i] = c.v[i] * win[e + i < c.hi ? qi[i] : 0];
  wave_lds_sync();
  const int pb = beg > c.c0 ? beg : c.c0;
  const int pe = end < c.hi ? end : c.hi;
  int p = pb;
#if KRCN_WIN_SUMU > 1
  // a chunk where some lane holds a long row (skewed data): that lane's slab
  // reads go out KRCN_WIN_SUMU at a time, one read latency per batch instead
  // of per element; the adds stay left to right (the same bits).  Short rows
  // (the uniform case, almost always) never enter it.  coop (slices mode over
  // S > 1 slices, whose partials are combined anyway, so not scipy's order):
  // a run longer than kWinCoopLen is summed by the whole wave — strided
  // partial sums, then a butterfly (every lane the same bits) — one run at a
  // time, instead of by its lane alone while the others wait: skewed news20
  // pass 1 41.5-41.7 -> 39.3-39.5 us, 11.4-11.5 k -> 11.8-12.2 k HVP/s
  // (profiles/r06u_news20_skew_coop_ab.txt).  The uniform news20 never has
  // such a run (5.35 elements a row and slice).  (Every run past 16 summed
  // this way was slower, 41.3 -> 48.1 us: many medium runs went one by one.)
  if (coop) {   // (wave-uniform) runs past kWinCoopLen: summed by the whole wave, one run at a time
    unsigned long long longm = __ballot(pe - pb > kWinCoopLen);
    while (longm != 0ull) {
      const int L = __builtin_ctzll(longm);
      longm &= longm - 1ull;
      const int lb = __builtin_amdgcn_readlane(pb, L), le = __builtin_amdgcn_readlane(pe, L);
      T part = T(0);
      for (int q = lb + lane; q < le; q += 64) part += slab[q - c.base];
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) part += __shfl_xor(part, off, 64);
      if (lane == L) s += part;
    }
    if (pe - pb > kWinCoopLen) p = pe;   // this lane's run is in s
  }
  if (__ballot(pe - p > 2 * KRCN_WIN_SUMU) != 0ull) {
    for (; p + KRCN_WIN_SUMU <= pe; p += KRCN_WIN_SUMU) {
      T a[KRCN_WIN_SUMU];
#pragma unroll
      for (int u = 0; u < KRCN_WIN_SUMU; ++u) a[u] = slab[p + u - c.base];
#pragma unroll
      for (int u = 0; u < KRCN_WIN_SUMU; ++u) s += a[u];
    }
  }
#endif
  for (; p < pe; ++p) s += slab[p - c.base];
  wave_lds_sync();
  return s;
#endif
}

// Block barrier that orders LDS only (the window), leaving global loads of
// the next chunks in flight.
__device__ __forceinline__ void lds_block_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// Window of slice `slice` into registers: piece q of the block's sweep (1024
// consecutive entries) lands in tmp[(q - rot) mod kPer].  Entries past the
// slice are not loaded (clamping whole pieces would send every such lane of
// every block to one cache line).  Issued as early as the pointer is known.
template <typename T>
__device__ __forceinline__ void win_fetch(T (&tmp)[WinGeom<T>::kPer], const T* __restrict__ x, int slice,
                                          const WinArgs& a, int rot) {
  constexpr int kPer = WinGeom<T>::kPer;
  const int64_t wbase = int64_t(slice) * a.W;
  const int len = a.cols - wbase < a.W ? int(a.cols - wbase) : a.W;
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    const int q = k + rot < kPer ? k + rot : k + rot - kPer;
    const int i = threadIdx.x + kWinNT * q;
    // a piece wholly past the slice is skipped (block-uniform test); inside
    // the piece that crosses the end, lanes clamp to the last entry
    if (kWinNT * q < len) tmp[k] = x[wbase + (i < len ? i : len - 1)];
  }
}

template <typename T>
__device__ __forceinline__ void win_store(const T (&tmp)[WinGeom<T>::kPer], T* win, int slice, const WinArgs& a,
                                          int rot) {
  constexpr int kPer = WinGeom<T>::kPer;
  const int64_t wbase = int64_t(slice) * a.W;
  const int len = a.cols - wbase < a.W ? int(a.cols - wbase) : a.W;
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    const int q = k + rot < kPer ? k + rot : k + rot - kPer;
    const int i = threadIdx.x + kWinNT * q;
    if (i < len) win[i] = tmp[k];
  }
}

// f(integral_constant<int, I>) for I = 0, 1, ... while I < n.
template <int... I, class F>
__device__ __forceinline__ void unroll_while(std::integer_sequence<int, I...>, int n, F&& f) {
  bool go = true;
  ((go = go && (I < n), go ? (f(std::integral_constant<int, I>{}), 0) : 0), ...);
}

// Wave-uniform bounds of tile t (clamped into [t0, t1)): rows [r0, r0 + nr),
// nonzeros [e0, e1) of the slice's CSR (tb: this slice's tile bases).
template <int R>
struct TileB {
  int r0, nr, e0, e1;
  __device__ __forceinline__ void load(const int* tb, int rows, int t, int t1) {
    t = t < t1 ? t : t1 - 1;
    t = t > 0 ? t : 0;
    r0 = t * R;
    nr = rows - r0 < R ? rows - r0 : R;
    e0 = tb[t];
    e1 = tb[t + 1];
  }
  // the same bounds from a WinTiles batch (no memory access)
  __device__ __forceinline__ void set(int rows, int t, int t1, int te0, int te1) {
    t = t < t1 ? t : t1 - 1;
    t = t > 0 ? t : 0;
    r0 = t * R;
    nr = rows - r0 < R ? rows - r0 : R;
    e0 = te0;
    e1 = te1;
  }
};

// Tile bases of a wave's tiles tw + 16 k, 64 tiles at a time: lane i holds
// e0 / e1 of tile k = kb + i (clamped into the segment), one vector load for
// all of them, read lane-wise (v_readlane) as the ring reaches each tile.
// Loading each tile's bases on its own and broadcasting them (readfirstlane)
// made every tile wait for its load, and vmcnt retires in issue order: that
// wait drained the whole ring of chunk loads once per tile (round 5, ISA of
// k_window_pass).
struct WinTiles {
  int e0, e1, kb;
  __device__ __forceinline__ void load(const int* tb, int tw, int t1, int kb_, int lane) {
    kb = kb_;
    int t = tw + kWinWaves * (kb + lane);
    t = t < t1 ? t : t1 - 1;
    t = t > 0 ? t : 0;   // an empty segment (t1 = 0: a slice with fewer tiles than its blocks) reads tile 0
    e0 = tb[t];
    e1 = tb[t + 1];
  }
};

// A tile's two row-end loads for this lane, issued a tile ahead; the lane's
// bounds are formed from them only when the tile is consumed (tile_row_bounds),
// so the wait for them is partial.  Unconditional clamped loads.
struct RowRaw {
  int o1, o0;
};
template <int R>
__device__ __forceinline__ RowRaw tile_row_load(const TileB<R>& b, const unsigned short* ro, int lane) {
  const int i1 = lane < b.nr ? lane : b.nr - 1;
  const int i0 = lane < b.nr ? (lane > 0 ? lane - 1 : 0) : b.nr - 1;
  return RowRaw{int(ro[b.r0 + i1]), int(ro[b.r0 + i0])};
}
template <int R>
__device__ __forceinline__ void tile_row_bounds(const TileB<R>& b, const RowRaw& q, int lane, int& bg, int& en) {
  const int ea = b.e0 + q.o1, eb = b.e0 + q.o0;
  en = lane < b.nr ? ea : b.e1;
  bg = lane < b.nr ? (lane > 0 ? eb : b.e0) : b.e1;
}

// ------------------------------------------------ slice-combine fold (A/B)
// VERDICT r05 item 4, tuning builds only (-DKRCN_FOLD=1): the early-alpha
// pass 1 of a window-slices plan (R = 32) combines its own slice partials
// instead of leaving them to k_slice_combine.  Lagged arrival: a wave stores
// tile t's slice partials (sc1), and two tiles later — after the loads of the
// tiles in between have gone out — waits with a counted vmcnt that retires
// those stores but leaves the ring's younger loads in flight, then draws a
// ticket on tile t (agent-scope fetch_add); the ticket comes back while two
// more tiles stream, and the wave that drew the S-th ticket records the tile
// in its block's list.  After the stream (the ring's registers dead) the
// block's waves combine the listed tiles: one round of partial loads (lane
// l: row pair l % 16, slices s = q, q + 4, ... for q = l / 16), the same
// per-phase sums and 8-phase tree as k_slice_combine (so u has the same
// bits), beta_{j-1} from the norm partials with block 0's reduction order,
// u = w (t / beta), and the tile's u.q partial into aq[t] (ntiles partials:
// who combines a tile varies from run to run, so the alpha partials are per
// tile, not per block).  The tickets spread the wins evenly (one tile in S of
// every wave's), so each block combines ~ntiles / grid tiles at its end.
#ifndef KRCN_FOLD
#define KRCN_FOLD 0
#endif
#ifndef KRCN_FOLD_ABL
#define KRCN_FOLD_ABL 0
#endif
constexpr int kFoldPad = 32;   // ints per ticket counter (one cache line: 85 draws a line contend otherwise)
template <typename T> struct EpiSliceFold {
  T* part; int64_t ld;          // slice partials, as EpiSlicePart (stored sc1)
  int* cnt;                     // per tile: tickets drawn, one 128-byte line each (kFoldPad ints; the combiner resets it)
  int* won;                     // per block: ntiles slots, the tiles its waves won
  int* nwon;                    // the block's count of them (LDS)
  int ntiles;
  double* aq;                   // per tile: partial of u.(t / beta)
  const T* w; T* u;
  LzCtl<T> c;                   // beta_{j-1}: c.pnorm / c.Pnorm, c.tol, c.st
  int S;
  static constexpr bool kReduce = false;
  struct Pre {};
  template <class Src> __device__ __forceinline__ void init(const Src&) {}
  __device__ __forceinline__ Pre pre(int) const { return Pre{}; }
  __device__ __forceinline__ double row(int r, T s, int slice, const Pre&) const {
    __hip_atomic_store(part + int64_t(slice) * ld + r, s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return 0.0;
  }
};
template <class E> struct IsFoldEpi : std::false_type {};
template <typename T> struct IsFoldEpi<EpiSliceFold<T>> : std::true_type {};

// beta of lz_step_prologue(_pre) in block 0 of the launch, computed by one
// wave with the same bits: thread t of a kNT block holds sum_{i = t, t + kNT,
// ...} p[i]; each 64-thread group is butterfly-summed; (s0 + s1) + (s2 + s3).
template <typename T>
__device__ __forceinline__ double fold_beta(const LzCtl<T>& c, int lane) {
  double g[kNT / 64];
#pragma unroll
  for (int w = 0; w < kNT / 64; ++w) {
    double v = 0.0;
    for (int i = 64 * w + lane; i < c.Pnorm; i += kNT) v += c.pnorm[i];
    g[w] = wave_sum(v);
  }
  return sqrt((g[0] + g[1]) + (g[2] + g[3]));
}

struct WinFold {
  int t1 = -1, t2 = -1;   // tiles stored one / two finishes ago, not yet ticketed
  int a1 = -1, a2 = -1;   // tiles ticketed one / two finishes ago, not yet resolved
  int o1 = 0, o2 = 0;     // their tickets
  int bstate = 0;         // 0: beta not formed yet, 1: formed, 2: the recurrence has ended
  double beta = 0.0;
};

template <typename T, int R>
__device__ __forceinline__ void fold_combine(const EpiSliceFold<T>& e, WinFold& f, int t, int rows, int lane) {
  if constexpr (R != 32) {   // the host folds 32-row tiles only (16 row pairs x 4 slice phases)
    return;
  } else {
  if (f.bstate == 0) {
    const int done = e.c.j > 0 ? __hip_atomic_load(&e.c.st->done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
    f.beta = fold_beta(e.c, lane);
    f.bstate = (done || (e.c.j > 0 && fabs(f.beta) < e.c.tol)) ? 2 : 1;
  }
  const int r0 = t * R;
  if (f.bstate == 1) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");   // the other waves' partials (rare: one tile in S)
    const int p = lane & 15, q = lane >> 4;
    const int ra = r0 + 2 * p;
    const int rA = ra < rows ? ra : rows - 1, rB = ra + 1 < rows ? ra + 1 : rows - 1;   // clamped (in bounds)
    T w0 = T(0), w1 = T(0);
    if (q == 0) {
      w0 = e.w[rA];
      w1 = e.w[rB];
    }
    // phases q (slices q, q + 8, ...) and q + 4 (q + 4, q + 12, ...), each
    // left to right; slices q + 4 k in two rounds of kH loads per row
    constexpr int kH = 12;   // 2 x 12 rounds: S <= 96
    T v0a = T(0), v4a = T(0), v0b = T(0), v4b = T(0);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      T a0[kH], a1[kH];
#pragma unroll
      for (int k = 0; k < kH; ++k) {
        const int s = q + 4 * (h * kH + k);
        const T* pp = e.part + int64_t(s < e.S ? s : q) * e.ld;
        a0[k] = __hip_atomic_load(pp + rA, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        a1[k] = __hip_atomic_load(pp + rB, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
#pragma unroll
      for (int k = 0; k < kH; ++k)
        if (q + 4 * (h * kH + k) < e.S) {
          if (k % 2 == 0) { v0a += a0[k]; v0b += a1[k]; }   // (kH even: k's parity is (h kH + k)'s)
          else { v4a += a0[k]; v4b += a1[k]; }
        }
    }
    // the tree of k_slice_combine: (0+1), (2+3), (4+5), (6+7); then pairs; then the root
    const T n0a = __shfl_down(v0a, 16, 64), n4a = __shfl_down(v4a, 16, 64);
    const T n0b = __shfl_down(v0b, 16, 64), n4b = __shfl_down(v4b, 16, 64);
    const T l1a = v0a + n0a, l5a = v4a + n4a, l1b = v0b + n0b, l5b = v4b + n4b;   // q = 0: (0+1), (4+5); q = 2: (2+3), (6+7)
    const T m1a = __shfl_down(l1a, 32, 64), m5a = __shfl_down(l5a, 32, 64);
    const T m1b = __shfl_down(l1b, 32, 64), m5b = __shfl_down(l5b, 32, 64);
    const T sa = (l1a + m1a) + (l5a + m5a), sb = (l1b + m1b) + (l5b + m5b);
    double acc = 0.0;
    if (q == 0) {
      const T div = T(f.beta);
      if (ra < rows) {
        const T qa = sa / div, ua = w0 * qa;
        e.u[ra] = ua;
        acc += double(ua) * double(qa);
      }
      if (ra + 1 < rows) {
        const T qb = sb / div, ub = w1 * qb;
        e.u[ra + 1] = ub;
        acc += double(ub) * double(qb);
      }
    }
    acc = wave_sum(acc);
    if (lane == 0) e.aq[t] = acc;
  } else if (lane == 0) {
    e.aq[t] = 0.0;
  }
  if (lane == 0) __hip_atomic_store(e.cnt + int64_t(t) * kFoldPad, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// A tile this wave drew the last ticket of: into the block's list.
template <typename T>
__device__ __forceinline__ void fold_won(const EpiSliceFold<T>& e, int t, int lane) {
  if (lane == 0) {
    const int i = __hip_atomic_fetch_add(e.nwon, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    e.won[int64_t(blockIdx.x) * e.ntiles + i] = t;
  }
}

// After tile t's partials went out (its finish): resolve the ticket drawn two
// finishes ago, and draw the ticket of the tile stored two finishes ago once a
// counted vmcnt has retired its stores (>= 12 vector-memory operations of the
// two tiles since: row ends, chunk loads and stores; a conservative 8 leaves
// the younger chunk in flight).
template <typename T, int R>
__device__ __forceinline__ void fold_after(const EpiSliceFold<T>& e, WinFold& f, int t, int rows, int lane) {
  if (f.a2 >= 0 && __builtin_amdgcn_readfirstlane(f.o2) == e.S - 1) fold_won(e, f.a2, lane);
  f.a2 = f.a1;
  f.o2 = f.o1;
  f.a1 = -1;
  if (f.t2 >= 0) {
    __builtin_amdgcn_s_waitcnt(0x0f78);   // vmcnt(8)
    int o = 0;
#if KRCN_FOLD_ABL   // ablation (timing only, wrong results): the counted wait without the tickets
    if (lane == 0) o = f.t2 % 97 == 0 ? 0 : 1;
#else
    if (lane == 0) o = __hip_atomic_fetch_add(e.cnt + int64_t(f.t2) * kFoldPad, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#endif
    f.o1 = o;   // read (readfirstlane: lane 0's) only when resolved, two finishes later
    f.a1 = f.t2;
  }
  f.t2 = f.t1;
  f.t1 = t;
}

// End of the wave's tiles: retire every store, ticket the pending tiles,
// resolve every pending ticket.
template <typename T, int R>
__device__ __forceinline__ void fold_drain(const EpiSliceFold<T>& e, WinFold& f, int rows, int lane) {
  __builtin_amdgcn_s_waitcnt(0x0f70);   // vmcnt(0)
  int ta[4] = {f.a2, f.a1, f.t2, f.t1};
  int oa[4] = {f.o2, f.o1, 0, 0};
#pragma unroll
  for (int i = 2; i < 4; ++i)
    if (ta[i] >= 0) {
      int o = 0;
      if (lane == 0) o = __hip_atomic_fetch_add(e.cnt + int64_t(ta[i]) * kFoldPad, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      oa[i] = o;
    }
#pragma unroll
  for (int i = 0; i < 4; ++i)
    if (ta[i] >= 0 && __builtin_amdgcn_readfirstlane(oa[i]) == e.S - 1) fold_won(e, ta[i], lane);
  f = WinFold{};
}

// Tiles of one segment in flush mode (every tile's row sums go to the
// epilogue when final): a runtime loop over the wave's tiles t0 + wave + 16 k
// with a ring of kWinRing chunk slots — while tile k is consumed the row
// bounds / epilogue operands of tile k + 1 and the chunk of tile k + 2 are in
// flight, and the scalar bounds of tile k + 3 are loading.  The window (if
// the segment loads one) is stored into LDS after the first chunks are issued.
template <typename T, int R, class Epi>
__device__ __forceinline__ void win_stream(int segno, const WinSeg& sg, const WinArgs& a,
                                           const T (&tmp)[WinGeom<T>::kPer], bool store_win, int rot, T* win,
                                           T* slab, const Epi& epi, int wave, int lane,
                                           typename RedOf<Epi>::type& red, WinTiles tl) {
  const int rows = a.rows;
  const int* tb = a.tb + int64_t(sg.slice) * (a.ntiles + 1);
  const unsigned short* ro = a.ro + int64_t(sg.slice) * rows;
  const unsigned short* widx = a.widx;
  const T* wval = static_cast<const T*>(a.wval);
  const int tw = sg.t0 + wave;
  const int nt = sg.t1 - tw > 0 ? (sg.t1 - tw + kWinWaves - 1) / kWinWaves : 0;
  // tiles in batches of kWinBatch: the ring's look-ahead (5 tiles) stays
  // inside one 64-lane batch of tile bases; a new batch (past 58 tiles of a
  // wave, rare) restarts the ring behind its load
  const int nb = (nt + kWinBatch - 1) / kWinBatch;
  WinFold fold;   // (the slice-combine fold only: IsFoldEpi)
  if (nb == 0 && store_win) {   // a wave without tiles still takes part in the window store
    lds_block_barrier();
    win_store<T>(tmp, win, sg.slice, a, rot);
    lds_block_barrier();
  }
  for (int bi = 0; bi < nb; ++bi) {
    const int kb = bi * kWinBatch;
    const int kn = nt - kb < kWinBatch ? nt - kb : kWinBatch;
    if (bi > 0) tl.load(tb, tw, sg.t1, kb, lane);
    auto bounds = [&](TileB<R>& b, int k) {   // tile kb + k, k < 64 (no memory access)
      b.set(rows, tw + (kb + k) * kWinWaves, sg.t1, __builtin_amdgcn_readlane(tl.e0, k),
            __builtin_amdgcn_readlane(tl.e1, k));
    };
    TileB<R> B0, B1, B2;
    bounds(B0, 0);
    bounds(B1, 1);
    bounds(B2, 2);
    WinChunk<T> c0, c1, c2;
    RowRaw q0, q1, q2;
    typename Epi::Pre p0, p1, p2;
    auto rows_of = [&](const TileB<R>& b, RowRaw& q, typename Epi::Pre& pr) {
      q = tile_row_load<R>(b, ro, lane);
      const int r = b.r0 + lane;
      pr = epi.pre(r < rows ? r : rows - 1);
    };
    const bool sw = bi == 0 && store_win;
    // vmcnt retires in issue order: a tile's row ends go out BEFORE the
    // chunks that must stay in flight while it is consumed
#if KRCN_WIN_FIRST
    // the window's loads go out alone: chunk loads issued beside them would
    // share the CU's memory queue with it while every CU starts up at once
    if (sw) {
      lds_block_barrier();   // every wave is done with the previous window
      win_store<T>(tmp, win, sg.slice, a, rot);
    }
    rows_of(B0, q0, p0);
    win_load(c0, B0.e0, B0.e1, widx, wval, lane);
    win_load(c1, B1.e0, B1.e1, widx, wval, lane);
    if (sw) lds_block_barrier();
#else
    rows_of(B0, q0, p0);
    win_load(c0, B0.e0, B0.e1, widx, wval, lane);
    win_load(c1, B1.e0, B1.e1, widx, wval, lane);
    if (sw) {
      lds_block_barrier();   // every wave is done with the previous window
      win_store<T>(tmp, win, sg.slice, a, rot);
      lds_block_barrier();
    }
#endif
    if (segno < 4 && bi == 0) KRCN_WIN_STAMP(2 + 2 * segno);
    auto finish = [&](const WinChunk<T>& c, const TileB<R>& b, const RowRaw& q, const typename Epi::Pre& pr,
                      int k) {
      int bg, en;
      tile_row_bounds<R>(b, q, lane, bg, en);
      const bool coop = KRCN_WIN_COOP && a.S > 1;
      T s = win_consume(c, bg, en, win, slab, lane, T(0), coop);
      for (int cc = c.hi; cc < b.e1;) {          // tiles longer than one chunk
        WinChunk<T> cx;
        win_load(cx, cc, b.e1, widx, wval, lane);
        s = win_consume(cx, bg, en, win, slab, lane, s, coop);
        cc = cx.hi;
      }
      if (k < kn && lane < b.nr) red += epi.row(b.r0 + lane, s, sg.slice, pr);
      if constexpr (IsFoldEpi<Epi>::value)
        if (k < kn) fold_after<T, R>(epi, fold, b.r0 / R, rows, lane);
    };
    for (int k = 0; k < kn; k += 3) {
      TileB<R> B3;
      bounds(B3, k + 3);
      rows_of(B1, q1, p1);
      win_load(c2, B2.e0, B2.e1, widx, wval, lane);
      finish(c0, B0, q0, p0, k);
      TileB<R> B4;
      bounds(B4, k + 4);
      rows_of(B2, q2, p2);
      win_load(c0, B3.e0, B3.e1, widx, wval, lane);
      finish(c1, B1, q1, p1, k + 1);
      TileB<R> B5;
      bounds(B5, k + 5);
      rows_of(B3, q0, p0);
      win_load(c1, B4.e0, B4.e1, widx, wval, lane);
      finish(c2, B2, q2, p2, k + 2);
      B0 = B3;
      B1 = B4;
      B2 = B5;
    }
  }
  if constexpr (IsFoldEpi<Epi>::value) fold_drain<T, R>(epi, fold, rows, lane);
}

// Tiles of one segment in accumulate mode: at most kWinTMax tiles per wave,
// row sums carried in registers across the block's segments (slices), the
// epilogue after the last one (FLUSH).  Same ring as win_stream, unrolled.
template <typename T, int R, class Epi, bool FLUSH>
__device__ __forceinline__ void win_accum(int segno, const WinSeg& sg, const WinArgs& a, const T (&tmp)[WinGeom<T>::kPer],
                                          bool store_win, int rot, T* win, T* slab, const Epi& epi, int wave,
                                          int lane, T (&acc)[kWinTMax], typename RedOf<Epi>::type& red,
                                          const WinTiles& tl) {
  constexpr int K = kWinTMax;
  constexpr int D = kWinRingAccum;
  const int rows = a.rows;
  const int* tb = a.tb + int64_t(sg.slice) * (a.ntiles + 1);
  const unsigned short* ro = a.ro + int64_t(sg.slice) * rows;
  const unsigned short* widx = a.widx;
  const T* wval = static_cast<const T*>(a.wval);
  const int nt = sg.t1 - sg.t0 - wave > 0 ? (sg.t1 - sg.t0 - wave + kWinWaves - 1) / kWinWaves : 0;
  (void)tb;
  TileB<R> B[K];   // K <= 64: the whole segment from the batch (kb = 0)
#pragma unroll
  for (int k = 0; k < K; ++k)
    B[k].set(rows, sg.t0 + wave + k * kWinWaves, sg.t1, __builtin_amdgcn_readlane(tl.e0, k),
             __builtin_amdgcn_readlane(tl.e1, k));
  WinChunk<T> ring[D];
  RowRaw rq[D];
  typename Epi::Pre pre[D];
  auto issue_chunk = [&](auto kc) {
    constexpr int k = decltype(kc)::value;
    win_load(ring[k % D], B[k].e0, B[k].e1, widx, wval, lane);
  };
  auto issue_rows = [&](auto kc) {
    constexpr int k = decltype(kc)::value;
    rq[k % D] = tile_row_load<R>(B[k], ro, lane);
    if constexpr (FLUSH) {
      const int r = B[k].r0 + lane;
      pre[k % D] = epi.pre(r < rows ? r : rows - 1);
    }
  };
#if KRCN_WIN_FIRST
  if (store_win) {
    lds_block_barrier();
    win_store<T>(tmp, win, sg.slice, a, rot);
  }
  issue_rows(std::integral_constant<int, 0>{});
  issue_chunk(std::integral_constant<int, 0>{});
  if constexpr (K > 1 && D > 2) issue_chunk(std::integral_constant<int, 1>{});
  if (store_win) lds_block_barrier();
#else
  issue_rows(std::integral_constant<int, 0>{});
  issue_chunk(std::integral_constant<int, 0>{});
  if constexpr (K > 1 && D > 2) issue_chunk(std::integral_constant<int, 1>{});
  if (store_win) {
    lds_block_barrier();
    win_store<T>(tmp, win, sg.slice, a, rot);
    lds_block_barrier();
  }
#endif
  if (segno < 4) KRCN_WIN_STAMP(2 + 2 * segno);
  auto step = [&](auto kc) {
    constexpr int k = decltype(kc)::value;
    if constexpr (k + 1 < K) issue_rows(std::integral_constant<int, k + 1>{});
    if constexpr (k + D - 1 < K && D > 1) issue_chunk(std::integral_constant<int, k + D - 1>{});
    const WinChunk<T>& cur = ring[k % D];
    int bg, en;
    tile_row_bounds<R>(B[k], rq[k % D], lane, bg, en);
    T s = win_consume(cur, bg, en, win, slab, lane, acc[k]);
    for (int c = cur.hi; c < B[k].e1;) {
      WinChunk<T> cx;
      win_load(cx, c, B[k].e1, widx, wval, lane);
      s = win_consume(cx, bg, en, win, slab, lane, s);
      c = cx.hi;
    }
    if constexpr (FLUSH) {
      if (lane < B[k].nr) red += epi.row(B[k].r0 + lane, s, sg.slice, pre[k % D]);
      acc[k] = T(0);
    } else {
      acc[k] = s;
    }
  };
  unroll_while(std::make_integer_sequence<int, K>{}, nt, step);
}

// Pass 1 of a Lanczos step that also runs pass 2's X^T u (one-piece
// window-accum plans with per-block X^T copies, PassPlan::xt; w8a's d = 300).
// u_i = w_i (t_i / div) as EpiLz1, kept in LDS for the block's rows instead of
// stored.  The block's X^T copy is column-major with every column's run padded
// to whole chunks of 4 (pad rows 0xFFFF).  After the tiles, thread t sums chunk
// t (4 elements in row order) into LDS, and thread c then adds its column's
// chunks in order into part[block][c]: one global round trip (the chunk and
// the column's chunk range load together) and no serial walk down a long
// column.  k_xt_combine then adds the blocks in a fixed order and runs step A
// (EpiLz2): pass 2 never re-reads the matrix and has no launch of its own.
constexpr int kXtChunk = 4;
constexpr int kXtRowCap = kWinWaves * kWinTMax * 64;   // rows of one accumulate block (<= 96 tiles of <= 64)
constexpr unsigned short kXtPad = 0xFFFF;
template <typename T> struct XtGeom {
  static constexpr int kChunks = WinGeom<T>::kW - kWinNT - kXtRowCap;   // chunk sums in LDS past lu
};
template <typename T> struct EpiLz1X {
  const T* w; T div;
  const int* xcp;               // per block: cols + 1 absolute chunk ids (column c: [xcp[c], xcp[c+1]))
  const unsigned short* xrow;   // row - (block's first row) per element; kXtPad in a chunk's pad
  const T* xval;
  T* part;                      // grid x cols partials
  int cols;
  T* lu; int rbase;             // set by the kernel: u of the block's rows in LDS
  static constexpr bool kReduce = false;
  static constexpr bool kPreEarly = true;
  struct Pre { T wr; };
  template <class S> __device__ __forceinline__ void init(const S& src) { div = src.v.div; }
  __device__ __forceinline__ Pre pre(int r) const { return Pre{w[r]}; }
  __device__ __forceinline__ double row(int r, T s, int, const Pre& p) const {
    lu[r - rbase] = p.wr * (s / div);
    return 0.0;
  }
  __device__ __forceinline__ void xt(int b, T* tp) const {
    const int* cp = xcp + int64_t(b) * (cols + 1);
    const int c = threadIdx.x;
    const int cb = cp[0], ce = cp[cols];
    int c0 = 0, c1 = 0;
    if (c < cols) {
      c0 = cp[c];
      c1 = cp[c + 1];
    }
    for (int t = cb + int(threadIdx.x); t < ce; t += kWinNT) {
      T v[kXtChunk];
      Quad<T>::load(xval + int64_t(t) * kXtChunk, v);
      const u16x4 q = *reinterpret_cast<const u16x4*>(xrow + int64_t(t) * kXtChunk);
      const unsigned short rr[kXtChunk] = {q.x, q.y, q.z, q.w};
      T s = T(0);
#pragma unroll
      for (int i = 0; i < kXtChunk; ++i) {
        const T pr = v[i] * lu[rr[i] != kXtPad ? rr[i] : 0];
        if (rr[i] != kXtPad) s += pr;
      }
      tp[t - cb] = s;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
    if (c < cols) {
      T s = T(0);
      for (int k = c0; k < c1; ++k) s += tp[k - cb];
      part[int64_t(b) * cols + c] = s;
    }
  }
};
template <class E> struct IsEpiXt : std::false_type {};
template <typename T> struct IsEpiXt<EpiLz1X<T>> : std::true_type {};

// Source of a Lanczos pass 1 with step B of the previous step fused into the
// window load (slices mode; krcn_api.hip lanczos_impl):
//   j = 0:  the window is g (cubic.py:85);
//   j >= 1: alpha_{j-1} = sum of pass 2's partials of v_{j-1}.w (every block,
//           fixed order; block 0 records alphas[j-1]), and the window is
//           z_j = w - alpha_{j-1} v_{j-1} (cubic.py:94-96, the expression of
//           k_lz_step_b); the blocks of each slice share the store of
//           their slice of z_j (unnormalised) into V[j], each writing the
//           partial of ||z_j||^2 of its share to pz[block].  The slice
//           combine then settles beta_{j-1} from pz (lz_step_prologue) and
//           normalises u by it.
// SrcLzZ / IsLzZ: krcn_tiled.hpp (the sorted pass fuses step B too).

// The window pass.  Block b runs its segments segs[b * stride + i]; the first
// segment and its window loads are issued before the source prologue (whose
// reductions / state reads then overlap them).
template <typename T, int R, class Src, class Epi, bool kAccum>
__global__ __launch_bounds__(kWinNT, 1) void k_window_pass(WinArgs a, Src src, Epi epi,
                                                           double* __restrict__ partials) {
  constexpr int kPer = WinGeom<T>::kPer;
  __shared__ double sm[kWinNT / 64];
  __shared__ T win[WinGeom<T>::kW];
  __shared__ T slab_all[kWinWaves][kWinChunk];
  __shared__ int fold_n;   // (the slice-combine fold: tiles won by the block)
  if constexpr (IsFoldEpi<Epi>::value) {
    if (threadIdx.x == 0) fold_n = 0;   // (ordered before every use by the window barriers)
    epi.nwon = &fold_n;
  }
  KRCN_WIN_STAMP(0);
  const WinSeg* bsegs = a.segs + int64_t(blockIdx.x) * a.stride;
  WinSeg sg = bsegs[0];
  const int nseg = sg.flags >> 8;
  const int rot = int((blockIdx.x >> 3) % kPer);
  // Slices mode: block b = slice + S c, so the window fetch goes out without
  // waiting for the segment (the tile bases follow it); accumulate mode: the
  // first segment's tile bases go out before the window fetch, whose wait
  // then does not hold the window burst.
  int slice0 = sg.slice, chunk0 = 0;
  if constexpr (!kAccum) win_block_slice(int(blockIdx.x), int(gridDim.x), a.S, a.kpb, slice0, chunk0);
  WinTiles tl;
  if constexpr (kAccum)
    tl.load(a.tb + int64_t(sg.slice) * (a.ntiles + 1), sg.t0 + __builtin_amdgcn_readfirstlane(int(threadIdx.x) >> 6),
            sg.t1, 0, int(threadIdx.x) & 63);
  T tmp[kPer];
  const T* x = nullptr;
  if constexpr (IsLzZ<Src>::value) {
    const int j = src.c.j;
    T tv[kPer];
    // The prologue's own operands (the state flag, pass 2's v.w partials) are
    // loaded BEFORE the two window fetches: loads retire in issue order, so
    // waiting for them then leaves the 2 x 85 KB window burst in flight while
    // alpha is reduced (issued after the burst, the flag's wait drained it).
    const bool early = src.Pa <= kNT;
    int flag = 0;
    double pv = 0.0;
    if (j > 0 && early) {
      if (threadIdx.x == 0) flag = __hip_atomic_load(&src.c.st->done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (threadIdx.x < src.Pa) pv = src.pa[threadIdx.x];
    }
    win_fetch<T>(tmp, j == 0 ? src.c.g : src.Wv, slice0, a, rot);
    if (j > 0) win_fetch<T>(tv, src.c.V + int64_t(j - 1) * src.c.ld, slice0, a, rot);
    if (j > 0 && early) {
      __shared__ int flag_sm;
      if (threadIdx.x == 0) flag_sm = flag;
      __syncthreads();
      const int done = flag_sm;
      __syncthreads();
      if (done) return;
      // = sum_partials(pa, Pa): one partial per thread, then the fixed tree
      const double al = block_sum(threadIdx.x < kNT ? 0.0 + pv : 0.0, sm);
      if (blockIdx.x == 0 && threadIdx.x == 0) src.alphas[j - 1] = al;
      src.alpha = T(al);
    } else if (src.begin(sm)) {
      return;
    }
    if (j > 0) {
      const int64_t wbase = int64_t(slice0) * a.W;
      const int len = a.cols - wbase < a.W ? int(a.cols - wbase) : a.W;
      const T ta = src.alpha;
#pragma unroll
      for (int k = 0; k < kPer; ++k) tmp[k] = tmp[k] - ta * tv[k];
      // the slice's kpb blocks (win_block_slice) share the store of z_j to
      // V[j] and its ||z_j||^2: block c takes the 1024-entry pieces q with
      // q % kpb == c; its partial lands in pz[b] (all blocks, fixed order)
      const int kpb = a.kpb ? a.kpb : int(gridDim.x) / a.S, cb = chunk0;
      T* z = src.c.V + int64_t(j) * src.c.ld + wbase;
      double nrm = 0.0;
#pragma unroll
      for (int k = 0; k < kPer; ++k) {
        const int q = k + rot < kPer ? k + rot : k + rot - kPer;
        const int i = threadIdx.x + kWinNT * q;
        if (q % kpb == cb && i < len) {
          if (src.store_z) store_policy<KRCN_VEC_ST>(z + i, tmp[k]);
          nrm += double(tmp[k]) * double(tmp[k]);
        }
      }
      const double bs = block_sum_nt<kWinNT>(nrm, sm);
      if (threadIdx.x == 0) src.pz[blockIdx.x] = bs;
    }
  } else if constexpr (IsLzSmall<Src>::value) {
    const int j = src.c.j;
    const int t = threadIdx.x;
    const int64_t d = src.c.ld;
    const bool in = t < d;
    const int tc = in ? t : 0;
    const T wv = (j == 0 ? src.c.g : src.Wv)[tc];
    const T vv = j == 0 ? T(0) : (src.c.V + int64_t(j - 1) * d)[tc];
    double al = 0.0;
    if (j > 0 && flag_and_sum(&src.c.st->done, src.pa, src.Pa, sm, &al)) return;
    const T zi = j == 0 ? wv : wv - T(al) * vv;   // the expression of k_lz_step_b
    const double nrm = sqrt(block_sum_nt<kWinNT>(in ? double(zi) * double(zi) : 0.0, sm));
    const bool lead = blockIdx.x == 0 && t == 0;
    if (j == 0) {
      if (lead) { src.c.st->done = 0; src.c.st->j_break = -1; src.c.st->gnorm = nrm; src.c.st->beta_last = 0.0; }
    } else {
      if (lead) src.alphas[j - 1] = al;
      if (fabs(nrm) < src.c.tol) {
        if (lead) { src.c.st->j_break = j - 1; src.c.st->beta_last = nrm; src.c.st->done = 1; }
        return;
      }
      if (lead) { src.c.betas[j - 1] = nrm; src.c.st->beta_last = nrm; }
      if (blockIdx.x == 0 && in) src.c.V[int64_t(j) * d + t] = zi;   // unnormalised; pass 2 divides in place
    }
    src.v = LzVec<T>{j == 0 ? src.c.g : src.c.V + int64_t(j) * d, T(nrm), j, 1};
#pragma unroll
    for (int k = 0; k < kPer; ++k) tmp[k] = (k + rot) % kPer == 0 ? zi : T(0);   // piece 0 holds all of z
  } else {
    if constexpr (HasPreload<Src>::value) src.preload();   // the prologue's operands before the window burst
    const T* xe = src.early();
    win_fetch<T>(tmp, xe, slice0, a, rot);
    if (src.begin(sm)) return;
    x = src.get();
    if (x != xe) win_fetch<T>(tmp, x, slice0, a, rot);   // the early guess was wrong (truncated Lanczos)
  }
  KRCN_WIN_STAMP(1);
  if constexpr (!kAccum)   // after the window fetch: its wait comes with the window's
    tl.load(a.tb + int64_t(sg.slice) * (a.ntiles + 1), sg.t0 + __builtin_amdgcn_readfirstlane(int(threadIdx.x) >> 6),
            sg.t1, 0, int(threadIdx.x) & 63);
  epi.init(src);
  if constexpr (IsEpiXt<Epi>::value) {   // u of the block's rows past the one-piece window
    epi.lu = win + kWinNT;
    epi.rbase = sg.t0 * R;
  }
  // wave index made explicitly uniform: tile bounds then live in SGPRs
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  T* slab = slab_all[wave];
  typename RedOf<Epi>::type red{};
  T acc[kWinTMax];
#pragma unroll
  for (int k = 0; k < kWinTMax; ++k) acc[k] = T(0);
  for (int si = 0; si < nseg; ++si) {
    bool store_win = si == 0;
    if (si > 0) {
      sg = bsegs[si];
      tl.load(a.tb + int64_t(sg.slice) * (a.ntiles + 1), sg.t0 + wave, sg.t1, 0, lane);   // before the window
      if (sg.flags & kSegLoad) {
        win_fetch<T>(tmp, x, sg.slice, a, rot);
        store_win = true;
      }
    }
    if constexpr (kAccum) {
      if (sg.flags & kSegFlush)
        win_accum<T, R, Epi, true>(si, sg, a, tmp, store_win, rot, win, slab, epi, wave, lane, acc, red, tl);
      else
        win_accum<T, R, Epi, false>(si, sg, a, tmp, store_win, rot, win, slab, epi, wave, lane, acc, red, tl);
    } else {
      win_stream<T, R, Epi>(si, sg, a, tmp, store_win, rot, win, slab, epi, wave, lane, red, tl);
    }
    if (si < 4) KRCN_WIN_STAMP(3 + 2 * si);
  }
  KRCN_WIN_WAVE_STAMP(16 + wave);
  if constexpr (IsEpiXt<Epi>::value) {
    lds_block_barrier();   // every row's u is in LDS
    epi.xt(int(blockIdx.x), win + kWinNT + kXtRowCap);
  }
  if constexpr (IsFoldEpi<Epi>::value) {
    __syncthreads();   // every wave has drained its stream and recorded its wins
    const int nw = fold_n;
    WinFold f;
    for (int i = wave; i < nw; i += kWinWaves)
      fold_combine<T, R>(epi, f, epi.won[int64_t(blockIdx.x) * epi.ntiles + i], a.rows, lane);
  }
  if constexpr (Epi::kReduce) store_block_red<kWinNT>(red, sm, partials, epi);
  KRCN_WIN_STAMP(10);
}

// Compact row pointers: tb[s (ntiles + 1) + t] = ptr[s rows + t R] (the tile
// bases; entry ntiles = the slice end) and ro[s rows + r] = ptr[s rows + r + 1]
// - (base of r's tile), 16 bits (the plan checks every tile fits).
[[maybe_unused]] static __global__ __launch_bounds__(kNT) void k_compact_rows(int S, int rows, int R, int ntiles,
                                                      const int* __restrict__ ptr, int* __restrict__ tb,
                                                      unsigned short* __restrict__ ro) {
  const int64_t total = int64_t(S) * rows;
  for (int64_t i = int64_t(blockIdx.x) * kNT + threadIdx.x; i < total; i += int64_t(gridDim.x) * kNT) {
    const int sl = int(i / rows), r = int(i % rows);
    const int t = r / R;
    const int base = ptr[int64_t(sl) * rows + int64_t(t) * R];
    ro[i] = static_cast<unsigned short>(ptr[i + 1] - base);
    if (r % R == 0) tb[int64_t(sl) * (ntiles + 1) + t] = base;
    if (r == rows - 1) tb[int64_t(sl) * (ntiles + 1) + ntiles] = ptr[int64_t(sl) * rows + rows];
  }
}

// 16-bit slice-local offsets of a uniformly sliced CSR (slice width W).
[[maybe_unused]] static __global__ __launch_bounds__(kNT) void k_local_u16(int64_t nnz, const int* __restrict__ idx, int W,
                                                   unsigned short* __restrict__ out) {
  for (int64_t e = int64_t(blockIdx.x) * kNT + threadIdx.x; e < nnz; e += int64_t(gridDim.x) * kNT)
    out[e] = static_cast<unsigned short>(idx[e] % W);
}

}  // namespace krcn
