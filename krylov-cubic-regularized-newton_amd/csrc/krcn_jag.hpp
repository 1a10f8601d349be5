// krcn_jag.hpp — jagged lane-per-row SpMV passes over a whole-LDS window.
//
// Why (DESIGN.md §3 "Jagged passes"): the tile formats of krcn_window.hpp stage
// each chunk's products in a per-wave LDS slab (32 KiB of slabs per CU) and
// hand every row to one lane that walks the slab.  When each lane OWNS a row
// and loads that row's elements itself, no slab is needed: the whole 160 KiB
// of LDS holds the gathered vector.  That buys two shapes:
//   * single window (S = 1): a vector of up to 20,448 fp64 entries sits in LDS
//     whole — news20's X^T u gathers from all of u (19,996 entries) with no
//     window switch inside the pass (the tile format needs two);
//   * accumulate (S > 1): two windows of 10,224 entries; the block owns a row
//     range for the whole pass and walks every column slice over it, loading
//     slice s + 1's window into registers while slice s is gathered — row sums
//     stay in registers, so there are no slice partials at all (synth: the
//     window-slices format wrote and re-read ~1 GB of partials per pass).
//
// Format (built by krcn_plan.hip build_jag):
//  * rows are cut into groups of 64 (lane l of a wave owns row 64 g + l);
//    block b owns groups [gcut[b], gcut[b+1]) (nonzero-balanced cuts), and
//    its wave w the groups gcut[b] + w + 16 i, i < K;
//  * columns are cut into S slices of W entries (slice bases 16-byte aligned);
//  * a UNIT is (block, slice, i, wave): one group restricted to one slice,
//    uid = ((b S + s) K + i) 16 + w.  Per unit: the count of every lane's
//    elements in the slice (4 or 8 bits; the K counts of a lane for one
//    (block, slice, wave) share one word, so one load fetches them all), the
//    position of its first element and its element count (umeta: per
//    (block, slice, wave) the K bases then the K sizes, one load);
//  * single window: a unit's elements are stored in PAIR-LEVEL order: pair
//    level q holds elements 2q and 2q + 1 (CSR order) of every lane with
//    count > 2q, in lane order, two slots a lane (odd counts padded with a
//    zero).  Lane l finds its pair q at base + 2 (pairs of levels < q) +
//    2 popcount(ballot(count > 2q) below l) — from its own count, with no
//    further metadata — and loads it with one 16-byte value load and one
//    4-byte offset load;
//  * accumulate: a unit's elements are row-major (lane 0's, lane 1's, ...),
//    padded to an even count (see k_jag_acc);
//  * elements: 16-bit slice-local column offsets + values (10 B / nonzero,
//    plus the pads).
//
// Pipeline: a wave's work is a fixed sequence of chunks (unit i, levels
// ch LC .. + LC) — K x CPG per slice, unrolled — and the loads of chunk q + 1
// are in flight while chunk q is gathered and summed; the counts, bases and
// the next window of slice s + 1 are loaded at the start of slice s.  All of
// it goes through the vector memory counter (bases are read by a vector load
// and broadcast), so the compiler's waits stay partial (a scalar load would be
// waited for by every LDS gather).  Levels past CPG x LC run in an
// overflow loop one chunk ahead.
//
// Summation order: each row's elements left to right in CSR order, slices in
// order — for column-sorted rows exactly scipy's csr_matvec / csc_matvec order
// (one lane per row, separate multiply and add: -ffp-contract=off), so a jag
// pass is bit-identical to scipy.  Deterministic, no atomics.
#pragma once
#include "krcn_window.hpp"

namespace krcn {

#ifndef KRCN_JAG_EARLY
#define KRCN_JAG_EARLY 1   // single-window pass: the first chunk goes out with the window fetch
#endif
constexpr int kJagNT = 1024;                     // one block per CU: the window takes the LDS
constexpr int kJagWaves = kJagNT / 64;
constexpr int kJagLdsBytes = 163840 - 256;       // window(s); 256 B stay for the block reduction
constexpr int kJagPieces = kJagLdsBytes / 16;    // 16-byte pieces of window: 10,224
constexpr int kJagSlab = 128;                    // accumulate mode: elements per unit (products slab)
constexpr int kJagPad = 2 * kJagSlab;            // element arrays' padding (unit loads past the end)

// Variants (host and device agree through these):
//   single window (k_jag_pass): K <= 6 groups per wave, 2 chunks of 8 levels,
//                               8-bit counts
//   accumulate (k_jag_acc):     K = 4 or 8 groups per wave, <= 128 elements
//                               per unit, 8-bit counts
#ifndef KRCN_JAG_CPG
#define KRCN_JAG_CPG 2   // static chunks per unit of K >= 3 plans (A/B: variant builds)
#endif
constexpr int kJagK1 = 6, kJagCPG1 = KRCN_JAG_CPG, kJagLC = 8;
// the first kJagCPGU chunks of a unit are loaded whatever its counts; later
// static chunks only when some lane of the wave has levels there (a wave-
// uniform test).  Measured (round 6, -DKRCN_JAG_CPG=3): news20's X^T rows
// (Poisson, mean 6.7) pass 16 levels in 3.9 % of the 64-row groups, so most
// blocks wait for one synchronous overflow round trip — but a third static
// chunk makes the fused Lanczos pass 2 spill 44 B and run 27.9 -> 38.9 us
// (profiles/r06ag_news20_cpg3_ab.txt); the default stays 2
constexpr int kJagCPGU = 2;
// K <= 2 plans (rcv1's X^T: rows to 60 levels) keep 2 static chunks and run
// the overflow one chunk ahead instead (a third static chunk would spill)
constexpr int jag_cpg(int K) { return K <= 2 ? 2 : kJagCPG1; }
constexpr int kJagK2 = 8;                        // largest accumulate K (4 when the groups allow)
// Single window, long rows: rows with more than kJagLong elements leave the
// lane-per-row units (a 64-row group would wait for its longest row) and are
// summed by whole waves in tasks of kJagTask elements, <= kJagLongTasks tasks a
// block (their partials sit in LDS past the window).
constexpr int kJagLong = 32, kJagTask = 128, kJagLongTasks = 256;

template <typename T> struct JagGeom {
  static constexpr int kE = 16 / int(sizeof(T));                       // entries per piece
  static constexpr int kW1 = kJagPieces * kE;                          // single window (fp64 20,448)
  static constexpr int kR1 = (kJagPieces + kJagNT - 1) / kJagNT;       // piece loads per thread
  // accumulate: two windows beside the 16 per-wave product slabs
  static constexpr int kPieces2 = (kJagLdsBytes - kJagWaves * (kJagSlab + 2) * int(sizeof(T))) / 32;
  static constexpr int kW2 = kPieces2 * kE;                            // fp64 9,200; fp32 19,424
  static constexpr int kR2 = (kPieces2 + kJagNT - 1) / kJagNT;
  static_assert(kW1 <= 65536, "16-bit slice-local offsets");
};

struct JagArgs {
  int rows, S, W, G;                  // accumulate: S slices per group, G slice groups (block b: group b % G)
  int64_t cols;
  const int* gcut;                    // row range r: groups [gcut[r], gcut[r+1]) (block b: range b / G)
  const int* umeta;                   // per (block, slice, wave): K unit bases, then K unit sizes
  const void* cnt;                    // per (block, slice, wave): 64 lane count words
  const unsigned short* widx;
  const void* wval;
  // single window, long rows (nlong > 0): block b sums long rows [lcut[b],
  // lcut[b+1]) through tasks [tcut[b], tcut[b+1]); task t = (element start,
  // count) at task[2t]; row i's tasks are [ltask[i], ltask[i+1]); the task
  // partials go to LDS at window piece lpiece (past the window)
  int nlong = 0, lpiece = 0;
  int xmap = 0;                       // single window: row range of block b = jag_xcd_range(b) (see there)
  const int* lcut = nullptr;
  const int* tcut = nullptr;
  const int* lrow = nullptr;
  const int* ltask = nullptr;
  const int* task = nullptr;
  const unsigned short* lidx = nullptr;
  const void* lval = nullptr;
};

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

#ifndef KRCN_JAG_XMAP
#define KRCN_JAG_XMAP 1   // 0: block b takes row range b (A/B: variant builds)
#endif
// Row range of block b when the ranges are dealt XCD-packed: the dispatcher
// deals blocks to the 8 XCDs round-robin (b % 8), so XCD x gets the
// contiguous ranges [x q + min(x, r), ...) (q = G / 8, r = G % 8) instead of
// every eighth one.  A single-window pass over X^T stores its rows' slice of
// z_{j+1} (EpiLz2E) into the L2 of the XCD whose pass-1 blocks gather that
// slice into their windows (krcn_window.hpp win_block_slice deals slices the
// same way).  A bijection on [0, G); partials stay indexed by range.
__host__ __device__ inline int jag_xcd_range(int b, int G) {
  const int x = b % 8, q = G / 8, r = G % 8;
  return x * q + (x < r ? x : r) + b / 8;
}

// Window pieces: piece q covers entries [e0 + q kE, + kE) of x (length cols).
// Loads are unconditional; a piece reaching past the vector's end is loaded
// from cols - kE and shifted into place (entries past the end are junk the
// kernel never gathers).  Piece indices past `np` are clamped (duplicate loads,
// not stored).
template <typename T>
__device__ __forceinline__ u32x4 jag_fetch1(const T* __restrict__ x, int64_t e0, int64_t cols, int np, int k) {
  constexpr int kE = JagGeom<T>::kE;
  constexpr int kWPE = int(sizeof(T)) / 4;   // 32-bit words per entry
  int q = int(threadIdx.x) + kJagNT * k;
  q = q < np ? q : np - 1;
  const int64_t e = e0 + int64_t(q) * kE;
  const int64_t ec = e <= cols - kE ? e : cols - kE;
  u32x4 v = *reinterpret_cast<const u32x4*>(x + ec);
  const int sh = int(e - ec) * kWPE;      // 0 unless the piece crosses the end
  if (sh > 0) {   // selects only (a dynamically indexed array would go to scratch)
    const unsigned w1 = v.y, w2 = v.z, w3 = v.w;
    v.x = sh == 1 ? w1 : sh == 2 ? w2 : w3;
    v.y = sh == 1 ? w2 : w3;
    v.z = w3;
  }
  return v;
}

template <typename T, int R>
__device__ __forceinline__ void jag_fetch(u32x4 (&tmp)[R], const T* __restrict__ x, int64_t e0, int64_t cols,
                                          int np) {
#pragma unroll
  for (int k = 0; k < R; ++k) tmp[k] = jag_fetch1<T>(x, e0, cols, np, k);
}

template <int R>
__device__ __forceinline__ void jag_store1(const u32x4& v, u32x4* win, int np, int k) {
  const int q = int(threadIdx.x) + kJagNT * k;
  if (k + 1 < R || q < np) win[q] = v;
}

template <int R>
__device__ __forceinline__ void jag_store(const u32x4 (&tmp)[R], u32x4* win, int np) {
#pragma unroll
  for (int k = 0; k < R; ++k) jag_store1<R>(tmp[k], win, np, k);
}

// Element pairs of a unit as the single-window pass stores them (PAIR-LEVEL
// order): pair level q holds elements 2q and 2q + 1 (CSR order) of every lane
// with count > 2q, in lane order, two slots a lane (a lane with count 2q + 1
// has a zero pad in its second slot).  So lane l's pair q sits at
// base + 2 (pair slots of levels < q) + 2 popcount(ballot(count > 2q) below l)
// and comes in with ONE 16-byte value load and ONE 4-byte offset load: half
// the vector-memory instructions of one load per level (the pass is bound by
// the texture addresser's per-instruction cost, profiles/r03_pmc_news20.txt).
template <typename T> struct JagPair;
template <> struct JagPair<double> { typedef f64x2 type; };
template <> struct JagPair<float> { typedef float type __attribute__((ext_vector_type(2))); };
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

// One chunk of LC levels (LC / 2 pair levels) of a unit in flight (a lane's
// level k is live when its count exceeds k: recomputed at consumption).
template <typename T, int LC> struct JagChunk {
  static_assert(LC % 2 == 0, "whole pair levels");
  u16x2 o[LC / 2];
  typename JagPair<T>::type v[LC / 2];
};

// Positions of pair levels [k0 / 2, (k0 + LC) / 2) for this lane (count c)
// and their loads; `cum` (wave-uniform) advances past the chunk's slots.
// Inactive lanes load from `cum` (an address shared by the wave, in bounds:
// the arrays are padded).
template <typename T, int LC>
__device__ __forceinline__ void jag_issue(JagChunk<T, LC>& C, int c, int k0, int& cum, const JagArgs& a) {
  typedef typename JagPair<T>::type T2;
  const unsigned short* __restrict__ widx = a.widx;
  const T* __restrict__ wval = static_cast<const T*>(a.wval);
#pragma unroll
  for (int j = 0; j < LC / 2; ++j) {
    const bool act = c > k0 + 2 * j;
    const unsigned long long M = __ballot(act);
    const int below = int(__builtin_amdgcn_mbcnt_hi(unsigned(M >> 32), __builtin_amdgcn_mbcnt_lo(unsigned(M), 0u)));
    const int p = act ? cum + 2 * below : cum;
    cum += 2 * __popcll(M);
    C.o[j] = KRCN_STREAM_LOAD(reinterpret_cast<const u16x2*>(widx + p));
    C.v[j] = KRCN_STREAM_LOAD(reinterpret_cast<const T2*>(wval + p));
  }
}

// Levels k0 .. k0 + LC - 1 added left to right (the CSR order of the row).
template <typename T, int LC>
__device__ __forceinline__ T jag_consume(const JagChunk<T, LC>& C, int c, int k0, const T* win, T acc) {
#pragma unroll
  for (int j = 0; j < LC / 2; ++j) {
    const T p0 = C.v[j].x * win[C.o[j].x];
    acc = c > k0 + 2 * j ? acc + p0 : acc;
    const T p1 = C.v[j].y * win[C.o[j].y];
    acc = c > k0 + 2 * j + 1 ? acc + p1 : acc;
  }
  return acc;
}

// Lane count words: per (block, slice, wave) one word per lane holding the
// lane's count in each of the wave's K units, CB bits apiece (unit i at bit
// CB i): 32-bit words for 4-bit counts, 64-bit for 8-bit.
template <int CB> struct JagWord { typedef unsigned long long type; };

template <int CB, class W>
__device__ __forceinline__ int jag_count(W w, int i) {
  return int((w >> (CB * i)) & W((1u << CB) - 1u));
}

// Long rows of a single-window plan (see JagArgs): wave w of block b takes the
// block's tasks w, w + 16, ... (at most kJagLongTasks / 16 = 16), each 128
// elements of one row: lane l loads elements 2l, 2l + 1 with one 4-byte
// offset and one 16-byte value load (the next task's loads go out before this
// one is gathered), gathers x from the LDS window and the wave sums the
// products by a butterfly (every lane the same bits).  After a block barrier
// thread i adds its row's task partials in task order and runs the epilogue.
// Deterministic; not scipy's order for these rows (tolerance-level).
template <typename T> __device__ __forceinline__ T wave_sum_t(T v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}
#ifndef KRCN_JAG_LONG_EARLY
#define KRCN_JAG_LONG_EARLY 0   // 1: the first long-row task's loads go out before the units (A/B: variant builds;
// with news20's X^T rows past 16 sent to tasks, KRCN_JAG_LONG=16, pass 2 ran 27.9-28.5 us against the
// default's 27.4-27.8: profiles/r06ah_news20_long16_ab.txt)
#endif
template <typename T> struct JagLong {
  typedef typename JagPair<T>::type T2;
  int t0, t1, ntw, dp, dn;
  u16x2 oc;
  T2 vc;
  __device__ __forceinline__ void ld(const JagArgs& a, int j, u16x2& o, T2& v, int lane) const {
    const int p = __builtin_amdgcn_readlane(dp, j) + 2 * lane;
    o = *reinterpret_cast<const u16x2*>(a.lidx + p);
    v = *reinterpret_cast<const T2*>(static_cast<const T*>(a.lval) + p);
  }
  // this wave's task list (lane j < 16: task j's start and count)
  __device__ __forceinline__ void desc(const JagArgs& a, int b, int wave, int lane) {
    t0 = a.tcut[b];
    t1 = a.tcut[b + 1];
    ntw = t1 - t0 > wave ? (t1 - t0 - wave + kJagWaves - 1) / kJagWaves : 0;
    const int tj = t0 + wave + kJagWaves * (lane & 15);
    const int tc = tj < t1 ? tj : t0;
    dp = a.task[2 * tc];
    dn = tj < t1 ? a.task[2 * tc + 1] : 0;
  }
  // the first task's loads
  __device__ __forceinline__ void first(const JagArgs& a, int lane) { ld(a, 0, oc, vc, lane); }
};
template <typename T, class Epi>
__device__ __forceinline__ typename RedOf<Epi>::type jag_long_rows(const JagArgs& a, const Epi& epi, const T* win, T* lpart, int b,
                                                int wave, int lane, JagLong<T>& L) {
  typedef typename JagPair<T>::type T2;
  if (!KRCN_JAG_LONG_EARLY) {
    L.desc(a, b, wave, lane);
    L.first(a, lane);
  }
  const int t0 = L.t0;
  // (one task ahead: four ahead, built and measured in round 6, left
  // news20-skew's and rcv1-skew's pass 2 unchanged, r06aj_skew_long_ahead_ab.txt)
  u16x2 oc = L.oc, on;
  T2 vc = L.vc, vn;
  for (int j = 0; j < L.ntw; ++j) {
    L.ld(a, j + 1 < 16 ? j + 1 : 15, on, vn, lane);   // unconditional (in bounds): the next task's loads in flight
    const int n = __builtin_amdgcn_readlane(L.dn, j);
    const T p0 = 2 * lane < n ? vc.x * win[oc.x] : T(0);
    const T p1 = 2 * lane + 1 < n ? vc.y * win[oc.y] : T(0);
    const T s = wave_sum_t<T>(p0 + p1);
    if (lane == 0) lpart[wave + kJagWaves * j] = s;
    oc = on;
    vc = vn;
  }
  __syncthreads();
  typename RedOf<Epi>::type red{};
  for (int i = a.lcut[b] + int(threadIdx.x); i < a.lcut[b + 1]; i += kJagNT) {
    const int r = a.lrow[i];
    const typename Epi::Pre pr = epi.pre(r);
    T s = T(0);
    for (int q = a.ltask[i]; q < a.ltask[i + 1]; ++q) s += lpart[q - t0];
    red += epi.row(r, s, 0, pr);
  }
  return red;
}

#ifdef KRCN_WIN_TIMING
// Diagnostic builds: the single-window pass stamps table 1 of the window
// passes' stamp array (tools/win_timeline.py): [0] entry, [1] after the source
// prologue, [2] window in LDS, [3] units done, [10] end, [16 + w] wave w done.
#define KRCN_JAG_STAMP(slot)                                                                             \
  do {                                                                                                 \
    if (threadIdx.x == 0 && blockIdx.x < 2048)                                                         \
      krcn_win_dbg[2048 * kWinDbgSlots + blockIdx.x * kWinDbgSlots + (slot)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#define KRCN_JAG_WAVE_STAMP(slot)                                                                        \
  do {                                                                                                 \
    if ((threadIdx.x & 63) == 0 && blockIdx.x < 2048)                                                  \
      krcn_win_dbg[2048 * kWinDbgSlots + blockIdx.x * kWinDbgSlots + (slot)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define KRCN_JAG_STAMP(slot) do {} while (0)
#define KRCN_JAG_WAVE_STAMP(slot) do {} while (0)
#endif

// End-of-pass reduction of a two-sum epilogue (Red2) with one barrier pair:
// once every wave is done with the window (first barrier) its LDS holds the
// 2 x 16 wave sums; the same pairwise tree over the waves as block_sum_nt,
// so the same bits as two store_block_red sums (which take two pairs).
template <class Epi>
__device__ __forceinline__ void jag_block_red(const Red2& v, double* ws, double*, double* partials, const Epi& epi,
                                              int pb) {
  const double a = wave_sum(v.a), b = wave_sum(v.b);
  const int w = int(threadIdx.x) >> 6;
  __syncthreads();   // every wave is done with the window it now overwrites
  if ((threadIdx.x & 63) == 0) {
    ws[w] = a;
    ws[kJagWaves + w] = b;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double ra[kJagWaves], rb[kJagWaves];
#pragma unroll
    for (int i = 0; i < kJagWaves; ++i) {
      ra[i] = ws[i];
      rb[i] = ws[kJagWaves + i];
    }
#pragma unroll
    for (int h = kJagWaves / 2; h > 0; h >>= 1)
#pragma unroll
      for (int i = 0; i < h; ++i) {
        ra[i] = ra[2 * i] + ra[2 * i + 1];
        rb[i] = rb[2 * i] + rb[2 * i + 1];
      }
    partials[pb] = ra[0];
    epi.part2[pb] = rb[0];
  }
}
template <class Epi>
__device__ __forceinline__ void jag_block_red(double v, double*, double* sm, double* partials, const Epi&, int pb) {
  const double t = block_sum_nt<kJagNT>(v, sm);   // = store_block_red, at the range's index
  if (threadIdx.x == 0) partials[pb] = t;
}

// The single-window jagged pass (S == 1): the vector in LDS whole, each unit
// flushed to the epilogue as soon as it is summed.
template <typename T, int K, int CPG, int CB, class Src, class Epi>
__global__ __launch_bounds__(kJagNT, 1) void k_jag_pass(JagArgs a, Src src, Epi epi, double* __restrict__ partials) {
  constexpr int LC = kJagLC;
  constexpr int Q = K * CPG;                 // chunks per wave
  constexpr int R = JagGeom<T>::kR1;
  constexpr int NP = kJagPieces;
  __shared__ double sm[kJagWaves];
  __shared__ u32x4 win_raw[kJagPieces];
  __shared__ double split_ls[8];   // a split source's wave sums (IsSplitSrc)
  __shared__ int split_lf;
  KRCN_JAG_STAMP(0);
  const int b = a.xmap ? jag_xcd_range(int(blockIdx.x), int(gridDim.x)) : int(blockIdx.x);
  const int g0 = a.gcut[b], g1 = a.gcut[b + 1];   // both before the window burst (waited for with it)
  const int wave = __builtin_amdgcn_readfirstlane(int(threadIdx.x) >> 6), lane = int(threadIdx.x) & 63;
  typedef typename JagWord<CB>::type CW;
  static_assert(CB * K <= int(8 * sizeof(CW)), "lane counts of K units must fit one word");
  // per-slice unit metadata of this wave: one count word per lane, and the K
  // bases (one load, lane i holds unit i's)
  auto load_counts = [&](int s, CW& cw, int& bvec) {
    const int64_t rec = (int64_t(b) * a.S + s) * kJagWaves + wave;
    cw = reinterpret_cast<const CW*>(a.cnt)[rec * 64 + lane];
    bvec = a.umeta[rec * 2 * K + (lane < 2 * K ? lane : 0)];
  };
  u32x4 tmp[R];
  CW cw;
  int bvec;
  load_counts(0, cw, bvec);
  if constexpr (HasPreload<Src>::value) src.preload();   // the prologue's operands before the window burst
  const T* xe = src.early();
  jag_fetch<T, R>(tmp, xe, 0, a.cols, NP);
  // long-row tasks: the descriptors behind the window burst, the first task's
  // loads before the units (KRCN_JAG_LONG_EARLY) or after them
  JagLong<T> jl;
  if (KRCN_JAG_LONG_EARLY && a.nlong > 0) jl.desc(a, b, wave, lane);
  // a count byte of 0xFF marks a long row (summed below, not in the units):
  // its lane counts 0 in the units and skips the unit epilogue (formed after
  // the window fetch is issued: the counts' wait then leaves the burst in flight)
  CW skipw;
  {
    const CW x = ~cw, lo7 = CW(0x7F7F7F7F7F7F7F7Full);
    skipw = ~(((x & lo7) + lo7) | x) & CW(0x8080808080808080ull);   // 0x80 in the bytes where cw is 0xFF
    cw &= ~((skipw >> 7) * CW(0xFF));
  }
  int cum[K];   // per unit: position of its next level (wave-uniform)
  auto decode = [&](int bv) {
#pragma unroll
    for (int i = 0; i < K; ++i) cum[i] = __builtin_amdgcn_readlane(bv, i);
  };
  JagChunk<T, LC> C[2];
#if KRCN_JAG_EARLY
  // the first chunk does not depend on the source: it streams in behind the
  // window fetch (the counts were loaded before it, so waiting for them does
  // not drain the window burst)
  decode(bvec);
  jag_issue<T, LC>(C[0], jag_count<CB>(cw, 0), 0, cum[0], a);
#endif
  bool split = false;
  if constexpr (IsSplitSrc<Src>::value) split = src.pre_ok;
  if (split) {
    if constexpr (IsSplitSrc<Src>::value) src.begin_split(split_ls, &split_lf);   // finished after the window barrier
  } else if (src.begin(sm)) {
    return;
  }
  KRCN_JAG_STAMP(1);
  const T* x = src.get();
  if (x != xe) jag_fetch<T, R>(tmp, x, 0, a.cols, NP);   // the early guess was wrong (truncated Lanczos)
  if constexpr (IsLzU<Src>::value) {   // u = u' / beta (pieces past the vector are never gathered)
    const T dv = src.v.div;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      T e[16 / sizeof(T)];
      __builtin_memcpy(e, &tmp[r], 16);
#pragma unroll
      for (int q = 0; q < int(16 / sizeof(T)); ++q) e[q] = e[q] / dv;
      __builtin_memcpy(&tmp[r], e, 16);
    }
  }
  jag_store<R>(tmp, win_raw, NP);
  lds_block_barrier();
  if constexpr (IsSplitSrc<Src>::value)
    if (split && src.after_split(split_ls, &split_lf)) return;
  KRCN_JAG_STAMP(2);
  epi.init(src);
  typename RedOf<Epi>::type red{};
#if !KRCN_JAG_EARLY
  decode(bvec);
  jag_issue<T, LC>(C[0], jag_count<CB>(cw, 0), 0, cum[0], a);
#endif
  // levels past the static chunks.  Plans of K <= 2 units a wave (rcv1's
  // X^T: 33-60-element rows past the 16 static levels, 2-6 chunks a wave)
  // pipeline them one chunk ahead, the first issued before the unit's last
  // static chunk is consumed (round 6; they used to be loaded and summed one
  // chunk at a time, a memory round trip each).  K >= 3 (news20's X^T, whose
  // rows past 32 go to the long-row tasks) keeps the synchronous loop: its
  // two more chunks would spill.  Same levels, same order: the bits do not
  // change.
  constexpr bool kOvfPipe = K <= 2;
  JagChunk<T, LC> X0, X1;
  auto overflow_issue = [&](int i) {
    if constexpr (!kOvfPipe) return true;
    const int c = jag_count<CB>(cw, i);
    const bool any = __ballot(c > CPG * LC) != 0ull;
    if (any) jag_issue<T, LC>(X0, c, CPG * LC, cum[i], a);
    return any;
  };
  auto overflow = [&](int i, const T* win, T acc) {
    const int c = jag_count<CB>(cw, i);
    int k0 = CPG * LC;
    if constexpr (!kOvfPipe) {
      while (__ballot(c > k0) != 0ull) {
        jag_issue<T, LC>(X0, c, k0, cum[i], a);
        acc = jag_consume<T, LC>(X0, c, k0, win, acc);
        k0 += LC;
      }
      return acc;
    }
    for (;;) {
      const bool m1 = __ballot(c > k0 + LC) != 0ull;
      if (m1) jag_issue<T, LC>(X1, c, k0 + LC, cum[i], a);
      acc = jag_consume<T, LC>(X0, c, k0, win, acc);
      k0 += LC;
      if (!m1) break;
      const bool m2 = __ballot(c > k0 + LC) != 0ull;
      if (m2) jag_issue<T, LC>(X0, c, k0 + LC, cum[i], a);
      acc = jag_consume<T, LC>(X1, c, k0, win, acc);
      k0 += LC;
      if (!m2) break;
    }
    return acc;
  };

  if (KRCN_JAG_LONG_EARLY && a.nlong > 0) jl.first(a, lane);
  {
    const T* win = reinterpret_cast<const T*>(win_raw);
    const int Gb = g1 - g0;
    typename Epi::Pre pre[2];
    auto row_of = [&](int i) { return (g0 + wave + kJagWaves * i) * 64 + lane; };
    auto pre_of = [&](int i) {
      const int r = row_of(i);
      return epi.pre(r < a.rows ? r : a.rows - 1);
    };
    pre[0] = pre_of(0);
    T acc = T(0);
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const int i = q / CPG, ch = q % CPG;
      if (q + 1 < Q) {
        const int i1 = (q + 1) / CPG, ch1 = (q + 1) % CPG;
        const int c1 = jag_count<CB>(cw, i1);
        if (ch1 < kJagCPGU || __ballot(c1 > ch1 * LC) != 0ull) jag_issue<T, LC>(C[(q + 1) & 1], c1, ch1 * LC, cum[i1], a);
        if (ch1 == 0) pre[i1 & 1] = pre_of(i1);
      }
      const bool ovf = ch == CPG - 1 && overflow_issue(i);
      const int ci = jag_count<CB>(cw, i);
      if (ch < kJagCPGU || __ballot(ci > ch * LC) != 0ull) acc = jag_consume<T, LC>(C[q & 1], ci, ch * LC, win, acc);
      if (ch == CPG - 1) {
        if (ovf) acc = overflow(i, win, acc);
        const int r = row_of(i);
        const bool skip = (skipw >> (CB * i + CB - 1)) & 1;
        if (wave + kJagWaves * i < Gb && r < a.rows && !skip) red += epi.row(r, acc, 0, pre[i & 1]);
        acc = T(0);
      }
    }
    KRCN_JAG_WAVE_STAMP(16 + wave);
    KRCN_JAG_STAMP(3);
    if (a.nlong > 0) red += jag_long_rows<T, Epi>(a, epi, win, reinterpret_cast<T*>(win_raw + a.lpiece), b, wave, lane, jl);
  }
  if constexpr (Epi::kReduce) jag_block_red(red, reinterpret_cast<double*>(win_raw), sm, partials, epi, b);
  KRCN_JAG_STAMP(10);
}

// The accumulate jagged pass (S > 1): two windows, slice s + 1's streaming
// into the back one while slice s is gathered; wave w keeps the row sums of
// its K groups in registers across all slices.  A unit's elements are stored
// row-major (lane 0's, then lane 1's, ...; the unit padded to an even count)
// and loaded two per lane with one 16-byte value load and one 4-byte offset
// load, a whole slice ahead: unit (s + 1, i) is issued as soon as unit (s, i)
// is consumed.  The products go to the wave's slab; lane l then adds slab
// entries [rs, rs + count) with rs = the exclusive lane prefix of the counts
// (one ballot per count bit).  The plan guarantees <= 128 elements a unit.
// (Loads cost the texture addresser ~13 cycles per wave instruction whatever
// their width, and the pass is issue-bound: profiles/r02_pmc_synth.txt — so
// every element load moves 16 bytes a lane, the row starts come from one DPP
// scan per four units, and levels past a lane's count read a zero slot.)
template <typename T> struct JagUnit {
  u16x2 o;
  typename JagPair<T>::type v;
};

// Inclusive prefix sum over the 64 lanes of a wave (DPP: row shifts, then the
// row broadcasts of lanes 15 and 31).  Packed byte fields scan independently
// as long as no field's total exceeds 255.
__device__ __forceinline__ unsigned wave_incl_scan(unsigned v) {
  v += unsigned(__builtin_amdgcn_update_dpp(0, int(v), 0x111, 0xf, 0xf, true));   // row_shr:1
  v += unsigned(__builtin_amdgcn_update_dpp(0, int(v), 0x112, 0xf, 0xf, true));   // row_shr:2
  v += unsigned(__builtin_amdgcn_update_dpp(0, int(v), 0x114, 0xf, 0xf, true));   // row_shr:4
  v += unsigned(__builtin_amdgcn_update_dpp(0, int(v), 0x118, 0xf, 0xf, true));   // row_shr:8
  v += unsigned(__builtin_amdgcn_update_dpp(0, int(v), 0x142, 0xa, 0xf, false));  // row_bcast:15
  v += unsigned(__builtin_amdgcn_update_dpp(0, int(v), 0x143, 0xc, 0xf, false));  // row_bcast:31
  return v;
}

// Row starts of a lane in each unit of a slice: the exclusive lane prefix of
// its counts, four 8-bit units a word (a unit holds <= 128 elements).
template <int K, class CW>
__device__ __forceinline__ void jag_row_starts(const CW& cw, unsigned (&rs)[(K + 3) / 4]) {
#pragma unroll
  for (int h = 0; h < (K + 3) / 4; ++h) {
    const unsigned c4 = unsigned(cw >> (h ? 32 : 0));
    rs[h] = wave_incl_scan(c4) - c4;
  }
}

#ifndef KRCN_JAG_LAG
#define KRCN_JAG_LAG 1   // units between a window piece's fetch and its LDS store (A/B: variant builds)
#endif
template <typename T, int K, class Src, class Epi>
__global__ __launch_bounds__(kJagNT, 1) void k_jag_acc(JagArgs a, Src src, Epi epi, double* __restrict__ partials) {
  constexpr int R = JagGeom<T>::kR2;
  constexpr int NP = JagGeom<T>::kPieces2;
  constexpr int RPU = (R + K - 1) / K;    // window piece rounds fetched per unit
  constexpr int kZero = kJagSlab;          // a zero slot past every wave's slab
  // one 8-bit count per unit: a 32-bit word for K <= 4, 64-bit for K <= 8
  typedef typename std::conditional<K <= 4, unsigned, unsigned long long>::type CW;
  typedef typename JagPair<T>::type T2;
  static_assert(K <= 8, "lane counts of K units must fit one 64-bit word");
  __shared__ double sm[kJagWaves];
  __shared__ u32x4 win_raw[2 * NP];
  __shared__ T2 slab_all[kJagWaves][kJagSlab / 2 + 1];
  const int b = blockIdx.x;
  const int sg = b % a.G, rr = b / a.G;   // slice group (blocks of a group share an XCD when G | 8), row range
  const int g0 = a.gcut[rr], Gb = a.gcut[rr + 1] - g0;
  const int64_t wbase = int64_t(sg) * a.S * a.W;   // first column of the group
  const int wave = __builtin_amdgcn_readfirstlane(int(threadIdx.x) >> 6), lane = int(threadIdx.x) & 63;
  T2* slab2 = slab_all[wave];
  const T* slab = reinterpret_cast<const T*>(slab2);
  if (lane == 0) slab2[kJagSlab / 2] = T2{};   // the zero slot (never written again)
  const unsigned short* __restrict__ widx = a.widx;
  const T* __restrict__ wval = static_cast<const T*>(a.wval);
  // slice metadata (clamped to the last slice: loads stay unconditional)
  auto meta = [&](int s, CW& cw, int& bv) {
    s = s < a.S ? s : a.S - 1;
    const int64_t rec = (int64_t(b) * a.S + s) * kJagWaves + wave;
    cw = reinterpret_cast<const CW*>(a.cnt)[rec * 64 + lane];
    bv = a.umeta[rec * 2 * K + (lane < 2 * K ? lane : 0)];
  };
  // lanes past the unit's elements load its first pair (a line the wave
  // fetches anyway): no over-fetch
  auto issue = [&](JagUnit<T>& U, int i, int bv) {
    const unsigned e0 = unsigned(__builtin_amdgcn_readlane(bv, i));
    const int n = __builtin_amdgcn_readlane(bv, K + i);
    const unsigned p = 2 * lane < n ? e0 + 2u * unsigned(lane) : e0;
    U.o = KRCN_STREAM_LOAD(reinterpret_cast<const u16x2*>(widx + p));
    U.v = KRCN_STREAM_LOAD(reinterpret_cast<const T2*>(wval + p));
  };
  CW cw0, cw1;
  int bv0, bv1;
  meta(0, cw0, bv0);
  meta(1, cw1, bv1);
  JagUnit<T> U[K];
#pragma unroll
  for (int i = 0; i < K; ++i) issue(U[i], i, bv0);
  {
    u32x4 tmp[R];
    if constexpr (HasPreload<Src>::value) src.preload();
    const T* xe = src.early();
    jag_fetch<T, R>(tmp, xe, wbase, a.cols, NP);
    if (src.begin(sm)) return;
    const T* x0 = src.get();
    if (x0 != xe) jag_fetch<T, R>(tmp, x0, wbase, a.cols, NP);   // the early guess was wrong (truncated Lanczos)
    jag_store<R>(tmp, win_raw, NP);
  }
  const T* x = src.get();
  lds_block_barrier();
  epi.init(src);
  T acc[K];
#pragma unroll
  for (int i = 0; i < K; ++i) acc[i] = T(0);
  for (int s = 0; s < a.S; ++s) {
    const T* win = reinterpret_cast<const T*>(win_raw + (s & 1) * NP);
    u32x4* nwin = win_raw + ((s + 1) & 1) * NP;
    const bool more = s + 1 < a.S;
    const int64_t e1 = wbase + int64_t(more ? s + 1 : s) * a.W;
    CW cw2;
    int bv2;
    meta(s + 2, cw2, bv2);
    unsigned rsw[(K + 3) / 4];
    jag_row_starts<K, CW>(cw0, rsw);
    // slice s + 1's window pieces: unit i's round is fetched at unit i and
    // stored LAG units later (into the other LDS window), so LAG units of work
    // cover its latency
    constexpr int LAG = KRCN_JAG_LAG < K ? KRCN_JAG_LAG : K - 1 > 0 ? K - 1 : 1;
    u32x4 pc[LAG + 1][RPU];
#pragma unroll
    for (int i = 0; i < K; ++i) {
#pragma unroll
      for (int r = 0; r < RPU; ++r)
        if (i * RPU + r < R) pc[i % (LAG + 1)][r] = jag_fetch1<T>(x, e1, a.cols, NP, i * RPU + r);
      const int c = int(cw0 >> (8 * i)) & 0xff;
      const int rs = int(rsw[i / 4] >> (8 * (i % 4))) & 0xff;
      T2 pr;
      pr.x = U[i].v.x * win[U[i].o.x];
      pr.y = U[i].v.y * win[U[i].o.y];
      slab2[lane] = pr;
      wave_lds_sync();
      // a lane's levels past its count read the zero slot: adding +0.0 leaves
      // a running sum unchanged (it is never -0.0: it starts at +0.0)
      T ai = acc[i];
#pragma unroll
      for (int k = 0; k < 4; ++k) ai += slab[c > k ? rs + k : kZero];
      if (__ballot(c > 4) != 0ull)   // rare: rows with more than 4 elements in the slice
        for (int k = 4; __ballot(c > k) != 0ull; ++k) ai += slab[c > k ? rs + k : kZero];
      acc[i] = ai;
      wave_lds_sync();
      issue(U[i], i, bv1);   // unit (s + 1, i) (clamped past the end)
      if (i >= LAG && more)
#pragma unroll
        for (int r = 0; r < RPU; ++r)
          if ((i - LAG) * RPU + r < R)
            jag_store1<R>(pc[(i - LAG) % (LAG + 1)][r], nwin, NP, (i - LAG) * RPU + r);
    }
    if (more) {
#pragma unroll
      for (int q = K - LAG; q < K; ++q)
#pragma unroll
        for (int r = 0; r < RPU; ++r)
          if (q >= 0 && q * RPU + r < R) jag_store1<R>(pc[q % (LAG + 1)][r], nwin, NP, q * RPU + r);
    }
    cw0 = cw1;
    bv0 = bv1;
    cw1 = cw2;
    bv1 = bv2;
    if (more) lds_block_barrier();
  }
  typename RedOf<Epi>::type red{};
  typename Epi::Pre pre[K];
#pragma unroll
  for (int i = 0; i < K; ++i) {
    const int r = (g0 + wave + kJagWaves * i) * 64 + lane;
    pre[i] = epi.pre(r < a.rows ? r : a.rows - 1);
  }
#pragma unroll
  for (int i = 0; i < K; ++i) {
    const int r = (g0 + wave + kJagWaves * i) * 64 + lane;
    if (wave + kJagWaves * i < Gb && r < a.rows) red += epi.row(r, acc[i], sg, pre[i]);
  }
  if constexpr (Epi::kReduce) store_block_red<kJagNT>(red, sm, partials, epi);
}

// ------------------------------------------------------------- plan build
// Per row r (one thread, elements in CSR order): the sort key of every
// element, (unit << 22) | ((level >> 1) << 7) | (lane << 1) | (level & 1)
// (pair-level order, the single-window pass) or (unit << 22) | (lane << 16) |
// level (row-major inside the unit, the accumulate pass), with level = rank
// of the element among the row's elements in the same slice; the lane counts
// per unit (8-bit, saturated at 255), the unit sizes and the largest count.
// Pair-level order pads every odd count to even: a row's last odd element
// gets a pad partner (key at keys[nnz + r], a sentinel past every real key
// when the row needs none; flags[2] counts the pads), so every (pair level,
// lane) takes exactly two slots and a lane loads its pair with one 16-byte
// value load and one 4-byte offset load.  Flags rows whose columns are not
// ascending (the level order would not be the CSR order).
// With G slice groups (accumulate), slice s belongs to group s / Sg and block
// (row range) * G + s / Sg; S here is Sg, the slices per group.
[[maybe_unused]] static __global__ __launch_bounds__(kNT) void k_jag_keys(int rows, int S, int G, int W, int K,
    int lane_major, int64_t nnz, unsigned long long sentinel, int long_len, const int* __restrict__ ptr,
    const int* __restrict__ idx, const int* __restrict__ gcut, const int* __restrict__ gblk,
    unsigned long long* __restrict__ keys, unsigned char* __restrict__ cnt8, int* __restrict__ usize,
    int* __restrict__ flags) {
  for (int r = blockIdx.x * kNT + threadIdx.x; r < rows; r += gridDim.x * kNT) {
    const int g = r >> 6, rr = gblk[g];
    const int gl = g - gcut[rr];
    const int lane = r & 63;
    int prev_s = -1, k = 0, prev_c = -1, mx = 0;
    auto unit = [&](int s) {
      const unsigned long long b = (unsigned long long)rr * G + s / S;
      return (((b * S + s % S) * K + gl / kJagWaves) * kJagWaves + gl % kJagWaves);
    };
    unsigned long long pad = sentinel;
    if (long_len > 0 && ptr[r + 1] - ptr[r] > long_len) {   // a long row (single window): summed apart
      for (int e = ptr[r]; e < ptr[r + 1]; ++e) keys[e] = sentinel;
      if (!lane_major) keys[nnz + r] = sentinel;
      cnt8[unit(0) * 64 + lane] = 0xFF;
      continue;
    }
    auto close_run = [&]() {
      if (prev_s < 0) return;
      cnt8[unit(prev_s) * 64 + lane] = static_cast<unsigned char>(k + 1 > 255 ? 255 : k + 1);
      const int c = k + 1;
      if (!lane_major && (c & 1)) {   // the odd last element's pad partner (one slice: one run per row)
        const unsigned long long kk = (unsigned long long)(c < 65535 ? c : 65535);
        pad = (unit(prev_s) << 22) | ((kk >> 1) << 7) | ((unsigned long long)lane << 1) | 1ull;
        atomicAdd(flags + 2, 1);
      }
      atomicAdd(usize + unit(prev_s), lane_major ? c : (c + 1) & ~1);
      mx = c > mx ? c : mx;
    };
    for (int e = ptr[r]; e < ptr[r + 1]; ++e) {
      const int c = idx[e];
      if (c < prev_c) flags[0] = 1;
      prev_c = c;
      const int s = c / W;
      if (s == prev_s) {
        ++k;
      } else {
        close_run();
        k = 0;
        prev_s = s;
      }
      const unsigned long long kk = (unsigned long long)(k < 65535 ? k : 65535);
      keys[e] = (unit(s) << 22) | (lane_major ? ((unsigned long long)lane << 16) | kk
                                              : ((kk >> 1) << 7) | ((unsigned long long)lane << 1) | (kk & 1));
    }
    close_run();
    if (!lane_major) keys[nnz + r] = pad;
    if (mx > 0) atomicMax(flags + 1, mx);
  }
}

// Long rows' elements into their own arrays (row i at lbeg[i], CSR order;
// the arrays are zeroed first, so each row's even padding holds zeros).
template <typename T>
__global__ __launch_bounds__(kNT) void k_jag_long_fill(int nl, int W, const int* __restrict__ lrow,
                                                       const int* __restrict__ lbeg, const int* __restrict__ ptr,
                                                       const int* __restrict__ idx, const T* __restrict__ val,
                                                       unsigned short* __restrict__ lidx, T* __restrict__ lval) {
  for (int i = blockIdx.x; i < nl; i += gridDim.x) {
    const int r = lrow[i], e0 = ptr[r], len = ptr[r + 1] - e0;
    for (int k = threadIdx.x; k < len; k += kNT) {
      lidx[lbeg[i] + k] = static_cast<unsigned short>(idx[e0 + k] % W);
      lval[lbeg[i] + k] = val[e0 + k];
    }
  }
}

// First sorted position of every unit (keys of units >= NU: sentinels).
[[maybe_unused]] static __global__ __launch_bounds__(kNT) void k_jag_firsts(int64_t n, int64_t NU,
    const unsigned long long* __restrict__ keys, int* __restrict__ first) {
  for (int64_t p = int64_t(blockIdx.x) * kNT + threadIdx.x; p < n; p += int64_t(gridDim.x) * kNT) {
    const unsigned long long u = keys[p] >> 22;
    if (u < (unsigned long long)NU && (p == 0 || (keys[p - 1] >> 22) != u)) first[u] = int(p);
  }
}

// Elements into place: sorted position p of unit u lands at p (pbase null) or
// at pbase[u] + (p - first[u]) (units padded to even element counts); sorted
// items past the real nonzeros (perm >= nnz) are pads: offset 0, value 0.
template <typename T>
__global__ __launch_bounds__(kNT) void k_jag_gather(int64_t n, int64_t nnz, int W, const int* __restrict__ perm,
                                                    const int* __restrict__ idx, const T* __restrict__ val,
                                                    const unsigned long long* __restrict__ keys,
                                                    const int* __restrict__ first, const int* __restrict__ pbase,
                                                    unsigned short* __restrict__ widx, T* __restrict__ wval) {
  for (int64_t p = int64_t(blockIdx.x) * kNT + threadIdx.x; p < n; p += int64_t(gridDim.x) * kNT) {
    const int e = perm[p];
    int64_t q = p;
    if (pbase) {
      const unsigned long long u = keys[p] >> 22;
      q = int64_t(pbase[u]) + (p - first[u]);
    }
    const bool real = e < nnz;
    widx[q] = real ? static_cast<unsigned short>(idx[e] % W) : static_cast<unsigned short>(0);
    wval[q] = real ? val[e] : T(0);
  }
}

// Even-padded unit sizes (accumulate layout).
[[maybe_unused]] static __global__ __launch_bounds__(kNT) void k_jag_pad2(int64_t n, const int* __restrict__ usize,
                                                                          int* __restrict__ psz) {
  for (int64_t i = int64_t(blockIdx.x) * kNT + threadIdx.x; i < n; i += int64_t(gridDim.x) * kNT)
    psz[i] = (usize[i] + 1) & ~1;
}

// Per (block, slice, wave) record: the K unit bases, then the K unit sizes.
[[maybe_unused]] static __global__ __launch_bounds__(kNT) void k_jag_umeta(int64_t nrec, int K,
    const int* __restrict__ bases, const int* __restrict__ usize, int* __restrict__ umeta) {
  for (int64_t t = int64_t(blockIdx.x) * kNT + threadIdx.x; t < nrec * 2 * K; t += int64_t(gridDim.x) * kNT) {
    const int64_t rec = t / (2 * K);
    const int j = int(t % (2 * K));
    const int i = j < K ? j : j - K;
    const int64_t uid = ((rec / kJagWaves) * K + i) * kJagWaves + rec % kJagWaves;
    umeta[t] = j < K ? bases[uid] : usize[uid];
  }
}

// 8-bit lane counts per unit -> the kernel's lane words: word (b, s, w, l)
// holds unit ((b S + s) K + i) 16 + w's count of lane l at bit 8 i.
template <class CW>
__global__ __launch_bounds__(kNT) void k_jag_words(int64_t nrec, int K, const unsigned char* __restrict__ c8,
                                                   CW* __restrict__ out) {
  constexpr int CB = 8;
  for (int64_t t = int64_t(blockIdx.x) * kNT + threadIdx.x; t < nrec * 64; t += int64_t(gridDim.x) * kNT) {
    const int64_t rec = t >> 6;            // (b S + s) 16 + w
    const int l = int(t & 63);
    const int64_t bs = rec / kJagWaves, w = rec % kJagWaves;
    CW word = 0;
    for (int i = 0; i < K; ++i) {
      const int64_t uid = (bs * K + i) * kJagWaves + w;
      word |= CW(c8[uid * 64 + l]) << (CB * i);
    }
    out[t] = word;
  }
}

}  // namespace krcn
