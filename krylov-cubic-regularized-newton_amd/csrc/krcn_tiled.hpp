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
#include <type_traits>
#include <utility>

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
// early(): the vector get() will return, known before begin() runs (a
// launch may start loading it while the prologue's reductions are in flight);
// a guess when it depends on device state — the caller re-checks get().
template <typename T> struct SrcPlain {
  const T* x;
  __device__ __forceinline__ bool begin(double*) { return false; }
  __device__ __forceinline__ const T* get() const { return x; }
  __device__ __forceinline__ const T* early() const { return x; }
};

// First launch of Lanczos loop step j: settles beta / breakdown (see
// lz_step_prologue) and gathers the unnormalised z_j.
// preload(): the prologue's operands (state flag, <= kNT norm partials) as
// early loads — a kernel that issues them before its own streams keeps those
// streams in flight through the prologue (loads retire in issue order).
template <typename T> struct SrcLzStep {
  LzCtl<T> c; LzVec<T> v;
  int pre_ok = 0, pre_flag = 0;
  double pre_pv = 0.0;
  __device__ __forceinline__ void preload() {
    if (c.Pnorm > kNT) return;
    pre_ok = 1;
    if (threadIdx.x == 0 && c.j > 0)
      pre_flag = __hip_atomic_load(&c.st->done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (threadIdx.x < c.Pnorm) pre_pv = c.pnorm[threadIdx.x];
  }
  __device__ __forceinline__ bool begin(double* sm) {
    return pre_ok ? lz_step_prologue_pre(c, sm, v, pre_flag, pre_pv) : lz_step_prologue(c, sm, v);
  }
  __device__ __forceinline__ const T* get() const { return v.z; }
  __device__ __forceinline__ const T* early() const { return c.j == 0 ? c.g : c.V + int64_t(c.j) * c.ld; }
};

template <class S> struct IsLzStep : std::false_type {};
template <typename T> struct IsLzStep<SrcLzStep<T>> : std::true_type {};

// Pass 1 of the early-alpha step (krcn_kernels.hpp EpiLz2E): its epilogue
// stores raw slice sums, so no block needs beta_{j-1}; only block 0 settles
// it (lz_step_prologue: the breakdown test, betas[j-1] and the state, which
// the slice combine reads after this launch) while every other block gathers
// z_j (g at j = 0) straight away, with no reduction or barrier in front of
// its window burst.  Once the recurrence has ended those blocks still run
// their slices (into partials nobody reads: the combine and pass 2 skip).
template <typename T> struct SrcLzBeta {
  LzCtl<T> c; LzVec<T> v;
  int pre_ok = 0, pre_flag = 0;
  double pre_pv = 0.0;
  __device__ __forceinline__ void preload() {
    if (blockIdx.x != 0 || c.Pnorm > kNT) return;
    pre_ok = 1;
    if (threadIdx.x == 0 && c.j > 0)
      pre_flag = __hip_atomic_load(&c.st->done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (threadIdx.x < c.Pnorm) pre_pv = c.pnorm[threadIdx.x];
  }
  __device__ __forceinline__ bool begin(double* sm) {
    if (blockIdx.x != 0) return false;
    if (pre_ok) lz_step_prologue_pre(c, sm, v, pre_flag, pre_pv);
    else lz_step_prologue(c, sm, v);
    return false;   // block 0 runs its slice whatever the test decided (see above)
  }
  __device__ __forceinline__ const T* get() const { return early(); }
  __device__ __forceinline__ const T* early() const { return c.j == 0 ? c.g : c.V + int64_t(c.j) * c.ld; }
};

// Pass 2 of the two-launch Lanczos step (sorted unsliced pass 1 + jagged
// single-window pass 2, krcn_lanczos_impl.hpp): pass 1 stored u' = w (.) X z_j
// unnormalised; every pass-2 block settles beta_{j-1} from pass 1's ||z||^2
// partials (lz_step_prologue: the breakdown test, block 0 records the state)
// and divides its window by it, u = u' / beta, before the gather.  EpiLz2
// takes v = z_j / beta from here (StepVecSrc).
template <typename T> struct SrcLzU {
  LzCtl<T> c; const T* x; LzVec<T> v;
  int pre_ok = 0, pre_flag = 0;
  double pre_pv = 0.0;
  static constexpr bool kStepVec = true;
  __device__ __forceinline__ void preload() {
    if (c.Pnorm > kNT) return;
    pre_ok = 1;
    if (threadIdx.x == 0 && c.j > 0)
      pre_flag = __hip_atomic_load(&c.st->done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (threadIdx.x < c.Pnorm) pre_pv = c.pnorm[threadIdx.x];
  }
  __device__ __forceinline__ bool begin(double* sm) {
    return pre_ok ? lz_step_prologue_pre(c, sm, v, pre_flag, pre_pv) : lz_step_prologue(c, sm, v);
  }
  __device__ __forceinline__ const T* get() const { return x; }
  __device__ __forceinline__ const T* early() const { return x; }
};
template <class S> struct IsLzU : std::false_type {};
template <typename T> struct IsLzU<SrcLzU<T>> : std::true_type {};

// Pass 2 of the early-alpha Lanczos step (EpiLz2E, krcn_kernels.hpp): gathers
// u and settles alpha_j in every block from the combine's partials of
// u.(t / beta) and the previous pass 2's partials of z_j . v_{j-1}
// (alpha_j = sum_q / n + l2 - sum_zv; block 0 records alphas[j]).  preload()
// issues those operands before the window burst (loads retire in issue order).
template <typename T> struct SrcLzAlpha {
  const T* x; const LanczosState* st;
  const double* pq; int Pq;       // combine partials (X v_j).(w (X v_j))
  const double* pzv; int Pzv;     // z_j . v_{j-1} partials (j >= 1)
  double* alphas; int j; double n, l2;
  T alpha = T(0);
  int pre_ok = 0, pre_flag = 0;
  double pre_q = 0.0, pre_z = 0.0;
  __device__ __forceinline__ void preload() {
    if (Pq > kNT || (j > 0 && Pzv > kNT)) return;
    pre_ok = 1;
    if (threadIdx.x == 0) pre_flag = __hip_atomic_load(&st->done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (threadIdx.x < Pq) pre_q = pq[threadIdx.x];
    if (j > 0 && threadIdx.x < Pzv) pre_z = pzv[threadIdx.x];
  }
  __device__ __forceinline__ bool begin(double* sm) {
    double a, zv = 0.0;
    if (pre_ok) {
      __shared__ int flag_sm;
      if (threadIdx.x == 0) flag_sm = pre_flag;
      __syncthreads();
      const int done = flag_sm;
      __syncthreads();
      if (done) return true;
      a = block_sum(threadIdx.x < kNT && int(threadIdx.x) < Pq ? 0.0 + pre_q : 0.0, sm);
      if (j > 0) zv = block_sum(threadIdx.x < kNT && int(threadIdx.x) < Pzv ? 0.0 + pre_z : 0.0, sm);
    } else {
      if (block_uniform_load(&st->done)) return true;
      a = sum_partials(pq, Pq, sm);
      if (j > 0) zv = sum_partials(pzv, Pzv, sm);
    }
    const double al = a / n + l2 - zv;
    if (blockIdx.x == 0 && threadIdx.x == 0) alphas[j] = al;
    alpha = T(al);
    return false;
  }
  // Split prologue (a kernel with a block barrier of its own after the window
  // store, k_jag_pass): the preloaded sums go through wave sums into LDS
  // before that barrier and are finished after it, so the prologue adds no
  // barrier of its own.  The same wave sums and the same fixed combination
  // as block_sum: the same alpha bits.  Only when pre_ok.
  static constexpr bool kSplit = true;
  __device__ __forceinline__ void begin_split(double* ls, int* lf) const {
    if (threadIdx.x < kNT) {   // waves 0..3, as block_sum
      const int t = int(threadIdx.x);
      const double q = wave_sum(t < Pq ? 0.0 + pre_q : 0.0);
      const double z = j > 0 ? wave_sum(t < Pzv ? 0.0 + pre_z : 0.0) : 0.0;
      if ((t & 63) == 0) {
        ls[t >> 6] = q;
        ls[4 + (t >> 6)] = z;
      }
      if (t == 0) *lf = pre_flag;
    }
  }
  __device__ __forceinline__ bool after_split(const double* ls, const int* lf) {
    if (*lf) return true;
    const double a = (ls[0] + ls[1]) + (ls[2] + ls[3]);
    const double zv = j > 0 ? (ls[4] + ls[5]) + (ls[6] + ls[7]) : 0.0;
    const double al = a / n + l2 - zv;
    if (blockIdx.x == 0 && threadIdx.x == 0) alphas[j] = al;
    alpha = T(al);
    return false;
  }
  __device__ __forceinline__ const T* get() const { return x; }
  __device__ __forceinline__ const T* early() const { return x; }
};
template <class S, class = void> struct IsSplitSrc : std::false_type {};
template <class S> struct IsSplitSrc<S, std::void_t<decltype(S::kSplit)>> : std::bool_constant<S::kSplit> {};



// Later launches of a Lanczos step (state settled by an earlier launch).
template <typename T> struct SrcLzState {
  LzCtl<T> c; LzVec<T> v;
  __device__ __forceinline__ bool begin(double*) {
    if (c.mode == 0 && c.st->done) return true;
    v = lz_vec_from_state(c);
    return false;
  }
  __device__ __forceinline__ const T* get() const { return v.z; }
  __device__ __forceinline__ const T* early() const {   // the untruncated choice of lz_vec_from_state
    const int jj = c.mode == 0 ? c.j : c.m - 1;
    return jj == 0 ? c.g : c.V + int64_t(jj) * c.ld;
  }
};

// An explicit vector, skipped once the recurrence has ended.
// Sources with operands a kernel may load before its window burst.
template <class S, class = void> struct HasPreload : std::false_type {};
template <class S> struct HasPreload<S, std::void_t<decltype(std::declval<S&>().preload())>> : std::true_type {};
template <class S, class = void> struct HasPreDone : std::false_type {};
template <class S> struct HasPreDone<S, std::void_t<decltype(std::declval<S&>().pre_done)>> : std::true_type {};

template <typename T> struct SrcGuard {
  const T* x; const LanczosState* st; int mode;
  int pre_ok = 0, pre_done = 0;
  // the flag loaded early by kernels that call preload() (a kernel's
  // prologue operands in one round trip); others read it in begin()
  __device__ __forceinline__ void preload() {
    pre_ok = 1;
    pre_done = mode == 0 ? st->done : 0;
  }
  __device__ __forceinline__ bool begin(double*) { return mode == 0 && (pre_ok ? pre_done != 0 : st->done != 0); }
  __device__ __forceinline__ const T* get() const { return x; }
  __device__ __forceinline__ const T* early() const { return x; }
};

// Pass 1 of the column-sharded early-alpha step (krcn_lanczos_impl.hpp,
// early_cols, j >= 1): SrcGuard, and block 0 first sums the previous pass 2's
// partials of ||z_p||^2 and z_p . v_p into the two elements past the row sums
// (u[n], u[n + 1]) that the all-reduce after this launch carries: the sums,
// and bits, of a separate two-block launch between pass 2 and this pass,
// without that launch.  Block 0 is dispatched first, so its two partial
// reductions overlap the other blocks' tiles.
template <typename T> struct SrcGuardPack {
  const T* x; const LanczosState* st;
  const double* pb; const double* pz; int P; double* out;
  int pre_ok = 0, pre_done = 0;
  __device__ __forceinline__ void preload() {
    pre_ok = 1;
    pre_done = st->done;
  }
  __device__ __forceinline__ bool begin(double* sm) {
    if (pre_ok ? pre_done != 0 : st->done != 0) return true;
    if (blockIdx.x == 0) {
      const double a = sum_partials(pb, P, sm);
      const double b = sum_partials(pz, P, sm);
      if (threadIdx.x == 0) {
        out[0] = a;
        out[1] = b;
      }
    }
    return false;
  }
  __device__ __forceinline__ const T* get() const { return x; }
  __device__ __forceinline__ const T* early() const { return x; }
};

// Fused Lanczos step B in pass 1 (window slices: k_window_pass; sorted tiles
// with slices: k_sorted_pass).  j >= 1: alpha_{j-1} from pass 2's partials
// (every block; block 0 records it), the gathered vector is
// z_j = w - alpha_{j-1} v_{j-1} (the expression of k_lz_step_b), stored
// unnormalised in V[j] by the blocks' shares with the partials of ||z_j||^2
// in pz[block]; the slice combine settles beta_{j-1} from pz.  j = 0: g.
template <typename T> struct SrcLzZ {
  LzCtl<T> c;
  const T* Wv;            // w of step j-1 (pass 2's output)
  const double* pa;       // partials of v_{j-1}.w
  int Pa;
  double* alphas;
  double* pz;
  T alpha;
  int store_z = 1;        // 0: pass 2 re-forms z_j (EpiLz2::zw), the window pass stores none
  __device__ __forceinline__ bool begin(double* sm) {
    if (c.j == 0) return false;
    double al;
    if (Pa <= 2 * kNT) {
      if (flag_and_sum(&c.st->done, pa, Pa, sm, &al)) return true;
    } else {
      if (block_uniform_load(&c.st->done)) return true;
      al = sum_partials(pa, Pa, sm);
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) alphas[c.j - 1] = al;
    alpha = T(al);
    return false;
  }
};
template <class S> struct IsLzZ : std::false_type {};
template <typename T> struct IsLzZ<SrcLzZ<T>> : std::true_type {};

// Fused Lanczos step B for a vector that fits one LDS window piece (d <=
// kWinNT, window-accum plans, w8a's d = 300): EVERY block forms all of
// z_j = w - alpha_{j-1} v_{j-1} and its norm beta_{j-1} itself (thread t owns
// element t, so the sums are the same bits in every block), settles the
// breakdown test and the state as lz_step_prologue does (block 0 records),
// and gathers z_j unnormalised with u = w (t / beta) in the epilogue — no
// k_lz_step_b launch and no slice combine.  j = 0: z = g, beta = ||g||.
template <typename T> struct SrcLzSmall {
  LzCtl<T> c;
  const T* Wv;            // w of step j-1
  const double* pa;       // partials of v_{j-1}.w
  int Pa;
  double* alphas;
  LzVec<T> v;
};
template <class S> struct IsLzSmall : std::false_type {};
template <typename T> struct IsLzSmall<SrcLzSmall<T>> : std::true_type {};

// Gathered-vector accessors of the sorted pass: a plain vector, or z = w - a v
// formed per element (the same rounding as k_lz_step_b's store).
template <typename T> struct GatherPtr {
  const T* x;
  __device__ __forceinline__ T operator()(int64_t i) const { return x[i]; }
};
template <typename T> struct GatherZ {
  const T* w; const T* v; T a;
  __device__ __forceinline__ T operator()(int64_t i) const { return w[i] - a * v[i]; }
};

// Per-slice partial store (sliced passes).
template <typename T> struct EpiSlicePart {
  T* part; int64_t ld;
  static constexpr bool kReduce = false;
  struct Pre {};
  template <class S> __device__ __forceinline__ void init(const S&) {}
  __device__ __forceinline__ Pre pre(int) const { return Pre{}; }
  __device__ __forceinline__ double row(int r, T s, int slice, const Pre&) const {
    store_policy<KRCN_PART_ST>(part + int64_t(slice) * ld + r, s);
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
  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  const int g = blockIdx.x % groups;
  // the group's tile range and the source's flag in one round trip (the
  // empty asm keeps the compiler from sinking the range loads past the
  // prologue's branch)
  const int t_beg = tbeg[g], t_end = tbeg[g + 1];
  if constexpr (HasPreload<Src>::value) src.preload();
  if constexpr (HasPreDone<Src>::value) asm volatile("" ::"s"(t_beg), "s"(t_end), "s"(src.pre_done));
  if (src.begin(sm)) return;
  __shared__ T prod_all[kWavesPerBlock][kProdSlots];
  __shared__ int rp_all[kWavesPerBlock][kWaveTileRows + 1];
  T* prod = prod_all[wave];
  int* rpl = rp_all[wave];
  const T* x = src.get();
  epi.init(src);
  const int j = (blockIdx.x / groups) * kWavesPerBlock + wave;
  const int stride = (gridDim.x / groups) * kWavesPerBlock;
  const int sub = lane & (L - 1);
  const int grp = lane / L;
  constexpr int kGroups = 64 / L;
  typename RedOf<Epi>::type acc{};
  for (int t = t_beg + j; t < t_end; t += stride) {
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
    store_block_red<kNT>(acc, sm, partials, epi);
  }
}

// Combine pass of a sliced SpMV.  A block owns 64 rows; wave q of 16 sums
// slices q, q+16, ... in order (coalesced 64-row loads, all issued before the
// adds), then s_r = pairwise sum of the 16 wave sums and the epilogue.
// Slice combine: block b owns rows [b R, b R + R) with R = ceil(rows / 256)
// (at most kCombineRows), so every CU ingests the same share of the S x rows
// partials in one round; thread (i, p) adds slices p, p + 8, p + 16, ... of
// row i left to right (all its loads issued before the first add), then a
// fixed tree over the 8 phases.  Deterministic; the order does not depend on
// the grid.
constexpr int kCombineRows = 128;
constexpr int kCombineNT = 1024;
constexpr int kCombinePh = kCombineNT / kCombineRows;
constexpr int kCombineU = 16;   // loads in flight per thread
constexpr int kCombineSpread = 256;   // one row range per CU (MI355X: 256 CUs)
__host__ inline int combine_rows(int rows) {
  const int R = (rows + kCombineSpread - 1) / kCombineSpread;
  return R < 1 ? 1 : (R > kCombineRows ? kCombineRows : R);
}
// at most one block per CU: past 256 x 128 rows a block walks several ranges
// (each block runs the source prologue, e.g. the beta reduction, once)
__host__ inline int combine_grid(int rows) {
  const int R = combine_rows(rows);
  const int g = (rows + R - 1) / R;
  return g < 1 ? 1 : (g > kCombineSpread ? kCombineSpread : g);
}
template <typename T, class Src, class Epi>
__global__ __launch_bounds__(kCombineNT) void k_slice_combine(int rows, int S, int R, const T* __restrict__ part,
                                                              Src src, Epi epi, double* __restrict__ partials) {
  constexpr int NW = kCombineNT / 64;
  __shared__ double sm[NW];
  __shared__ T qs[kCombinePh][kCombineRows];
  const int i = threadIdx.x % kCombineRows, ph = threadIdx.x / kCombineRows;
  // the first range's loads go out before the source prologue (beta, the
  // breakdown test): they do not depend on it
  T a[kCombineU];
  auto issue = [&](int rc, int k0) {
#pragma unroll
    for (int u = 0; u < kCombineU; ++u) {
      const int k = k0 + u * kCombinePh;
      a[u] = part[int64_t(k < S ? k : S - 1) * rows + rc];
    }
  };
  int r0 = blockIdx.x * R;
  if constexpr (IsLzStep<Src>::value) src.preload();
  issue(r0 + i < rows && i < R ? r0 + i : (r0 < rows ? r0 : rows - 1), ph);
  typename Epi::Pre pre0{};
  if constexpr (PreEarly<Epi>::value)
    if (ph == 0) pre0 = epi.pre(r0 + i < rows && i < R ? r0 + i : (r0 < rows ? r0 : rows - 1));
  if (src.begin(sm)) return;
  epi.init(src);
  typename RedOf<Epi>::type acc{};
  for (bool first = true; r0 < rows; r0 += gridDim.x * R, first = false) {
    const int r = r0 + i;
    const bool live = i < R && r < rows;
    const int rc = live ? r : r0;
    typename Epi::Pre pre{};
    if (ph == 0) pre = PreEarly<Epi>::value && first ? pre0 : epi.pre(rc);
    T sq = T(0);
    for (int k0 = ph; k0 < S; k0 += kCombineU * kCombinePh) {
      if (!first || k0 != ph) issue(rc, k0);
#pragma unroll
      for (int u = 0; u < kCombineU; ++u)
        if (k0 + u * kCombinePh < S) sq += a[u];
    }
    qs[ph][i] = sq;
    __syncthreads();
    if (ph == 0 && live) {
      T v[kCombinePh];
#pragma unroll
      for (int j = 0; j < kCombinePh; ++j) v[j] = qs[j][i];
#pragma unroll
      for (int h = kCombinePh / 2; h > 0; h >>= 1)
#pragma unroll
        for (int j = 0; j < h; ++j) v[j] = v[2 * j] + v[2 * j + 1];
      acc += epi.row(r, v[0], 0, pre);
    }
    __syncthreads();
  }
  if constexpr (Epi::kReduce) {
    store_block_red<kCombineNT>(acc, sm, partials, epi);
  }
}

// Slice combine with 16-byte partial loads (many slices: news20's 128): a
// thread owns VW = 16 / sizeof(T) adjacent rows and adds slices p, p + PH,
// p + 2 PH, ... left to right (one 16-byte load per slice, all in flight),
// then a fixed pairwise tree over the PH = 32 phases.  Blocks of 1024
// threads cover 32 VW-row groups.  Half the load instructions of
// k_slice_combine (TA-bound at 8 bytes a lane).  Needs rows % VW == 0.
constexpr int kCombWPh = 32;
constexpr int kCombWGroups = kCombineNT / kCombWPh;   // row groups per block
template <typename T> struct CombW {
  static constexpr int VW = 16 / int(sizeof(T));
  using V = typename std::conditional<sizeof(T) == 8, f64x2, f32x4>::type;
};
__host__ inline int combine_w_grid(int rows, int vw) { return (rows / vw + kCombWGroups - 1) / kCombWGroups; }
template <typename T, class Src, class Epi>
__global__ __launch_bounds__(kCombineNT) void k_slice_combine_w(int rows, int S, const T* __restrict__ part, Src src,
                                                                Epi epi, double* __restrict__ partials) {
  using CW = CombW<T>;
  constexpr int VW = CW::VW, U = 8;
  using V = typename CW::V;
  __shared__ double sm[kCombineNT / 64];
  __shared__ V qs[kCombWPh][kCombWGroups];
  const int i = threadIdx.x % kCombWGroups, ph = threadIdx.x / kCombWGroups;
  const int ngroups = rows / VW;
  const int gi = int(blockIdx.x) * kCombWGroups + i;
  const int gc = gi < ngroups ? gi : ngroups - 1;
  const V* pv = reinterpret_cast<const V*>(part);
  const int64_t ldv = rows / VW;
  V a[U];
  auto issue = [&](int k0) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = k0 + u * kCombWPh;
      a[u] = pv[int64_t(k < S ? k : S - 1) * ldv + gc];
    }
  };
  if constexpr (IsLzStep<Src>::value) src.preload();
  issue(ph);
  typename Epi::Pre pre[VW];
  if (ph == 0) {
#pragma unroll
    for (int v = 0; v < VW; ++v) pre[v] = epi.pre(gc * VW + v);
  }
  if (src.begin(sm)) return;
  epi.init(src);
  V sq = V(T(0));
  for (int k0 = ph; k0 < S; k0 += U * kCombWPh) {
    if (k0 != ph) issue(k0);
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (k0 + u * kCombWPh < S) sq += a[u];
  }
  qs[ph][i] = sq;
  __syncthreads();
  typename RedOf<Epi>::type acc{};
  if (ph == 0 && gi < ngroups) {
    V v[kCombWPh];
#pragma unroll
    for (int j = 0; j < kCombWPh; ++j) v[j] = qs[j][i];
#pragma unroll
    for (int h = kCombWPh / 2; h > 0; h >>= 1)
#pragma unroll
      for (int j = 0; j < h; ++j) v[j] = v[2 * j] + v[2 * j + 1];
#pragma unroll
    for (int e = 0; e < VW; ++e) acc += epi.row(gi * VW + e, v[0][e], 0, pre[e]);
  }
  if constexpr (Epi::kReduce) {
    store_block_red<kCombineNT>(acc, sm, partials, epi);
  }
}

// Combine of many partial arrays over few rows (the fused X^T partials of
// one-piece plans: S = the pass-1 grid, 256, over d <= 1,024 rows): blocks of
// RB rows x PH = 1024 / RB phases, phase p adds arrays p, p + PH, ... left to
// right with all its loads in one round, then a fixed pairwise tree over the
// phases.  Deterministic.  (k_slice_combine spreads such a matrix over 150
// blocks of two live rows each, with its loads in two rounds.)
template <typename T, class Src, class Epi, int RB>
__global__ __launch_bounds__(kCombineNT) void k_xt_combine(int rows, int S, const T* __restrict__ part, Src src,
                                                           Epi epi, double* __restrict__ partials) {
  constexpr int PH = kCombineNT / RB;
  constexpr int U = 8;
  __shared__ double sm[kCombineNT / 64];
  __shared__ T qs[PH][RB];
  const int i = threadIdx.x % RB, ph = threadIdx.x / RB;
  const int r = int(blockIdx.x) * RB + i;
  const int rc = r < rows ? r : rows - 1;
  T a[U];
  auto issue = [&](int k0) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = k0 + u * PH;
      a[u] = part[int64_t(k < S ? k : S - 1) * rows + rc];
    }
  };
  issue(ph);   // the first round goes out before the source prologue
  if (src.begin(sm)) return;
  epi.init(src);
  typename Epi::Pre pre{};
  if (ph == 0) pre = epi.pre(rc);
  T sq = T(0);
  for (int k0 = ph; k0 < S; k0 += U * PH) {
    if (k0 != ph) issue(k0);
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (k0 + u * PH < S) sq += a[u];
  }
  qs[ph][i] = sq;
  __syncthreads();
  typename RedOf<Epi>::type acc{};
  if (ph == 0 && r < rows) {
    T v[PH];
#pragma unroll
    for (int j = 0; j < PH; ++j) v[j] = qs[j][i];
#pragma unroll
    for (int h = PH / 2; h > 0; h >>= 1)
#pragma unroll
      for (int j = 0; j < h; ++j) v[j] = v[2 * j] + v[2 * j + 1];
    acc = epi.row(r, v[0], 0, pre);
  }
  if constexpr (Epi::kReduce) {
    store_block_red<kCombineNT>(acc, sm, partials, epi);
  }
}
constexpr int kXtCombineRows = 32;

// Slice combine for few partial arrays (S <= 16: jagged slice groups, small
// window / sorted plans): one row per thread, all S loads in flight, <= one
// block per CU walking rows in strides.  The same sums in the same order as
// k_slice_combine (phase p adds slices p, p + 8 left to right from 0, then the
// 8-phase tree): bitwise the same result, without its 8-phase LDS exchange and
// per-range barriers (a range loop of k_slice_combine is latency-bound at
// 250 K rows: 16.6 us for 8 arrays, tools/bench --rehearse-shard 8 synth).
constexpr int kCombineSmallS = 16;
// Block size of the small combine: 256 threads while that still gives <= 256
// blocks (rcv1's 20 K rows: 79 blocks instead of 20 of 1024), else 1024.
__host__ inline int combine_small_nt(int rows) { return rows <= 256 * 256 ? 256 : kCombineNT; }
__host__ inline int combine_small_grid(int rows) {
  const int nt = combine_small_nt(rows);
  const int g = (rows + nt - 1) / nt;
  return g < 1 ? 1 : (g > kCombineSpread ? kCombineSpread : g);
}
// SM: loads per row (the smallest of 2, 4, 8, 16 >= S; no duplicate loads).
template <typename T, class Src, class Epi, int SM, int NT>
__global__ __launch_bounds__(NT) void k_slice_combine_small(int rows, int S, const T* __restrict__ part, Src src,
                                                            Epi epi, double* __restrict__ partials) {
  __shared__ double sm[NT / 64];
  T a[SM];
  auto issue = [&](int r) {
    const int rc = r < rows ? r : rows - 1;
#pragma unroll
    for (int k = 0; k < SM; ++k) a[k] = part[int64_t(k < S ? k : S - 1) * rows + rc];
  };
  int r = int(blockIdx.x) * NT + int(threadIdx.x);
  if constexpr (IsLzStep<Src>::value) src.preload();
  issue(r);
  typename Epi::Pre pre0{};
  if constexpr (PreEarly<Epi>::value) pre0 = epi.pre(r < rows ? r : rows - 1);
  if (src.begin(sm)) return;
  epi.init(src);
  typename RedOf<Epi>::type acc{};
  for (bool first = true; r - int(threadIdx.x) < rows; r += int(gridDim.x) * NT, first = false) {
    const int rc = r < rows ? r : rows - 1;
    const typename Epi::Pre pre = PreEarly<Epi>::value && first ? pre0 : epi.pre(rc);
    T v[kCombinePh];
#pragma unroll
    for (int j = 0; j < kCombinePh; ++j) {
      T q = T(0);
#pragma unroll
      for (int u = 0; u < (SM + kCombinePh - 1) / kCombinePh; ++u)
        if (j + u * kCombinePh < S && j + u * kCombinePh < SM) q += a[j + u * kCombinePh];
      v[j] = q;
    }
#pragma unroll
    for (int h = kCombinePh / 2; h > 0; h >>= 1)
#pragma unroll
      for (int j = 0; j < h; ++j) v[j] = v[2 * j] + v[2 * j + 1];
    const int rn = r + int(gridDim.x) * NT;
    if (rn - int(threadIdx.x) < rows) issue(rn);   // next stride's loads before this row's epilogue
    if (r < rows) acc += epi.row(r, v[0], 0, pre);
  }
  if constexpr (Epi::kReduce) {
    store_block_red<NT>(acc, sm, partials, epi);
  }
}

// Elementwise run of an epilogue over rows with precomputed sums (sharded
// modes: after the all-reduce of raw partial row sums).
// kU rows a thread per round, all their operand loads issued before the
// first row is applied (round 5: one row at a time left the synth row apply a
// chain of dependent round trips, 1 M rows on 1,024 blocks).  Its grid:
// apply_grid(rows) blocks, each with rows to apply (every block runs the
// source prologue and writes one partial).
constexpr int kApplyU = 4;
__host__ inline int apply_grid(int64_t rows) {
  int64_t b = (rows + int64_t(kNT) * kApplyU - 1) / (int64_t(kNT) * kApplyU);
  return int(b < 1 ? 1 : (b > 1024 ? 1024 : b));
}
template <typename T, class Src, class Epi>
__global__ __launch_bounds__(kNT) void k_rows_apply(int rows, const T* __restrict__ sums, Src src, Epi epi,
                                                    double* __restrict__ partials) {
  // (kPreEarly epilogues: the first round's loads go out before the source
  // prologue, whose partial sums then overlap them)
  constexpr int kU = kApplyU;
  __shared__ double sm[kNT / 64];
  T sv[kU];
  typename Epi::Pre pv[kU];
  auto issue = [&](int rb) {
#pragma unroll
    for (int k = 0; k < kU; ++k) {
      const int r = rb + k * kNT;
      const int rc = r < rows ? r : rows - 1;
      sv[k] = sums[rc];
      pv[k] = epi.pre(rc);
    }
  };
  int r0 = blockIdx.x * kNT * kU + threadIdx.x;
  if constexpr (PreEarly<Epi>::value) issue(r0);
  if (src.begin(sm)) return;
  epi.init(src);
  typename RedOf<Epi>::type acc{};
  for (bool first = true; r0 < rows; r0 += gridDim.x * kNT * kU, first = false) {
    if (!(PreEarly<Epi>::value && first)) issue(r0);
#pragma unroll
    for (int k = 0; k < kU; ++k)
      if (r0 + k * kNT < rows) acc += epi.row(r0 + k * kNT, sv[k], 0, pv[k]);
  }
  if constexpr (Epi::kReduce) {
    store_block_red<kNT>(acc, sm, partials, epi);
  }
}

// ---------------------------------------------------------- slice builder
// slice id of every nonzero: largest s with bounds[s] <= col.
[[maybe_unused]] static __global__ __launch_bounds__(kNT) void k_slice_of(int64_t nnz, const int* __restrict__ idx,
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
[[maybe_unused]] static __global__ __launch_bounds__(kNT) void k_slice_counts(int rows, const int* __restrict__ ptr,
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
// LDS slot swizzle of the sorted tiles: XOR the low 4 bits of a slot with
// bits 4..7.  A double's bank pair is slot mod 16, and the lanes of one
// scatter instruction often hold the same in-row offset of consecutive
// equal-length rows (slot = 8 r + k); the swizzle spreads those over all
// banks.  It permutes each aligned 256-slot block, so every consumer of the
// tile just reads prod[lds_sw(p)].
#ifndef KRCN_SORT_SWIZZLE
#define KRCN_SORT_SWIZZLE 1
#endif
__device__ __forceinline__ int lds_sw(int p) { return KRCN_SORT_SWIZZLE ? p ^ ((p >> 4) & 15) : p; }

constexpr int kSortPerThread = 8;
constexpr int ilog2(int v) { return v <= 1 ? 0 : 1 + ilog2(v / 2); }
// Occupancy the sorted pass is built for: 8 waves per SIMD (2 blocks of 1024, 4 blocks
// of 512 or 8 of 256 threads per CU, matching the LDS footprint), so the
// register allocator keeps to 64 VGPRs.
#ifndef KRCN_SORT_WAVES
#define KRCN_SORT_WAVES 8
#endif
template <int NT> struct SortGeom {
  static constexpr int kTile = NT * kSortPerThread;   // nonzeros per block tile / sort segment
  static constexpr int kRows = kTile / 4;             // rows per block tile (cap)
  static constexpr int kRowRegs = (kRows + 1 + NT - 1) / NT;   // row pointers per thread
  static constexpr int kSlotBits = ilog2(kTile);
  static_assert((1 << kSlotBits) == kTile, "slot field must address a whole tile");
  // packed word: (column - tile's column base) << kSlotBits | slot
  static constexpr int64_t kMaxWindow = int64_t(1) << (32 - kSlotBits);
};

// Per-thread staging of one sorted tile.  Every load is unconditional (index
// clamped into the tile, result selected): a branch around a load makes the
// compiler wait for all outstanding loads (vmcnt(0)) where its value is
// used, which serialises the block on memory latency.
template <typename T, int NT, int L, class Epi>
struct SortedStage {
  using G = SortGeom<NT>;
  static constexpr int PER = kSortPerThread, kTile = G::kTile, kBits = G::kSlotBits, kRR = G::kRowRegs;
  static constexpr int kGroups = NT / L;
  unsigned w[PER];     // packed (column, slot), raw: lanes past the tile's end hold a clamped copy
  T v[PER];            // values
  T gx[PER];           // gathered x
  int rr[kRR];         // raw row pointers (tile offset subtracted at the LDS store)
  typename Epi::Pre q0, q1;   // epilogue operands of a group's first two rows

  __device__ __forceinline__ void load_nz(const TileDesc& d, const unsigned* __restrict__ gword,
                                          const T* __restrict__ gval) {
    const int t = threadIdx.x;
    const int last = d.p1 > 0 ? d.p1 - 1 : 0;
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int e = d.p0 + t + NT * k;
      const int ec = e < last ? e : last;
      w[k] = gword[ec];   // no select here: it would wait for the load on the spot
      v[k] = gval[ec];
    }
  }
  static __device__ __forceinline__ bool valid(const TileDesc& d, int k) {
    return d.p0 + int(threadIdx.x) + NT * k < d.p1;
  }
  __device__ __forceinline__ void load_rows(const TileDesc& d, const int* __restrict__ ptr, int rows,
                                            const Epi& epi) {
    const int t = threadIdx.x, sub = t & (L - 1), grp = t / L;
    const int* rp = ptr + int64_t(d.slice) * rows + d.row0;
    const int nr = d.row1 - d.row0;
#pragma unroll
    for (int k = 0; k < kRR; ++k) {
      const int i = t + NT * k;
      rr[k] = rp[i < nr ? i : nr];
    }
    (void)sub;
    const int r0 = grp < nr ? grp : nr - 1;
    const int r1 = grp + kGroups < nr ? grp + kGroups : nr - 1;
    q0 = epi.pre(d.row0 + r0);
    q1 = epi.pre(d.row0 + r1);
  }
  template <class X> __device__ __forceinline__ void gather(const TileDesc& d, const X& x) {
#pragma unroll
    for (int k = 0; k < PER; ++k) gx[k] = x(int64_t(d.pad0) + (valid(d, k) ? (w[k] >> kBits) : 0u));
  }
  // prod has kTile + 1 slots; lanes past the tile's end write the spare one
  __device__ __forceinline__ void store(const TileDesc& d, T* prod, int* rpl) const {
    const int t = threadIdx.x, nr = d.row1 - d.row0;
#pragma unroll
    for (int k = 0; k < kRR; ++k) {
      const int i = t + NT * k;
      if (i <= nr) rpl[i] = rr[k] - d.p0;
    }
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int slot = valid(d, k) ? lds_sw(int(w[k] & (kTile - 1))) : kTile;
      prod[slot] = v[k] * gx[k];
    }
  }
};

// Row sums of a staged tile out of LDS (lane-strided over L lanes); the first
// two rows of each group are returned, later ones go through the epilogue.
template <typename T, int NT, int L, class Epi>
__device__ __forceinline__ void sorted_reduce(const TileDesc& d, const T* prod, const int* rpl, const Epi& epi,
                                              T& s0, T& s1, typename RedOf<Epi>::type& acc) {
  const int t = threadIdx.x, sub = t & (L - 1), grp = t / L;
  constexpr int kGroups = NT / L;
  const int nr = d.row1 - d.row0;
  s0 = T(0);
  s1 = T(0);
  int kk = 0;
  for (int r = grp; r < nr; r += kGroups, ++kk) {
    const int beg = rpl[r], end = rpl[r + 1];
    T s = T(0);
    for (int p = beg + sub; p < end; p += L) s += prod[lds_sw(p)];
    if constexpr (L > 1) {
#pragma unroll
      for (int off = L / 2; off > 0; off >>= 1) s += __shfl_xor(s, off, L);
    }
    if (kk == 0) s0 = s;
    else if (kk == 1) s1 = s;
    else if (sub == 0) acc += epi.row(d.row0 + r, s, d.slice, epi.pre(d.row0 + r));
  }
}

template <typename T, int NT, int L, class Epi>
__device__ __forceinline__ void sorted_finish(const TileDesc& d, const SortedStage<T, NT, L, Epi>& st, T s0, T s1,
                                              const Epi& epi, typename RedOf<Epi>::type& acc) {
  const int t = threadIdx.x, sub = t & (L - 1), grp = t / L;
  constexpr int kGroups = NT / L;
  const int nr = d.row1 - d.row0;
  if (sub == 0) {
    if (grp < nr) acc += epi.row(d.row0 + grp, s0, d.slice, st.q0);
    if (grp + kGroups < nr) acc += epi.row(d.row0 + grp + kGroups, s1, d.slice, st.q1);
  }
}

// One single long row in sort segments of kTile (a multiple of L): row
// element q sits in segment q / kTile, slot q % kTile; the first group keeps
// its lane-strided sums across segments.
template <typename T, int NT, int L, class Epi, class X>
__device__ __forceinline__ void sorted_long_row(const TileDesc& td, const unsigned* __restrict__ gword,
                                                const T* __restrict__ gval, const X& x, T* prod,
                                                const Epi& epi, typename RedOf<Epi>::type& acc) {
  using G = SortGeom<NT>;
  constexpr int kTile = G::kTile, kBits = G::kSlotBits;
  const int t = threadIdx.x, sub = t & (L - 1), grp = t / L;
  T s = T(0);
  for (int c0 = td.p0; c0 < td.p1; c0 += kTile) {
    const int c1 = c0 + kTile < td.p1 ? c0 + kTile : td.p1;
#pragma unroll
    for (int k = 0; k < kSortPerThread; ++k) {
      const int e = c0 + t + NT * k;
      if (e < c1) {
        const unsigned wv = gword[e];
        prod[lds_sw(int(wv & (kTile - 1)))] = gval[e] * x(int64_t(td.pad0) + (wv >> kBits));
      }
    }
    __syncthreads();
    if (grp == 0)
      for (int p = sub; p < c1 - c0; p += L) s += prod[lds_sw(p)];
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

#ifdef KRCN_SORT_TIMING
// Debug builds only (-DKRCN_SORT_TIMING): per-wave phase cycles of the 1024-thread sorted pass.
__device__ unsigned long long krcn_dbg_cycles[1024 * 16 * 8];
#endif

// The tile loop of k_sorted_pass over gathered-vector accessor x.
template <typename T, int L, int NT, class X, class Epi>
__device__ __forceinline__ void sorted_tiles(int rows, int groups, const int* __restrict__ ptr,
                                             const unsigned* __restrict__ gword, const T* __restrict__ gval,
                                             const TileDesc* __restrict__ tiles, const int* __restrict__ tbeg,
                                             const int* __restrict__ tmid, const X& x, const Epi& epi,
                                             double* __restrict__ partials, T* prod, int* rpl, double* sm) {
  const int g = blockIdx.x % groups;
  const int j = blockIdx.x / groups;
  const int stride = gridDim.x / groups;
  typename RedOf<Epi>::type acc{};
  SortedStage<T, NT, L, Epi> st;
#ifdef KRCN_SORT_TIMING
  unsigned long long tc[7] = {0, 0, 0, 0, 0, 0, 0};
#define KRCN_TS(k) { const unsigned long long now = __builtin_amdgcn_s_memtime(); tc[k] += now - tl; tl = now; }
  unsigned long long tl = __builtin_amdgcn_s_memtime();
#else
#define KRCN_TS(k)
#endif
  // the next tile's descriptor is fetched one tile ahead (a scalar load
  // whose latency would otherwise open every tile)
  const int tm = tmid[g];
  TileDesc tn = tbeg[g] + j < tm ? tiles[tbeg[g] + j] : TileDesc{};
  for (int ti = tbeg[g] + j; ti < tm; ti += stride) {
    const TileDesc td = tn;
    if (ti + stride < tm) tn = tiles[ti + stride];
    st.load_nz(td, gword, gval);
    st.load_rows(td, ptr, rows, epi);
    KRCN_TS(0);
    st.gather(td, x);
    KRCN_TS(1);
    st.store(td, prod, rpl);
    KRCN_TS(2);
    __syncthreads();
    KRCN_TS(3);
    T s0, s1;
    sorted_reduce<T, NT, L>(td, prod, rpl, epi, s0, s1, acc);
    KRCN_TS(4);
    sorted_finish<T, NT, L>(td, st, s0, s1, epi, acc);
    KRCN_TS(5);
    __syncthreads();
    KRCN_TS(6);
  }
#ifdef KRCN_SORT_TIMING
  if ((threadIdx.x & 63) == 0 && blockIdx.x < 1024 && NT == 1024) {
    const int wv = threadIdx.x >> 6;
    for (int k = 0; k < 7; ++k) atomicAdd(&krcn_dbg_cycles[(blockIdx.x * 16 + wv) * 8 + k], tc[k]);
  }
#endif
#undef KRCN_TS
  for (int ti = tmid[g] + j; ti < tbeg[g + 1]; ti += stride)
    sorted_long_row<T, NT, L>(tiles[ti], gword, gval, x, prod, epi, acc);
  if constexpr (Epi::kReduce) {
    store_block_red<NT>(acc, sm, partials, epi);
  }
}

// Sorted pass: each block stages, scatters and reduces one tile at a
// time (two barriers per tile); several blocks per CU overlap.
// (the fused step B gathers two vectors: 4 waves per SIMD, 128 VGPRs, no spills)
template <typename T, int L, int NT, class Src, class Epi>
__global__ __launch_bounds__(NT, IsLzZ<Src>::value ? 4 : KRCN_SORT_WAVES) void k_sorted_pass(int rows, int groups, const int* __restrict__ ptr,
                                                    const unsigned* __restrict__ gword,
                                                    const T* __restrict__ gval,
                                                    const TileDesc* __restrict__ tiles,
                                                    const int* __restrict__ tbeg, const int* __restrict__ tmid,
                                                    Src src, Epi epi, double* __restrict__ partials) {
  using G = SortGeom<NT>;
  // Src::begin reduces over the first kNT threads only (sum_partials), so
  // every block size derives the same beta bits
  __shared__ double sm[NT / 64];
  if (src.begin(sm)) return;
  __shared__ T prod[G::kTile + 1];
  __shared__ int rpl[G::kRows + 1];
  epi.init(src);
  if constexpr (IsLzZ<Src>::value) {
    // fused step B: the tiles gather z_j = w - alpha v_{j-1} element by
    // element; this block's share of z_j goes to V[j] with its ||z_j||^2
    // partial (one element per thread loaded before the tiles, so its latency
    // hides behind them; wider shares loop after)
    const int j = src.c.j;
    const T* wz = j == 0 ? src.c.g : src.Wv;
    const T* vz = j == 0 ? src.c.g : src.c.V + int64_t(j - 1) * src.c.ld;
    const T az = j == 0 ? T(0) : src.alpha;
    // the first min(grid, kNT) blocks write z (the combine's beta prologue
    // then preloads one partial per thread)
    const int nw = int(gridDim.x) < kNT ? int(gridDim.x) : kNT;
    const bool writer = j > 0 && int(blockIdx.x) < nw;
    const int64_t d = src.c.ld;
    const int64_t cs = (d + nw - 1) / nw;
    const int64_t c0 = int64_t(blockIdx.x) * cs, c1 = c0 + cs < d ? c0 + cs : d;
    const int64_t i0 = c0 + threadIdx.x;
    const bool one = cs <= NT, has = i0 < c1;
    T w0 = T(0), v0 = T(0);
    if (writer && one) {
      const int64_t ic = has ? i0 : 0;
      w0 = wz[ic];
      v0 = vz[ic];
    }
    sorted_tiles<T, L, NT>(rows, groups, ptr, gword, gval, tiles, tbeg, tmid, GatherZ<T>{wz, vz, az}, epi,
                           partials, prod, rpl, sm);
    if (writer) {
      T* zo = src.c.V + int64_t(j) * d;
      double nz = 0.0;
      if (one) {
        const T zi = w0 - az * v0;
        if (has) {
          zo[i0] = zi;
          nz = double(zi) * double(zi);
        }
      } else {
        for (int64_t i = i0; i < c1; i += NT) {
          const T zi = wz[i] - az * vz[i];
          zo[i] = zi;
          nz += double(zi) * double(zi);
        }
      }
      const double t = block_sum_nt<NT>(nz, sm);
      if (threadIdx.x == 0) src.pz[blockIdx.x] = t;
    }
  } else {
    sorted_tiles<T, L, NT>(rows, groups, ptr, gword, gval, tiles, tbeg, tmid, GatherPtr<T>{src.get()}, epi,
                           partials, prod, rpl, sm);
  }
}


// ------------------------------------------------- sorted-tile builder
// key[e] = (segment of e) << 32 | column of e, for the segments [segs[s], segs[s+1]).
[[maybe_unused]] static __global__ __launch_bounds__(kNT) void k_seg_keys(int nseg, const int* __restrict__ segs,
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
