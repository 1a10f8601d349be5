// krcn_kernels.hpp — CDNA4 (gfx950) device code of the Krylov-CRN hot path.
//
// Everything here is memory-bound (≈0.17 flop/B): no MFMA.  Design rules:
//   * 64-lane waves; CSR rows are reduced by groups of L lanes (L = 1..64) with
//     __shfl_xor butterflies inside the group (width L), so every lane of a
//     group ends with the bit-identical row sum.
//   * Deterministic reductions only (no float atomics): each block reduces its
//     contribution in a fixed tree and stores one partial; the NEXT kernel's
//     blocks each re-sum the partials in the same fixed order (the "combine in
//     the consumer's prologue" form), so every block sees the identical scalar.
//   * The build compiles with -ffp-contract=off so elementwise epilogues round
//     exactly like numpy (separate multiply and add), and a 1-lane row sums left
//     to right like scipy's csr_matvec / csc_matvec.
//
// Reference semantics are cited per kernel (optimizer/loss.py, optimizer/cubic.py).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

namespace krcn {

constexpr int kNT = 256;           // threads per block for every kernel here
constexpr int kUnroll = 4;         // elementwise kernels: independent loads per array per thread

constexpr int kMaxPartials = 2048;  // upper bound on blocks of a reducing launch

// Device-resident Lanczos control state (one per matrix handle).
struct LanczosState {
  int done;        // 1 once |beta| < tol fired (cubic.py:98-99)
  int j_break;     // loop index of the breakdown, -1 otherwise
  int pad0, pad1;
  double gnorm;    // ||g|| (cubic.py:85)
  double beta_last;
};

// ---------------------------------------------------------------- reductions
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// Block-wide sum of one double per thread (kNT threads), fixed order; every
// thread returns the same value.  `sm` must hold kNT/64 doubles.
__device__ __forceinline__ double block_sum(double v, double* sm) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) sm[w] = v;
  __syncthreads();
  double r = (sm[0] + sm[1]) + (sm[2] + sm[3]);
  __syncthreads();
  return r;
}

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

// Sum of P per-block partials, identical in every block that calls it.
// Larger blocks (sorted tiles) leave threads >= kNT out, so the bits match.
__device__ __forceinline__ double sum_partials(const double* __restrict__ p, int P, double* sm) {
  double v = 0.0;
  if (threadIdx.x < kNT)
    for (int i = threadIdx.x; i < P; i += kNT) v += p[i];
  return block_sum(v, sm);
}

// Two per-block partial sums reduced together: an epilogue whose row()
// returns Red2 names the array of the second (EpiLz2E: ||z||^2 and z.v).
// Kernels hold `typename RedOf<Epi>::type red` and finish with
// store_block_red, which writes one partial per block in a fixed order.
struct Red2 {
  double a = 0.0, b = 0.0;
  __device__ __forceinline__ Red2& operator+=(const Red2& o) {
    a += o.a;
    b += o.b;
    return *this;
  }
};
template <class E, class = void> struct RedOf { using type = double; };
template <class E> struct RedOf<E, std::void_t<typename E::Red>> { using type = typename E::Red; };

template <int NT, class Epi>
__device__ __forceinline__ void store_block_red(double v, double* sm, double* partials, const Epi&) {
  const double t = block_sum_nt<NT>(v, sm);
  if (threadIdx.x == 0) partials[blockIdx.x] = t;
}
template <int NT, class Epi>
__device__ __forceinline__ void store_block_red(const Red2& v, double* sm, double* partials, const Epi& epi) {
  const double ta = block_sum_nt<NT>(v.a, sm);
  const double tb = block_sum_nt<NT>(v.b, sm);
  if (threadIdx.x == 0) {
    partials[blockIdx.x] = ta;
    epi.part2[blockIdx.x] = tb;
  }
}

// The Lanczos state flag and sum_partials(p, P) (P <= 2 kNT) with both loads
// issued together: one memory latency instead of two.  Same sums in the same
// order as sum_partials.  Returns the flag (every thread).
__device__ __forceinline__ int flag_and_sum(const int* flag, const double* __restrict__ p, int P, double* sm,
                                            double* out) {
  __shared__ int fl;
  int f = 0;
  double a = 0.0, b = 0.0;
  if (threadIdx.x == 0) f = __hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (threadIdx.x < kNT && int(threadIdx.x) < P) a = p[threadIdx.x];
  if (threadIdx.x < kNT && int(threadIdx.x) + kNT < P) b = p[threadIdx.x + kNT];
  if (threadIdx.x == 0) fl = f;
  double v = 0.0;
  if (threadIdx.x < kNT && int(threadIdx.x) < P) v += a;
  if (threadIdx.x < kNT && int(threadIdx.x) + kNT < P) v += b;
  const double r = block_sum(v, sm);   // its barriers publish fl
  *out = r;
  return fl;
}

// ------------------------------------------------------------- store policy
// Stores whose bytes the NEXT launch reads (slice partials, Lanczos vectors)
// may leave the XCD's L2 during the launch instead of at its end:
//   0 plain (line kept dirty in L2, written back at the kernel boundary),
//   1 sc1 write-through (agent-scope relaxed atomic store; the line is dropped),
//   2 nontemporal.
// A/B knobs for now (-DKRCN_PART_ST=..., -DKRCN_VEC_ST=...); results are
// bitwise the same under every policy.
#ifndef KRCN_PART_ST
#define KRCN_PART_ST 0
#endif
#ifndef KRCN_VEC_ST
#define KRCN_VEC_ST 0
#endif
template <int kPolicy, typename T>
__device__ __forceinline__ void store_policy(T* p, T v) {
  if constexpr (kPolicy == 1) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  } else if constexpr (kPolicy == 2) {
    __builtin_nontemporal_store(v, p);
  } else {
    *p = v;
  }
}

// ------------------------------------------------------- logistic functions
// scipy.special.expit (loss.py:225,296): 1 / (1 + exp(-x)).
template <typename T> __device__ __forceinline__ T expit(T x) { return T(1) / (T(1) + exp(-x)); }

// logsig, loss.py:161-176 (piecewise, http://fa.bianp.net/blog/2019/evaluate_logistic/).
template <typename T> __device__ __forceinline__ T logsig(T x) {
  if (x < T(-33)) return x;
  if (x < T(-18)) return x - exp(x);
  if (x < T(37)) return -log1p(exp(-x));
  return -exp(-x);
}

// --------------------------------------------------------------- epilogues
// Epilogues receive (row r, row sum s) on the group's lane 0 and return a
// double contribution to the block partial (0 when the launch does not reduce).
// The row passes themselves live in krcn_tiled.hpp.

// Epilogue interface: init(src) once per block (after the source's prologue),
// pre(r) loads the row's operands (issued before the tile's LDS phase so the
// loads overlap it), row(r, s, slice, pre) consumes the row sum and returns a
// double contribution to the block partial (0 when the launch does not reduce).

// out[r] = s                                (A @ x, loss.py:270; raw shard partials)
template <typename T> struct EpiStore {
  T* out;
  static constexpr bool kReduce = false;
  struct Pre {};
  template <class S> __device__ __forceinline__ void init(const S&) {}
  __device__ __forceinline__ Pre pre(int) const { return Pre{}; }
  __device__ __forceinline__ double row(int r, T s, int, const Pre&) const { out[r] = s; return 0.0; }
};

// u[r] = w[r] * s                           (np.multiply(weights, Av), loss.py:301)
template <typename T> struct EpiWeighted {
  const T* w; T* u;
  static constexpr bool kReduce = false;
  struct Pre { T wr; };
  template <class S> __device__ __forceinline__ void init(const S&) {}
  __device__ __forceinline__ Pre pre(int r) const { return Pre{w[r]}; }
  __device__ __forceinline__ double row(int r, T s, int, const Pre& p) const { u[r] = p.wr * s; return 0.0; }
};

// y[r] = s / n + l2 * v[r]                  (A.T @ u / self.n + self.l2 * v, loss.py:302)
// kL2 = false (l2 == 0): y = s / n without reading v.  The reference's
// s / n + 0 * v has the same bits for every finite v (s is never -0: every
// row sum starts from +0), so the d-vector read the algorithmic byte count
// does not include is skipped (news20: 10.8 MB of pass 2).
template <typename T, bool kL2 = true> struct EpiHvpOut {
  const T* v; T* y; T n; T l2;
  static constexpr bool kReduce = false;
  struct Pre { T vr; };
  template <class S> __device__ __forceinline__ void init(const S&) {}
  __device__ __forceinline__ Pre pre(int r) const {
    if constexpr (kL2) return Pre{v[r]};
    else return Pre{T(0)};
  }
  __device__ __forceinline__ double row(int r, T s, int, const Pre& p) const {
    if constexpr (kL2) y[r] = s / n + l2 * p.vr;
    else y[r] = s / n;
    return 0.0;
  }
};

// g[r] = s / n (+ l2 * x[r])               (loss.py:227 / :229)
template <typename T> struct EpiGrad {
  const T* x; T* g; T n; T l2; int has_l2;
  static constexpr bool kReduce = false;
  struct Pre { T xr; };
  template <class S> __device__ __forceinline__ void init(const S&) {}
  // x may be null when l2 == 0: never touch it then
  __device__ __forceinline__ Pre pre(int r) const { return Pre{has_l2 ? x[r] : T(0)}; }
  __device__ __forceinline__ double row(int r, T s, int, const Pre& p) const {
    const T q = s / n;
    g[r] = has_l2 ? q + l2 * p.xr : q;
    return 0.0;
  }
};

// -------------------------------------------------------- vector kernels
// w_i = s (1 - s), s = expit(Ax_i)            (loss.py:296-297)
template <typename T>
__global__ __launch_bounds__(kNT) void k_weights(int64_t n, const T* __restrict__ Ax, T* __restrict__ w) {
  for (int64_t i = int64_t(blockIdx.x) * kNT + threadIdx.x; i < n; i += int64_t(gridDim.x) * kNT) {
    const T a = expit(Ax[i]);
    w[i] = a * (T(1) - a);
  }
}

// r_i = expit(Ax_i) - b_i                     (activation - self.b, loss.py:225,227)
template <typename T>
__global__ __launch_bounds__(kNT) void k_residual(int64_t n, const T* __restrict__ Ax,
                                                  const T* __restrict__ b, T* __restrict__ r) {
  for (int64_t i = int64_t(blockIdx.x) * kNT + threadIdx.x; i < n; i += int64_t(gridDim.x) * kNT)
    r[i] = expit(Ax[i]) - b[i];
}

// partial sums of (1 - b_i) Ax_i - logsig(Ax_i)   (loss.py:220)
template <typename T>
__global__ __launch_bounds__(kNT) void k_loss_terms(int64_t n, const T* __restrict__ Ax,
                                                    const T* __restrict__ b,
                                                    double* __restrict__ partials) {
  double acc = 0.0;
  for (int64_t i = int64_t(blockIdx.x) * kNT + threadIdx.x; i < n; i += int64_t(gridDim.x) * kNT) {
    const T a = Ax[i];
    const T t = (T(1) - b[i]) * a - logsig(a);
    acc += double(t);
  }
  __shared__ double sm[kNT / 64];
  const double t = block_sum(acc, sm);
  if (threadIdx.x == 0) partials[blockIdx.x] = t;
}

// partial sums of (a_i - b_i)^2 or a_i^2 (b == nullptr) or a_i*b_i (dot)
template <typename T, int kMode>  // 0: dot(a,b)  1: ||a||^2  2: ||a-b||^2
__global__ __launch_bounds__(kNT) void k_reduce2(int64_t n, const T* __restrict__ a,
                                                 const T* __restrict__ b,
                                                 double* __restrict__ partials) {
  double acc = 0.0;
  for (int64_t i = int64_t(blockIdx.x) * kNT + threadIdx.x; i < n; i += int64_t(gridDim.x) * kNT) {
    if constexpr (kMode == 0) acc += double(a[i]) * double(b[i]);
    if constexpr (kMode == 1) { const double t = a[i]; acc += t * t; }
    if constexpr (kMode == 2) { const T t = a[i] - b[i]; acc += double(t) * double(t); }
  }
  __shared__ double sm[kNT / 64];
  const double t = block_sum(acc, sm);
  if (threadIdx.x == 0) partials[blockIdx.x] = t;
}

// One block: out[0] = scale(sum of partials).  kSqrt: out = sqrt(sum).
template <int kSqrt>
__global__ __launch_bounds__(kNT) void k_finish(const double* __restrict__ partials, int P,
                                                double* __restrict__ out) {
  __shared__ double sm[kNT / 64];
  const double s = sum_partials(partials, P, sm);
  if (threadIdx.x == 0) out[0] = kSqrt ? sqrt(s) : s;
}

// ----------------------------------------------------- Lanczos recurrence
// Device-side control of the three-term Lanczos of cubic.py:77-111.
//
// Storage: row j of V (m x ld) is the reference's column V[:, j].  Each new
// vector is stored UNNORMALISED (z_{j+1} = w - alpha v_j, written by step B)
// together with the partial sums of ||z||^2; the next iteration's pass 1
// reduces them to beta (in every block, identical), applies the reference's
// absolute breakdown test |beta| < tol (cubic.py:98), and pass 2 divides
// z by beta in place — the reference's v = w / beta (cubic.py:102), same
// IEEE division.  Iteration 0 treats g the same way with ||g|| (cubic.py:85).
// Per iteration this is pass 1 (+ slice combine), pass 2 (+ step A), step B.
template <typename T> struct LzCtl {
  T* V; const T* g; int64_t ld; int m; int j; int mode;  // mode 0: loop step j; 1: final quotient
  LanczosState* st; double* betas; const double* pnorm; int Pnorm; double tol;
};

// The vector a pass works on: z (to be divided by div when normalize).
template <typename T> struct LzVec {
  const T* z; T div; int jc; int normalize;
};

// Read an int that another block of the SAME launch may be writing, once per
// block, so that every thread takes the same branch.
__device__ __forceinline__ int block_uniform_load(const int* p) {
  __shared__ int v;
  if (threadIdx.x == 0) v = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  const int r = v;
  __syncthreads();
  return r;
}

// State written by earlier launches (kernel boundaries order it): which
// vector the current step uses and how to normalise it.
template <typename T>
__device__ __forceinline__ LzVec<T> lz_vec_from_state(const LzCtl<T>& c) {
  LzVec<T> r;
  if (c.mode == 0) {
    r.jc = c.j;
    r.normalize = 1;
    r.z = c.j == 0 ? c.g : c.V + int64_t(c.j) * c.ld;
    r.div = c.j == 0 ? T(c.st->gnorm) : T(c.betas[c.j - 1]);
  } else if (c.st->done) {            // truncated basis: quotient of the last kept vector
    r.jc = c.st->j_break;
    r.normalize = 0;
    r.z = c.V + int64_t(r.jc) * c.ld;
    r.div = T(1);
  } else {
    r.jc = c.m - 1;
    r.normalize = 1;
    r.z = c.m == 1 ? c.g : c.V + int64_t(c.m - 1) * c.ld;
    r.div = c.m == 1 ? T(c.st->gnorm) : T(c.betas[c.m - 2]);
  }
  return r;
}

// First launch of loop step j: beta_{j-1} (or ||g|| at j = 0) from the norm
// partials, the breakdown test, and the state update (block 0).  Returns
// true when the block must skip (the recurrence has ended).
template <typename T>
__device__ __forceinline__ bool lz_step_prologue(const LzCtl<T>& c, double* sm, LzVec<T>& out) {
  if (c.j > 0 && block_uniform_load(&c.st->done)) return true;
  const double nrm = sqrt(sum_partials(c.pnorm, c.Pnorm, sm));
  const bool lead = blockIdx.x == 0 && threadIdx.x == 0;
  if (c.j == 0) {
    if (lead) { c.st->done = 0; c.st->j_break = -1; c.st->gnorm = nrm; c.st->beta_last = 0.0; }
    out.z = c.g; out.div = T(nrm); out.jc = 0; out.normalize = 1;
    return false;
  }
  if (fabs(nrm) < c.tol) {
    if (lead) { c.st->j_break = c.j - 1; c.st->beta_last = nrm; c.st->done = 1; }
    return true;
  }
  if (lead) { c.betas[c.j - 1] = nrm; c.st->beta_last = nrm; }
  out.z = c.V + int64_t(c.j) * c.ld; out.div = T(nrm); out.jc = c.j; out.normalize = 1;
  return false;
}

// lz_step_prologue with its operands loaded early by the caller (SrcLzStep::
// preload): flag = st->done (thread 0), pv = pnorm[tid] (tid < Pnorm <= kNT).
// The same reductions in the same order: bitwise the same beta.
template <typename T>
__device__ __forceinline__ bool lz_step_prologue_pre(const LzCtl<T>& c, double* sm, LzVec<T>& out, int flag,
                                                     double pv) {
  if (c.j > 0) {
    __shared__ int flag_sm;
    if (threadIdx.x == 0) flag_sm = flag;
    __syncthreads();
    const int done = flag_sm;
    __syncthreads();
    if (done) return true;
  }
  const double nrm = sqrt(block_sum(threadIdx.x < kNT && threadIdx.x < c.Pnorm ? 0.0 + pv : 0.0, sm));
  const bool lead = blockIdx.x == 0 && threadIdx.x == 0;
  if (c.j == 0) {
    if (lead) { c.st->done = 0; c.st->j_break = -1; c.st->gnorm = nrm; c.st->beta_last = 0.0; }
    out.z = c.g; out.div = T(nrm); out.jc = 0; out.normalize = 1;
    return false;
  }
  if (fabs(nrm) < c.tol) {
    if (lead) { c.st->j_break = c.j - 1; c.st->beta_last = nrm; c.st->done = 1; }
    return true;
  }
  if (lead) { c.betas[c.j - 1] = nrm; c.st->beta_last = nrm; }
  out.z = c.V + int64_t(c.j) * c.ld; out.div = T(nrm); out.jc = c.j; out.normalize = 1;
  return false;
}

// Pass-2 epilogue (step A, cubic.py:93-94 with the deferred v = z / beta):
//   v = z / div (stored back in place), y = s/n + l2 v,
//   mode 0: w = y - beta_{j-1} v_pre (w = y at j = 0), W = w, partial v.w;
//   mode 1: partial v.y (the final alphas[-1] = v . A(v), cubic.py:109).
//   zw (the window-slices fused pass 1 stores no z_j): z_j is formed here from
//   w of step j-1 (still in W: this row's read precedes its write) and
//   v_{j-1}, z_j = W - alpha_{j-1} v_{j-1} — the expression and operands of
//   the pass-1 window (SrcLzZ), so the same bits — saving pass 1 its store of
//   z_j and this pass its read of it.
// Sources that settle beta themselves in this launch (SrcLzU: the pass-2
// prologue of the two-launch step) hand their LzVec to EpiLz2 instead of the
// betas array, which the same launch's block 0 is writing.
template <class S, class = void> struct StepVecSrc : std::false_type {};
template <class S> struct StepVecSrc<S, std::void_t<decltype(S::kStepVec)>> : std::bool_constant<S::kStepVec> {};

template <typename T> struct EpiLz2 {
  LzCtl<T> c; T* W; T n; T l2;
  const double* alphas = nullptr; int zw = 0;
  LzVec<T> lv; T* vout; const T* vpre; T bsub; int first; int zon; T alz;
  static constexpr bool kReduce = true;
  struct Pre { T z, vp; };
  template <class S> __device__ __forceinline__ void init(const S& src) {
    if constexpr (StepVecSrc<S>::value) lv = src.v;
    else lv = lz_vec_from_state(c);
    vout = c.V + int64_t(lv.jc) * c.ld;
    first = c.mode == 1 || lv.jc == 0;
    vpre = first ? lv.z : c.V + int64_t(lv.jc - 1) * c.ld;
    if constexpr (StepVecSrc<S>::value) bsub = first ? T(0) : lv.div;   // = betas[jc - 1], settled in this launch
    else bsub = first ? T(0) : T(c.betas[lv.jc - 1]);
    zon = zw && !first && lv.normalize;
    alz = zon ? T(alphas[lv.jc - 1]) : T(0);
  }
  __device__ __forceinline__ Pre pre(int r) const {
    return Pre{zon ? W[r] : lv.z[r], first ? T(0) : vpre[r]};
  }
  __device__ __forceinline__ double row(int r, T s, int, const Pre& p) const {
    const T z = zon ? p.z - alz * p.vp : p.z;
    const T v = lv.normalize ? z / lv.div : z;
    if (lv.normalize) store_policy<KRCN_VEC_ST>(vout + r, v);
    const T y = s / n + l2 * v;
    if (c.mode == 1) return double(v) * double(y);
    const T w = first ? y : y - bsub * p.vp;
    store_policy<KRCN_VEC_ST>(W + r, w);
    return double(v) * double(w);
  }
};

// Epilogues whose pre() does not depend on init() / the source prologue
// (kPreEarly): a combine loads their operands together with the partials.
template <class E, class = void> struct PreEarly : std::false_type {};
template <class E> struct PreEarly<E, std::void_t<decltype(E::kPreEarly)>> : std::bool_constant<E::kPreEarly> {};

// Pass-1 epilogue of a Lanczos step: u_i = w_i * (t_i / div)  (t = X z).
template <typename T> struct EpiLz1 {
  const T* w; T* u; T div;
  static constexpr bool kReduce = false;
  static constexpr bool kPreEarly = true;   // pre() reads only w: loadable before the source prologue
  struct Pre { T wr; };
  template <class S> __device__ __forceinline__ void init(const S& src) { div = src.v.div; }
  __device__ __forceinline__ Pre pre(int r) const { return Pre{w[r]}; }
  __device__ __forceinline__ double row(int r, T s, int, const Pre& p) const {
    u[r] = p.wr * (s / div);
    return 0.0;
  }
};

// ------------------------------------------------- early-alpha Lanczos step
// Window-slices plans (news20's pass 1, krcn_lanczos_impl.hpp) settle
// alpha_j before pass 2 instead of after it, so step B runs inside pass 2's
// epilogue and pass 1 gathers a stored z_j (one window stream, no alpha
// reduction in its prologue) instead of forming z_j = w - alpha v_{j-1} from
// two.  The reference's alpha_j = v_j . w (cubic.py:93-95) with
// w = A(v_j) - beta_{j-1} v_{j-1} and A(v) = X^T (D (X v)) / n + l2 v
// (loss.py:299-302) is, by X^T's adjoint,
//   alpha_j = (X v_j).(D (X v_j)) / n + l2 ||v_j||^2 - beta_{j-1} v_j.v_{j-1}
// with v_j = z_j / beta_{j-1}, so beta_{j-1} v_j.v_{j-1} = z_j . v_{j-1}:
//   * (X v_j).(D (X v_j)) = sum_r u_r q_r over the slice combine's rows
//     (q = t / beta, u = w q: EpiLz1A's partials);
//   * ||v_j||^2 = 1 (v_j is z_j over its own norm; rounding-level);
//   * z_j . v_{j-1}: partials that the previous pass 2 formed beside
//     ||z_j||^2 (EpiLz2E), keeping the modified-Gram-Schmidt form of the
//     reference (dropping the term would let local orthogonality errors carry
//     from step to step scaled by beta_{j-1} / beta_j).
// Equal to the reference's v.w in exact arithmetic; the computed values differ
// at the rounding level, like any reordering of the HVP's sums (tests: the
// golden Lanczos and breakdown fixtures on window-slices plans at 1e-11,
// news20 within its measured 1e-7 envelope).

// Combine epilogue: u = w (t / div) as EpiLz1, plus the partials of u.(t / div).
template <typename T> struct EpiLz1A {
  const T* w; T* u; T div;
  static constexpr bool kReduce = true;
  static constexpr bool kPreEarly = true;
  struct Pre { T wr; };
  template <class S> __device__ __forceinline__ void init(const S& src) { div = src.v.div; }
  __device__ __forceinline__ Pre pre(int r) const { return Pre{w[r]}; }
  __device__ __forceinline__ double row(int r, T s, int, const Pre& p) const {
    const T q = s / div;
    const T ur = p.wr * q;
    u[r] = ur;
    return double(ur) * double(q);
  }
};

// Pass-2 epilogue (the source, SrcLzAlpha, settled alpha_j in the prologue):
//   v_j = z_j / beta_{j-1} stored in place (z_0 = g over ||g||: V[0]),
//   y = s/n + l2 v, w = y - beta_{j-1} v_{j-1} (w = y at j = 0),
//   z_{j+1} = w - alpha_j v_j stored unnormalised in V[j+1] (cubic.py:93-96,
//   the reference's expressions in its order); partials of ||z_{j+1}||^2
//   (the next pass 1 settles beta_j from them) and of z_{j+1}.v_j (the next
//   alpha) — two sums per block (Red2).
template <typename T> struct EpiLz2E {
  LzCtl<T> c; T n; T l2; double* part2;
  LzVec<T> lv; T* znext; const T* vpre; T bsub; T al; int first;
  static constexpr bool kReduce = true;
  using Red = Red2;
  struct Pre { T z, vp; };
  template <class S> __device__ __forceinline__ void init(const S& src) {
    lv = lz_vec_from_state(c);
    znext = c.V + int64_t(lv.jc + 1) * c.ld;
    first = lv.jc == 0;
    vpre = first ? lv.z : c.V + int64_t(lv.jc - 1) * c.ld;
    bsub = first ? T(0) : T(c.betas[lv.jc - 1]);
    al = src.alpha;
  }
  // pre() reads no state (loop steps are mode 0: z_j = V[j], or g at j = 0,
  // as lz_vec_from_state gives them), so its loads may precede init()
  static constexpr bool kPreEarly = true;
  __device__ __forceinline__ Pre pre(int r) const {
    const T* z = c.j == 0 ? c.g : c.V + int64_t(c.j) * c.ld;
    return Pre{z[r], c.j == 0 ? T(0) : c.V[int64_t(c.j - 1) * c.ld + r]};
  }
  __device__ __forceinline__ Red2 row(int r, T s, int, const Pre& p) const {
    const T v = p.z / lv.div;
    store_policy<KRCN_VEC_ST>(c.V + int64_t(lv.jc) * c.ld + r, v);
    const T y = s / n + l2 * v;
    const T w = first ? y : y - bsub * p.vp;
    const T z = w - al * v;
    store_policy<KRCN_VEC_ST>(znext + r, z);
    return Red2{double(z) * double(z), double(z) * double(v)};
  }
};

// Step B (cubic.py:94-97): alpha = v.w (pass-2 partials), alphas[j] = alpha,
// z_{j+1} = W - alpha v stored unnormalised in V[j+1], partials of ||z||^2.
template <typename T>
__global__ __launch_bounds__(kNT) void k_lz_step_b(int64_t d, const T* __restrict__ W, LzCtl<T> c,
                                                   const double* __restrict__ pa, int Pa,
                                                   double* __restrict__ alphas_dev,
                                                   double* __restrict__ pnorm_out) {
  if (c.st->done) return;
  __shared__ double sm[kNT / 64];
  const double alpha = sum_partials(pa, Pa, sm);
  const T ta = T(alpha);
  const T* v = c.V + int64_t(c.j) * c.ld;
  T* z = c.V + int64_t(c.j + 1) * c.ld;
  double acc = 0.0;
  // kUnroll independent coalesced loads per array in flight per thread
  constexpr int U = kUnroll;
  for (int64_t i0 = int64_t(blockIdx.x) * (kNT * U) + threadIdx.x; i0 < d; i0 += int64_t(gridDim.x) * (kNT * U)) {
    T wv[U], vv[U];
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const int64_t i = i0 + int64_t(k) * kNT;
      wv[k] = i < d ? W[i] : T(0);
      vv[k] = i < d ? v[i] : T(0);
    }
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const int64_t i = i0 + int64_t(k) * kNT;
      if (i < d) {
        const T zi = wv[k] - ta * vv[k];
        z[i] = zi;
        acc += double(zi) * double(zi);
      }
    }
  }
  const double t = block_sum(acc, sm);
  if (threadIdx.x == 0) pnorm_out[blockIdx.x] = t;
  if (blockIdx.x == 0 && threadIdx.x == 0) alphas_dev[c.j] = alpha;
}

// Start of a recurrence: zero alphas[0..m) and betas[0..m) (block 0) and the
// partials of ||g||^2 (cubic.py:85).
template <typename T>
__global__ __launch_bounds__(kNT) void k_lz_begin(int64_t d, const T* __restrict__ g, int m,
                                                  double* __restrict__ alphas, double* __restrict__ betas,
                                                  double* __restrict__ partials) {
  if (blockIdx.x == 0)
    for (int i = threadIdx.x; i < m; i += kNT) {
      alphas[i] = 0.0;
      betas[i] = 0.0;
    }
  double acc = 0.0;
  for (int64_t i = int64_t(blockIdx.x) * kNT + threadIdx.x; i < d; i += int64_t(gridDim.x) * kNT) {
    const double t = g[i];
    acc += t * t;
  }
  __shared__ double sm[kNT / 64];
  const double t = block_sum(acc, sm);
  if (threadIdx.x == 0) partials[blockIdx.x] = t;
}

// Before the final quotient: settle beta_{m-2} (breakdown at j = m-2 keeps a
// zero last column, cubic.py:105-108) or, for m = 1, reset the state.
template <typename T>
__global__ __launch_bounds__(kNT) void k_lz_final_check(LzCtl<T> c) {
  __shared__ double sm[kNT / 64];
  const double nrm = sqrt(sum_partials(c.pnorm, c.Pnorm, sm));
  if (threadIdx.x != 0) return;
  if (c.m == 1) {
    c.st->done = 0; c.st->j_break = -1; c.st->gnorm = nrm; c.st->beta_last = 0.0;
    return;
  }
  if (c.st->done) return;
  if (fabs(nrm) < c.tol) {
    c.st->done = 1; c.st->j_break = c.m - 2; c.st->beta_last = nrm;
  } else {
    c.betas[c.m - 2] = nrm; c.st->beta_last = nrm;
  }
}

// Final (cubic.py:105-109): alphas[slot] = v.A(v), slot = j_break when the
// basis was truncated (j_break < m-2) and m-1 otherwise; a breakdown at
// j = m-2 zeroes the unnormalised V[m-1] (the reference never wrote it).
// Block 0 then packs the state, alphas[0..m) and betas[0..m-1) into `out`
// (one D2H of 2 m + 3 doubles).
template <typename T>
__global__ __launch_bounds__(kNT) void k_lz_final(const double* __restrict__ pa, int Pa, LzCtl<T> c,
                                                  double* __restrict__ alphas_dev, double* __restrict__ out) {
  const bool quirk = c.st->done && c.st->j_break == c.m - 2;
  if (blockIdx.x == 0) {
    __shared__ double sm[kNT / 64];
    const double alpha = sum_partials(pa, Pa, sm);
    const int slot = (c.st->done && c.st->j_break < c.m - 2) ? c.st->j_break : c.m - 1;
    for (int i = threadIdx.x; i < c.m; i += kNT) out[4 + i] = i == slot ? alpha : alphas_dev[i];
    for (int i = threadIdx.x; i + 1 < c.m; i += kNT) out[4 + c.m + i] = c.betas[i];
    if (threadIdx.x == 0) *reinterpret_cast<LanczosState*>(out) = *c.st;
  }
  if (quirk) {
    T* z = c.V + int64_t(c.m - 1) * c.ld;
    for (int64_t i = int64_t(blockIdx.x) * kNT + threadIdx.x; i < c.ld; i += int64_t(gridDim.x) * kNT)
      z[i] = T(0);
  }
}

// ---------------------------------------------------------- basis combine
// x_new = x + V^T s (cubic.py:291): per column, sum_j V[j,i] s_j in j order.
// s is staged in LDS and each thread issues kBasisU row loads before it adds
// them (in j order: the same sums as one load at a time), so a CU keeps
// enough loads in flight to stream V (m x d, 1.08 GB at news20 m = 100).
constexpr int kBasisMaxM = 2048;   // >= the Lanczos workspace's largest m (krcn_lanczos: m <= 2044)
constexpr int kBasisU = 16;
template <typename T>
__global__ __launch_bounds__(kNT) void k_basis_combine(int64_t d, int m, const T* __restrict__ V,
                                                       const double* __restrict__ s,
                                                       const T* __restrict__ x, T* __restrict__ xn) {
  __shared__ T ss[kBasisMaxM];
  for (int j = threadIdx.x; j < m; j += kNT) ss[j] = T(s[j]);
  __syncthreads();
  for (int64_t i = int64_t(blockIdx.x) * kNT + threadIdx.x; i < d; i += int64_t(gridDim.x) * kNT) {
    T acc = T(0);
    int j = 0;
    for (; j + kBasisU <= m; j += kBasisU) {
      T v[kBasisU];
#pragma unroll
      for (int u = 0; u < kBasisU; ++u) v[u] = V[int64_t(j + u) * d + i];
#pragma unroll
      for (int u = 0; u < kBasisU; ++u) acc += v[u] * ss[j + u];
    }
    for (; j < m; ++j) acc += V[int64_t(j) * d + i] * ss[j];
    xn[i] = x[i] + acc;
  }
}

// ------------------------------------------------------ transpose helpers
// row id of every nonzero (expands indptr).
[[maybe_unused]] static __global__ __launch_bounds__(kNT) void k_expand_rows(int n, const int* __restrict__ ptr,
                                                     int* __restrict__ rowid) {
  const int lane = threadIdx.x & 63;
  const int wv = (blockIdx.x * kNT + threadIdx.x) >> 6;
  const int W = (gridDim.x * kNT) >> 6;
  for (int r = wv; r < n; r += W)
    for (int p = ptr[r] + lane; p < ptr[r + 1]; p += 64) rowid[p] = r;
}

[[maybe_unused]] static __global__ __launch_bounds__(kNT) void k_iota(int64_t n, int* __restrict__ out) {
  for (int64_t i = int64_t(blockIdx.x) * kNT + threadIdx.x; i < n; i += int64_t(gridDim.x) * kNT)
    out[i] = int(i);
}

// colptr[c] = first position of key c in the sorted key array (lower bound),
// computed per column by binary search; colptr[d] = nnz.
[[maybe_unused]] static __global__ __launch_bounds__(kNT) void k_colptr_from_sorted(int64_t d, int64_t nnz,
                                                            const int* __restrict__ keys,
                                                            int* __restrict__ colptr) {
  for (int64_t c = int64_t(blockIdx.x) * kNT + threadIdx.x; c <= d; c += int64_t(gridDim.x) * kNT) {
    int64_t lo = 0, hi = nnz;
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if (keys[mid] < c) lo = mid + 1; else hi = mid;
    }
    colptr[c] = int(lo);
  }
}

template <typename T>
__global__ __launch_bounds__(kNT) void k_gather_transpose(int64_t nnz, const int* __restrict__ perm,
                                                          const int* __restrict__ rowid,
                                                          const T* __restrict__ val,
                                                          int* __restrict__ t_idx, T* __restrict__ t_val) {
  for (int64_t p = int64_t(blockIdx.x) * kNT + threadIdx.x; p < nnz; p += int64_t(gridDim.x) * kNT) {
    const int e = perm[p];
    t_idx[p] = rowid[e];
    t_val[p] = val[e];
  }
}

}  // namespace krcn
