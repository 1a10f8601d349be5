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

namespace krcn {

constexpr int kNT = 256;           // threads per block for every kernel here
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

// Sum of P per-block partials, identical in every block that calls it.
__device__ __forceinline__ double sum_partials(const double* __restrict__ p, int P, double* sm) {
  double v = 0.0;
  for (int i = threadIdx.x; i < P; i += kNT) v += p[i];
  return block_sum(v, sm);
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

// out[r] = s                                (A @ x, loss.py:270; raw shard partials)
template <typename T> struct EpiStore {
  T* out;
  static constexpr bool kReduce = false;
  __device__ __forceinline__ double row(int r, T s) const { out[r] = s; return 0.0; }
};

// u[r] = w[r] * s                           (np.multiply(weights, Av), loss.py:301)
template <typename T> struct EpiWeighted {
  const T* w; T* u;
  static constexpr bool kReduce = false;
  __device__ __forceinline__ double row(int r, T s) const { u[r] = w[r] * s; return 0.0; }
};

// y[r] = s / n + l2 * v[r]                  (A.T @ u / self.n + self.l2 * v, loss.py:302)
template <typename T> struct EpiHvpOut {
  const T* v; T* y; T n; T l2;
  static constexpr bool kReduce = false;
  __device__ __forceinline__ double row(int r, T s) const { y[r] = s / n + l2 * v[r]; return 0.0; }
};

// g[r] = s / n (+ l2 * x[r])               (loss.py:227 / :229)
template <typename T> struct EpiGrad {
  const T* x; T* g; T n; T l2; int has_l2;
  static constexpr bool kReduce = false;
  __device__ __forceinline__ double row(int r, T s) const {
    const T q = s / n;
    if (has_l2) g[r] = q + l2 * x[r];   // x may be null when l2 == 0: never touch it
    else g[r] = q;
    return 0.0;
  }
};

// Lanczos step A, fused into pass 2 (cubic.py:93-94):
//   y = s/n + l2 v ; w = y - beta * v_pre ; W[r] = w ; alpha partial += v * w.
// first (j == 0): the reference subtracts 0 * zeros, i.e. w = y exactly.
template <typename T> struct EpiLanczosA {
  const T* v; const T* vpre; T* W; T n; T l2; T beta; int first; int store;
  static constexpr bool kReduce = true;
  __device__ __forceinline__ double row(int r, T s) const {
    const T vr = v[r];
    const T y = s / n + l2 * vr;
    const T w = first ? y : y - beta * vpre[r];
    if (store) W[r] = w;
    return double(vr) * double(w);
  }
};

// A Lanczos vector selector: loop iteration j (mode 0, x = V[j]) or the final
// Rayleigh quotient (mode 1, cubic.py:109) whose vector comes from the state.
template <typename T> struct LanczosRef {
  const T* V; int64_t ld; int m; int j; int mode;
  const LanczosState* st;
  __device__ __forceinline__ int cur() const {
    if (mode == 0) return j;
    return st->done ? st->j_break : (m - 1);
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

// ----------------------------------------------------- Lanczos vector steps
// Start (cubic.py:82-88): V[0] = g / ||g||, state reset.  Runs after a
// k_reduce2<T,1> over g wrote the partials of ||g||^2.
template <typename T>
__global__ __launch_bounds__(kNT) void k_lanczos_start(int64_t d, const T* __restrict__ g,
                                                       T* __restrict__ V0,
                                                       const double* __restrict__ partials, int P,
                                                       LanczosState* st) {
  __shared__ double sm[kNT / 64];
  const double nrm = sqrt(sum_partials(partials, P, sm));
  const T tn = T(nrm);
  for (int64_t i = int64_t(blockIdx.x) * kNT + threadIdx.x; i < d; i += int64_t(gridDim.x) * kNT)
    V0[i] = g[i] / tn;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    st->done = 0; st->j_break = -1; st->gnorm = nrm; st->beta_last = 0.0;
  }
}

// Step B (cubic.py:94-97): alpha = v.w (from pass-2 partials); alphas[j] = alpha;
// W = W - alpha v; partial ||W||^2.
template <typename T>
__global__ __launch_bounds__(kNT) void k_lanczos_b(int64_t d, T* __restrict__ W, const T* __restrict__ v,
                                                   const double* __restrict__ pa, int Pa,
                                                   double* __restrict__ alphas_dev, int j,
                                                   const LanczosState* st,
                                                   double* __restrict__ pb) {
  if (st->done) return;
  __shared__ double sm[kNT / 64];
  const double alpha = sum_partials(pa, Pa, sm);
  const T ta = T(alpha);
  double acc = 0.0;
  for (int64_t i = int64_t(blockIdx.x) * kNT + threadIdx.x; i < d; i += int64_t(gridDim.x) * kNT) {
    const T w = W[i] - ta * v[i];
    W[i] = w;
    acc += double(w) * double(w);
  }
  const double t = block_sum(acc, sm);
  if (threadIdx.x == 0) pb[blockIdx.x] = t;
  if (blockIdx.x == 0 && threadIdx.x == 0) alphas_dev[j] = alpha;
}

// Step C (cubic.py:97-103): beta = ||W||; breakdown test |beta| < tol (absolute);
// else betas[j] = beta; V[j+1] = W / beta.
template <typename T>
__global__ __launch_bounds__(kNT) void k_lanczos_c(int64_t d, const T* __restrict__ W,
                                                   T* __restrict__ Vnext,
                                                   const double* __restrict__ pb, int Pb,
                                                   double* __restrict__ betas_dev, int j,
                                                   double tol, LanczosState* st) {
  if (st->done) return;
  __shared__ double sm[kNT / 64];
  const double beta = sqrt(sum_partials(pb, Pb, sm));
  if (fabs(beta) < tol) {
    if (blockIdx.x == 0 && threadIdx.x == 0) { st->done = 1; st->j_break = j; st->beta_last = beta; }
    return;
  }
  const T tb = T(beta);
  for (int64_t i = int64_t(blockIdx.x) * kNT + threadIdx.x; i < d; i += int64_t(gridDim.x) * kNT)
    Vnext[i] = W[i] / tb;
  if (blockIdx.x == 0 && threadIdx.x == 0) { betas_dev[j] = beta; st->beta_last = beta; }
}

// Final (cubic.py:105-109): alphas[-1] = v.A(v) after truncation.
// Output slot: j_break if the basis was truncated (j_break < m-2), else m-1.
__global__ __launch_bounds__(kNT) void k_lanczos_final(const double* __restrict__ pa, int Pa,
                                                       double* __restrict__ alphas_dev, int m,
                                                       const LanczosState* st) {
  __shared__ double sm[kNT / 64];
  const double alpha = sum_partials(pa, Pa, sm);
  if (threadIdx.x == 0) {
    const int slot = (st->done && st->j_break < m - 2) ? st->j_break : m - 1;
    alphas_dev[slot] = alpha;
  }
}

// ------------------------------------------ full reorthogonalisation (CGS2)
// Build-only extension (the reference has none, cubic.py:92-103).
// h_r = V[r] . W for r < k: each block reduces a column slab of all k rows.
// partials layout: [block][r], kMaxRows rows per pass chunk.
template <typename T>
__global__ __launch_bounds__(kNT) void k_reorth_dots(int64_t d, int k, const T* __restrict__ V,
                                                     const T* __restrict__ W,
                                                     double* __restrict__ partials,
                                                     const LanczosState* st) {
  if (st->done) return;
  __shared__ double sm[kNT / 64];
  // Each block owns a contiguous slab of columns and loops over the k rows.
  const int64_t per = (d + gridDim.x - 1) / gridDim.x;
  const int64_t lo = int64_t(blockIdx.x) * per;
  const int64_t hi = lo + per < d ? lo + per : d;
  for (int r = 0; r < k; ++r) {
    const T* vr = V + int64_t(r) * d;
    double acc = 0.0;
    for (int64_t i = lo + threadIdx.x; i < hi; i += kNT) acc += double(vr[i]) * double(W[i]);
    const double t = block_sum(acc, sm);
    if (threadIdx.x == 0) partials[int64_t(blockIdx.x) * k + r] = t;
  }
}

// h_r = sum over blocks of partials[b][r] (fixed order), one thread per r.
__global__ __launch_bounds__(kNT) void k_reorth_coeffs(const double* __restrict__ partials, int P, int k,
                                                       double* __restrict__ h,
                                                       const LanczosState* st) {
  if (st->done) return;
  const int r = blockIdx.x * kNT + threadIdx.x;
  if (r >= k) return;
  double s = 0.0;
  for (int b = 0; b < P; ++b) s += partials[int64_t(b) * k + r];
  h[r] = s;
}

// W -= sum_r h_r V[r]   (columns independent; rows summed in order)
template <typename T>
__global__ __launch_bounds__(kNT) void k_reorth_update(int64_t d, int k, const T* __restrict__ V,
                                                       const double* __restrict__ h,
                                                       T* __restrict__ W, const LanczosState* st) {
  if (st->done) return;
  for (int64_t i = int64_t(blockIdx.x) * kNT + threadIdx.x; i < d; i += int64_t(gridDim.x) * kNT) {
    double acc = 0.0;
    for (int r = 0; r < k; ++r) acc += h[r] * double(V[int64_t(r) * d + i]);
    W[i] = T(double(W[i]) - acc);
  }
}

// Partial ||W||^2 after reorthogonalisation (feeds k_lanczos_c).
template <typename T>
__global__ __launch_bounds__(kNT) void k_norm2_partials(int64_t d, const T* __restrict__ W,
                                                        double* __restrict__ pb,
                                                        const LanczosState* st) {
  if (st->done) return;
  double acc = 0.0;
  for (int64_t i = int64_t(blockIdx.x) * kNT + threadIdx.x; i < d; i += int64_t(gridDim.x) * kNT) {
    const double w = W[i];
    acc += w * w;
  }
  __shared__ double sm[kNT / 64];
  const double t = block_sum(acc, sm);
  if (threadIdx.x == 0) pb[blockIdx.x] = t;
}

// ---------------------------------------------------------- basis combine
// x_new = x + V^T s (cubic.py:291): per column, sum_j V[j,i] s_j in j order.
template <typename T>
__global__ __launch_bounds__(kNT) void k_basis_combine(int64_t d, int m, const T* __restrict__ V,
                                                       const double* __restrict__ s,
                                                       const T* __restrict__ x, T* __restrict__ xn) {
  for (int64_t i = int64_t(blockIdx.x) * kNT + threadIdx.x; i < d; i += int64_t(gridDim.x) * kNT) {
    T acc = T(0);
    for (int j = 0; j < m; ++j) acc += V[int64_t(j) * d + i] * T(s[j]);
    xn[i] = x[i] + acc;
  }
}

// ------------------------------------------------------ transpose helpers
// row id of every nonzero (expands indptr).
__global__ __launch_bounds__(kNT) void k_expand_rows(int n, const int* __restrict__ ptr,
                                                     int* __restrict__ rowid) {
  const int lane = threadIdx.x & 63;
  const int wv = (blockIdx.x * kNT + threadIdx.x) >> 6;
  const int W = (gridDim.x * kNT) >> 6;
  for (int r = wv; r < n; r += W)
    for (int p = ptr[r] + lane; p < ptr[r + 1]; p += 64) rowid[p] = r;
}

__global__ __launch_bounds__(kNT) void k_iota(int64_t n, int* __restrict__ out) {
  for (int64_t i = int64_t(blockIdx.x) * kNT + threadIdx.x; i < n; i += int64_t(gridDim.x) * kNT)
    out[i] = int(i);
}

// colptr[c] = first position of key c in the sorted key array (lower bound),
// computed per column by binary search; colptr[d] = nnz.
__global__ __launch_bounds__(kNT) void k_colptr_from_sorted(int64_t d, int64_t nnz,
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
