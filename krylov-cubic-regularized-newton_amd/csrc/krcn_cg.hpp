// krcn_cg.hpp — device conjugate gradients on the logistic Hessian, the inner
// solver of the full-space CRN with cubic_solver="CG" (optimizer/cubic.py:152-182:
// scipy.sparse.linalg.cg on the LinearOperator v -> hess_vec_prod(x, v) + lam v).
//
// Iteration k (the loop of scipy's cg, unpreconditioned, x0 = 0):
//   q = (H + shift I) p        pass 1 (u = w (.) X p) + pass 2 with EpiCgQ, which
//                              also writes the partials of p.q
//   k_cg_update:  alpha = rho_k / (p.q);  x += alpha p;  r -= alpha q;
//                 partials of r.r
//   k_cg_dir:     rho_{k+1} = r.r; stop when sqrt(rho_{k+1}) < atol
//                 (scipy: norm(r) < atol, atol = rtol ||b||); else
//                 p = p beta + r, beta = rho_{k+1} / rho_k
// Control stays on the device (CgState.done): once it is set every launch of
// the remaining iterations returns at once, so the host checks the flag only
// every few iterations.  rho is double-buffered by iteration parity because
// every block of k_cg_dir reads rho_k while block 0 records rho_{k+1}.
// Deterministic: every block re-sums the partials in the same fixed order.
#pragma once
#include <cstddef>

#include "krcn_kernels.hpp"

namespace krcn {

struct CgState {
  int done;        // shares its offset with LanczosState::done (SrcGuard reads it)
  int iters;       // updates of x performed
  int pad0, pad1;
  double rho[2];   // r.r of iterations k (slot k & 1) and k + 1
  double atol;     // rtol * ||b||
  double pq;
};
static_assert(offsetof(CgState, done) == offsetof(LanczosState, done), "SrcGuard reads done");

// q[r] = s / n + shift p[r] (the HVP epilogue with l2 + lam as the shift,
// cubic.py:156-157) and the partial of p.q.
template <typename T> struct EpiCgQ {
  const T* p; T* q; T n; T shift;
  static constexpr bool kReduce = true;
  struct Pre { T pr; };
  template <class S> __device__ __forceinline__ void init(const S&) {}
  __device__ __forceinline__ Pre pre(int r) const { return Pre{p[r]}; }
  __device__ __forceinline__ double row(int r, T s, int, const Pre& a) const {
    const T v = s / n + shift * a.pr;
    q[r] = v;
    return double(a.pr) * double(v);
  }
};

// x = 0, r = b, p = b, partials of b.b.
template <typename T>
__global__ __launch_bounds__(kNT) void k_cg_begin(int64_t d, const T* __restrict__ b, T* __restrict__ x,
                                                  T* __restrict__ r, T* __restrict__ p,
                                                  double* __restrict__ partials) {
  double acc = 0.0;
  for (int64_t i = int64_t(blockIdx.x) * kNT + threadIdx.x; i < d; i += int64_t(gridDim.x) * kNT) {
    const T bi = b[i];
    x[i] = T(0);
    r[i] = bi;
    p[i] = bi;
    acc += double(bi) * double(bi);
  }
  __shared__ double sm[kNT / 64];
  const double t = block_sum(acc, sm);
  if (threadIdx.x == 0) partials[blockIdx.x] = t;
}

// rho_0 = b.b, atol = rtol ||b||; ||b|| = 0 returns x = b = 0 (scipy's early exit).
[[maybe_unused]] static __global__ __launch_bounds__(kNT) void k_cg_init(const double* __restrict__ partials, int P, double rtol,
                                                 CgState* st) {
  __shared__ double sm[kNT / 64];
  const double rho = sum_partials(partials, P, sm);
  if (threadIdx.x == 0) {
    st->rho[0] = rho;
    st->rho[1] = 0.0;
    st->atol = rtol * sqrt(rho);
    st->iters = 0;
    st->done = rho == 0.0 ? 1 : 0;
  }
}

// alpha = rho_k / p.q; x += alpha p; r -= alpha q; partials of r.r.
template <typename T>
__global__ __launch_bounds__(kNT) void k_cg_update(int64_t d, int k, const double* __restrict__ pq_part, int P,
                                                   CgState* st, T* __restrict__ x, T* __restrict__ r,
                                                   const T* __restrict__ p, const T* __restrict__ q,
                                                   double* __restrict__ rr_part) {
  if (st->done) return;
  __shared__ double sm[kNT / 64];
  const double pq = sum_partials(pq_part, P, sm);
  const T alpha = T(st->rho[k & 1] / pq);
  double acc = 0.0;
  for (int64_t i = int64_t(blockIdx.x) * kNT + threadIdx.x; i < d; i += int64_t(gridDim.x) * kNT) {
    x[i] = x[i] + alpha * p[i];
    const T ri = r[i] - alpha * q[i];
    r[i] = ri;
    acc += double(ri) * double(ri);
  }
  const double t = block_sum(acc, sm);
  if (threadIdx.x == 0) rr_part[blockIdx.x] = t;
  if (blockIdx.x == 0 && threadIdx.x == 0) st->pq = pq;
}

// rho_{k+1} = r.r; converged (norm(r) < atol) or p = p beta + r.
template <typename T>
__global__ __launch_bounds__(kNT) void k_cg_dir(int64_t d, int k, const double* __restrict__ rr_part, int P,
                                                CgState* st, const T* __restrict__ r, T* __restrict__ p) {
  if (st->done) return;
  __shared__ double sm[kNT / 64];
  const double rho = sum_partials(rr_part, P, sm);
  const bool lead = blockIdx.x == 0 && threadIdx.x == 0;
  if (sqrt(rho) < st->atol) {
    if (lead) { st->rho[(k + 1) & 1] = rho; st->iters = k + 1; st->done = 1; }
    return;
  }
  const T beta = T(rho / st->rho[k & 1]);
  for (int64_t i = int64_t(blockIdx.x) * kNT + threadIdx.x; i < d; i += int64_t(gridDim.x) * kNT)
    p[i] = p[i] * beta + r[i];
  if (lead) { st->rho[(k + 1) & 1] = rho; st->iters = k + 1; }
}

}  // namespace krcn
