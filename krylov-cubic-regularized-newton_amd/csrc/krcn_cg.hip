// krcn_cg.hip — krcn_cg_solve: scipy-style conjugate gradients on
// (H + shift I) x = b with the device HVP (krcn_cg.hpp), the linear solver of
// Cubic_LS.cubic_solver_root_CG (optimizer/cubic.py:152-182).
#include "krcn_cg.hpp"
#include "krcn_internal.hpp"

namespace {

constexpr int kCgCheckEvery = 16;   // iterations between host reads of the done flag

krcn_status ensure_cg_ws(krcn_csr* h) {
  if (h->cg_r) return KRCN_OK;
  char* p = nullptr;
  CHK(dalloc(h, &p, size_t(3) * size_t(h->d) * h->vs));
  h->cg_r = p;
  CHK(dalloc(h, &h->cg_st, 1));
  return KRCN_OK;
}

template <typename T>
krcn_status cg_impl(krcn_csr* h, const T* w, const T* b, double shift, double rtol, int maxiter, T* x,
                    krcn_cg_info* info, hipStream_t s) {
  const int64_t d = h->d;
  CHK(plans_for_compute(h));
  CHK(ensure_cg_ws(h));
  T* r = static_cast<T*>(h->cg_r);
  T* p = r + d;
  T* q = p + d;
  T* u = static_cast<T*>(h->u);
  CgState* st = h->cg_st;
  const LanczosState* guard = reinterpret_cast<const LanczosState*>(st);
  const int P = vec_grid(d);
  hipLaunchKernelGGL((k_cg_begin<T>), dim3(P), dim3(kNT), 0, s, d, b, x, r, p, h->pb);
  LAUNCHCHK();
  hipLaunchKernelGGL(k_cg_init, dim3(1), dim3(kNT), 0, s, h->pb, P, rtol, st);
  LAUNCHCHK();
  const T tn = T(h->n_global), tshift = T(shift);
  CgState hs{};
  int k = 0;
  for (; k < maxiter; ++k) {
    if (k % kCgCheckEvery == 0) {
      HIPCHK(hipMemcpyAsync(h->hostbuf, st, sizeof(CgState), hipMemcpyDeviceToHost, s));
      HIPCHK(hipStreamSynchronize(s));
      std::memcpy(&hs, h->hostbuf, sizeof(CgState));
      if (hs.done) break;
    }
    CHK(run_pass<T>(h->p1, SrcGuard<T>{p, guard, 0}, SrcGuard<T>{p, guard, 0}, EpiWeighted<T>{w, u}, nullptr,
                    nullptr, s));
    int Pq = 0;
    CHK(run_pass<T>(h->p2, SrcGuard<T>{u, guard, 0}, SrcGuard<T>{u, guard, 0}, EpiCgQ<T>{p, q, tn, tshift}, h->pa,
                    &Pq, s));
    hipLaunchKernelGGL((k_cg_update<T>), dim3(P), dim3(kNT), 0, s, d, k, h->pa, Pq, st, x, r,
                       static_cast<const T*>(p), static_cast<const T*>(q), h->pb);
    LAUNCHCHK();
    hipLaunchKernelGGL((k_cg_dir<T>), dim3(P), dim3(kNT), 0, s, d, k, h->pb, P, st, static_cast<const T*>(r), p);
    LAUNCHCHK();
  }
  HIPCHK(hipMemcpyAsync(h->hostbuf, st, sizeof(CgState), hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  std::memcpy(&hs, h->hostbuf, sizeof(CgState));
  info->converged = hs.done;
  info->iterations = hs.iters;
  info->info = hs.done ? 0 : maxiter;
  info->residual_norm = std::sqrt(hs.rho[hs.iters & 1]);
  return KRCN_OK;
}

}  // namespace

extern "C" krcn_status krcn_cg_solve(krcn_csr* h, const void* w, const void* b, double shift, double rtol,
                                     int maxiter, void* x, krcn_cg_info* info_host, void* stream) {
  if (!h || !b || !x || !info_host || (h->n && !w)) return fail(KRCN_ERR_INVALID, "krcn_cg_solve: null argument");
  if (h->shard != KRCN_SHARD_NONE)
    return fail(KRCN_ERR_UNSUPPORTED, "krcn_cg_solve: sharded handles are not supported");
  if (maxiter < 0) return fail(KRCN_ERR_INVALID, "krcn_cg_solve: maxiter must be >= 0");
  if (!(rtol >= 0.0)) return fail(KRCN_ERR_INVALID, "krcn_cg_solve: rtol must be >= 0");
  CHK(set_device(h));
  *info_host = krcn_cg_info{};
  if (h->d == 0) return KRCN_OK;
  return h->dtype == KRCN_F64
             ? cg_impl<double>(h, static_cast<const double*>(w), static_cast<const double*>(b), shift, rtol, maxiter,
                               static_cast<double*>(x), info_host, S(stream))
             : cg_impl<float>(h, static_cast<const float*>(w), static_cast<const float*>(b), shift, rtol, maxiter,
                              static_cast<float*>(x), info_host, S(stream));
}
