// krcn_ops.hip — objective pieces of optimizer/loss.py on the device: X x,
// X^T u, the Hessian weights, the HVP, the gradient, the loss mean, the basis
// combine and the dense reductions; and the krcn_lanczos entry point, which
// dispatches to the per-dtype recurrence units.
#include "krcn_internal.hpp"

using namespace krcn;

// ------------------------------------------------------ objective pieces
template <typename T>
static krcn_status matvec_impl(krcn_csr* h, const T* x, T* Ax, hipStream_t s) {
  CHK(launch_rows_x<T>(h, x, EpiStore<T>{Ax}, nullptr, nullptr, s));
  if (h->shard == KRCN_SHARD_COLS) CHK(allreduce(h, Ax, h->n, h->dtype, s));
  return KRCN_OK;
}

extern "C" krcn_status krcn_matvec(krcn_csr* h, const void* x, void* Ax, void* stream) {
  if (!h || (!x && h->d) || (!Ax && h->n)) return fail(KRCN_ERR_INVALID, "krcn_matvec: null argument");
  CHK(set_device(h));
  if (h->n == 0) return KRCN_OK;
  return h->dtype == KRCN_F64
             ? matvec_impl<double>(h, static_cast<const double*>(x), static_cast<double*>(Ax), S(stream))
             : matvec_impl<float>(h, static_cast<const float*>(x), static_cast<float*>(Ax), S(stream));
}

// X^T r with epilogue `epi`; in ROWS mode the raw partial is all-reduced
// first and the epilogue runs elementwise over d.
template <typename T, class Epi>
static krcn_status xt_pass(krcn_csr* h, const T* r, const Epi& epi, hipStream_t s) {
  if (h->d == 0) return KRCN_OK;
  if (h->shard == KRCN_SHARD_ROWS) {
    T* raw = static_cast<T*>(h->td);
    CHK(launch_rows_xt<T>(h, r, EpiStore<T>{raw}, nullptr, nullptr, s));
    CHK(allreduce(h, raw, h->d, h->dtype, s));
    hipLaunchKernelGGL((k_rows_apply<T, SrcPlain<T>, Epi>), dim3(apply_grid(h->d)), dim3(kNT), 0, s, int(h->d),
                       static_cast<const T*>(raw), SrcPlain<T>{raw}, epi, static_cast<double*>(nullptr));
    LAUNCHCHK();
    return KRCN_OK;
  }
  return launch_rows_xt<T>(h, r, epi, nullptr, nullptr, s);
}

template <typename T>
static krcn_status rmatvec_impl(krcn_csr* h, const T* u, T* y, hipStream_t s) {
  return xt_pass<T>(h, u, EpiGrad<T>{nullptr, y, T(h->n_global), T(0), 0}, s);
}

extern "C" krcn_status krcn_rmatvec(krcn_csr* h, const void* u, void* y, void* stream) {
  if (!h || (!u && h->n) || (!y && h->d)) return fail(KRCN_ERR_INVALID, "krcn_rmatvec: null argument");
  CHK(set_device(h));
  return h->dtype == KRCN_F64
             ? rmatvec_impl<double>(h, static_cast<const double*>(u), static_cast<double*>(y), S(stream))
             : rmatvec_impl<float>(h, static_cast<const float*>(u), static_cast<float*>(y), S(stream));
}

extern "C" krcn_status krcn_weights(krcn_csr* h, const void* Ax, void* w, void* stream) {
  if (!h || (h->n && (!Ax || !w))) return fail(KRCN_ERR_INVALID, "krcn_weights: null argument");
  CHK(set_device(h));
  if (h->n == 0) return KRCN_OK;
  if (h->dtype == KRCN_F64)
    hipLaunchKernelGGL((k_weights<double>), dim3(vec_grid(h->n)), dim3(kNT), 0, S(stream), h->n,
                       static_cast<const double*>(Ax), static_cast<double*>(w));
  else
    hipLaunchKernelGGL((k_weights<float>), dim3(vec_grid(h->n)), dim3(kNT), 0, S(stream), h->n,
                       static_cast<const float*>(Ax), static_cast<float*>(w));
  LAUNCHCHK();
  return KRCN_OK;
}

template <typename T>
static krcn_status hvp_impl(krcn_csr* h, const T* w, const T* v, T* y, double l2, hipStream_t s) {
  ProfRec* pr = prof_next(h);
  if (pr) HIPCHK(hipEventRecord(pr->e0, s));
  T* u = static_cast<T*>(h->u);
  if (h->shard == KRCN_SHARD_COLS) {
    CHK(launch_rows_x<T>(h, v, EpiStore<T>{u}, nullptr, nullptr, s));
    CHK(allreduce(h, u, h->n, h->dtype, s));
    hipLaunchKernelGGL((k_rows_apply<T, SrcPlain<T>, EpiWeighted<T>>), dim3(apply_grid(h->n)), dim3(kNT), 0, s,
                       int(h->n), static_cast<const T*>(u), SrcPlain<T>{u}, EpiWeighted<T>{w, u},
                       static_cast<double*>(nullptr));
    LAUNCHCHK();
  } else {
    CHK(launch_rows_x<T>(h, v, EpiWeighted<T>{w, u}, nullptr, nullptr, s));
  }
  if (pr) HIPCHK(hipEventRecord(pr->e1, s));
  if (l2 != 0.0) CHK(xt_pass<T>(h, u, EpiHvpOut<T, true>{v, y, T(h->n_global), T(l2)}, s));
  else CHK(xt_pass<T>(h, u, EpiHvpOut<T, false>{v, y, T(h->n_global), T(0)}, s));
  if (pr) HIPCHK(hipEventRecord(pr->e2, s));
  return KRCN_OK;
}

extern "C" krcn_status krcn_hvp(krcn_csr* h, const void* w, const void* v, void* y, double l2,
                                void* stream) {
  if (!h || (h->n && !w) || (h->d && (!v || !y))) return fail(KRCN_ERR_INVALID, "krcn_hvp: null argument");
  CHK(set_device(h));
  if (h->d == 0) return KRCN_OK;
  return h->dtype == KRCN_F64
             ? hvp_impl<double>(h, static_cast<const double*>(w), static_cast<const double*>(v),
                                static_cast<double*>(y), l2, S(stream))
             : hvp_impl<float>(h, static_cast<const float*>(w), static_cast<const float*>(v),
                               static_cast<float*>(y), l2, S(stream));
}

// The placement probe (krcn_plan.hip tune_placement): the two local passes of
// an HVP (pass 1 with the weighting, pass 2 with y = s / n; no collective, so
// a rank of a sharded handle probes alone) over the handle's own scratch:
// w = tn, v = W, y = td.  Their values do not change the memory traffic.
template <typename T>
static krcn_status probe_impl(krcn_csr* h, hipStream_t s, int reps, float* us) {
  T* u = static_cast<T*>(h->u);
  const T* w = static_cast<const T*>(h->tn);
  const T* v = static_cast<const T*>(h->W);
  T* y = static_cast<T*>(h->td);
  auto one = [&]() -> krcn_status {
    CHK(run_pass<T>(h->p1, SrcPlain<T>{v}, SrcPlain<T>{v}, EpiWeighted<T>{w, u}, nullptr, nullptr, s));
    return run_pass<T>(h->p2, SrcPlain<T>{u}, SrcPlain<T>{u}, EpiHvpOut<T, false>{v, y, T(h->n_global), T(0)},
                       nullptr, nullptr, s);
  };
  hipEvent_t e0 = nullptr, e1 = nullptr;
  HIPCHK(hipEventCreate(&e0));
  HIPCHK(hipEventCreate(&e1));
  krcn_status r = KRCN_OK;
  float best = 0.0f;
  for (int k = 0; k < 2 && r == KRCN_OK; ++k) r = one();   // warm the caches
  // the fastest of three batches: the slow placement is systematic, a
  // disturbance of one batch is not
  for (int b = 0; b < 3 && r == KRCN_OK; ++b) {
    if (hipEventRecord(e0, s) != hipSuccess) r = fail(KRCN_ERR_HIP, "placement probe: hipEventRecord");
    for (int k = 0; k < reps && r == KRCN_OK; ++k) r = one();
    if (r == KRCN_OK && hipEventRecord(e1, s) != hipSuccess) r = fail(KRCN_ERR_HIP, "placement probe: hipEventRecord");
    float ms = 0.0f;
    if (r == KRCN_OK && (hipEventSynchronize(e1) != hipSuccess || hipEventElapsedTime(&ms, e0, e1) != hipSuccess))
      r = fail(KRCN_ERR_HIP, "placement probe: event timing");
    const float t = 1e3f * ms / float(reps);
    if (r == KRCN_OK && (b == 0 || t < best)) best = t;
  }
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  CHK(r);
  *us = best;
  return KRCN_OK;
}

krcn_status placement_probe(krcn_csr* h, hipStream_t s, int reps, float* us) {
  return h->dtype == KRCN_F64 ? probe_impl<double>(h, s, reps, us) : probe_impl<float>(h, s, reps, us);
}

template <typename T>
static krcn_status gradient_impl(krcn_csr* h, const T* Ax, const T* b, const T* x, double l2, T* g,
                                 hipStream_t s) {
  T* r = static_cast<T*>(h->tn);
  if (h->n) {
    hipLaunchKernelGGL((k_residual<T>), dim3(vec_grid(h->n)), dim3(kNT), 0, s, h->n, Ax, b, r);
    LAUNCHCHK();
  }
  const int has_l2 = l2 != 0.0;
  return xt_pass<T>(h, r, EpiGrad<T>{x, g, T(h->n_global), T(l2), has_l2}, s);
}

extern "C" krcn_status krcn_gradient(krcn_csr* h, const void* Ax, const void* b, const void* x,
                                     double l2, void* grad, void* stream) {
  if (!h || (h->n && (!Ax || !b)) || (h->d && !grad) || (l2 != 0.0 && h->d && !x))
    return fail(KRCN_ERR_INVALID, "krcn_gradient: null argument");
  CHK(set_device(h));
  return h->dtype == KRCN_F64
             ? gradient_impl<double>(h, static_cast<const double*>(Ax), static_cast<const double*>(b),
                                     static_cast<const double*>(x), l2, static_cast<double*>(grad), S(stream))
             : gradient_impl<float>(h, static_cast<const float*>(Ax), static_cast<const float*>(b),
                                    static_cast<const float*>(x), l2, static_cast<float*>(grad), S(stream));
}

// Reduce `partials` (P values) to device scalar scal[slot], optionally
// all-reduced over the communicator, then (if host) copied to *host.
static krcn_status finish_scalar(krcn_csr* h, int P, int slot, bool over_ranks, double* host,
                                 hipStream_t s, bool do_sqrt = false) {
  hipLaunchKernelGGL((k_finish<0>), dim3(1), dim3(kNT), 0, s, h->pa, P, h->scal + slot);
  LAUNCHCHK();
  if (over_ranks) CHK(allreduce(h, h->scal + slot, 1, KRCN_F64, s));
  HIPCHK(hipMemcpyAsync(h->hostbuf, h->scal + slot, sizeof(double), hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  *host = do_sqrt ? std::sqrt(h->hostbuf[0]) : h->hostbuf[0];
  return KRCN_OK;
}

template <typename T>
static krcn_status loss_mean_impl(krcn_csr* h, const T* Ax, const T* b, double* out, hipStream_t s) {
  const int P = vec_grid(h->n);
  hipLaunchKernelGGL((k_loss_terms<T>), dim3(P), dim3(kNT), 0, s, h->n, Ax, b, h->pa);
  LAUNCHCHK();
  double sum = 0.0;
  CHK(finish_scalar(h, P, 0, h->shard == KRCN_SHARD_ROWS, &sum, s));
  *out = sum / double(h->n_global);
  return KRCN_OK;
}

extern "C" krcn_status krcn_loss_mean(krcn_csr* h, const void* Ax, const void* b, double* out_host,
                                      void* stream) {
  if (!h || !out_host || (h->n && (!Ax || !b))) return fail(KRCN_ERR_INVALID, "krcn_loss_mean: null argument");
  CHK(set_device(h));
  return h->dtype == KRCN_F64
             ? loss_mean_impl<double>(h, static_cast<const double*>(Ax), static_cast<const double*>(b), out_host, S(stream))
             : loss_mean_impl<float>(h, static_cast<const float*>(Ax), static_cast<const float*>(b), out_host, S(stream));
}

// k loss values in one submission: per iterate the launches of krcn_matvec and
// krcn_loss_mean (so every value is bitwise the single call's), the k sums
// kept on the device, one all-reduce of all k (ROWS), one D2H, one sync.
template <typename T>
static krcn_status loss_values_impl(krcn_csr* h, int k, const void* const* xs, const T* b, double* out,
                                    hipStream_t s) {
  T* Ax = static_cast<T*>(h->tn);
  const int P = vec_grid(h->n);
  for (int c0 = 0; c0 < k; c0 += int(h->pcap)) {
    const int kc = std::min<int64_t>(k - c0, h->pcap);
    for (int i = 0; i < kc; ++i) {
      CHK(matvec_impl<T>(h, static_cast<const T*>(xs[c0 + i]), Ax, s));
      hipLaunchKernelGGL((k_loss_terms<T>), dim3(P), dim3(kNT), 0, s, h->n, static_cast<const T*>(Ax), b, h->pa);
      LAUNCHCHK();
      hipLaunchKernelGGL((k_finish<0>), dim3(1), dim3(kNT), 0, s, h->pa, P, h->pb + i);
      LAUNCHCHK();
    }
    if (h->shard == KRCN_SHARD_ROWS) CHK(allreduce(h, h->pb, kc, KRCN_F64, s));
    HIPCHK(hipMemcpyAsync(out + c0, h->pb, size_t(kc) * sizeof(double), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    for (int i = 0; i < kc; ++i) out[c0 + i] = out[c0 + i] / double(h->n_global);
  }
  return KRCN_OK;
}

extern "C" krcn_status krcn_loss_values(krcn_csr* h, int k, const void* const* xs_host, const void* b,
                                        double* out_host, void* stream) {
  if (!h || k < 0 || (k && (!xs_host || !out_host)) || (h->n && k && !b))
    return fail(KRCN_ERR_INVALID, "krcn_loss_values: null argument");
  for (int i = 0; i < k; ++i)
    if (!xs_host[i] && h->d) return fail(KRCN_ERR_INVALID, "krcn_loss_values: iterate %d is null", i);
  CHK(set_device(h));
  if (k == 0) return KRCN_OK;
  if (h->n == 0) {
    std::fill(out_host, out_host + k, 0.0);
    return KRCN_OK;
  }
  CHK(plans_for_compute(h));
  return h->dtype == KRCN_F64
             ? loss_values_impl<double>(h, k, xs_host, static_cast<const double*>(b), out_host, S(stream))
             : loss_values_impl<float>(h, k, xs_host, static_cast<const float*>(b), out_host, S(stream));
}

extern "C" krcn_status krcn_lanczos(krcn_csr* h, const void* w, const void* g, int m, int reorth,
                                    double tol, double l2, void* V, double* alphas_host,
                                    double* betas_host, krcn_lanczos_info* info_host, void* stream) {
  if (!h || !g || !V || !alphas_host || !betas_host || !info_host || (h->n && !w))
    return fail(KRCN_ERR_INVALID, "krcn_lanczos: null argument");
  if (m < 1) return fail(KRCN_ERR_INVALID, "krcn_lanczos: m must be >= 1 (got %d)", m);
  if (m > 2044) return fail(KRCN_ERR_UNSUPPORTED, "krcn_lanczos: m > 2044 not supported");
  CHK(set_device(h));
  return h->dtype == KRCN_F64
             ? lanczos_f64(h, static_cast<const double*>(w), static_cast<const double*>(g), m, reorth,
                                    tol, l2, static_cast<double*>(V), alphas_host, betas_host, info_host,
                                    S(stream))
             : lanczos_f32(h, static_cast<const float*>(w), static_cast<const float*>(g), m, reorth, tol,
                                   l2, static_cast<float*>(V), alphas_host, betas_host, info_host, S(stream));
}

extern "C" krcn_status krcn_basis_combine(krcn_csr* h, int m_eff, const void* V, const double* s_host,
                                          const void* x, void* x_new, void* stream) {
  if (!h || !V || !s_host || !x || !x_new) return fail(KRCN_ERR_INVALID, "krcn_basis_combine: null argument");
  if (m_eff < 1 || m_eff > h->mcap || m_eff > kBasisMaxM)
    return fail(KRCN_ERR_INVALID, "krcn_basis_combine: m_eff %d outside [1, %d]", m_eff, std::min(h->mcap, kBasisMaxM));
  CHK(set_device(h));
  hipStream_t s = S(stream);
  // h->hcoef is free between Lanczos calls; stage s through it (pageable H2D
  // copies are staged synchronously by the runtime, so s_host may be reused).
  HIPCHK(hipMemcpyAsync(h->hcoef, s_host, size_t(m_eff) * sizeof(double), hipMemcpyHostToDevice, s));
  if (h->d == 0) return KRCN_OK;
  if (h->dtype == KRCN_F64)
    hipLaunchKernelGGL((k_basis_combine<double>), dim3(vec_grid(h->d)), dim3(kNT), 0, s, h->d, m_eff,
                       static_cast<const double*>(V), h->hcoef, static_cast<const double*>(x),
                       static_cast<double*>(x_new));
  else
    hipLaunchKernelGGL((k_basis_combine<float>), dim3(vec_grid(h->d)), dim3(kNT), 0, s, h->d, m_eff,
                       static_cast<const float*>(V), h->hcoef, static_cast<const float*>(x),
                       static_cast<float*>(x_new));
  LAUNCHCHK();
  return KRCN_OK;
}

template <typename T>
static krcn_status reduce_impl(krcn_csr* h, int space, int mode, const T* a, const T* b, double* out,
                               hipStream_t s) {
  const int64_t len = space == KRCN_SPACE_N ? h->n : h->d;
  const bool sharded = (space == KRCN_SPACE_N && h->shard == KRCN_SHARD_ROWS) ||
                       (space == KRCN_SPACE_D && h->shard == KRCN_SHARD_COLS);
  const int P = vec_grid(len);
  if (mode == 0)
    hipLaunchKernelGGL((k_reduce2<T, 0>), dim3(P), dim3(kNT), 0, s, len, a, b, h->pa);
  else if (mode == 1)
    hipLaunchKernelGGL((k_reduce2<T, 1>), dim3(P), dim3(kNT), 0, s, len, a, b, h->pa);
  else
    hipLaunchKernelGGL((k_reduce2<T, 2>), dim3(P), dim3(kNT), 0, s, len, a, b, h->pa);
  LAUNCHCHK();
  return finish_scalar(h, P, 4, sharded, out, s, mode != 0);
}

extern "C" krcn_status krcn_dot(krcn_csr* h, int space, const void* a, const void* b, double* out_host,
                                void* stream) {
  if (!h || !a || !b || !out_host) return fail(KRCN_ERR_INVALID, "krcn_dot: null argument");
  if (space != KRCN_SPACE_N && space != KRCN_SPACE_D) return fail(KRCN_ERR_INVALID, "krcn_dot: bad space");
  CHK(set_device(h));
  return h->dtype == KRCN_F64
             ? reduce_impl<double>(h, space, 0, static_cast<const double*>(a), static_cast<const double*>(b), out_host, S(stream))
             : reduce_impl<float>(h, space, 0, static_cast<const float*>(a), static_cast<const float*>(b), out_host, S(stream));
}

extern "C" krcn_status krcn_diff_norm(krcn_csr* h, int space, const void* a, const void* b,
                                      double* out_host, void* stream) {
  if (!h || !a || !out_host) return fail(KRCN_ERR_INVALID, "krcn_diff_norm: null argument");
  if (space != KRCN_SPACE_N && space != KRCN_SPACE_D) return fail(KRCN_ERR_INVALID, "krcn_diff_norm: bad space");
  CHK(set_device(h));
  const int mode = b ? 2 : 1;
  return h->dtype == KRCN_F64
             ? reduce_impl<double>(h, space, mode, static_cast<const double*>(a), static_cast<const double*>(b), out_host, S(stream))
             : reduce_impl<float>(h, space, mode, static_cast<const float*>(a), static_cast<const float*>(b), out_host, S(stream));
}

#ifdef KRCN_WIN_TIMING
extern "C" int krcn_debug_win_stamps_ops(unsigned long long* out, int n, int reset) {
  return krcn::win_stamps_read(out, n, reset);
}
#endif
