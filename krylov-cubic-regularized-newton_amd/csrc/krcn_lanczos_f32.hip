// krcn_lanczos_f32.hip — the f32 instantiation of the device Lanczos recurrence.
#include "krcn_lanczos_impl.hpp"

krcn_status lanczos_f32(krcn_csr* h, const float* w, const float* g, int m, int reorth, double tol, double l2,
                        float* V, double* alphas_host, double* betas_host, krcn_lanczos_info* info, hipStream_t s) {
  return lanczos_impl<float>(h, w, g, m, reorth, tol, l2, V, alphas_host, betas_host, info, s);
}

#ifdef KRCN_WIN_TIMING
extern "C" int krcn_debug_win_stamps_lz32(unsigned long long* out, int n, int reset) {
  return krcn::win_stamps_read(out, n, reset);
}
#endif
