// krcn_vec.hip — handle-free dense vector kernels: the Lanczos recurrence over
// an EXTERNAL operator (optimizer/cubic.py:77-111 called with any callable A,
// which the fused krcn_lanczos cannot see inside) and the vector helpers of the
// host loops (dot, scale, axpy).  A krcn_vctx owns only reduction scratch and a
// pinned staging buffer, so it serves vectors of any length on its device.
//
// Lanczos step j (krcn_lz_ext_step), given y = A(v) computed by the caller:
//   w = y - beta v_pre          (cubic.py:93; y alone at j = 0, v_pre = 0)
//   alpha = v.w                 (cubic.py:94)
//   z = w - alpha v             (cubic.py:96)
//   beta' = ||z||               (cubic.py:97)
// three launches (w + partials of v.w; alpha + z + partials of z.z; both
// scalars) and one 16-byte D2H.  The caller applies the breakdown test and
// v = z / beta' (krcn_vec_div, cubic.py:102).  Deterministic fixed-order
// reductions; -ffp-contract=off keeps every elementwise expression numpy's.
#include "krcn_internal.hpp"

struct krcn_vctx {
  int device = 0;
  double* part = nullptr;      // 2 x kMaxPartials partials + 2 scalars
  double* host = nullptr;      // pinned staging
};

namespace {

constexpr int kVecMaxGrid = 1024;   // vec_grid's cap: partials per reduction

template <typename T>
__global__ __launch_bounds__(kNT) void k_lzx_a(int64_t n, const T* __restrict__ y, const T* __restrict__ v,
                                               const T* __restrict__ v_pre, T beta, T* __restrict__ w,
                                               double* __restrict__ part) {
  double acc = 0.0;
  for (int64_t i = int64_t(blockIdx.x) * kNT + threadIdx.x; i < n; i += int64_t(gridDim.x) * kNT) {
    const T wi = v_pre ? y[i] - beta * v_pre[i] : y[i];
    w[i] = wi;
    acc += double(v[i]) * double(wi);
  }
  __shared__ double sm[kNT / 64];
  const double t = block_sum(acc, sm);
  if (threadIdx.x == 0) part[blockIdx.x] = t;
}

template <typename T>
__global__ __launch_bounds__(kNT) void k_lzx_b(int64_t n, const T* __restrict__ v, T* __restrict__ w,
                                               const double* __restrict__ part_a, int P, double* __restrict__ part_b) {
  __shared__ double sm[kNT / 64];
  const T alpha = T(sum_partials(part_a, P, sm));
  double acc = 0.0;
  for (int64_t i = int64_t(blockIdx.x) * kNT + threadIdx.x; i < n; i += int64_t(gridDim.x) * kNT) {
    const T zi = w[i] - alpha * v[i];
    w[i] = zi;
    acc += double(zi) * double(zi);
  }
  const double t = block_sum(acc, sm);
  if (threadIdx.x == 0) part_b[blockIdx.x] = t;
}

__global__ __launch_bounds__(kNT) void k_lzx_fin(const double* __restrict__ part_a, const double* __restrict__ part_b,
                                                 int P, double* __restrict__ out2) {
  __shared__ double sm[kNT / 64];
  const double a = sum_partials(part_a, P, sm);
  const double b = sum_partials(part_b, P, sm);
  if (threadIdx.x == 0) {
    out2[0] = a;
    out2[1] = sqrt(b);
  }
}

template <typename T>
__global__ __launch_bounds__(kNT) void k_vec_div(int64_t n, const T* __restrict__ a, T div, T* __restrict__ out) {
  for (int64_t i = int64_t(blockIdx.x) * kNT + threadIdx.x; i < n; i += int64_t(gridDim.x) * kNT) out[i] = a[i] / div;
}

template <typename T>
__global__ __launch_bounds__(kNT) void k_vec_axpy(int64_t n, T alpha, const T* __restrict__ x, const T* __restrict__ y,
                                                  T* __restrict__ out) {
  for (int64_t i = int64_t(blockIdx.x) * kNT + threadIdx.x; i < n; i += int64_t(gridDim.x) * kNT)
    out[i] = y[i] + alpha * x[i];
}

krcn_status check(const krcn_vctx* c, int dtype, int64_t n) {
  if (!c) return fail(KRCN_ERR_INVALID, "krcn_vec: null context");
  if (dtype != KRCN_F64 && dtype != KRCN_F32) return fail(KRCN_ERR_INVALID, "krcn_vec: bad dtype");
  if (n < 0) return fail(KRCN_ERR_INVALID, "krcn_vec: negative length");
  HIPCHK(hipSetDevice(c->device));
  return KRCN_OK;
}

template <typename T>
krcn_status lz_step(krcn_vctx* c, int64_t n, const T* y, const T* v, const T* v_pre, double beta, T* z,
                    double* ab, hipStream_t s) {
  const int P = vec_grid(n);
  double* pa = c->part;
  double* pb = c->part + kVecMaxGrid;
  double* out = c->part + 2 * kVecMaxGrid;
  hipLaunchKernelGGL((k_lzx_a<T>), dim3(P), dim3(kNT), 0, s, n, y, v, v_pre, T(beta), z, pa);
  LAUNCHCHK();
  hipLaunchKernelGGL((k_lzx_b<T>), dim3(P), dim3(kNT), 0, s, n, v, z, static_cast<const double*>(pa), P, pb);
  LAUNCHCHK();
  hipLaunchKernelGGL(k_lzx_fin, dim3(1), dim3(kNT), 0, s, pa, pb, P, out);
  LAUNCHCHK();
  HIPCHK(hipMemcpyAsync(c->host, out, 2 * sizeof(double), hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  ab[0] = c->host[0];
  ab[1] = c->host[1];
  return KRCN_OK;
}

}  // namespace

extern "C" krcn_status krcn_vctx_create(int device, krcn_vctx** out) {
  if (!out) return fail(KRCN_ERR_INVALID, "krcn_vctx_create: out is null");
  *out = nullptr;
  HIPCHK(hipSetDevice(device));
  krcn_vctx* c = new krcn_vctx();
  c->device = device;
  if (hipMalloc(&c->part, sizeof(double) * (2 * kVecMaxGrid + 2)) != hipSuccess ||
      hipHostMalloc(reinterpret_cast<void**>(&c->host), 16 * sizeof(double), 0) != hipSuccess) {
    if (c->part) (void)hipFree(c->part);
    delete c;
    return fail(KRCN_ERR_HIP, "krcn_vctx_create: allocation failed");
  }
  *out = c;
  return KRCN_OK;
}

extern "C" krcn_status krcn_vctx_destroy(krcn_vctx* c) {
  if (!c) return KRCN_OK;
  (void)hipSetDevice(c->device);
  (void)hipFree(c->part);
  (void)hipHostFree(c->host);
  delete c;
  return KRCN_OK;
}

extern "C" krcn_status krcn_lz_ext_step(krcn_vctx* c, int dtype, int64_t n, const void* y, const void* v,
                                        const void* v_pre, double beta, void* z, double* alpha_beta_host,
                                        void* stream) {
  CHK(check(c, dtype, n));
  if (!alpha_beta_host || (n && (!y || !v || !z))) return fail(KRCN_ERR_INVALID, "krcn_lz_ext_step: null argument");
  if (n == 0) {
    alpha_beta_host[0] = alpha_beta_host[1] = 0.0;
    return KRCN_OK;
  }
  return dtype == KRCN_F64
             ? lz_step<double>(c, n, static_cast<const double*>(y), static_cast<const double*>(v),
                               static_cast<const double*>(v_pre), beta, static_cast<double*>(z), alpha_beta_host,
                               S(stream))
             : lz_step<float>(c, n, static_cast<const float*>(y), static_cast<const float*>(v),
                              static_cast<const float*>(v_pre), beta, static_cast<float*>(z), alpha_beta_host,
                              S(stream));
}

extern "C" krcn_status krcn_vec_dot(krcn_vctx* c, int dtype, int64_t n, const void* a, const void* b,
                                    double* out_host, void* stream) {
  CHK(check(c, dtype, n));
  if (!out_host || (n && (!a || !b))) return fail(KRCN_ERR_INVALID, "krcn_vec_dot: null argument");
  hipStream_t s = S(stream);
  const int P = vec_grid(n);
  if (dtype == KRCN_F64)
    hipLaunchKernelGGL((k_reduce2<double, 0>), dim3(P), dim3(kNT), 0, s, n, static_cast<const double*>(a),
                       static_cast<const double*>(b), c->part);
  else
    hipLaunchKernelGGL((k_reduce2<float, 0>), dim3(P), dim3(kNT), 0, s, n, static_cast<const float*>(a),
                       static_cast<const float*>(b), c->part);
  LAUNCHCHK();
  hipLaunchKernelGGL((k_finish<0>), dim3(1), dim3(kNT), 0, s, c->part, P, c->part + 2 * kVecMaxGrid);
  LAUNCHCHK();
  HIPCHK(hipMemcpyAsync(c->host, c->part + 2 * kVecMaxGrid, sizeof(double), hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  *out_host = c->host[0];
  return KRCN_OK;
}

extern "C" krcn_status krcn_vec_div(krcn_vctx* c, int dtype, int64_t n, const void* a, double div, void* out,
                                    void* stream) {
  CHK(check(c, dtype, n));
  if (n && (!a || !out)) return fail(KRCN_ERR_INVALID, "krcn_vec_div: null argument");
  if (n == 0) return KRCN_OK;
  if (dtype == KRCN_F64)
    hipLaunchKernelGGL((k_vec_div<double>), dim3(vec_grid(n)), dim3(kNT), 0, S(stream), n,
                       static_cast<const double*>(a), div, static_cast<double*>(out));
  else
    hipLaunchKernelGGL((k_vec_div<float>), dim3(vec_grid(n)), dim3(kNT), 0, S(stream), n,
                       static_cast<const float*>(a), float(div), static_cast<float*>(out));
  LAUNCHCHK();
  return KRCN_OK;
}

extern "C" krcn_status krcn_vec_axpy(krcn_vctx* c, int dtype, int64_t n, double alpha, const void* x, const void* y,
                                     void* out, void* stream) {
  CHK(check(c, dtype, n));
  if (n && (!x || !y || !out)) return fail(KRCN_ERR_INVALID, "krcn_vec_axpy: null argument");
  if (n == 0) return KRCN_OK;
  if (dtype == KRCN_F64)
    hipLaunchKernelGGL((k_vec_axpy<double>), dim3(vec_grid(n)), dim3(kNT), 0, S(stream), n, alpha,
                       static_cast<const double*>(x), static_cast<const double*>(y), static_cast<double*>(out));
  else
    hipLaunchKernelGGL((k_vec_axpy<float>), dim3(vec_grid(n)), dim3(kNT), 0, S(stream), n, float(alpha),
                       static_cast<const float*>(x), static_cast<const float*>(y), static_cast<float*>(out));
  LAUNCHCHK();
  return KRCN_OK;
}
