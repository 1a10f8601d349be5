/* Multi-core CPU restatement of the reference HVP -- TEST INFRASTRUCTURE ONLY.
 *
 * Used by tests/ (checked against the golden vectors of the reference, F1)
 * and by bench.py's cpu_baseline as the "strong CPU" line SURVEY.md §8(d)
 * asks for.  The product path (libkrcn) never links or calls this file.
 *
 * LogisticRegression.hess_vec_prod, optimizer/loss.py:289-302:
 *     t = X v                    (loss.py:299, scipy csr_matvec)
 *     u = w * t                  (loss.py:301, w = s (1 - s), s = expit(X x))
 *     y = X^T u / n + l2 v       (loss.py:302, scipy csc_matvec on A.T)
 * Summation order is scipy's: row i of X v left to right over its CSR row;
 * y_k accumulates u_i X_ik over i ascending, which is row k of the
 * transposed CSR (column-sorted transpose, rows ascending) left to right.  So
 * with -ffp-contract=off the result is bitwise scipy's.  Rows of X and of X^T
 * are split over OpenMP threads (no shared accumulators).
 *
 * Build (done by __graft_entry__.build()):
 *   gcc -O3 -fopenmp -ffp-contract=off -shared -fPIC oracle/krcn_hvp_omp.c \
 *       -o oracle/_build/libkrcn_hvp_omp.so
 */
#include <omp.h>
#include <stdint.h>

int krcn_oracle_hvp_omp(int64_t n, int64_t d, const int32_t* ptr, const int32_t* idx, const double* val,
                        const int32_t* tptr, const int32_t* tidx, const double* tval, const double* w,
                        const double* v, double l2, double* u, double* y, int threads) {
  if (n <= 0 || d < 0) return 1;
  if (threads > 0) omp_set_num_threads(threads);
  const double dn = (double)n;
#pragma omp parallel
  {
#pragma omp for schedule(dynamic, 256)
    for (int64_t i = 0; i < n; ++i) {
      double s = 0.0;
      for (int32_t e = ptr[i]; e < ptr[i + 1]; ++e) s += val[e] * v[idx[e]];
      u[i] = w[i] * s;
    }
#pragma omp for schedule(dynamic, 1024)
    for (int64_t k = 0; k < d; ++k) {
      double s = 0.0;
      for (int32_t e = tptr[k]; e < tptr[k + 1]; ++e) s += tval[e] * u[tidx[e]];
      y[k] = s / dn + l2 * v[k];
    }
  }
  return 0;
}
