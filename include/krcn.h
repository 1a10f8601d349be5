/*
 * krcn.h — C ABI of the MI355X-native Krylov cubic-regularized-Newton hot path.
 *
 * The hot path is the Lanczos + logistic Hessian-vector-product (HVP) inner loop
 * of Krylov CRN.  Every entry point below replaces one reference (Python/scipy)
 * operation; the reference location it replaces is cited on each declaration.
 * Reference root: Raymond30/Krylov-Cubic-Regularized-Newton (optimizer/loss.py,
 * optimizer/cubic.py).
 *
 * Conventions
 *   - All array arguments are DEVICE pointers (HIP global memory, e.g. the
 *     data_ptr() of a torch tensor) unless the name ends in _host.
 *   - Values are fp64 (KRCN_F64) or fp32 (KRCN_F32), chosen when the matrix
 *     handle is created; every vector passed with that handle has that dtype.
 *     Indices and row pointers are int32 (the reference's scipy CSR downcasts
 *     to int32 whenever nnz < 2^31).
 *   - Calls are asynchronous on `stream` (a hipStream_t, 0 = legacy default)
 *     unless documented as synchronous (they return a scalar to the host).
 *   - The caller owns every buffer it passes.  The library allocates device
 *     memory in krcn_csr_create (transposed CSR, vectors, the Lanczos results
 *     block for m <= 2044), when it builds a handle's pass plans and their
 *     partials (krcn_csr_reserve, krcn_csr_attach_comm of a multi-rank
 *     communicator, the plan queries, or the first compute call of any other
 *     handle), in krcn_csr_reserve(.., reorth = 1) (CGS2 workspace) and in the
 *     first krcn_cg_solve.  krcn_lanczos allocates nothing on a handle that is
 *     reserved for its m; a handle of a multi-rank communicator never builds
 *     or allocates inside a compute call (that call fails instead), so no
 *     rank synchronises the device while its peers wait in a collective.
 *   - Errors: every call returns a krcn_status (0 = OK).  The message of the
 *     last failure on the calling thread is krcn_last_error_string().  No C++
 *     exception crosses this boundary.
 *   - A handle is not thread-safe; one host thread drives one device.
 *   - A handle is single-stream: its scratch (u, w, partials, the Lanczos
 *     state, the pinned staging buffer) lives on the handle, not per call, so
 *     every call on one handle must go to the same stream, or the caller must
 *     order calls on different streams itself (events).  Calls on different
 *     handles are independent.
 *   - Sharded handles (KRCN_SHARD_ROWS / _COLS) must hold at least one row and
 *     one column: every rank joins the collectives of every call, and an empty
 *     block is rejected by krcn_csr_create rather than left to hang its peers.
 */
#ifndef KRCN_H
#define KRCN_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef int krcn_status;
enum {
  KRCN_OK = 0,
  KRCN_ERR_INVALID = 1,     /* bad argument (null pointer, shape, dtype, m < 1) */
  KRCN_ERR_HIP = 2,         /* a HIP runtime call failed                        */
  KRCN_ERR_RCCL = 3,        /* an RCCL call failed                              */
  KRCN_ERR_UNSUPPORTED = 4  /* valid request this build does not implement      */
};

enum { KRCN_F64 = 0, KRCN_F32 = 1 };

/* How a matrix shard relates to the global X (n_global x d_global).
 * KRCN_SHARD_NONE: the handle holds all of X.
 * KRCN_SHARD_ROWS: the handle holds a contiguous block of rows; d-vectors are
 *                  replicated and the HVP all-reduces its d-length partial.
 * KRCN_SHARD_COLS: the handle holds a contiguous block of columns (local column
 *                  indices); d-vectors are sharded, the HVP all-reduces X_p v_p
 *                  (n-length) and Lanczos dots all-reduce one scalar each. */
enum { KRCN_SHARD_NONE = 0, KRCN_SHARD_ROWS = 1, KRCN_SHARD_COLS = 2 };

/* Row-group width policy of the CSR row kernels (lanes of a 64-wide wave that
 * cooperate on one row).  KRCN_LANES_AUTO picks from the mean row length;
 * KRCN_LANES_SEQUENTIAL (1 lane per row, left-to-right sum, no FMA contraction)
 * reproduces scipy's csr_matvec / csc_matvec summation order bit for bit. */
enum { KRCN_LANES_AUTO = 0, KRCN_LANES_SEQUENTIAL = 1 };

/* Column slicing of the two SpMV passes ("Slices"):
 * KRCN_SLICING_AUTO slices a pass when the vector it gathers exceeds ~3 MiB,
 * KRCN_SLICING_OFF never slices, a value k >= 8 (multiple of 8) forces k. */
enum { KRCN_SLICING_AUTO = 0, KRCN_SLICING_OFF = 1 };

/* Tile format of the SpMV passes ("Sorted tiles", "LDS windows"):
 * KRCN_FORMAT_AUTO picks per pass from a cost model, KRCN_FORMAT_WAVE uses
 * per-wave tiles in CSR order, KRCN_FORMAT_SORTED uses block tiles whose
 * nonzeros are stored sorted by gather index (same results, fewer distinct
 * cache lines per gather), KRCN_FORMAT_WINDOW copies column slices of the
 * gathered vector into LDS and sums each row in one lane (short rows),
 * KRCN_FORMAT_JAG gives every lane a row and stores the elements level by level
 * so that the whole LDS holds the gathered vector (one window, or two
 * double-buffered windows walked by every block; scipy's summation order). */
enum { KRCN_FORMAT_AUTO = 0, KRCN_FORMAT_WAVE = 1, KRCN_FORMAT_SORTED = 2, KRCN_FORMAT_WINDOW = 3,
       KRCN_FORMAT_JAG = 4 };

/* Formats reported by krcn_csr_plan_format. */
enum { KRCN_PLAN_WAVE = 1, KRCN_PLAN_SORTED = 2, KRCN_PLAN_WINDOW_SLICES = 3, KRCN_PLAN_WINDOW_ACCUM = 4,
       KRCN_PLAN_JAG = 5 };

typedef struct krcn_csr krcn_csr;
typedef struct krcn_comm krcn_comm;
typedef struct krcn_vctx krcn_vctx;

/* Result summary of krcn_lanczos (mirrors the reference's return values and
 * its truncation rule, optimizer/cubic.py:105-111). */
typedef struct {
  int m_eff;         /* number of basis vectors returned (columns of the reference V)   */
  int breakdown;     /* 1 if |beta| < tol ended the recurrence early (cubic.py:98-99)   */
  int j_break;       /* loop index j at which the breakdown happened, -1 if none        */
  int hvps;          /* Hessian-vector products executed (m when there is no breakdown) */
  double beta_last;  /* the reference's 4th return value `beta` (cubic.py:111)          */
  double gnorm;      /* ||g||_2, the normaliser of the first vector (cubic.py:85)       */
} krcn_lanczos_info;

/* Result summary of krcn_cg_solve (scipy.sparse.linalg.cg's return code, plus
 * what it does not report). */
typedef struct {
  int converged;         /* 1 if norm(r) < rtol ||b|| was reached (scipy info = 0) */
  int info;              /* scipy's info: 0 converged, maxiter if not              */
  int iterations;        /* updates of x performed                                 */
  int pad;
  double residual_norm;  /* ||r|| after the last update                            */
} krcn_cg_info;

/* ---- library ------------------------------------------------------------ */
const char* krcn_last_error_string(void);
int krcn_version(void);

/* ---- matrix handle ------------------------------------------------------ */
/* Upload-side constructor.  indptr (n+1), indices (nnz), data (nnz) are the
 * caller's device CSR arrays of the local block (borrowed: they must outlive
 * the handle).  The handle builds and owns the transposed CSR (X^T stored
 * explicitly, stable in row order so per-column sums run in the order of the
 * reference's csc_matvec scatter).
 * Replaces: the scipy CSR held by LogisticRegression (optimizer/loss.py:188,211)
 * and the zero-copy CSC view A.T it multiplies by (loss.py:227,302).
 * n_global: the reference's self.n (the 1/n of loss.py:227,302);
 * shard_mode: KRCN_SHARD_* (a COLS shard uses local column indices 0..d-1). */
krcn_status krcn_csr_create(int device, int64_t n, int64_t d, int64_t nnz,
                            const int32_t* indptr, const int32_t* indices,
                            const void* data, int dtype, int64_t n_global,
                            int shard_mode, krcn_csr** out);
krcn_status krcn_csr_destroy(krcn_csr* h);
/* Device bytes owned by the handle (transpose + workspace). */
krcn_status krcn_csr_owned_bytes(const krcn_csr* h, int64_t* bytes_host);
/* Row-group policy for X (pass 1) and X^T (pass 2): KRCN_LANES_AUTO,
 * KRCN_LANES_SEQUENTIAL, or an explicit power of two 2..64. */
krcn_status krcn_csr_set_lanes(krcn_csr* h, int lanes_x, int lanes_xt);
/* Slicing policy (KRCN_SLICING_*, or a forced slice count). */
krcn_status krcn_csr_set_slicing(krcn_csr* h, int slicing);
/* Tile format policy (KRCN_FORMAT_*) of both passes. */
krcn_status krcn_csr_set_format(krcn_csr* h, int format);
/* Tile format policy of one pass (1: X, 2: X^T), overriding krcn_csr_set_format
 * for it; -1 returns the pass to the handle's policy. */
krcn_status krcn_csr_set_pass_format(krcn_csr* h, int pass, int format);
/* Execution plan summary (builds the plan if needed):
 * out8_host = {slices, lanes, tiles, grid} of pass 1 (X) then pass 2 (X^T);
 * a sorted-tile pass reports its slice count negated. */
krcn_status krcn_csr_plan_info(krcn_csr* h, int* out8_host);
/* Format of each pass's plan (KRCN_PLAN_*): out2_host = {pass 1, pass 2}. */
krcn_status krcn_csr_plan_format(krcn_csr* h, int* out2_host);
/* Read back the transposed CSR (tests): colptr (d+1), rowidx (nnz), vals (nnz). */
krcn_status krcn_csr_get_transpose(const krcn_csr* h, int32_t* colptr,
                                   int32_t* rowidx, void* vals, void* stream);
/* hipGraph replay of krcn_lanczos (unsharded handles, profiling off): on = 1
 * records the whole launch sequence of a call the second time the same
 * arguments arrive and replays it with one hipGraphLaunch from then on
 * (bitwise the eager sequence).  Off by default: measured no faster on the
 * BASELINE shapes.  Replaces no reference call: the
 * reference's Lanczos loop is Python (optimizer/cubic.py:92-103). */
krcn_status krcn_csr_set_graph(krcn_csr* h, int on);
/* Placement probe of the hot buffers at every plan build (DESIGN.md §5
 * "Placement"): when the handle's per-HVP working set is within reach of the
 * 256 MiB Infinity Cache (96-400 MB), its plan arrays, partials and scratch
 * vectors are copied to trials - 1 further placements, each is timed with the
 * same local HVP (no collective) and the fastest is kept; the rest are freed.
 * Results are bitwise unchanged.  trials: -1 auto (4 in that band, else off;
 * the default), 0 off, 1..8 forced.  Invalidates the plans.  Replaces no
 * reference call (scipy's arrays live in host memory, optimizer/loss.py:188). */
krcn_status krcn_csr_set_placement_trials(krcn_csr* h, int trials);
/* The same search continues over the first krcn_lanczos calls of such a
 * handle (unsharded or single-rank, no graph replay, m >= 8): call 1 runs
 * untimed, the next `trials` calls of the same m each run on one placement
 * (the probe's, then fresh copies), timed by events, and the fastest is kept
 * — the recurrence also streams the caller's V, which the plan-build probe
 * cannot see.  Results of every call are unchanged.
 * krcn_csr_placement_info (builds the plans if needed): out24_host =
 * {placements probed at the plan build, the one kept (-1: none), hot set MB,
 * policy, us per probe HVP of each placement (8 slots), Lanczos calls timed,
 * the placement kept after them (-1: not finished), their m, the search
 * stage, ms per timed call (8 slots)}. */
krcn_status krcn_csr_placement_info(krcn_csr* h, double* out24_host);
/* Attach a communicator for sharded operation (ROWS / COLS modes).  With a
 * communicator of more than one rank the pass plans are built here, before
 * any collective, and the call is COLLECTIVE for ROWS handles: every rank
 * calls it (each on its own thread for a virtual communicator), and the ranks
 * agree on the packed length of their one all-reduce per Lanczos step (the
 * pass-1 alpha partials ride past the d-vector; their count depends on the
 * rank's block).  krcn_csr_reserve after a policy change agrees again. */
krcn_status krcn_csr_attach_comm(krcn_csr* h, krcn_comm* comm);
/* Build the pass plans now (if a policy call invalidated them) and reserve
 * the workspace of krcn_lanczos up to m_max (1..2044; reorth = 1 adds the
 * CGS2 partials for m_max), so that later krcn_lanczos calls with m <= m_max
 * allocate and free nothing.  Required on a handle of a multi-rank
 * communicator after a policy change and before reorthogonalised calls.
 * Replaces no reference call (the reference allocates per numpy call). */
krcn_status krcn_csr_reserve(krcn_csr* h, int m_max, int reorth);

/* ---- objective pieces (optimizer/loss.py) -------------------------------- */
/* Ax = X x.                       Replaces LogisticRegression.mat_vec_product,
 *                                 loss.py:266-277 (the A @ x of :270).        */
krcn_status krcn_matvec(krcn_csr* h, const void* x, void* Ax, void* stream);
/* y = (X^T u) / n_global.         Replaces A.T @ u / self.n, loss.py:227,302. */
krcn_status krcn_rmatvec(krcn_csr* h, const void* u, void* y, void* stream);
/* w_i = s(1 - s), s = expit(Ax_i). Replaces loss.py:296-297 (hoisted: it
 *                                 depends on x only, not on v).               */
krcn_status krcn_weights(krcn_csr* h, const void* Ax, void* w, void* stream);
/* y = X^T (w (.) X v) / n + l2 v. Replaces LogisticRegression.hess_vec_prod,
 *                                 loss.py:289-302 (grad_dif=False branch).
 * l2 == 0 stores X^T(..)/n without reading v: the reference's + 0 * v gives
 * the same bits for every finite v, the sign of a zero included — a row sum
 * s is never -0 (it starts from +0; +0 + (-0) and x + (-x) round to +0), so
 * s/n + (+-0) = s/n — and would turn an inf / nan v into nan
 * (tests/test_gpu_hvp.py::test_l2_zero_hvp_signed_zeros). */
krcn_status krcn_hvp(krcn_csr* h, const void* w, const void* v, void* y,
                     double l2, void* stream);
/* grad = X^T (expit(Ax) - b) / n (+ l2 x when l2 != 0).
 *                                 Replaces LogisticRegression.gradient,
 *                                 loss.py:223-232.                            */
krcn_status krcn_gradient(krcn_csr* h, const void* Ax, const void* b,
                          const void* x, double l2, void* grad, void* stream);
/* SYNCHRONOUS.  *out_host = mean((1 - b) Ax - logsig(Ax)) (without the l2
 * term, which the host adds as the reference does).
 *                                 Replaces LogisticRegression._value,
 *                                 loss.py:215-220, and logsig, loss.py:161-176. */
krcn_status krcn_loss_mean(krcn_csr* h, const void* Ax, const void* b,
                           double* out_host, void* stream);

/* SYNCHRONOUS.  out_host[i] = mean((1 - b) X x_i - logsig(X x_i)) for k
 * iterates x_i (device d-vectors; xs_host is a HOST array of k device
 * pointers), without the l2 term — each value bitwise what krcn_matvec +
 * krcn_loss_mean return for that iterate, with all 2k launches in one
 * submission, one all-reduce of the k sums (ROWS) and one D2H.  Uses the
 * handle's n-vector scratch.
 * Replaces the loop `[self.loss.value(x) for x in self.xs]` of
 * Trace.compute_loss_of_iterates, optimizer/opt_trace.py:39-41 (with
 * optimizer.py:164-166), over iterates kept on the device. */
krcn_status krcn_loss_values(krcn_csr* h, int k, const void* const* xs_host, const void* b,
                             double* out_host, void* stream);

/* ---- Lanczos (optimizer/cubic.py:77-111) -------------------------------- */
/* SYNCHRONOUS on return of alphas/betas/info.  Runs the reference three-term
 * Lanczos on the operator v -> hess_vec_prod(x, v) (w = weights at x), started
 * from g.  V is the caller's device basis of m rows x ld columns (row j = the
 * reference's column V[:, j], contiguous; ld = local d).  alphas_host[m],
 * betas_host[max(m-1,1)] receive the reference's alphas/betas (already
 * truncated to info->m_eff / m_eff-1 entries; entries past that are zero).
 * reorth = 0 reproduces the reference (no reorthogonalisation, the default);
 * reorth = 1 adds classical Gram-Schmidt twice (CGS2) against all previous
 * basis vectors (build-only extension; not in the reference).  An unsharded
 * handle whose V is 16-byte aligned with rows of whole 16-byte vectors
 * (ld * sizeof(T) % 16 == 0) runs the 1 KiB-row-piece sweeps with step B in
 * the first; otherwise the batched sweeps run (the same CGS2, summed in
 * another fixed order).
 * tol is the reference's absolute breakdown threshold (1e-6, cubic.py:98). */
krcn_status krcn_lanczos(krcn_csr* h, const void* w, const void* g, int m,
                         int reorth, double tol, double l2, void* V,
                         double* alphas_host, double* betas_host,
                         krcn_lanczos_info* info_host, void* stream);

/* x_new = x + V^T s over the first m_eff basis rows (the reference's
 * x + V @ s_new, cubic.py:291,301).  V is the handle's basis (m rows x local d),
 * s_host an m_eff-vector on the host; x, x_new are local d-vectors. */
krcn_status krcn_basis_combine(krcn_csr* h, int m_eff, const void* V,
                               const double* s_host, const void* x, void* x_new,
                               void* stream);

/* ---- conjugate gradients on the Hessian (full-space CRN) ---------------- */
/* SYNCHRONOUS.  Solves (H + shift I) x = b, H = X^T diag(w) X / n_global,
 * by unpreconditioned conjugate gradients from x0 = 0 with scipy's loop and
 * stopping rule (scipy.sparse.linalg.cg: stop when ||r|| < rtol ||b||, at most
 * maxiter updates; ||b|| = 0 returns x = 0).  Each iteration is one HVP on the
 * device plus two vector launches; control stays on the device.
 * Replaces the cg(LinearOperator(v -> hess_vec_prod(x, v) + lam v), -g, tol)
 * calls of Cubic_LS.cubic_solver_root_CG, optimizer/cubic.py:152-182 (pass the
 * reference's l2 + lam as shift).  Unsharded handles only. */
krcn_status krcn_cg_solve(krcn_csr* h, const void* w, const void* b, double shift,
                          double rtol, int maxiter, void* x,
                          krcn_cg_info* info_host, void* stream);

/* ---- dense vector helpers (host glue of optimizer.py / utils.py) -------- */
/* Vector spaces of a handle: n-vectors (one entry per sample row) and
 * d-vectors (one entry per feature).  In a sharded handle the helper reduces
 * over all ranks when that space is sharded (ROWS: n, COLS: d). */
enum { KRCN_SPACE_N = 0, KRCN_SPACE_D = 1 };
/* SYNCHRONOUS.  *out_host = sum_i a_i b_i, deterministic tree order
 * (np.dot, cubic.py:94,109). */
krcn_status krcn_dot(krcn_csr* h, int space, const void* a, const void* b,
                     double* out_host, void* stream);
/* SYNCHRONOUS.  *out_host = ||a - b||_2 (b may be NULL for ||a||_2).
 * Replaces loss.norm(x - x_old) of optimizer.py:110 and np.linalg.norm. */
krcn_status krcn_diff_norm(krcn_csr* h, int space, const void* a, const void* b,
                           double* out_host, void* stream);

/* ---- handle-free vector context ------------------------------------------ */
/* Reduction scratch + pinned staging on one device, for vectors of any length
 * and either dtype (no matrix handle needed). */
krcn_status krcn_vctx_create(int device, krcn_vctx** out);
krcn_status krcn_vctx_destroy(krcn_vctx* c);
/* SYNCHRONOUS.  One Lanczos step over an external operator, y = A(v) supplied
 * by the caller: w = y - beta v_pre (w = y when v_pre is NULL), alpha = v.w,
 * z = w - alpha v, beta' = ||z||; z receives the unnormalised next vector,
 * alpha_beta_host = {alpha, beta'}.  Replaces cubic.py:93-97 for Lanczos(A, v, m)
 * with a callable A the fused krcn_lanczos cannot run. */
krcn_status krcn_lz_ext_step(krcn_vctx* c, int dtype, int64_t n, const void* y,
                             const void* v, const void* v_pre, double beta,
                             void* z, double* alpha_beta_host, void* stream);
/* SYNCHRONOUS.  *out_host = a.b (fixed-order tree; np.dot, cubic.py:109). */
krcn_status krcn_vec_dot(krcn_vctx* c, int dtype, int64_t n, const void* a,
                         const void* b, double* out_host, void* stream);
/* out = a / div (the reference's v = w / beta, cubic.py:85,102). */
krcn_status krcn_vec_div(krcn_vctx* c, int dtype, int64_t n, const void* a,
                         double div, void* out, void* stream);
/* out = y + alpha x (x + s of Cubic_LS.step, cubic.py:209; out may alias y). */
krcn_status krcn_vec_axpy(krcn_vctx* c, int dtype, int64_t n, double alpha,
                          const void* x, const void* y, void* out, void* stream);

/* ---- multi-GPU (RCCL over xGMI; one process per GPU) -------------------- */
/* 128-byte RCCL unique id, produced on rank 0 and broadcast by the caller. */
krcn_status krcn_comm_unique_id(void* uid128_host);
krcn_status krcn_comm_create(int nranks, int rank, const void* uid128_host,
                             int device, krcn_comm** out);
krcn_status krcn_comm_destroy(krcn_comm* c);
/* nranks VIRTUAL ranks on one device (tests and rehearsals of a sharded run
 * without nranks GPUs; RCCL refuses two ranks on one device): out[0..nranks)
 * receive one communicator per rank, each to be attached to that rank's
 * handle and driven by its own host thread on its own stream.  Every
 * all-reduce drains the caller's stream and waits for the other ranks; the
 * last to arrive sums the ranks' buffers in rank order on the device.  A rank
 * missing for 90 s breaks the group (every waiting call fails, and the error
 * string lists how many all-reduces each rank has entered, the count of its
 * last one and which ranks were waiting).  Destroy
 * each communicator; the group goes with the last one.  Not in the
 * reference: it has no parallelism ("P virtual shards"). */
krcn_status krcn_comm_create_virtual(int nranks, int device, krcn_comm** out);
/* In-place sum all-reduce of n values of dtype (plumbing for tests/bench). */
krcn_status krcn_comm_allreduce(krcn_comm* c, int dtype, void* buf, int64_t n,
                                void* stream);

/* ---- LIBSVM / svmlight text (host) ---------------------------------------- */
/* Parse svmlight text (text[0..len), not NUL-terminated) on `threads` host
 * threads (<= 0: all cores) into a parsed set: info4_host = {rows, nnz, the
 * largest index, the smallest index (-1 without nonzeros)}.  The grammar and
 * the errors are sklearn.datasets.load_svmlight_file's (comments, blank
 * lines, a leading qid:, correctly rounded decimal floats; a negative index or
 * indices not strictly increasing in a row are KRCN_ERR_INVALID with sklearn's
 * message).  Replaces the reference's load_svmlight_file(path)
 * (cubic_newton.py:52-53). */
typedef struct krcn_svm krcn_svm;
krcn_status krcn_svm_parse(const char* text, int64_t len, int threads, krcn_svm** out,
                           int64_t* info4_host);
/* Copy a parsed set into the caller's HOST arrays: indptr (rows + 1) and
 * indices (nnz) as int32 with every index lowered by `shift` (1 for one-based
 * files), data (nnz) and labels (rows) as float64. */
krcn_status krcn_svm_export(const krcn_svm* p, int64_t shift, int32_t* indptr, int32_t* indices,
                            double* data, double* labels);
krcn_status krcn_svm_destroy(krcn_svm* p);

/* ---- profiling ----------------------------------------------------------- */
/* When enabled, krcn_hvp / krcn_lanczos record HIP events around every
 * pass-1 (X v) and pass-2 (X^T u) launch on the call's stream and accumulate
 * their durations; krcn_prof_read returns {calls, ms} for pass 1 (with its
 * slice combine), pass 2 and the whole HVP (pass 1 start to pass 2 end), then
 * the ms of pass 1's main launch alone and of its slice combine, and resets
 * the counters: out8_host = {c, p1, c, p2, c, hvp, p1_kernel, p1_combine}. */
krcn_status krcn_prof_enable(krcn_csr* h, int on);
krcn_status krcn_prof_read(krcn_csr* h, double* out8_host);

#ifdef __cplusplus
}
#endif
#endif /* KRCN_H */
