// krcn_plan.hip — handle lifecycle, the transposed CSR, the pass plans (tile /
// sorted / LDS-window formats), the RCCL communicator and profiling readout.
#include "krcn_internal.hpp"

#include <hipcub/hipcub.hpp>

using namespace krcn;

// ------------------------------------------------------------------ errors
static thread_local std::string g_err;

krcn_status fail(krcn_status s, const char* fmt, ...) {
  char buf[2048];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
  return s;
}

// ---------------------------------------------------------------- library
extern "C" const char* krcn_last_error_string(void) { return g_err.c_str(); }

std::mutex& build_mutex() {
  static std::mutex m;
  return m;
}
extern "C" int krcn_version(void) { return 1; }

// ---------------------------------------------------------- matrix handle
template <typename T>
static krcn_status build_transpose(krcn_csr* h, hipStream_t s) {
  const int64_t n = h->n, d = h->d, nnz = h->nnz;
  CHK(dalloc(h, &h->tptr, size_t(d + 1)));
  CHK(dalloc(h, &h->tidx, size_t(nnz)));
  T* tval = nullptr;
  CHK(dalloc(h, &tval, size_t(nnz)));
  h->tval = tval;
  if (nnz == 0) {
    HIPCHK(hipMemsetAsync(h->tptr, 0, size_t(d + 1) * sizeof(int), s));
    return KRCN_OK;
  }
  int *rowid = nullptr, *iota = nullptr, *keys_out = nullptr, *perm = nullptr;
  HIPCHK(hipMalloc(&rowid, size_t(nnz) * sizeof(int)));
  HIPCHK(hipMalloc(&iota, size_t(nnz) * sizeof(int)));
  HIPCHK(hipMalloc(&keys_out, size_t(nnz) * sizeof(int)));
  HIPCHK(hipMalloc(&perm, size_t(nnz) * sizeof(int)));
  hipLaunchKernelGGL(k_expand_rows, dim3(vec_grid(n * 64)), dim3(kNT), 0, s, int(n), h->ptr, rowid);
  LAUNCHCHK();
  hipLaunchKernelGGL(k_iota, dim3(vec_grid(nnz)), dim3(kNT), 0, s, nnz, iota);
  LAUNCHCHK();
  int bits = 1;
  while ((int64_t(1) << bits) < d) ++bits;
  size_t tmpb = 0;
  HIPCHK(hipcub::DeviceRadixSort::SortPairs(nullptr, tmpb, h->idx, keys_out, iota, perm, int(nnz), 0,
                                            bits, s));
  void* tmp = nullptr;
  HIPCHK(hipMalloc(&tmp, tmpb));
  // LSD radix sort is stable: inside every column the entries keep their CSR
  // (row-ascending) order, i.e. the order csc_matvec scatters them in.
  HIPCHK(hipcub::DeviceRadixSort::SortPairs(tmp, tmpb, h->idx, keys_out, iota, perm, int(nnz), 0,
                                            bits, s));
  hipLaunchKernelGGL(k_colptr_from_sorted, dim3(vec_grid(d + 1)), dim3(kNT), 0, s, d, nnz,
                     keys_out, h->tptr);
  LAUNCHCHK();
  hipLaunchKernelGGL((k_gather_transpose<T>), dim3(vec_grid(nnz)), dim3(kNT), 0, s, nnz, perm,
                     rowid, static_cast<const T*>(h->val), h->tidx, tval);
  LAUNCHCHK();
  HIPCHK(hipStreamSynchronize(s));
  HIPCHK(hipFree(tmp));
  HIPCHK(hipFree(rowid));
  HIPCHK(hipFree(iota));
  HIPCHK(hipFree(keys_out));
  HIPCHK(hipFree(perm));
  return KRCN_OK;
}

static krcn_status destroy_impl(krcn_csr* h) {
  if (!h) return KRCN_OK;
  (void)hipSetDevice(h->device);
  void* bufs[] = {h->tptr, h->tidx, h->tval, h->pa, h->pb, h->scal, h->st, h->u, h->tn, h->W,
                  h->td, h->alphas_dev, h->hcoef, h->pr, h->pr2, h->cy, h->ccnt, h->pz, h->pq, h->cg_r, h->cg_st,
                  h->fcnt};
  for (void* b : bufs)
    if (b) (void)hipFree(b);
  if (h->hostbuf) (void)hipHostFree(h->hostbuf);
  if (h->hostres) (void)hipHostFree(h->hostres);
  if (h->gexec) (void)hipGraphExecDestroy(h->gexec);
  if (h->gstream) (void)hipStreamDestroy(h->gstream);
  lzp_abort(h);
  if (h->lzp_e0) (void)hipEventDestroy(h->lzp_e0);
  if (h->lzp_e1) (void)hipEventDestroy(h->lzp_e1);
  free_plan(h->p1);
  free_plan(h->p2);
  for (auto& r : h->prof_pool) {
    (void)hipEventDestroy(r.e0);
    (void)hipEventDestroy(r.e1);
    (void)hipEventDestroy(r.e2);
    (void)hipEventDestroy(r.em);
  }
  delete h;
  return KRCN_OK;
}

extern "C" krcn_status krcn_csr_create(int device, int64_t n, int64_t d, int64_t nnz,
                                       const int32_t* indptr, const int32_t* indices,
                                       const void* data, int dtype, int64_t n_global,
                                       int shard_mode, krcn_csr** out) {
  if (!out) return fail(KRCN_ERR_INVALID, "krcn_csr_create: out is null");
  *out = nullptr;
  if (n < 0 || d < 0 || nnz < 0) return fail(KRCN_ERR_INVALID, "krcn_csr_create: negative shape");
  if (nnz >= (int64_t(1) << 31) || n >= (int64_t(1) << 31) || d >= (int64_t(1) << 31))
    return fail(KRCN_ERR_UNSUPPORTED, "krcn_csr_create: int32 indices require n, d, nnz < 2^31");
  if (dtype != KRCN_F64 && dtype != KRCN_F32) return fail(KRCN_ERR_INVALID, "krcn_csr_create: bad dtype");
  if (shard_mode < KRCN_SHARD_NONE || shard_mode > KRCN_SHARD_COLS)
    return fail(KRCN_ERR_INVALID, "krcn_csr_create: bad shard_mode");
  if (!indptr || (nnz > 0 && (!indices || !data)))
    return fail(KRCN_ERR_INVALID, "krcn_csr_create: null CSR array");
  if ((reinterpret_cast<uintptr_t>(indices) | reinterpret_cast<uintptr_t>(data)) % 16 != 0)
    return fail(KRCN_ERR_INVALID, "krcn_csr_create: indices and data must be 16-byte aligned (16-B vector loads)");
  // every rank of a sharded run joins the collectives of each call: a rank
  // with an empty block would skip them (early returns on empty work) and
  // leave the others blocked, so an empty shard is rejected up front
  if (shard_mode != KRCN_SHARD_NONE && (n == 0 || d == 0))
    return fail(KRCN_ERR_INVALID, "krcn_csr_create: a shard must hold at least one row and one column (got %lld x %lld)",
                (long long)n, (long long)d);
  if (n_global <= 0) n_global = n;
  krcn_csr* h = new krcn_csr();
  if (const char* e = tuning_env("KRCN_SORT_NT")) h->sort_nt = atoi(e) == 256 || atoi(e) == 512 || atoi(e) == 1024 ? atoi(e) : 0;  // tuning knob
  h->device = device;
  h->dtype = dtype;
  h->vs = dtype == KRCN_F64 ? 8 : 4;
  h->shard = shard_mode;
  h->n = n;
  h->d = d;
  h->nnz = nnz;
  h->n_global = n_global;
  h->ptr = indptr;
  h->idx = indices;
  h->val = data;
  krcn_status st = KRCN_OK;
  auto init = [&]() -> krcn_status {
    std::lock_guard<std::mutex> lk(build_mutex());
    HIPCHK(hipSetDevice(device));
    hipStream_t s = nullptr;
    HIPCHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    krcn_status r = dtype == KRCN_F64 ? build_transpose<double>(h, s) : build_transpose<float>(h, s);
    const hipError_t se = hipStreamSynchronize(s);
    (void)hipStreamDestroy(s);
    CHK(r);
    HIPCHK(se);
    CHK(dalloc(h, &h->pa, kMaxPartials));
    CHK(dalloc(h, &h->pb, kMaxPartials));
    CHK(dalloc(h, &h->scal, 16));
    CHK(dalloc(h, &h->st, 1));
    char* p = nullptr;
    CHK(dalloc(h, &p, size_t(n + 2) * h->vs)); h->u = p;   // + 2: the packed d-space sums (lanczos_impl)
    CHK(dalloc(h, &p, size_t(n) * h->vs)); h->tn = p;
    CHK(dalloc(h, &p, size_t(d) * h->vs)); h->W = p;
    CHK(dalloc(h, &p, size_t(d + kMaxPartials) * h->vs)); h->td = p;   // + the packed alpha partials (lanczos_impl)
    // the Lanczos recurrence's alphas | betas for every m <= kLzMaxM (+ 4 spare
    // doubles), and the CGS2 coefficients (which read kCgsHPad zeros past k);
    // the packed results go to the mapped host block hostres (k_lz_final)
    CHK(dalloc(h, &h->alphas_dev, size_t(2 * kLzMaxM + 4)));
    h->betas_dev = h->alphas_dev + kLzMaxM;
    CHK(dalloc(h, &h->hcoef, size_t(kLzMaxM + kCgsHPad)));
    h->mcap = kLzMaxM;
    HIPCHK(hipHostMalloc(reinterpret_cast<void**>(&h->hostbuf), 4096 * sizeof(double), 0));
    // the Lanczos results block: mapped, coherent host memory that k_lz_final
    // stores into (one kernel store stream over PCIe instead of a copy launch
    // per call: round 5, w8a's m = 10 calls)
    HIPCHK(hipHostMalloc(reinterpret_cast<void**>(&h->hostres), size_t(kLzOut) * sizeof(double),
                         hipHostMallocMapped | hipHostMallocCoherent));
    HIPCHK(hipHostGetDevicePointer(reinterpret_cast<void**>(&h->hostres_dev), h->hostres, 0));
    HIPCHK(hipMemset(h->st, 0, sizeof(LanczosState)));
    HIPCHK(hipMemset(h->scal, 0, 16 * sizeof(double)));
    return KRCN_OK;
  };
  st = init();
  if (st != KRCN_OK) {
    std::string keep = g_err;
    destroy_impl(h);
    g_err = keep;
    return st;
  }
  *out = h;
  return KRCN_OK;
}

extern "C" krcn_status krcn_csr_destroy(krcn_csr* h) { return destroy_impl(h); }

extern "C" krcn_status krcn_csr_owned_bytes(const krcn_csr* h, int64_t* bytes_host) {
  if (!h || !bytes_host) return fail(KRCN_ERR_INVALID, "krcn_csr_owned_bytes: null argument");
  *bytes_host = int64_t(h->owned + h->p1.owned + h->p2.owned);
  return KRCN_OK;
}

static bool lanes_ok(int L) {
  return L == KRCN_LANES_AUTO || L == KRCN_LANES_SEQUENTIAL || L == 2 || L == 4 || L == 8 ||
         L == 16 || L == 32 || L == 64;
}

extern "C" krcn_status krcn_csr_set_lanes(krcn_csr* h, int lanes_x, int lanes_xt) {
  if (!h) return fail(KRCN_ERR_INVALID, "krcn_csr_set_lanes: null handle");
  if (!lanes_ok(lanes_x) || !lanes_ok(lanes_xt))
    return fail(KRCN_ERR_INVALID, "krcn_csr_set_lanes: lanes must be 0 (auto), 1 (sequential) or a power of two <= 64");
  if (h->lanes_x != lanes_x || h->lanes_xt != lanes_xt) h->plans_ready = false;
  h->lanes_x = lanes_x;
  h->lanes_xt = lanes_xt;
  return KRCN_OK;
}

extern "C" krcn_status krcn_csr_get_transpose(const krcn_csr* h, int32_t* colptr, int32_t* rowidx,
                                              void* vals, void* stream) {
  if (!h) return fail(KRCN_ERR_INVALID, "krcn_csr_get_transpose: null handle");
  CHK(set_device(h));
  hipStream_t s = S(stream);
  if (colptr) HIPCHK(hipMemcpyAsync(colptr, h->tptr, size_t(h->d + 1) * sizeof(int), hipMemcpyDeviceToDevice, s));
  if (rowidx && h->nnz) HIPCHK(hipMemcpyAsync(rowidx, h->tidx, size_t(h->nnz) * sizeof(int), hipMemcpyDeviceToDevice, s));
  if (vals && h->nnz) HIPCHK(hipMemcpyAsync(vals, h->tval, size_t(h->nnz) * h->vs, hipMemcpyDeviceToDevice, s));
  return KRCN_OK;
}

// Row shards of a multi-rank communicator pack the pass-1 combine's alpha
// partials past the d-vector of their one all-reduce per Lanczos step
// (krcn_lanczos_impl.hpp early_rows).  Each rank's count depends on its own
// block (the partition balances nonzeros, not rows), so the ranks agree here,
// after every plan build and before any compute call: the packed length is
// the maximum over ranks (a rank with fewer zero-fills the rest), and the
// step runs only if every rank's grids fit.  One all-reduce of 2 x nranks
// doubles (rank r fills slots r and nranks + r).  Collective: every rank of
// the communicator calls it (krcn_csr_attach_comm, krcn_csr_reserve).
static krcn_status agree_rows(krcn_csr* h) {
  if (!h->comm || h->comm->nranks <= 1 || h->shard != KRCN_SHARD_ROWS || h->rows_pq >= 0) return KRCN_OK;
  const int P = h->comm->nranks, me = h->comm->rank;
  std::vector<double> v(size_t(2 * P), 0.0);
  v[size_t(me)] = pass_partials(h->p1);
  v[size_t(P + me)] = std::max(h->p1.grid, h->p1.combine_grid) <= kMaxPartials ? 1.0 : 0.0;
  double* dv = nullptr;
  hipStream_t s = nullptr;
  HIPCHK(hipMalloc(&dv, v.size() * sizeof(double)));
  krcn_status r = KRCN_OK;
  if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess ||
      hipMemcpyAsync(dv, v.data(), v.size() * sizeof(double), hipMemcpyHostToDevice, s) != hipSuccess)
    r = fail(KRCN_ERR_HIP, "agree_rows: staging");
  if (r == KRCN_OK) r = allreduce(h, dv, int64_t(v.size()), KRCN_F64, s);
  if (r == KRCN_OK && (hipMemcpyAsync(v.data(), dv, v.size() * sizeof(double), hipMemcpyDeviceToHost, s) != hipSuccess ||
                       hipStreamSynchronize(s) != hipSuccess))
    r = fail(KRCN_ERR_HIP, "agree_rows: readback");
  if (s) (void)hipStreamDestroy(s);
  (void)hipFree(dv);
  CHK(r);
  int pq = 0, ok = 1;
  for (int i = 0; i < P; ++i) {
    pq = std::max(pq, int(v[size_t(i)]));
    ok = ok && v[size_t(P + i)] == 1.0;
  }
  h->rows_pq = pq;
  h->rows_early = ok && pq <= kMaxPartials;
  return KRCN_OK;
}

extern "C" krcn_status krcn_csr_attach_comm(krcn_csr* h, krcn_comm* comm) {
  if (!h) return fail(KRCN_ERR_INVALID, "krcn_csr_attach_comm: null handle");
  if (comm && h->shard == KRCN_SHARD_NONE && comm->nranks > 1)
    return fail(KRCN_ERR_INVALID, "krcn_csr_attach_comm: an unsharded handle cannot join a %d-rank communicator", comm->nranks);
  h->comm = comm;
  h->rows_pq = -1;
  // a multi-rank handle builds its plans now, before any collective (plans_for_compute)
  if (comm && comm->nranks > 1) {
    CHK(set_device(h));
    CHK(ensure_plans(h));
    CHK(agree_rows(h));
  }
  return KRCN_OK;
}

// ----------------------------------------------------------- pass plans
static constexpr int64_t kSliceThresholdBytes = 3 << 20;   // gathered vector above this: slice
static constexpr int64_t kSliceTargetBytes = 2 << 20;      // x window per slice
static constexpr int kBlocksPerGroup = 256;                // sliced: 8 groups x 256 = 2048 blocks (8 per CU)
static constexpr int kMaxGrid = 2048;
static constexpr int kNumCUs = 256;                        // MI355X: 8 XCDs x 32 CUs

void free_plan(PassPlan& P) {
  void* bufs[] = {P.own_ptr, P.own_idx, P.own_val, P.tiles, P.tbeg, P.part, P.gword, P.gval, P.tmid,
                  P.widx, P.segs, P.tb, P.ro, P.jgcut, P.jumeta, P.jcnt, P.jlcut, P.jlrow, P.jltask,
                  P.jtask, P.jlidx, P.jlval, P.xcp, P.xrow, P.xval, P.xpart};
  for (void* b : bufs)
    if (b) (void)hipFree(b);
  P = PassPlan();
}

static int slices_for(int64_t bytes) {
  if (bytes <= kSliceThresholdBytes) return 1;
  const int64_t per8 = 8 * kSliceTargetBytes;
  return int(8 * ((bytes + per8 - 1) / per8));
}

// Sliced copy of a CSR: slice s holds columns [bounds[s], bounds[s+1]) with
// global column ids, rows in order; row pointers flattened slice-major.
template <typename T>
static krcn_status build_slices(PassPlan& P, const int* ptr, const int* idx, const T* val, hipStream_t s,
                                const std::vector<int>* bounds_in = nullptr, int64_t pad = 0) {
  const int S = P.S, rows = P.rows;
  const int64_t nnz = P.nnz, cols = P.cols;
  std::vector<int> hb(S + 1);
  for (int k = 0; k <= S; ++k) hb[k] = bounds_in ? (*bounds_in)[k] : int((cols * k) / S);
  int *bounds = nullptr, *sid = nullptr, *sid_out = nullptr, *iota = nullptr, *perm = nullptr, *counts = nullptr;
  HIPCHK(hipMalloc(&bounds, sizeof(int) * (S + 1)));
  HIPCHK(hipMemcpyAsync(bounds, hb.data(), sizeof(int) * (S + 1), hipMemcpyHostToDevice, s));
  const size_t nptr = size_t(S) * rows + 1;
  HIPCHK(hipMalloc(&P.own_ptr, sizeof(int) * nptr));
  HIPCHK(hipMalloc(&P.own_idx, sizeof(int) * std::max<int64_t>(nnz, 1)));
  HIPCHK(hipMalloc(&P.own_val, sizeof(T) * size_t(std::max<int64_t>(nnz, 1) + pad)));
  if (pad) HIPCHK(hipMemsetAsync(static_cast<T*>(P.own_val) + nnz, 0, sizeof(T) * size_t(pad), s));
  P.owned += sizeof(int) * nptr + (sizeof(int) + sizeof(T)) * size_t(std::max<int64_t>(nnz, 1)) + sizeof(T) * pad;
  HIPCHK(hipMalloc(&counts, sizeof(int) * nptr));
  HIPCHK(hipMemsetAsync(counts, 0, sizeof(int) * nptr, s));
  if (nnz > 0) {
    HIPCHK(hipMalloc(&sid, sizeof(int) * nnz));
    HIPCHK(hipMalloc(&sid_out, sizeof(int) * nnz));
    HIPCHK(hipMalloc(&iota, sizeof(int) * nnz));
    HIPCHK(hipMalloc(&perm, sizeof(int) * nnz));
    hipLaunchKernelGGL(k_slice_of, dim3(vec_grid(nnz)), dim3(kNT), 0, s, nnz, idx, bounds, S, sid);
    LAUNCHCHK();
    hipLaunchKernelGGL(k_iota, dim3(vec_grid(nnz)), dim3(kNT), 0, s, nnz, iota);
    LAUNCHCHK();
    int bits = 1;
    while ((1 << bits) < S) ++bits;
    size_t tmpb = 0;
    HIPCHK(hipcub::DeviceRadixSort::SortPairs(nullptr, tmpb, sid, sid_out, iota, perm, int(nnz), 0, bits, s));
    void* tmp = nullptr;
    HIPCHK(hipMalloc(&tmp, tmpb));
    // stable: inside a slice the nonzeros keep their row-major order
    HIPCHK(hipcub::DeviceRadixSort::SortPairs(tmp, tmpb, sid, sid_out, iota, perm, int(nnz), 0, bits, s));
    hipLaunchKernelGGL(k_slice_counts, dim3(vec_grid(int64_t(rows) * 64)), dim3(kNT), 0, s, rows, ptr, sid, counts);
    LAUNCHCHK();
    hipLaunchKernelGGL((k_slice_gather<T>), dim3(vec_grid(nnz)), dim3(kNT), 0, s, nnz, perm, idx, val,
                       P.own_idx, static_cast<T*>(P.own_val));
    LAUNCHCHK();
    size_t tmp2 = 0;
    HIPCHK(hipcub::DeviceScan::InclusiveSum(nullptr, tmp2, counts, P.own_ptr, int(nptr), s));
    void* t2 = nullptr;
    HIPCHK(hipMalloc(&t2, tmp2));
    HIPCHK(hipcub::DeviceScan::InclusiveSum(t2, tmp2, counts, P.own_ptr, int(nptr), s));
    HIPCHK(hipStreamSynchronize(s));
    HIPCHK(hipFree(t2));
    HIPCHK(hipFree(tmp));
  } else {
    HIPCHK(hipMemsetAsync(P.own_ptr, 0, sizeof(int) * nptr, s));
  }
  HIPCHK(hipStreamSynchronize(s));
  void* frees[] = {bounds, sid, sid_out, iota, perm, counts};
  for (void* f : frees)
    if (f) HIPCHK(hipFree(f));
  P.ptr = P.own_ptr;
  P.idx = P.own_idx;
  P.val = P.own_val;
  return KRCN_OK;
}

// Tile list (host greedy over the row pointers), grouped by XCD group.
// Wave tiles: <= kWaveTileNnz nonzeros in the 4-aligned window, <= kWaveTileRows
// rows.  Sorted block tiles: <= kSortTile nonzeros, <= kSortTileRows rows, and
// `segs` receives the sort segments (a normal tile, or kSortTile chunks of a
// long row) as nonzero offsets.
static krcn_status build_tiles(PassPlan& P, hipStream_t s, std::vector<int>* segs, std::vector<int>* segbase) {
  const int S = P.S, rows = P.rows;
  const bool sorted = P.sorted != 0;
  const int sort_tile = P.sort_nt * kSortPerThread;
  const int cap_nnz = sorted ? sort_tile : kWaveTileNnz;
  const int cap_rows = sorted ? sort_tile / 4 : kWaveTileRows;
  const int per_block = sorted ? 1 : kWavesPerBlock;
  const size_t nptr = size_t(S) * rows + 1;
  std::vector<int> hp(nptr);
  HIPCHK(hipMemcpyAsync(hp.data(), P.ptr, sizeof(int) * nptr, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  auto win = [&](const int* rp, int a, int b) { return sorted ? rp[b] - rp[a] : rp[b] - (rp[a] & ~3); };
  // Greedy tiling of one slice with nonzero cap `cap`; emit(long, r0, r1).
  auto walk = [&](int sl, int cap, auto&& emit) {
    const int* rp = hp.data() + size_t(sl) * rows;
    int r = 0;
    while (r < rows) {
      // a tile's nonzero window must fit one wave slab / block tile
      if (win(rp, r, r + 1) > cap) {
        emit(1, r, r + 1);
        ++r;
        continue;
      }
      int r1 = r + 1;
      while (r1 < rows && r1 - r < cap_rows && win(rp, r, r1 + 1) <= cap) ++r1;
      emit(0, r, r1);
      r = r1;
    }
  };
  // Sorted tiles run one resident wave of B blocks per XCD group: shrink
  // the tiles of a group until its tile count fills whole rounds of B blocks
  // (smallest cap with count(cap) <= R * B, R = rounds at the full tile), so
  // no block runs a last round alone.
  // sorted tiles: one resident wave of blocks (8 waves per SIMD)
  const int per_group = sorted ? kBlocksPerGroup * kNT / P.sort_nt : kBlocksPerGroup;
  const int max_grid = sorted ? kMaxGrid * kNT / P.sort_nt : kMaxGrid;
  std::vector<int> gcap(P.groups, cap_nnz);
  if (sorted) {
    const int B = P.groups > 1 ? per_group : max_grid;
    for (int g = 0; g < P.groups; ++g) {
      auto count = [&](int cap) {
        int64_t c = 0;
        for (int sl = g; sl < S; sl += P.groups) walk(sl, cap, [&](int, int, int) { ++c; });
        return c;
      };
      const int64_t n0 = count(cap_nnz);
      if (n0 == 0) continue;
      const int64_t R = (n0 + B - 1) / B;
      if (R < 2) continue;   // a single partial round: keep the tiles whole
      int lo = std::max(64, cap_nnz / 16), hi = cap_nnz;   // count(hi) <= R * B
      if (count(lo) <= R * B) { gcap[g] = lo; continue; }
      while (hi - lo > 32) {
        const int mid = (lo + hi) / 2;
        if (count(mid) <= R * B) hi = mid; else lo = mid;
      }
      gcap[g] = hi;
    }
  }
  std::vector<std::vector<TileDesc>> per(P.groups);
  if (segs) segs->clear();
  if (segbase) segbase->clear();
  for (int sl = 0; sl < S; ++sl) {
    const int* rp = hp.data() + size_t(sl) * rows;
    const int g = sl % P.groups;
    // sorted tiles gather relative to their slice's first column (slice_bounds)
    const int base = sorted ? int((P.cols * sl) / S) : 0;
    auto seg = [&](int c) {
      if (segs) segs->push_back(c);
      if (segbase) segbase->push_back(base);
    };
    walk(sl, gcap[g], [&](int lng, int r0, int r1) {
      per[g].push_back(TileDesc{sl, lng, r0, r1, rp[r0], rp[r1], base, 0});
      if (!sorted) return;
      if (lng) {
        for (int c = rp[r0]; c < rp[r1]; c += sort_tile) seg(c);
      } else if (rp[r1] > rp[r0]) {
        seg(rp[r0]);
      }
    });
  }
  if (segs) segs->push_back(hp[nptr - 1]);
  std::vector<TileDesc> all;
  std::vector<int> beg(P.groups + 1, 0), mid(P.groups, 0);
  int maxg = 0;
  for (int g = 0; g < P.groups; ++g) {
    beg[g] = int(all.size());
    // sorted tiles: ordinary tiles first, single long rows after tmid[g]
    if (sorted)
      std::stable_partition(per[g].begin(), per[g].end(), [](const TileDesc& d) { return d.long_row == 0; });
    int nshort = 0;
    for (const TileDesc& d : per[g]) nshort += d.long_row == 0;
    mid[g] = beg[g] + nshort;
    all.insert(all.end(), per[g].begin(), per[g].end());
    maxg = std::max<int>(maxg, int(per[g].size()));
  }
  beg[P.groups] = int(all.size());
  if (sorted) {
    HIPCHK(hipMalloc(&P.tmid, sizeof(int) * mid.size()));
    P.owned += sizeof(int) * mid.size();
    HIPCHK(hipMemcpyAsync(P.tmid, mid.data(), sizeof(int) * mid.size(), hipMemcpyHostToDevice, s));
  }
  P.ntiles = int(all.size());
  HIPCHK(hipMalloc(&P.tiles, sizeof(TileDesc) * std::max<size_t>(all.size(), 1)));
  HIPCHK(hipMalloc(&P.tbeg, sizeof(int) * beg.size()));
  P.owned += sizeof(TileDesc) * std::max<size_t>(all.size(), 1) + sizeof(int) * beg.size();
  if (!all.empty())
    HIPCHK(hipMemcpyAsync(P.tiles, all.data(), sizeof(TileDesc) * all.size(), hipMemcpyHostToDevice, s));
  HIPCHK(hipMemcpyAsync(P.tbeg, beg.data(), sizeof(int) * beg.size(), hipMemcpyHostToDevice, s));
  HIPCHK(hipStreamSynchronize(s));
  const int units = (maxg + per_block - 1) / per_block;
  if (P.groups > 1)
    P.grid = P.groups * std::max(1, std::min(units, per_group));
  else
    P.grid = std::max(1, std::min((P.ntiles + per_block - 1) / per_block, max_grid));
  P.combine_grid = combine_grid(rows);
  return KRCN_OK;
}

// Store the pass's nonzeros sorted by gather index inside every sort segment
// (stable: ties keep CSR order), with their slot in the segment.
template <typename T>
static krcn_status build_sorted(PassPlan& P, const std::vector<int>& segs, const std::vector<int>& segbase,
                               hipStream_t s) {
  const int64_t nnz = P.nnz;
  const int nseg = int(segs.size()) - 1;
  HIPCHK(hipMalloc(&P.gword, sizeof(unsigned) * std::max<int64_t>(nnz, 1)));
  HIPCHK(hipMalloc(&P.gval, sizeof(T) * std::max<int64_t>(nnz, 1)));
  P.owned += (sizeof(unsigned) + sizeof(T)) * size_t(std::max<int64_t>(nnz, 1));
  if (nnz == 0 || nseg <= 0) return KRCN_OK;
  int *dsegs = nullptr, *dbase = nullptr, *iota = nullptr, *perm = nullptr;
  unsigned long long *key = nullptr, *skey = nullptr;
  HIPCHK(hipMalloc(&dsegs, sizeof(int) * segs.size()));
  HIPCHK(hipMemcpyAsync(dsegs, segs.data(), sizeof(int) * segs.size(), hipMemcpyHostToDevice, s));
  HIPCHK(hipMalloc(&dbase, sizeof(int) * segbase.size()));
  HIPCHK(hipMemcpyAsync(dbase, segbase.data(), sizeof(int) * segbase.size(), hipMemcpyHostToDevice, s));
  HIPCHK(hipMalloc(&key, sizeof(unsigned long long) * nnz));
  HIPCHK(hipMalloc(&skey, sizeof(unsigned long long) * nnz));
  HIPCHK(hipMalloc(&iota, sizeof(int) * nnz));
  HIPCHK(hipMalloc(&perm, sizeof(int) * nnz));
  hipLaunchKernelGGL(k_seg_keys, dim3(std::min(nseg, 65535)), dim3(kNT), 0, s, nseg, dsegs, P.idx, key);
  LAUNCHCHK();
  hipLaunchKernelGGL(k_iota, dim3(vec_grid(nnz)), dim3(kNT), 0, s, nnz, iota);
  LAUNCHCHK();
  int sbits = 1;
  while ((int64_t(1) << sbits) < nseg) ++sbits;
  int slot_bits = 0;
  while ((1 << slot_bits) < P.sort_nt * kSortPerThread) ++slot_bits;
  size_t tmpb = 0;
  HIPCHK(hipcub::DeviceRadixSort::SortPairs(nullptr, tmpb, key, skey, iota, perm, int(nnz), 0, 32 + sbits, s));
  void* tmp = nullptr;
  HIPCHK(hipMalloc(&tmp, tmpb));
  HIPCHK(hipcub::DeviceRadixSort::SortPairs(tmp, tmpb, key, skey, iota, perm, int(nnz), 0, 32 + sbits, s));
  hipLaunchKernelGGL((k_sorted_gather<T>), dim3(vec_grid(nnz)), dim3(kNT), 0, s, nnz, perm, skey, dsegs, dbase,
                     static_cast<const T*>(P.val), slot_bits, P.gword, static_cast<T*>(P.gval));
  LAUNCHCHK();
  HIPCHK(hipStreamSynchronize(s));
  void* frees[] = {tmp, dsegs, dbase, key, skey, iota, perm};
  for (void* f : frees) HIPCHK(hipFree(f));
  // the sorted arrays replace the slice copies (the row pointers stay)
  if (P.own_idx) { HIPCHK(hipFree(P.own_idx)); P.own_idx = nullptr; }
  if (P.own_val) { HIPCHK(hipFree(P.own_val)); P.own_val = nullptr; }
  P.idx = nullptr;
  P.val = nullptr;
  return KRCN_OK;
}

// Sorted tiles pay when the gathered window per slice is dense enough for a
// 2 K-nonzero tile to put several lanes on one cache line: at most
// kSortWindow entries per slice, and the slice partials (S x rows, written
// and re-read) cheap next to the matrix stream.
static constexpr int64_t kSortWindowDefault = 24576;

static int64_t sort_window() {
  static const int64_t w = [] {
    const char* e = tuning_env("KRCN_SORT_WINDOW");   // tuning knob
    const long long v = e ? atoll(e) : 0;
    return v >= 1024 ? int64_t(v) : kSortWindowDefault;
  }();
  return w;
}

static int sorted_slices(int64_t cols) {
  const int64_t kSortWindow = sort_window();
  if (cols <= kSortWindow) return 1;
  const int64_t per8 = 8 * kSortWindow;
  return int(8 * ((cols + per8 - 1) / per8));
}

// ------------------------------------------------------ LDS-window plans
// (krcn_window.hpp.)  Slices of W columns, 16-bit slice-local offsets, tiles
// of R rows, and per-block segment lists.
//   accum:  S = ceil(cols / Wmax) slices of equal width; blocks own contiguous
//           tile ranges of equal nonzero count and walk every slice over them
//           (row sums carry across slices: no partials).
//   slices: S = the smallest divisor of 256 >= ceil(cols / Wmax) (or, past
//           256, a multiple of 8), k = 256 / S blocks per slice, each owning a
//           nonzero-balanced row range of it; block s + S c holds chunk c of
//           slice s, so a slice's blocks share an XCD (b % 8) and its window
//           is fetched from HBM once per XCD.  Per-slice partial row sums,
//           combined in slice order by k_slice_combine.
static constexpr int kWinTileCost = 24;   // fixed per-tile work, in nonzero equivalents

template <typename T>
static int64_t win_width() { return WinGeom<T>::kW; }

static int win_slices_mode(int64_t cols, int64_t Wmax, int* k_out) {
  const int64_t smin = (cols + Wmax - 1) / Wmax;
  static const int k_env = [] {   // A/B knob: blocks per slice (S = 256 / k slices, e.g. k = 3: 85)
    const char* e = tuning_env("KRCN_WIN_KPB");
    return e ? atoi(e) : 0;
  }();
  if (k_env >= 2 && k_env <= 8 && kNumCUs / k_env >= smin) {
    *k_out = k_env;
    return kNumCUs / k_env;
  }
  // 65-85 slices needed (news20: 83): 85 slices x 3 blocks (255 blocks,
  // XCD-packed, win_block_slice) instead of 128 x 2 — a third fewer slice
  // partials (20.5 -> 13.6 MB written and re-read per pass on news20) for a
  // 50 % larger window per block; interleaved on one box 16.6-17.3 k against
  // 16.5-17.1 k HVP/s, the combine 6.6-6.8 us against 7.7-7.8
  // (profiles/r05h_news20_kpb_ab.txt; KRCN_WIN_KPB=2 restores 128 x 2)
  if (k_env == 0 && smin > kNumCUs / 4 && smin <= kNumCUs / 3) {
    *k_out = 3;
    return kNumCUs / 3;
  }
  static const int s_env = [] {   // A/B knob: minimum slice count (a power of two)
    const char* e = tuning_env("KRCN_WIN_MIN_SLICES");
    return e ? atoi(e) : 0;
  }();
  for (int S = 8; S <= kNumCUs; S *= 2)
    if (S >= smin && S >= s_env) { *k_out = kNumCUs / S; return S; }
  for (int S = 8; S <= kNumCUs; S *= 2)
    if (S >= smin) { *k_out = kNumCUs / S; return S; }
  *k_out = 1;
  return int(8 * ((smin + 7) / 8));
}

// A/B knob KRCN_PLAN_RELOC (placement): 1 moves a plan's element
// arrays into physically contiguous allocations (hipDeviceMallocContiguous),
// 2 into fresh plain allocations made after the build's temporaries are gone.
static int plan_reloc_env() {
  static const int v = [] {
    const char* e = tuning_env("KRCN_PLAN_RELOC");
    return e ? atoi(e) : 0;
  }();
  return v;
}

static krcn_status plan_reloc(void** p, size_t bytes, hipStream_t s) {
  const int mode = plan_reloc_env();
  if (mode == 0 || !*p || bytes == 0) return KRCN_OK;
  void* q = nullptr;
  if (mode == 1) HIPCHK(hipExtMallocWithFlags(&q, bytes, hipDeviceMallocContiguous));
  else HIPCHK(hipMalloc(&q, bytes));
  HIPCHK(hipMemcpyAsync(q, *p, bytes, hipMemcpyDeviceToDevice, s));
  HIPCHK(hipStreamSynchronize(s));
  HIPCHK(hipFree(*p));
  *p = q;
  return KRCN_OK;
}

// 0: no window format, 1: accumulate, 2: slices (auto policy).
static double slice_min_mat() {   // matrix bytes below which slices + combine do not pay
  static const double v = [] {
    const char* e = tuning_env("KRCN_SLICE_MIN_MB");   // A/B knob
    return e ? atof(e) * 1e6 : 48e6;
  }();
  return v;
}
static int window_choice(int rows, int64_t cols, int64_t nnz, size_t vs) {
  if (nnz == 0 || rows == 0 || cols == 0) return 0;
  const int64_t Wmax = vs == 8 ? win_width<double>() : win_width<float>();
  const int64_t S = (cols + Wmax - 1) / Wmax;
  const double mean = double(nnz) / (double(rows) * double(S));   // nonzeros per row and slice
  if (mean > 24.0) return 0;                 // one lane per row: short rows only
  const double mat = double(nnz) * double(vs + 2);
  const double win = double(std::min<int64_t>(cols, Wmax)) * double(vs);
  if (S <= 4 && double(kNumCUs) * double(S) * win <= mat) return 1;
  int k = 1;
  const int Ss = win_slices_mode(cols, Wmax, &k);
  const double part = 2.0 * double(Ss) * double(rows) * double(vs);
  const double wbytes = double(Ss) * double(k) * double((cols + Ss - 1) / Ss) * double(vs);
  // partials (written once, read once by the combine) up to 1.25x the matrix
  // bytes still pay against cache-served gathers: synth 2M x 1M (100 nnz per
  // row, part / mat = 1.02) HVP 2,753 -> 2,173 us against the wave format
  // and the combine launch (≈5 us of latency) must be small next to the pass:
  // rcv1's X^T (15 MB) ran 34.9 us per HVP with window slices + combine
  // against 29.6 us with unsliced sorted tiles (tools/lz_fmt.py)
  if (Ss > 1 && part <= 1.25 * mat && wbytes <= 0.6 * mat && mat >= slice_min_mat()) return 2;
  return 0;
}

// One-piece window-accum plans (d <= kWinNT): each block's rows once more as a
// column-major copy, so the fused Lanczos pass 1 also forms the block's share
// of X^T u (EpiLz1X, krcn_window.hpp).  Every column's run (rows ascending) is
// padded to whole chunks of kXtChunk (value 0, row kXtPad); xcp holds per
// block the cols + 1 absolute chunk ids.  Skipped (P.xt = 0) when a block's
// chunk sums do not fit the LDS past the window and its rows.
template <typename T>
static krcn_status build_xt(PassPlan& P, const std::vector<int>& hp, const std::vector<int>& cut, int B,
                            hipStream_t s) {
  const int rows = P.rows, R = P.R, cols = int(P.cols);
  const int64_t nnz = P.nnz;
  std::vector<unsigned short> hidx(size_t(std::max<int64_t>(nnz, 1)));
  std::vector<T> hval(size_t(std::max<int64_t>(nnz, 1)));
  if (nnz > 0) {
    HIPCHK(hipMemcpy(hidx.data(), P.widx, sizeof(unsigned short) * size_t(nnz), hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(hval.data(), P.val, sizeof(T) * size_t(nnz), hipMemcpyDeviceToHost));
  }
  const size_t ncp = size_t(B) * (size_t(cols) + 1);
  std::vector<int> cp(ncp);
  std::vector<int> cnt(static_cast<size_t>(cols));
  int64_t chunks = 0;   // first pass: chunk ids
  for (int b = 0; b < B; ++b) {
    const int r0 = std::min(rows, cut[b] * R), r1 = std::min(rows, cut[b + 1] * R);
    if (r1 - r0 > kXtRowCap) return KRCN_OK;
    std::fill(cnt.begin(), cnt.end(), 0);
    for (int e = hp[r0]; e < hp[r1]; ++e) ++cnt[hidx[size_t(e)]];
    int* bcp = cp.data() + size_t(b) * (size_t(cols) + 1);
    const int64_t c0 = chunks;
    for (int c = 0; c < cols; ++c) {
      bcp[c] = int(chunks);
      chunks += (cnt[size_t(c)] + kXtChunk - 1) / kXtChunk;
    }
    bcp[cols] = int(chunks);
    if (chunks - c0 > XtGeom<T>::kChunks) return KRCN_OK;
    if (chunks * kXtChunk >= (int64_t(1) << 31)) return KRCN_OK;
  }
  std::vector<unsigned short> xr(size_t(chunks) * kXtChunk, kXtPad);
  std::vector<T> xv(size_t(chunks) * kXtChunk, T(0));
  std::vector<int64_t> pos(static_cast<size_t>(cols));
  for (int b = 0; b < B; ++b) {   // second pass: rows in order, so each column's run stays in row order
    const int r0 = std::min(rows, cut[b] * R), r1 = std::min(rows, cut[b + 1] * R);
    const int* bcp = cp.data() + size_t(b) * (size_t(cols) + 1);
    for (int c = 0; c < cols; ++c) pos[size_t(c)] = int64_t(bcp[c]) * kXtChunk;
    for (int r = r0; r < r1; ++r)
      for (int e = hp[r]; e < hp[r + 1]; ++e) {
        const int64_t k = pos[hidx[size_t(e)]]++;
        xr[size_t(k)] = static_cast<unsigned short>(r - r0);
        xv[size_t(k)] = hval[size_t(e)];
      }
  }
  const size_t ne = std::max<size_t>(xr.size(), kXtChunk);
  xr.resize(ne, kXtPad);
  xv.resize(ne, T(0));
  HIPCHK(hipMalloc(&P.xcp, sizeof(int) * ncp));
  HIPCHK(hipMalloc(&P.xrow, sizeof(unsigned short) * ne));
  HIPCHK(hipMalloc(&P.xval, sizeof(T) * ne));
  HIPCHK(hipMalloc(&P.xpart, sizeof(T) * size_t(B) * size_t(cols)));
  P.owned += sizeof(int) * ncp + (sizeof(unsigned short) + sizeof(T)) * ne + sizeof(T) * size_t(B) * size_t(cols);
  HIPCHK(hipMemcpyAsync(P.xcp, cp.data(), sizeof(int) * ncp, hipMemcpyHostToDevice, s));
  HIPCHK(hipMemcpyAsync(P.xrow, xr.data(), sizeof(unsigned short) * ne, hipMemcpyHostToDevice, s));
  HIPCHK(hipMemcpyAsync(P.xval, xv.data(), sizeof(T) * ne, hipMemcpyHostToDevice, s));
  HIPCHK(hipStreamSynchronize(s));
  P.xt = 1;
  return KRCN_OK;
}

template <typename T>
static krcn_status build_window(PassPlan& P, const int* ptr, const int* idx, const T* val, int accum,
                                hipStream_t s) {
  const int64_t Wmax = WinGeom<T>::kW;
  const int rows = P.rows;
  const int64_t cols = P.cols, nnz = P.nnz;
  int S = 1, kpb = 1;
  if (accum) {
    S = int((cols + Wmax - 1) / Wmax);
  } else {
    S = win_slices_mode(cols, Wmax, &kpb);
  }
  const int W = int((cols + S - 1) / S);
  P.S = S;
  P.W = W;
  P.win = 1;
  P.accum = accum;
  P.L = 1;
  P.groups = 1;
  std::vector<int> hb(S + 1);
  for (int k = 0; k <= S; ++k) hb[k] = int(std::min<int64_t>(int64_t(k) * W, cols));
  CHK(build_slices<T>(P, ptr, idx, val, s, &hb, kWinPad));
  HIPCHK(hipMalloc(&P.widx, sizeof(unsigned short) * size_t(nnz + kWinPad)));
  P.owned += sizeof(unsigned short) * size_t(nnz + kWinPad);
  HIPCHK(hipMemsetAsync(P.widx, 0, sizeof(unsigned short) * size_t(nnz + kWinPad), s));
  if (nnz > 0) {
    hipLaunchKernelGGL(k_local_u16, dim3(vec_grid(nnz)), dim3(kNT), 0, s, nnz, P.own_idx, W, P.widx);
    LAUNCHCHK();
  }
  HIPCHK(hipStreamSynchronize(s));
  HIPCHK(hipFree(P.own_idx));
  P.owned -= sizeof(int) * size_t(std::max<int64_t>(nnz, 1));
  P.own_idx = nullptr;
  P.idx = nullptr;
  const size_t nptr = size_t(S) * rows + 1;
  std::vector<int> hp(nptr);
  HIPCHK(hipMemcpy(hp.data(), P.ptr, sizeof(int) * nptr, hipMemcpyDeviceToHost));
  // rows per tile: up to one staging chunk of nonzeros per tile and slice.
  // The tile stream is latency-bound (a wave keeps two tiles' chunks in
  // flight), so the tiles are taken as large as a chunk allows: news20's X
  // (3.55 nonzeros per row and slice, 227 per 64-row tile) ran its fused
  // pass 1 in 32.5 us with 64-row tiles against 38.0 us with 32-row tiles
  // (profiles/r03_news20_winR.txt); the few tiles past 256 take one extra chunk.
  const double mean = double(nnz) / (double(rows) * double(S));
  P.R = mean * 64.0 <= 0.95 * kWinChunk ? 64 : mean * 32.0 <= 0.95 * kWinChunk ? 32 : 16;
  if (const char* e = tuning_env("KRCN_WIN_R")) {   // A/B knob: rows per tile (16 / 32 / 64)
    const int r = atoi(e);
    if (r == 16 || r == 32 || r == 64) P.R = r;
  }
  const int R = P.R;
  const int ntiles = (rows + R - 1) / R;
  auto tnnz = [&](int sl, int t) -> int64_t {
    const int* rp = hp.data() + size_t(sl) * rows;
    const int r0 = t * R, r1 = std::min(rows, r0 + R);
    return int64_t(rp[r1]) - rp[r0];
  };
  // compact row pointers (16-bit row ends inside a tile): every tile of every
  // slice must hold < 65536 nonzeros, else the format does not apply
  for (int sl = 0; sl < S; ++sl)
    for (int t = 0; t < ntiles; ++t)
      if (tnnz(sl, t) > 65535) return fail(KRCN_ERR_UNSUPPORTED, "window plan: a tile holds > 65535 nonzeros");
  {
    void* wi = P.widx;
    CHK(plan_reloc(&wi, sizeof(unsigned short) * size_t(nnz + kWinPad), s));
    P.widx = static_cast<unsigned short*>(wi);
    void* wv = P.own_val;
    CHK(plan_reloc(&wv, sizeof(T) * size_t(std::max<int64_t>(nnz, 1) + kWinPad), s));
    P.own_val = wv;
    P.val = wv;
  }
  HIPCHK(hipMalloc(&P.tb, sizeof(int) * size_t(S) * (ntiles + 1)));
  HIPCHK(hipMalloc(&P.ro, sizeof(unsigned short) * std::max<size_t>(size_t(S) * rows, 1)));
  P.owned += sizeof(int) * size_t(S) * (ntiles + 1) + sizeof(unsigned short) * size_t(S) * rows;
  hipLaunchKernelGGL(k_compact_rows, dim3(vec_grid(int64_t(S) * rows)), dim3(kNT), 0, s, S, rows, R, ntiles, P.ptr,
                     P.tb, P.ro);
  LAUNCHCHK();
  HIPCHK(hipStreamSynchronize(s));
  // the kernels read the compact form only
  HIPCHK(hipFree(P.own_ptr));
  P.owned -= sizeof(int) * nptr;
  P.own_ptr = nullptr;
  P.ptr = nullptr;
  // cut [0, ntiles) into B ranges of equal cost(t) (prefix-sum cuts)
  auto cut_ranges = [&](int B, auto&& cost) {
    std::vector<int64_t> pre(ntiles + 1, 0);
    for (int t = 0; t < ntiles; ++t) pre[t + 1] = pre[t] + cost(t);
    std::vector<int> cut(B + 1, 0);
    int t = 0;
    for (int b = 1; b < B; ++b) {
      const int64_t target = (pre[ntiles] * b) / B;
      while (t < ntiles && pre[t] < target) ++t;
      cut[b] = t;
    }
    cut[B] = ntiles;
    return cut;
  };
  std::vector<WinSeg> segs;
  if (accum) {
    auto cost = [&](int t) {
      int64_t c = kWinTileCost * int64_t(S);
      for (int sl = 0; sl < S; ++sl) c += tnnz(sl, t);
      return c;
    };
    const int cap = kWinWaves * kWinTMax;   // tiles per block (register sums)
    int B = kNumCUs;
    if (const char* e = tuning_env("KRCN_WIN_ACC_B")) B = std::max(1, atoi(e));   // A/B knob: first grid tried
    std::vector<int> cut;
    for (;;) {
      cut = cut_ranges(B, cost);
      int mx = 0;
      for (int b = 0; b < B; ++b) mx = std::max(mx, cut[b + 1] - cut[b]);
      if (mx <= cap || B >= 64 * kNumCUs) break;
      B += kNumCUs;
    }
    P.stride = S;
    segs.assign(size_t(B) * S, WinSeg{0, 0, 0, 0});
    for (int b = 0; b < B; ++b) {
      if (cut[b + 1] == cut[b]) continue;      // an empty block: segment count 0
      for (int sl = 0; sl < S; ++sl)
        segs[size_t(b) * S + sl] =
            WinSeg{sl, cut[b], cut[b + 1], kSegLoad | (sl == S - 1 ? kSegFlush : 0) | (sl == 0 ? S << 8 : 0)};
    }
    P.grid = B;
    if (S == 1 && cols <= kWinNT) CHK(build_xt<T>(P, hp, cut, B, s));
  } else {
    P.stride = 1;
    P.grid = S * kpb;
    P.kpb = (kpb & (kpb - 1)) != 0 ? kpb : 0;   // win_block_slice's mapping
    // a block whose row chunk is empty still names its slice (no segments to
    // run): the fused Lanczos prologue has it store its share of that slice
    std::vector<std::vector<int>> cuts(static_cast<size_t>(S));
    for (int sl = 0; sl < S; ++sl)
      cuts[size_t(sl)] = cut_ranges(kpb, [&](int t) { return tnnz(sl, t) + kWinTileCost; });
    segs.resize(size_t(S) * kpb);
    for (int b = 0; b < P.grid; ++b) {
      int sl = 0, c = 0;
      win_block_slice(b, P.grid, S, P.kpb, sl, c);
      const std::vector<int>& cut = cuts[size_t(sl)];
      segs[size_t(b)] = cut[c + 1] > cut[c] ? WinSeg{sl, cut[c], cut[c + 1], kSegLoad | kSegFlush | (1 << 8)}
                                           : WinSeg{sl, 0, 0, 0};
    }
    HIPCHK(hipMalloc(&P.part, sizeof(T) * size_t(S) * std::max(rows, 1)));
    P.owned += sizeof(T) * size_t(S) * std::max(rows, 1);
    P.combine_grid = combine_grid(rows);
  }
  P.nseg = int(segs.size());
  P.ntiles = ntiles;
  HIPCHK(hipMalloc(&P.segs, sizeof(WinSeg) * std::max<size_t>(segs.size(), 1)));
  P.owned += sizeof(WinSeg) * std::max<size_t>(segs.size(), 1);
  if (!segs.empty())
    HIPCHK(hipMemcpy(P.segs, segs.data(), sizeof(WinSeg) * segs.size(), hipMemcpyHostToDevice));
  return KRCN_OK;
}

// ------------------------------------------------------ jagged plans
// (krcn_jag.hpp.)  S = 1 when the gathered vector fits one LDS window (fp64:
// 20,448 entries), else S slices of W <= 10,224 entries that every block
// walks over its own rows (double-buffered windows, register row sums).
static constexpr int kJagGroupCost = 96;   // fixed work per group and slice, in nonzero equivalents

// KRCN_JAG (A/B knob): 0 never by the auto policy, 1 the cost model (default),
// 2 every pass the format can run
static int jag_env() {
  static const int v = [] {
    const char* e = tuning_env("KRCN_JAG");
    return e ? atoi(e) : 1;
  }();
  return v;
}

template <typename T>
static int jag_slices(int64_t cols, int* W_out) {
  constexpr int kE = JagGeom<T>::kE;
  if (cols <= JagGeom<T>::kW1) {
    *W_out = int(cols);
    return 1;
  }
  const int64_t s0 = (cols + JagGeom<T>::kW2 - 1) / JagGeom<T>::kW2;
  int64_t W = (cols + s0 - 1) / s0;
  W = (W + kE - 1) / kE * kE;   // slice bases stay 16-byte aligned
  *W_out = int(W);
  return int((cols + W - 1) / W);
}

// Accumulate mode, slice groups: with G groups, block b walks the S / G
// slices of group b % G over row range b / G (256 / G ranges) and writes
// per-group partial row sums that k_slice_combine adds in group order.  More
// groups give each block fewer slices and more row groups per wave (K, at
// most 8).  Per-block time model, fitted on the synth passes at HEAD (round 3:
// pass 1 S = 109, K = 8: 485 us; pass 2 S = 218, K = 4: 608 us; pass 2 at
// G = 2, S = 109 a block, K = 8: 486-502 us with its combine): every slice
// costs ~1.13 us (window pieces, lane counts, the barrier) plus ~0.415 us per
// unit a wave carries.  G > 1 adds the group partials (written and read once)
// and a combine launch (~8 us); it changes the summation order (no longer
// scipy's), so it is taken only when the model gains 10 % or more.
template <typename T>
static int jag_groups(int rows, int64_t cols, int64_t nnz, int S, int pass) {
  const double vs = double(sizeof(T));
  const int64_t groups = (int64_t(rows) + 63) / 64;
  constexpr double kSliceUs = 1.13, kUnitUs = 0.415, kCombineUs = 8.0, kPartBps = 5e12;
  int best = 0;
  double bc = 1e300;
  for (int G = 1; G <= 8 && G <= S; G *= 2) {
    const int R = std::max(1, kNumCUs / G);
    const int64_t per_block = (groups + R - 1) / R;
    const int64_t K = (per_block + kJagWaves - 1) / kJagWaves;
    if (K > kJagK2) continue;
    const double slices = double((S + G - 1) / G);
    double c = slices * (kSliceUs + double(std::max<int64_t>(K, 1)) * kUnitUs);
    if (G > 1) c = (c + 2.0 * G * double(rows) * vs / kPartBps * 1e6 + kCombineUs) / 0.9;
    if (c < bc) {
      bc = c;
      best = G;
    }
  }
  // An X^T pass whose window (the whole gathered vector, walked by every
  // block) outweighs a block's share of the matrix by more than half takes
  // two groups even where the model keeps one: the synth rank-of-8 pass 2
  // (250 K-entry u = 2 MB a block against 1 MB of matrix) ran 97.8-98.4 ->
  // 93.4-93.6 us per step with G = 2 (1 MB of window a block), 5,428-5,443 ->
  // 5,615-5,621 HVP/s (round 6, profiles/r06w_synth8_pass2_groups.txt;
  // a layout whose window bytes do not exceed its matrix
  // bytes).
  if (best == 1 && pass == 2 && S >= 2 && nnz >= (int64_t(1) << 23)) {   // (heavy passes only: >= 8 M nonzeros)
    const double win = double(cols) * vs, mat = double(nnz) * (vs + 2.0) / double(kNumCUs);
    const int64_t K2 = ((groups + kNumCUs / 2 - 1) / (kNumCUs / 2) + kJagWaves - 1) / kJagWaves;
    if (win > 1.5 * mat && K2 <= kJagK2) best = 2;
  }
  return best;
}

// Auto policy: enough row groups to give every wave work, short rows per
// slice (one lane per row), and — with several slices — a block's share of
// the matrix not small next to the windows it loads (L2/MALL-served).
// Single-window X^T passes (pass 2: the gathered u fits one LDS window) need
// only a row group per CU: rcv1's X^T (738 groups) ran 13.2 -> 10.5 us a pass
// on 123 blocks against the sorted tiles (interleaved, profiles/r03_rcv1_jag_ab.txt).
// Pass 1 keeps the full bar: a one-piece X z (w8a) keeps its fused step B.
static constexpr int kJagS1MinGroupsXt = kNumCUs;
static constexpr int kJagS1GroupsPerBlock = 6;   // below a group per wave: blocks of >= 6 groups
template <typename T>
static bool jag_choice(int rows, int64_t cols, int64_t nnz, int pass) {
  const int mode = jag_env();
  if (mode == 0 || nnz == 0 || rows == 0 || cols < 16) return false;
  const int64_t G = (int64_t(rows) + 63) / 64;
  int W = 0;
  const int S = jag_slices<T>(cols, &W);
  const double mean = double(nnz) / double(rows) / double(S);   // elements per row and slice
  if (S == 1) {
    // A/B knob: KRCN_JAG_S1G=g sets the row groups a single-window plan needs
    static const int64_t genv = [] {
      const char* e = tuning_env("KRCN_JAG_S1G");
      return e ? int64_t(atoi(e)) : int64_t(0);
    }();
    const bool relaxed = pass == 2 && sizeof(T) == 8;   // (fp32 rcv1 stress: 10.4 -> 14.7 us, kept off)
    const int64_t gmin = genv > 0 ? genv : relaxed ? int64_t(kJagS1MinGroupsXt) : int64_t(kNumCUs) * kJagWaves;
    return G >= gmin && mean <= 48.0;
  }
  if (G < int64_t(kNumCUs) * 4) return false;   // accumulate: >= 4 groups a block
  if (mean > 1.5) return false;   // a 64-row group's slice must fit the 128-entry products slab
  const int sg = jag_groups<T>(rows, cols, nnz, S, pass);
  if (sg == 0) return false;
  if (mode == 2) return true;
  const double mat = double(nnz) * double(sizeof(T) + 2) / double(kNumCUs);
  const double win = double(cols) * double(sizeof(T)) / sg;
  return mat >= 0.25 * win;
}

template <typename T>
static krcn_status build_jag(PassPlan& P, const int* ptr, const int* idx, const T* val, int pass, bool seq,
                             hipStream_t s) {
  const int rows = P.rows;
  const int64_t cols = P.cols, nnz = P.nnz;
  if (cols < JagGeom<T>::kE || rows == 0 || nnz == 0)
    return fail(KRCN_ERR_UNSUPPORTED, "jag plan: empty or too narrow (%lld columns)", (long long)cols);
  int W = 0;
  const int S = jag_slices<T>(cols, &W);
  const int Kmax = S == 1 ? kJagK1 : kJagK2;
  const int G = (rows + 63) / 64;
  // A/B knob: force the slice-group count of accumulate plans, KRCN_JAG_G=g
  // (both passes) or g1,g2 (pass 1 / pass 2; 0 keeps the cost model's)
  static const std::pair<int, int> g_env = [] {
    const char* e = tuning_env("KRCN_JAG_G");
    int a = 0, b = 0;
    if (e && std::sscanf(e, "%d,%d", &a, &b) == 1) b = a;
    return std::make_pair(a, b);
  }();
  const int gf = pass == 1 ? g_env.first : g_env.second;
  // slice groups (their partials change the summation order: never under the
  // sequential lane policy, whose contract is scipy's order bit for bit)
  int SG = S == 1 || seq ? 1 : (gf > 0 ? std::min(gf, S) : jag_groups<T>(rows, cols, nnz, S, pass));
  if (SG == 0) SG = 1;                                       // (forced format: block count grows instead)
  const int Sg = (S + SG - 1) / SG;                          // slices per group
  std::vector<int> hp(size_t(rows) + 1);
  HIPCHK(hipMemcpy(hp.data(), ptr, sizeof(int) * (size_t(rows) + 1), hipMemcpyDeviceToHost));
  // single window: rows longer than kJagLong are summed apart by whole waves
  // (jag_long_rows) when their task partials fit the LDS past the window.
  // Their wave-tree order is not scipy's, so the sequential lane policy keeps
  // such rows lane-per-row (a row over 255 elements then refuses the plan)
  std::vector<int> lrows;
  const int lpiece = int((cols * int64_t(sizeof(T)) + 15) / 16);
  // task partials a block can keep in the LDS past the window (round 6: a
  // window within 256 tasks' partials of the LDS — rcv1's 20,242-entry u —
  // used to refuse the plan, and a skewed rcv1 X^T then ran sorted tiles at
  // 318 us a pass; a block now takes at most as many tasks as fit)
  const int tcap = std::min<int64_t>(kJagLongTasks, int64_t(kJagPieces - lpiece) * 16 / int64_t(sizeof(T)));
  // which rows go long: past kJagLong when the window leaves room for all 256
  // task partials (round 5's rule: news20's X^T); with less room only when some
  // row is longer than the 8-bit lane counts hold (> 254, since a count byte
  // of 0xFF marks a long row: a skewed rcv1's hot columns) —
  // sending a uniform rcv1's 33-60-element X^T rows to 128-element tasks cost
  // its pass 2 11.2 -> 17.5 us (profiles/r06t_bench_rcv1.json)
  int lthr = 0;
  if (S == 1 && !seq && tcap >= kJagWaves) {
    if (lpiece + kJagLongTasks * int(sizeof(T)) / 16 <= kJagPieces) {
      lthr = kJagLong;
    } else {
      // (the rows past 32 then go long too: a skewed rcv1 ran 24.6 k HVP/s so,
      // 19.7 k with only the rows past 254 long, r06t / r06t2)
      for (int r = 0; r < rows && lthr == 0; ++r)
        if (hp[r + 1] - hp[r] > 254) lthr = kJagLong;
    }
  }
  {
    // A/B knob KRCN_JAG_LONG=t: rows past t elements go long (8..254)
    static const int long_env = [] {
      const char* e = tuning_env("KRCN_JAG_LONG");
      return e ? atoi(e) : 0;
    }();
    if (lthr > 0 && long_env >= 8 && long_env <= 254) lthr = long_env;
  }
  if (lthr > 0)
    for (int r = 0; r < rows; ++r)
      if (hp[r + 1] - hp[r] > lthr) lrows.push_back(r);
  std::vector<char> is_long(lrows.empty() ? 0 : size_t(rows), 0);
  for (int r : lrows) is_long[size_t(r)] = 1;
  std::vector<int64_t> pre(size_t(G) + 1, 0);
  for (int g = 0; g < G; ++g) {
    int64_t e = int64_t(hp[std::min(rows, 64 * (g + 1))]) - hp[64 * g];
    if (!lrows.empty())
      for (int r = 64 * g; r < std::min(rows, 64 * (g + 1)); ++r)
        if (is_long[size_t(r)]) e -= hp[r + 1] - hp[r];
    pre[g + 1] = pre[g] + e + int64_t(kJagGroupCost) * S;
  }
  // nonzero-balanced row ranges of at most 16 K groups (K per wave); the
  // grid is R ranges x SG slice groups
  const int Rstep = std::max(1, kNumCUs / SG);
  int R = std::min(G, Rstep), mx = 0;
  if (S == 1) {
    // fewer groups than waves: blocks of >= kJagS1GroupsPerBlock groups, so
    // fewer blocks load the whole window (A/B knob: KRCN_JAG_R=r caps them)
    static const int rcap = [] {
      const char* e = tuning_env("KRCN_JAG_R");
      return e ? atoi(e) : 0;
    }();
    if (G < kNumCUs * kJagWaves) R = std::max(1, std::min(R, G / kJagS1GroupsPerBlock));
    if (rcap > 0) R = std::min(R, rcap);
  }
  std::vector<int> cut;
  for (;;) {
    cut.assign(size_t(R) + 1, 0);
    int g = 0;
    for (int b = 1; b < R; ++b) {
      const int64_t target = pre[G] * b / R;
      while (g < G && pre[g] < target) ++g;
      cut[b] = g;
    }
    cut[R] = G;
    mx = 0;
    for (int b = 0; b < R; ++b) mx = std::max(mx, cut[b + 1] - cut[b]);
    if (mx <= kJagWaves * Kmax) break;
    if (R * SG >= 64 * kNumCUs) return fail(KRCN_ERR_UNSUPPORTED, "jag plan: %d row groups exceed the block cap", G);
    R += Rstep;
  }
  const int B = R * SG;
  // the smallest unrolled variant the block's groups allow: a wave issues the
  // loads of all K unit slots whether they hold a group or not (a sharded
  // news20 X^T with 21 groups per block ran its jagged pass 2 at rank-of-4 in
  // the same 26 us as at rank-of-2 with K = 6)
  const int K = S == 1 ? (mx <= kJagWaves ? 1 : mx <= 2 * kJagWaves ? 2 : mx <= 3 * kJagWaves ? 3 : kJagK1)
                       : (mx <= kJagWaves * 4 ? 4 : 8);
  std::vector<int> gblk(G);
  for (int b = 0; b < R; ++b)
    for (int g = cut[b]; g < cut[b + 1]; ++g) gblk[g] = b;
  const int64_t NU = int64_t(B) * Sg * K * kJagWaves;   // units
  int ubits = 1;
  while ((int64_t(1) << ubits) <= NU) ++ubits;
  if (ubits + 22 > 63) return fail(KRCN_ERR_UNSUPPORTED, "jag plan: too many units");
  const int64_t nrec = int64_t(B) * Sg * kJagWaves;   // (block, slice, wave) records

  // long rows: tasks of kJagTask elements, rows cut into B contiguous ranges by
  // task count (a block's tasks' partials must fit its tcap LDS slots)
  const int nl = int(lrows.size());
  std::vector<int> ltask, lbeg, lcut, tasks;
  if (nl > 0) {
    ltask.assign(size_t(nl) + 1, 0);
    lbeg.assign(size_t(nl) + 1, 0);
    for (int i = 0; i < nl; ++i) {
      const int len = hp[lrows[i] + 1] - hp[lrows[i]];
      ltask[i + 1] = ltask[i] + (len + kJagTask - 1) / kJagTask;
      lbeg[i + 1] = lbeg[i] + ((len + 1) & ~1);
    }
    const int64_t tt = ltask[nl];
    lcut.assign(2 * (size_t(B) + 1), 0);
    int i = 0;
    for (int bb = 1; bb < B; ++bb) {
      const int64_t target = tt * bb / B;
      while (i < nl && ltask[i] < target) ++i;
      lcut[bb] = i;
    }
    lcut[B] = nl;
    for (int bb = 0; bb <= B; ++bb) lcut[B + 1 + bb] = ltask[lcut[bb]];
    for (int bb = 0; bb < B; ++bb)
      if (lcut[B + 2 + bb] - lcut[B + 1 + bb] > tcap)
        return fail(KRCN_ERR_UNSUPPORTED, "jag plan: a block's long rows need %d tasks (max %d)",
                    lcut[B + 2 + bb] - lcut[B + 1 + bb], tcap);
    tasks.assign(2 * (size_t(tt) + 1), 0);   // one spare entry: the clamped read of an empty block
    for (int k = 0; k < nl; ++k) {
      const int len = hp[lrows[k] + 1] - hp[lrows[k]];
      for (int t = ltask[k]; t < ltask[k + 1]; ++t) {
        const int off = (t - ltask[k]) * kJagTask;
        tasks[2 * size_t(t)] = lbeg[k] + off;
        tasks[2 * size_t(t) + 1] = std::min(kJagTask, len - off);
      }
    }
  }
  HIPCHK(hipMalloc(&P.jgcut, sizeof(int) * (size_t(R) + 1)));
  HIPCHK(hipMalloc(&P.jumeta, sizeof(int) * size_t(nrec) * 2 * K));
  P.owned += sizeof(int) * (size_t(R) + 1) + sizeof(int) * size_t(nrec) * 2 * K;
  HIPCHK(hipMemcpyAsync(P.jgcut, cut.data(), sizeof(int) * (size_t(R) + 1), hipMemcpyHostToDevice, s));
  if (SG > 1) {   // per-group partial row sums
    HIPCHK(hipMalloc(&P.part, sizeof(T) * size_t(SG) * size_t(rows)));
    P.owned += sizeof(T) * size_t(SG) * size_t(rows);
    P.combine_grid = combine_grid(rows);
  }

  int *gblk_d = nullptr, *flags = nullptr, *iota = nullptr, *perm = nullptr, *usize = nullptr, *first = nullptr;
  int* pbase = nullptr;
  unsigned long long *keys = nullptr, *keys_out = nullptr;
  unsigned char* cnt8 = nullptr;
  void* tmp = nullptr;
  auto cleanup = [&]() {
    void* fr[] = {gblk_d, flags, iota, perm, usize, first, pbase, keys, keys_out, cnt8, tmp};
    for (void* f : fr)
      if (f) (void)hipFree(f);
  };
  int hflags[3] = {0, 0, 0};
  // single window: pair-level order, one pad key slot per row after the nonzeros
  const bool pairs = S == 1;
  const int64_t nitems = pairs ? nnz + rows : nnz;
  const unsigned long long sentinel = (1ull << (ubits + 22)) - 1ull;   // unit id >= NU: sorts past every real key
  if (nitems >= (int64_t(1) << 31)) return fail(KRCN_ERR_UNSUPPORTED, "jag plan: too many elements");
  auto body = [&]() -> krcn_status {
    HIPCHK(hipMalloc(&gblk_d, sizeof(int) * size_t(G)));
    HIPCHK(hipMalloc(&flags, 3 * sizeof(int)));
    HIPCHK(hipMalloc(&iota, sizeof(int) * size_t(nitems)));
    HIPCHK(hipMalloc(&perm, sizeof(int) * size_t(nitems)));
    HIPCHK(hipMalloc(&keys, sizeof(unsigned long long) * size_t(nitems)));
    HIPCHK(hipMalloc(&keys_out, sizeof(unsigned long long) * size_t(nitems)));
    HIPCHK(hipMalloc(&cnt8, size_t(NU) * 64));
    HIPCHK(hipMalloc(&usize, sizeof(int) * size_t(NU)));
    HIPCHK(hipMalloc(&first, sizeof(int) * size_t(NU)));
    HIPCHK(hipMemsetAsync(first, 0, sizeof(int) * size_t(NU), s));
    HIPCHK(hipMemsetAsync(usize, 0, sizeof(int) * size_t(NU), s));
    HIPCHK(hipMemcpyAsync(gblk_d, gblk.data(), sizeof(int) * size_t(G), hipMemcpyHostToDevice, s));
    HIPCHK(hipMemsetAsync(flags, 0, 3 * sizeof(int), s));
    HIPCHK(hipMemsetAsync(cnt8, 0, size_t(NU) * 64, s));
    hipLaunchKernelGGL(k_jag_keys, dim3(vec_grid(rows)), dim3(kNT), 0, s, rows, Sg, SG, W, K, pairs ? 0 : 1, nnz,
                       sentinel, nl > 0 ? lthr : 0, ptr, idx, P.jgcut, gblk_d, keys, cnt8, usize, flags);
    LAUNCHCHK();
    HIPCHK(hipMemcpyAsync(hflags, flags, 3 * sizeof(int), hipMemcpyDeviceToHost, s));
    std::vector<int> hsz(S > 1 ? size_t(NU) : 0);
    if (S > 1) HIPCHK(hipMemcpyAsync(hsz.data(), usize, sizeof(int) * size_t(NU), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    if (hflags[0]) return fail(KRCN_ERR_UNSUPPORTED, "jag plan: rows with descending column indices");
    if (hflags[1] > 255) return fail(KRCN_ERR_UNSUPPORTED, "jag plan: %d elements of a row in one slice (max 255)", hflags[1]);
    const int umax = hsz.empty() ? 0 : *std::max_element(hsz.begin(), hsz.end());
    if (umax > kJagSlab)
      return fail(KRCN_ERR_UNSUPPORTED, "jag plan: a group holds %d elements of one slice (accumulate mode: max %d)",
                  umax, kJagSlab);
    hipLaunchKernelGGL(k_iota, dim3(vec_grid(nitems)), dim3(kNT), 0, s, nitems, iota);
    LAUNCHCHK();
    size_t tb = 0;
    HIPCHK(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, keys, keys_out, iota, perm, int(nitems), 0, ubits + 22, s));
    HIPCHK(hipMalloc(&tmp, tb));
    HIPCHK(hipcub::DeviceRadixSort::SortPairs(tmp, tb, keys, keys_out, iota, perm, int(nitems), 0, ubits + 22, s));
    hipLaunchKernelGGL(k_jag_firsts, dim3(vec_grid(nitems)), dim3(kNT), 0, s, nitems, NU, keys_out, first);
    LAUNCHCHK();
    // single window: the nonzeros and their pads in sorted (pair-level) order
    // (long rows' elements sort past them, as sentinels); accumulate layout:
    // every unit padded to an even count (two elements a lane)
    int64_t total = pairs ? nnz + hflags[2] : nnz;
    if (nl > 0) {
      int64_t lnnz = 0;
      for (int r : lrows) lnnz += hp[r + 1] - hp[r];
      total -= lnnz;
    }
    if (S > 1) {
      HIPCHK(hipMalloc(&pbase, sizeof(int) * size_t(NU)));
      hipLaunchKernelGGL(k_jag_pad2, dim3(vec_grid(NU)), dim3(kNT), 0, s, NU, usize, first);   // first := padded sizes
      LAUNCHCHK();
      HIPCHK(hipStreamSynchronize(s));
      HIPCHK(hipFree(tmp));
      tmp = nullptr;
      size_t tb2 = 0;
      HIPCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, tb2, first, pbase, int(NU), s));
      HIPCHK(hipMalloc(&tmp, tb2));
      HIPCHK(hipcub::DeviceScan::ExclusiveSum(tmp, tb2, first, pbase, int(NU), s));
      int last[2] = {0, 0};
      HIPCHK(hipMemcpyAsync(&last[0], pbase + NU - 1, sizeof(int), hipMemcpyDeviceToHost, s));
      HIPCHK(hipMemcpyAsync(&last[1], first + NU - 1, sizeof(int), hipMemcpyDeviceToHost, s));
      HIPCHK(hipStreamSynchronize(s));
      total = int64_t(last[0]) + last[1];
      hipLaunchKernelGGL(k_jag_firsts, dim3(vec_grid(nnz)), dim3(kNT), 0, s, nnz, NU, keys_out, first);   // restore
      LAUNCHCHK();
    }
    HIPCHK(hipMalloc(&P.widx, sizeof(unsigned short) * size_t(total + kJagPad)));
    HIPCHK(hipMalloc(&P.own_val, sizeof(T) * size_t(total + kJagPad)));
    P.owned += (sizeof(unsigned short) + sizeof(T)) * size_t(total + kJagPad);
    HIPCHK(hipMemsetAsync(P.widx, 0, sizeof(unsigned short) * size_t(total + kJagPad), s));
    HIPCHK(hipMemsetAsync(P.own_val, 0, sizeof(T) * size_t(total + kJagPad), s));
    hipLaunchKernelGGL((k_jag_gather<T>), dim3(vec_grid(pairs ? total : nnz)), dim3(kNT), 0, s, pairs ? total : nnz,
                       nnz, W, perm, idx, val, keys_out, first, pbase, P.widx, static_cast<T*>(P.own_val));
    LAUNCHCHK();
    hipLaunchKernelGGL(k_jag_umeta, dim3(vec_grid(nrec * 2 * K)), dim3(kNT), 0, s, nrec, K, pbase ? pbase : first,
                       usize, P.jumeta);
    LAUNCHCHK();
    {
      void* wi = P.widx;
      CHK(plan_reloc(&wi, sizeof(unsigned short) * size_t(total + kJagPad), s));
      P.widx = static_cast<unsigned short*>(wi);
      CHK(plan_reloc(&P.own_val, sizeof(T) * size_t(total + kJagPad), s));
    }
    if (nl > 0) {
      const size_t lsz = size_t(lbeg[nl]) + kJagPad;
      HIPCHK(hipMalloc(&P.jlcut, sizeof(int) * lcut.size()));
      HIPCHK(hipMalloc(&P.jlrow, sizeof(int) * size_t(nl)));
      HIPCHK(hipMalloc(&P.jltask, sizeof(int) * ltask.size()));
      HIPCHK(hipMalloc(&P.jtask, sizeof(int) * tasks.size()));
      HIPCHK(hipMalloc(&P.jlidx, sizeof(unsigned short) * lsz));
      HIPCHK(hipMalloc(&P.jlval, sizeof(T) * lsz));
      P.owned += sizeof(int) * (lcut.size() + size_t(nl) + ltask.size() + tasks.size()) +
                 (sizeof(unsigned short) + sizeof(T)) * lsz;
      int* lbeg_d = nullptr;
      HIPCHK(hipMalloc(&lbeg_d, sizeof(int) * size_t(nl)));
      HIPCHK(hipMemcpyAsync(P.jlcut, lcut.data(), sizeof(int) * lcut.size(), hipMemcpyHostToDevice, s));
      HIPCHK(hipMemcpyAsync(P.jlrow, lrows.data(), sizeof(int) * size_t(nl), hipMemcpyHostToDevice, s));
      HIPCHK(hipMemcpyAsync(P.jltask, ltask.data(), sizeof(int) * ltask.size(), hipMemcpyHostToDevice, s));
      HIPCHK(hipMemcpyAsync(P.jtask, tasks.data(), sizeof(int) * tasks.size(), hipMemcpyHostToDevice, s));
      HIPCHK(hipMemcpyAsync(lbeg_d, lbeg.data(), sizeof(int) * size_t(nl), hipMemcpyHostToDevice, s));
      HIPCHK(hipMemsetAsync(P.jlidx, 0, sizeof(unsigned short) * lsz, s));
      HIPCHK(hipMemsetAsync(P.jlval, 0, sizeof(T) * lsz, s));
      hipLaunchKernelGGL((k_jag_long_fill<T>), dim3(std::min(nl, 4096)), dim3(kNT), 0, s, nl, W, P.jlrow, lbeg_d, ptr,
                         idx, val, P.jlidx, static_cast<T*>(P.jlval));
      LAUNCHCHK();
      HIPCHK(hipStreamSynchronize(s));
      HIPCHK(hipFree(lbeg_d));
    }
    // 8-bit lane counts: a 32-bit word for the K = 4 accumulate kernel, else 64-bit
    const bool w32 = S > 1 && K <= 4;
    const size_t cbytes = size_t(nrec) * 64 * (w32 ? 4 : 8);
    HIPCHK(hipMalloc(&P.jcnt, cbytes));
    P.owned += cbytes;
    if (w32)
      hipLaunchKernelGGL((k_jag_words<unsigned>), dim3(vec_grid(nrec * 64)), dim3(kNT), 0, s, nrec, K, cnt8,
                         reinterpret_cast<unsigned*>(P.jcnt));
    else
      hipLaunchKernelGGL((k_jag_words<unsigned long long>), dim3(vec_grid(nrec * 64)), dim3(kNT), 0, s, nrec, K,
                         cnt8, reinterpret_cast<unsigned long long*>(P.jcnt));
    LAUNCHCHK();
    HIPCHK(hipStreamSynchronize(s));
    return KRCN_OK;
  };
  const krcn_status r = body();
  cleanup();
  CHK(r);
  P.jag = 1;
  P.jlong = nl;
  P.jlpiece = lpiece;
  P.jK = K;
  P.jG = SG;
  P.jSg = Sg;
  P.S = S;
  P.W = W;
  P.L = 1;
  P.groups = 1;
  P.grid = B;
  P.ntiles = G;
  P.val = P.own_val;
  return KRCN_OK;
}

template <typename T>
static krcn_status build_plan(krcn_csr* h, PassPlan& P, int rows, int64_t cols, int64_t nnz, const int* ptr,
                              const int* idx, const T* val, int lanes, hipStream_t s) {
  free_plan(P);
  P.rows = rows;
  P.cols = cols;
  P.nnz = nnz;
  const bool seq = lanes == KRCN_LANES_SEQUENTIAL;
  // A/B knobs KRCN_FMT1 / KRCN_FMT2: the format policy of one pass only
  // (KRCN_FORMAT_* values; unset keeps the handle's)
  int fmt = h->format_pass[&P == &h->p2 ? 1 : 0] >= 0 ? h->format_pass[&P == &h->p2 ? 1 : 0] : h->format;
  {
    static const int f1 = [] { const char* e = tuning_env("KRCN_FMT1"); return e ? atoi(e) : -1; }();
    static const int f2 = [] { const char* e = tuning_env("KRCN_FMT2"); return e ? atoi(e) : -1; }();
    const int f = &P == &h->p2 ? f2 : f1;
    if (f >= KRCN_FORMAT_AUTO && f <= KRCN_FORMAT_JAG) fmt = f;
  }
  // jagged format: forced, or by the auto policy (its summation order is
  // scipy's, so the sequential lane policy may use it too)
  if (fmt == KRCN_FORMAT_JAG ||
      (fmt == KRCN_FORMAT_AUTO && h->slicing == KRCN_SLICING_AUTO && jag_choice<T>(rows, cols, nnz, &P == &h->p2 ? 2 : 1))) {
    const krcn_status r = build_jag<T>(P, ptr, idx, val, &P == &h->p2 ? 2 : 1, seq, s);
    if (r != KRCN_ERR_UNSUPPORTED || fmt == KRCN_FORMAT_JAG) return r;
    free_plan(P);
    P.rows = rows;
    P.cols = cols;
    P.nnz = nnz;
  }
  // LDS-window format: forced, or by the auto policy (never under the
  // sequential lane policy, whose sliced passes must stay unsliced)
  {
    int wc = 0;
    if (fmt == KRCN_FORMAT_WINDOW) {
      const int64_t W = win_width<T>();
      wc = (cols + W - 1) / W <= 4 ? 1 : 2;
    } else if (fmt == KRCN_FORMAT_AUTO && !seq && h->slicing == KRCN_SLICING_AUTO) {
      wc = window_choice(rows, cols, nnz, sizeof(T));
    }
    if (wc) {
      const krcn_status r = build_window<T>(P, ptr, idx, val, wc == 1, s);
      if (r != KRCN_ERR_UNSUPPORTED || fmt == KRCN_FORMAT_WINDOW) return r;
      free_plan(P);   // not applicable to this matrix: fall through to the other formats
      P.rows = rows;
      P.cols = cols;
      P.nnz = nnz;
    }
  }
  // format
  bool sorted = false;
  int S_sorted = sorted_slices(cols);
  // sharded passes run without the fused step B, so the slices' combine is
  // pure overhead while the gathered vector is L2-sized: a news20 rank of 8
  // (170 K columns, 1.36 MB) ran 27.4 k HVP/s unsliced against 25.3 k sliced;
  // a rank of 4 (2.7 MB) 20.4 k against 23.8 k
  if (h->shard != KRCN_SHARD_NONE && cols * int64_t(sizeof(T)) <= int64_t(3) << 19) S_sorted = 1;
  // pass 1 beside a single-window jagged pass 2: unsliced sorted tiles (no
  // slice partials, no combine launch: the two-launch Lanczos step)
  if (&P == &h->p1 && h->p1_unsliced) S_sorted = 1;
  if (h->slicing >= 8) S_sorted = h->slicing;
  // largest block tile that still leaves >= one tile per CU
  int sort_nt = h->sort_nt;
  if (sort_nt == 0)
    sort_nt = nnz >= int64_t(kNumCUs) * 1024 * kSortPerThread ? 1024
              : nnz >= int64_t(kNumCUs) * 512 * kSortPerThread ? 512 : 256;
  const int64_t max_window = sort_nt == 256 ? SortGeom<256>::kMaxWindow
                             : sort_nt == 512 ? SortGeom<512>::kMaxWindow : SortGeom<1024>::kMaxWindow;
  const bool one_slice = h->slicing == KRCN_SLICING_OFF || seq;
  if (one_slice) S_sorted = 1;
  // the packed gather word addresses kSortMaxWindow columns past a slice's base
  while (!one_slice && (cols + S_sorted - 1) / S_sorted >= max_window) S_sorted = S_sorted < 8 ? 8 : S_sorted + 8;
  const bool sortable = (cols + S_sorted - 1) / S_sorted < max_window;
  const bool unsliced_pick = &P == &h->p1 && h->p1_unsliced && S_sorted == 1;
  if (fmt == KRCN_FORMAT_SORTED && sortable) {
    sorted = true;
  } else if (fmt == KRCN_FORMAT_AUTO && !seq && nnz > 0) {
    const double part_bytes = S_sorted > 1 ? 16.0 * double(S_sorted) * double(rows) : 0.0;
    const double mat_bytes = double(nnz) * (sizeof(T) + sizeof(int));
    const int64_t window = (cols + S_sorted - 1) / S_sorted;
    sorted = (window <= sort_window() || unsliced_pick) && part_bytes <= 0.25 * mat_bytes;
  }
  if (sorted) {
    P.S = S_sorted;
  } else if (seq || h->slicing == KRCN_SLICING_OFF) {
    P.S = 1;
  } else if (h->slicing >= 8) {
    P.S = h->slicing;
  } else {
    P.S = slices_for(cols * int64_t(sizeof(T)));
  }
  if (P.S > 1 && cols < P.S) P.S = 1;
  P.sorted = sorted ? 1 : 0;
  P.sort_nt = sort_nt;
  P.groups = P.S > 1 ? 8 : 1;
  // a sliced row holds ~1/S of its nonzeros: pick lanes from the slice-local mean
  P.L = resolve_lanes(lanes, int64_t(rows) * P.S, nnz);
  if (sorted && lanes == KRCN_LANES_AUTO && &P == &h->p1 && rows > 0 && nnz > 0) {
    // skewed rows: a row's lane group walks ceil(len / L) staged products,
    // so a wave waits on the longest of its rows, not on the mean one. When
    // the nonzero-weighted mean row (sum len^2 / nnz) is >= 2x the plain
    // mean, lanes come from 4x the weighted slice-local mean (auto_lanes: the
    // largest L with 8 L <= that): rcv1 with a power-law row tail (max 2160,
    // mean 71, weighted 189, 8 slices: 94) takes L = 8, 37.0 -> 28.4 us per
    // HVP, best of L = 1..32 on two boxes (L = 4 29.4, L = 16 30.8; calibrated
    // on this one tail shape;
    // profiles/r06aa_rcv1skew_lanes.txt); uniform rows (ratio 1.0) keep the
    // plain mean (rcv1: L = 1 18.0 us, L = 4 19.0 us)
    std::vector<int> hp(size_t(rows) + 1);
    HIPCHK(hipMemcpyAsync(hp.data(), ptr, sizeof(int) * hp.size(), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    double sq = 0.0;
    for (int r = 0; r < rows; ++r) {
      const double len = double(hp[r + 1] - hp[r]);
      sq += len * len;
    }
    const double mean = double(nnz) / double(rows);
    const double wmean = sq / double(nnz);
    if (wmean >= 2.0 * mean) P.L = std::max(P.L, auto_lanes(int64_t(P.S), int64_t(4.0 * wmean)));
  }
  if (P.S == 1) {
    P.ptr = ptr;
    P.idx = idx;
    P.val = val;
  } else {
    CHK(build_slices<T>(P, ptr, idx, val, s));
    HIPCHK(hipMalloc(&P.part, sizeof(T) * size_t(P.S) * std::max(rows, 1)));
    P.owned += sizeof(T) * size_t(P.S) * std::max(rows, 1);
  }
  std::vector<int> segs, segbase;
  CHK(build_tiles(P, s, P.sorted ? &segs : nullptr, P.sorted ? &segbase : nullptr));
  if (P.sorted) CHK(build_sorted<T>(P, segs, segbase, s));
  return KRCN_OK;
}

// ------------------------------------------------------ placement probe
// DESIGN.md §5 *Placement*: a news20-sized working set (both plans, the slice
// partials, the Lanczos vectors: ~235 MB) fills ~90 % of the 256 MiB
// Infinity Cache, and whether a handle runs fast or ~7 % slow is decided by
// where its buffers' pages land (fresh handles in one process flip between
// the two states; moving the pass-1 partials alone flipped one).  So after a
// plan build whose hot set is within reach of the cache, the handle's hot
// buffers are copied to k - 1 further placements (each allocated while the
// others are alive, so each lands elsewhere), every placement is timed with
// the same local HVP, and the fastest is kept; the others are freed.
// Results are unchanged: only addresses move.
static constexpr double kPlaceHotLoMB = 96.0;    // below: the hot set sits in the cache whatever its placement
static constexpr double kPlaceHotHiMB = 400.0;   // above: streamed from HBM, placement-blind
static constexpr int kPlaceAutoTrials = 4;
static constexpr int kPlaceReps = 6;

static void hot_slots(krcn_csr* h, std::vector<void**>& out) {
  for (PassPlan* P : {&h->p1, &h->p2}) {
    void** f[] = {reinterpret_cast<void**>(&P->own_ptr), reinterpret_cast<void**>(&P->own_idx), &P->own_val,
                  reinterpret_cast<void**>(&P->tiles), reinterpret_cast<void**>(&P->tbeg), &P->part,
                  reinterpret_cast<void**>(&P->gword), &P->gval, reinterpret_cast<void**>(&P->tmid),
                  reinterpret_cast<void**>(&P->widx), reinterpret_cast<void**>(&P->segs),
                  reinterpret_cast<void**>(&P->tb), reinterpret_cast<void**>(&P->ro),
                  reinterpret_cast<void**>(&P->jgcut), reinterpret_cast<void**>(&P->jumeta),
                  reinterpret_cast<void**>(&P->jcnt), reinterpret_cast<void**>(&P->jlcut),
                  reinterpret_cast<void**>(&P->jlrow), reinterpret_cast<void**>(&P->jltask),
                  reinterpret_cast<void**>(&P->jtask), reinterpret_cast<void**>(&P->jlidx), &P->jlval,
                  reinterpret_cast<void**>(&P->xcp), reinterpret_cast<void**>(&P->xrow), &P->xval, &P->xpart};
    for (void** s : f)
      if (*s) out.push_back(s);
  }
  void** v[] = {&h->u, &h->tn, &h->W, &h->td, reinterpret_cast<void**>(&h->pa), reinterpret_cast<void**>(&h->pb),
                reinterpret_cast<void**>(&h->pz), reinterpret_cast<void**>(&h->pq)};
  for (void** s : v)
    if (*s) out.push_back(s);
}

// The handle's hot buffers as relocatable slots: their allocation sizes and
// the plan fields that alias the owned arrays (ptr / idx / val).
struct PlaceSet {
  std::vector<void**> slots;
  std::vector<size_t> bytes;
  PassPlan* Ps[2] = {nullptr, nullptr};
  bool al_ptr[2] = {}, al_idx[2] = {}, al_val[2] = {};
  double hot = 0.0;
  krcn_status init(krcn_csr* h) {
    hot_slots(h, slots);
    bytes.assign(slots.size(), 0);
    for (size_t i = 0; i < slots.size(); ++i) {
      void* base = nullptr;
      HIPCHK(hipMemGetAddressRange(&base, &bytes[i], *slots[i]));
      if (base != *slots[i]) return fail(KRCN_ERR_HIP, "placement probe: a plan buffer is not an allocation base");
      hot += double(bytes[i]);
    }
    std::vector<void*> seen = current();
    std::sort(seen.begin(), seen.end());
    if (std::adjacent_find(seen.begin(), seen.end()) != seen.end())
      return fail(KRCN_ERR_HIP, "placement probe: two plan fields share one allocation");
    Ps[0] = &h->p1;
    Ps[1] = &h->p2;
    for (int i = 0; i < 2; ++i) {
      al_ptr[i] = Ps[i]->own_ptr && Ps[i]->ptr == Ps[i]->own_ptr;
      al_idx[i] = Ps[i]->own_idx && Ps[i]->idx == Ps[i]->own_idx;
      al_val[i] = Ps[i]->own_val && Ps[i]->val == Ps[i]->own_val;
    }
    return KRCN_OK;
  }
  std::vector<void*> current() const {
    std::vector<void*> c;
    for (void** sl : slots) c.push_back(*sl);
    return c;
  }
  void apply(const std::vector<void*>& c) {
    for (size_t i = 0; i < slots.size(); ++i) *slots[i] = c[i];
    for (int i = 0; i < 2; ++i) {
      if (al_ptr[i]) Ps[i]->ptr = Ps[i]->own_ptr;
      if (al_idx[i]) Ps[i]->idx = Ps[i]->own_idx;
      if (al_val[i]) Ps[i]->val = Ps[i]->own_val;
    }
  }
  // a fresh placement holding a copy of `from` (allocated while every other
  // placement is alive, so it lands elsewhere); c's entries are set as they
  // are allocated, so a failure leaves them to be freed by the caller
  krcn_status copy(std::vector<void*>& c, const std::vector<void*>& from, hipStream_t s) const {
    c.assign(slots.size(), nullptr);
    for (size_t i = 0; i < slots.size(); ++i) {
      HIPCHK(hipMalloc(&c[i], bytes[i]));
      HIPCHK(hipMemcpyAsync(c[i], from[i], bytes[i], hipMemcpyDeviceToDevice, s));
    }
    return KRCN_OK;
  }
};

static int place_auto_trials(const krcn_csr* h) {
  int k = h->place_trials;
  if (k < 0) k = (h->place_hot_mb >= kPlaceHotLoMB && h->place_hot_mb <= kPlaceHotHiMB) ? kPlaceAutoTrials : 0;
  return std::min(k, krcn_csr::kPlaceMax);
}

static void free_placements(std::vector<std::vector<void*>>& cand, int keep) {
  for (size_t t = 0; t < cand.size(); ++t)
    if (int(t) != keep)
      for (void* p : cand[t])
        if (p) (void)hipFree(p);
  cand.clear();
}

static krcn_status tune_placement(krcn_csr* h) {
  h->place_ran = 0;
  h->place_best = -1;
  PlaceSet ps;
  CHK(ps.init(h));
  h->place_hot_mb = (ps.hot + 3.0 * double(h->d) * double(h->vs)) / 1e6;   // + the Lanczos vectors a step touches
  const int k = place_auto_trials(h);
  if (k <= 1 || h->n == 0 || h->d == 0) return KRCN_OK;
  std::vector<std::vector<void*>> cand(1, ps.current());
  hipStream_t s = nullptr;
  HIPCHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  krcn_status r = KRCN_OK;
  // the probe's operands: zero vectors (the traffic does not depend on them)
  for (void* b : {h->tn, h->W}) {
    void* base = nullptr;
    size_t sz = 0;
    if (r == KRCN_OK && hipMemGetAddressRange(&base, &sz, b) == hipSuccess)
      r = hipMemsetAsync(b, 0, sz, s) == hipSuccess ? KRCN_OK : fail(KRCN_ERR_HIP, "placement probe: memset");
  }
  for (int t = 0; t < k && r == KRCN_OK; ++t) {
    if (t > 0) {
      cand.emplace_back();
      r = ps.copy(cand.back(), cand[0], s);   // (freed below whatever happened)
      if (r != KRCN_OK) break;
      ps.apply(cand.back());
    }
    r = placement_probe(h, s, kPlaceReps, &h->place_us[t]);
    if (r == KRCN_OK) h->place_ran = t + 1;
  }
  if (hipStreamSynchronize(s) != hipSuccess && r == KRCN_OK) r = fail(KRCN_ERR_HIP, "placement probe: sync");
  (void)hipStreamDestroy(s);
  int best = 0;
  for (int t = 1; t < h->place_ran; ++t)
    if (h->place_us[t] < h->place_us[best]) best = t;
  if (r != KRCN_OK) best = 0;   // a failed probe keeps the built placement
  ps.apply(cand[best]);
  free_placements(cand, best);
  h->place_best = best;
  ++h->ws_gen;
  return r;
}

// ------------------------------------------- placement over Lanczos calls
// The plan-build probe times a standalone HVP on the handle's own scratch;
// the recurrence also streams the caller's basis V and weights, allocated
// later, and which placement runs a Lanczos step fastest can differ (round 6:
// a probe-picked placement still drew the slow state in 1 of 4 processes,
// profiles/r06c_news20_placement_probe_ab.txt).  So the first Lanczos calls of
// an eligible handle (unsharded or single-rank, no graph replay, m >= 8, hot
// set in the probe's band) continue it on the real workload: call 1 runs
// untimed (warm), calls 2 .. k + 1 with the same m each run on one placement
// (the current one, then fresh copies) bracketed by events, and after the
// k-th the fastest is kept and the others freed.  Each call's results are
// the same whatever the placement (addresses move between calls, never
// inside one).
static bool lzp_eligible(const krcn_csr* h, int m) {
  return (h->shard == KRCN_SHARD_NONE || !h->comm || h->comm->nranks <= 1) && !h->graph && m >= 8 &&
         place_auto_trials(h) > 1;
}

void lzp_abort(krcn_csr* h) {
  // (the applied placement stays: it is the handle's; the rest are freed)
  if (!h->lzp_cand.empty()) {
    const std::vector<void*> cur = [&] {
      PlaceSet ps;
      hot_slots(h, ps.slots);
      return ps.current();
    }();
    for (auto& c : h->lzp_cand)
      if (c != cur)
        for (void* p : c)
          if (p) (void)hipFree(p);
    h->lzp_cand.clear();
  }
  h->lzp_stage = 0;
}

krcn_status lzp_begin(krcn_csr* h, int m, hipStream_t s, bool* timed) {
  *timed = false;
  if (h->lzp_stage < 0 || !lzp_eligible(h, m)) return KRCN_OK;
  if (h->lzp_stage == 0) {   // the warm call
    h->lzp_m = m;
    h->lzp_ran = 0;
    h->lzp_stage = 1;
    return KRCN_OK;
  }
  if (m != h->lzp_m) return KRCN_OK;   // only calls of the same m compete
  const int t = h->lzp_stage - 1;
  PlaceSet ps;
  CHK(ps.init(h));
  if (t == 0) {
    h->lzp_cand.assign(1, ps.current());
  } else {
    h->lzp_cand.emplace_back();
    CHK(ps.copy(h->lzp_cand.back(), h->lzp_cand[0], s));   // (on the call's stream: ordered before it)
    ps.apply(h->lzp_cand.back());
    ++h->ws_gen;
  }
  if (!h->lzp_e0) HIPCHK(hipEventCreate(&h->lzp_e0));
  if (!h->lzp_e1) HIPCHK(hipEventCreate(&h->lzp_e1));
  HIPCHK(hipEventRecord(h->lzp_e0, s));
  *timed = true;
  return KRCN_OK;
}

krcn_status lzp_end(krcn_csr* h, hipStream_t s, bool timed) {
  if (!timed) return KRCN_OK;
  HIPCHK(hipEventRecord(h->lzp_e1, s));
  return KRCN_OK;
}

krcn_status lzp_done(krcn_csr* h, bool timed) {   // after the call's stream synchronisation
  if (!timed) return KRCN_OK;
  const int t = h->lzp_stage - 1;
  float ms = 0.0f;
  HIPCHK(hipEventElapsedTime(&ms, h->lzp_e0, h->lzp_e1));
  h->lzp_ms[t] = ms;
  h->lzp_ran = t + 1;
  ++h->lzp_stage;
  if (h->lzp_ran == place_auto_trials(h)) {
    int best = 0;
    for (int i = 1; i < h->lzp_ran; ++i)
      if (h->lzp_ms[i] < h->lzp_ms[best]) best = i;
    PlaceSet ps;
    CHK(ps.init(h));
    ps.apply(h->lzp_cand[size_t(best)]);
    free_placements(h->lzp_cand, best);
    h->lzp_best = best;
    h->lzp_stage = -1;
    ++h->ws_gen;
  }
  return KRCN_OK;
}

krcn_status ensure_plans(krcn_csr* h) {
  if (h->plans_ready) return KRCN_OK;
  std::lock_guard<std::mutex> lk(build_mutex());
  h->rows_pq = -1;   // new plans: row shards agree again (agree_rows)
  lzp_abort(h);      // (and the Lanczos-call placement search starts over)
  h->lzp_best = -1;
  h->lzp_ran = 0;
  hipStream_t s = nullptr;
  HIPCHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  krcn_status r;
  // pass 2 first: whether it is a single-window jagged plan may decide pass
  // 1's slicing.  Off by default: unslicing rcv1's sorted pass 1 for the
  // two-launch step ran 33.4-34.1 k HVP/s against 43.3-44.2 k for the sliced
  // pass + combine (pass 1 16 against 10 us, pass 2 13.7 against 10.3 us;
  // profiles/r04_rcv1_lz2.txt).  A/B knob KRCN_LZ2=1 turns it on.
  static const bool lz2_env = [] {
    const char* e = tuning_env("KRCN_LZ2");
    return e && e[0] == '1';
  }();
  if (h->dtype == KRCN_F64) {
    r = build_plan<double>(h, h->p2, int(h->d), h->n, h->nnz, h->tptr, h->tidx, static_cast<const double*>(h->tval), h->lanes_xt, s);
    h->p1_unsliced = lz2_env && h->p2.jag && h->p2.S == 1 && h->shard == KRCN_SHARD_NONE;
    if (r == KRCN_OK)
      r = build_plan<double>(h, h->p1, int(h->n), h->d, h->nnz, h->ptr, h->idx, static_cast<const double*>(h->val), h->lanes_x, s);
  } else {
    r = build_plan<float>(h, h->p2, int(h->d), h->n, h->nnz, h->tptr, h->tidx, static_cast<const float*>(h->tval), h->lanes_xt, s);
    h->p1_unsliced = lz2_env && h->p2.jag && h->p2.S == 1 && h->shard == KRCN_SHARD_NONE;
    if (r == KRCN_OK)
      r = build_plan<float>(h, h->p1, int(h->n), h->d, h->nnz, h->ptr, h->idx, static_cast<const float*>(h->val), h->lanes_x, s);
  }
  (void)hipStreamDestroy(s);
  CHK(r);
  // size the partials buffers to the plans' largest reducing grid (an
  // accumulate-mode window plan over a tall X^T can run up to 64 x 256 blocks)
  int64_t need = kMaxPartials;
  for (const PassPlan* P : {&h->p1, &h->p2}) need = std::max<int64_t>(need, std::max(P->grid, P->combine_grid));
  if (need > h->pcap) {
    for (double** b : {&h->pa, &h->pb, &h->pz, &h->pq}) {
      if (*b) HIPCHK(hipFree(*b));
      *b = nullptr;
      CHK(dalloc(h, b, size_t(need)));
    }
    h->pcap = need;
  } else if (!h->pz) {   // the fused step B's ||z||^2 (early-alpha step: z.v) and the combine's alpha partials
    CHK(dalloc(h, &h->pz, size_t(h->pcap)));
    CHK(dalloc(h, &h->pq, size_t(h->pcap)));
  }
  h->p1.pcap = h->p2.pcap = h->pcap;
#if KRCN_FOLD
  if (h->fcnt) HIPCHK(hipFree(h->fcnt));
  h->fcnt = nullptr;
  if (h->p1.win && !h->p1.accum && h->p1.ntiles > 0) {   // tickets (ntiles), then the per-block won lists
    const size_t cnt = size_t(h->p1.ntiles) * size_t(kFoldPad + h->p1.grid);
    HIPCHK(hipMalloc(&h->fcnt, sizeof(int) * cnt));
    HIPCHK(hipMemset(h->fcnt, 0, sizeof(int) * cnt));
  }
#endif
  h->plans_ready = true;
  ++h->ws_gen;   // a recorded Lanczos graph points into the old plans
  return tune_placement(h);
}

krcn_status reserve_reorth(krcn_csr* h, int m) {
  // dot partials: k_cgs_rowdots (chunks x rows, <= kCgsRdParts + rows) in
  // pr, k_cgs_update_dots ((column slabs) x rows) in pr2
  if (m <= h->reorth_m) return KRCN_OK;
  std::lock_guard<std::mutex> lk(build_mutex());
  const int64_t cap = ((h->d + kCgsUpdCols - 1) / kCgsUpdCols) * int64_t(m);
  // the previous reservation's buffers leave the handle's accounting as they are freed
  size_t old = size_t(h->prv_cap + h->pr_cap) * sizeof(double);
  if (h->cy) old += size_t(h->cy_q) * size_t(h->d) * sizeof(double) + size_t((h->d + 63) / 64) * sizeof(int);
  h->owned -= std::min(old, h->owned);
  for (double** b : {&h->pr, &h->pr2}) {
    if (*b) HIPCHK(hipFree(*b));
    *b = nullptr;
  }
  h->pr_cap = 0;
  h->prv_cap = 0;
  h->reorth_m = 0;
  // chunk partials of either path: the batched k_cgs_rowdots (C k <= kCgsRdPartsV)
  // and k_cgs_rowdots_v (C k, C = the 1 KiB-piece chunks of a row: past
  // 16 x 16 x 256 vectors a row takes more than kCgsRdChunksV of them)
  const int64_t nv = h->d / int64_t(16 / h->vs);
  const int64_t cv = std::max<int64_t>(kCgsRdChunksV, nv > 0 ? cgs_rdv_chunks_of(nv) : 0);
  const int64_t prv = std::max<int64_t>(kCgsRdPartsV, cv * m) + 4 * int64_t(m);
  CHK(dalloc(h, &h->pr, size_t(prv)));
  h->prv_cap = prv;
  CHK(dalloc(h, &h->pr2, size_t(cap)));
  // k_cgs_colsweep: the row ranges of a sweep over up to m - 1 rows (one range
  // needs no partials), V^T h partials of each, and one arrival counter per
  // 64-vector column group; not allocated where the 1 KiB-piece path never
  // runs (column shards, rows not whole 16-byte vectors)
  if (h->cy) HIPCHK(hipFree(h->cy));
  if (h->ccnt) HIPCHK(hipFree(h->ccnt));
  h->cy = nullptr;
  h->ccnt = nullptr;
  h->cy_q = 0;
  const int q = cgs_col_ranges(m);
  if (q > 1 && h->shard != KRCN_SHARD_COLS && h->d % int64_t(16 / h->vs) == 0) {
    const int64_t ncg = (h->d + 63) / 64;   // >= the column groups of either dtype
    CHK(dalloc(h, &h->cy, size_t(q) * size_t(h->d)));
    CHK(dalloc(h, &h->ccnt, size_t(ncg)));
    HIPCHK(hipMemsetAsync(h->ccnt, 0, sizeof(int) * size_t(ncg), nullptr));
    HIPCHK(hipStreamSynchronize(nullptr));   // zero before any stream of the handle counts on it
    h->cy_q = q;
  }
  h->pr_cap = cap;
  h->reorth_m = m;
  ++h->ws_gen;
  return KRCN_OK;
}

extern "C" krcn_status krcn_csr_reserve(krcn_csr* h, int m_max, int reorth) {
  if (!h) return fail(KRCN_ERR_INVALID, "krcn_csr_reserve: null handle");
  if (m_max < 1 || m_max > kLzMaxM) return fail(KRCN_ERR_INVALID, "krcn_csr_reserve: m_max must be 1..%d", kLzMaxM);
  CHK(set_device(h));
  CHK(ensure_plans(h));
  CHK(agree_rows(h));   // (outside the build lock: virtual ranks are threads of one process)
  if (reorth) CHK(reserve_reorth(h, m_max));
  return KRCN_OK;
}

extern "C" krcn_status krcn_csr_set_slicing(krcn_csr* h, int slicing) {
  if (!h) return fail(KRCN_ERR_INVALID, "krcn_csr_set_slicing: null handle");
  if (!(slicing == KRCN_SLICING_AUTO || slicing == KRCN_SLICING_OFF || (slicing >= 8 && slicing % 8 == 0)))
    return fail(KRCN_ERR_INVALID, "krcn_csr_set_slicing: expected 0 (auto), 1 (off) or a multiple of 8");
  if (h->slicing != slicing) {
    h->slicing = slicing;
    h->plans_ready = false;
  }
  return KRCN_OK;
}

extern "C" krcn_status krcn_csr_set_format(krcn_csr* h, int format) {
  if (!h) return fail(KRCN_ERR_INVALID, "krcn_csr_set_format: null handle");
  if (format < KRCN_FORMAT_AUTO || format > KRCN_FORMAT_JAG)
    return fail(KRCN_ERR_INVALID, "krcn_csr_set_format: expected 0 (auto), 1 (wave), 2 (sorted), 3 (window) or 4 (jagged)");
  if (h->format != format) {
    h->format = format;
    h->plans_ready = false;
  }
  return KRCN_OK;
}

extern "C" krcn_status krcn_csr_set_pass_format(krcn_csr* h, int pass, int format) {
  if (!h) return fail(KRCN_ERR_INVALID, "krcn_csr_set_pass_format: null handle");
  if (pass != 1 && pass != 2) return fail(KRCN_ERR_INVALID, "krcn_csr_set_pass_format: pass must be 1 (X) or 2 (X^T)");
  if (format < -1 || format > KRCN_FORMAT_JAG)
    return fail(KRCN_ERR_INVALID, "krcn_csr_set_pass_format: expected -1 (the handle's format) or a KRCN_FORMAT_* value");
  if (h->format_pass[pass - 1] != format) {
    h->format_pass[pass - 1] = format;
    h->plans_ready = false;
  }
  return KRCN_OK;
}

extern "C" krcn_status krcn_csr_set_placement_trials(krcn_csr* h, int trials) {
  if (!h) return fail(KRCN_ERR_INVALID, "krcn_csr_set_placement_trials: null handle");
  if (trials < -1 || trials > krcn_csr::kPlaceMax)
    return fail(KRCN_ERR_INVALID, "krcn_csr_set_placement_trials: expected -1 (auto), 0 (off) or 1..%d",
                krcn_csr::kPlaceMax);
  if (h->place_trials != trials) {
    h->place_trials = trials;
    h->plans_ready = false;   // probed at the next plan build
  }
  return KRCN_OK;
}

extern "C" krcn_status krcn_csr_placement_info(krcn_csr* h, double* out24_host) {
  if (!h || !out24_host) return fail(KRCN_ERR_INVALID, "krcn_csr_placement_info: null argument");
  CHK(set_device(h));
  CHK(ensure_plans(h));
  double* o = out24_host;
  o[0] = h->place_ran;
  o[1] = h->place_best;
  o[2] = h->place_hot_mb;
  o[3] = h->place_trials;
  for (int i = 0; i < krcn_csr::kPlaceMax; ++i) o[4 + i] = i < h->place_ran ? h->place_us[i] : 0.0;
  o[12] = h->lzp_ran;
  o[13] = h->lzp_stage < 0 ? h->lzp_best : -1;
  o[14] = h->lzp_m;
  o[15] = h->lzp_stage;
  for (int i = 0; i < krcn_csr::kPlaceMax; ++i) o[16 + i] = i < h->lzp_ran ? h->lzp_ms[i] : 0.0;
  return KRCN_OK;
}

extern "C" krcn_status krcn_csr_set_graph(krcn_csr* h, int on) {
  if (!h) return fail(KRCN_ERR_INVALID, "krcn_csr_set_graph: null handle");
  h->graph = on != 0;
  return KRCN_OK;
}

extern "C" krcn_status krcn_csr_plan_info(krcn_csr* h, int* out8_host) {
  if (!h || !out8_host) return fail(KRCN_ERR_INVALID, "krcn_csr_plan_info: null argument");
  CHK(set_device(h));
  CHK(ensure_plans(h));
  const PassPlan* ps[2] = {&h->p1, &h->p2};
  for (int i = 0; i < 2; ++i) {
    out8_host[4 * i + 0] = ps[i]->sorted ? -ps[i]->S : ps[i]->S;
    out8_host[4 * i + 1] = ps[i]->L;
    out8_host[4 * i + 2] = ps[i]->ntiles;
    out8_host[4 * i + 3] = ps[i]->grid;
  }
  return KRCN_OK;
}

extern "C" krcn_status krcn_csr_plan_format(krcn_csr* h, int* out2_host) {
  if (!h || !out2_host) return fail(KRCN_ERR_INVALID, "krcn_csr_plan_format: null argument");
  CHK(set_device(h));
  CHK(ensure_plans(h));
  const PassPlan* ps[2] = {&h->p1, &h->p2};
  for (int i = 0; i < 2; ++i)
    out2_host[i] = ps[i]->jag   ? KRCN_PLAN_JAG
                   : ps[i]->win ? (ps[i]->accum ? KRCN_PLAN_WINDOW_ACCUM : KRCN_PLAN_WINDOW_SLICES)
                   : ps[i]->sorted ? KRCN_PLAN_SORTED : KRCN_PLAN_WAVE;
  return KRCN_OK;
}

// ------------------------------------------------------------- comm
extern "C" krcn_status krcn_comm_unique_id(void* uid128_host) {
  if (!uid128_host) return fail(KRCN_ERR_INVALID, "krcn_comm_unique_id: null argument");
  static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId is 128 bytes");
  ncclUniqueId id;
  NCCLCHK(ncclGetUniqueId(&id));
  std::memcpy(uid128_host, &id, sizeof(id));
  return KRCN_OK;
}

extern "C" krcn_status krcn_comm_create(int nranks, int rank, const void* uid128_host, int device,
                                        krcn_comm** out) {
  if (!out || !uid128_host) return fail(KRCN_ERR_INVALID, "krcn_comm_create: null argument");
  if (nranks < 1 || rank < 0 || rank >= nranks) return fail(KRCN_ERR_INVALID, "krcn_comm_create: bad rank %d of %d", rank, nranks);
  HIPCHK(hipSetDevice(device));
  ncclUniqueId id;
  std::memcpy(&id, uid128_host, sizeof(id));
  krcn_comm* c = new krcn_comm();
  c->nranks = nranks;
  c->rank = rank;
  c->device = device;
  ncclResult_t r = ncclCommInitRank(&c->comm, nranks, id, rank);
  if (r != ncclSuccess) {
    delete c;
    return fail(KRCN_ERR_RCCL, "ncclCommInitRank -> %s", ncclGetErrorString(r));
  }
  *out = c;
  return KRCN_OK;
}

// ------------------------------------------------- virtual communicator
// P ranks on ONE device, one host thread each (SURVEY.md §4 "P virtual shards
// on 1 GPU"): the partition, the rank-level plans and every sharded kernel
// run exactly as in a P-GPU job; only the collective differs — a rendezvous
// of the rank threads and a device sum in rank order stand in for RCCL's
// all-reduce (RCCL refuses two ranks on one device).
struct VirtualGroup : krcn::Rendezvous {
  int device = 0;
};

template <typename T>
__global__ __launch_bounds__(kNT) void k_virtual_sum(int P, int64_t count, VirtualBufs b) {
  for (int64_t i = int64_t(blockIdx.x) * kNT + threadIdx.x; i < count; i += int64_t(gridDim.x) * kNT) {
    T s = static_cast<const T*>(b.p[0])[i];
    for (int r = 1; r < P; ++r) s = s + static_cast<const T*>(b.p[r])[i];
    for (int r = 0; r < P; ++r) static_cast<T*>(b.p[r])[i] = s;
  }
}

krcn_status virtual_allreduce(krcn_comm* c, void* buf, int64_t count, int dtype, hipStream_t s) {
  HIPCHK(hipStreamSynchronize(s));   // this rank's buffer is final
  // the last to arrive sums every rank's buffer in rank order on its own stream
  auto sum = [s](void* const* bufs, int P, int64_t cnt, int dt) -> int {
    VirtualBufs vb{};
    for (int r = 0; r < P; ++r) vb.p[r] = bufs[r];
    const int grid = vec_grid(cnt);
    if (dt == KRCN_F64)
      hipLaunchKernelGGL(k_virtual_sum<double>, dim3(grid), dim3(kNT), 0, s, P, cnt, vb);
    else
      hipLaunchKernelGGL(k_virtual_sum<float>, dim3(grid), dim3(kNT), 0, s, P, cnt, vb);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    return e == hipSuccess ? KRCN_OK : KRCN_ERR_HIP;
  };
  std::string msg;
  const int r = c->vg->arrive(c->rank, &c->seq, buf, count, dtype, sum, &msg);
  if (r != KRCN_OK) return fail(r, "%s", msg.c_str());
  return KRCN_OK;
}

extern "C" krcn_status krcn_comm_create_virtual(int nranks, int device, krcn_comm** out) {
  if (!out) return fail(KRCN_ERR_INVALID, "krcn_comm_create_virtual: null argument");
  if (nranks < 1 || nranks > kVirtualMaxRanks)
    return fail(KRCN_ERR_INVALID, "krcn_comm_create_virtual: nranks must be 1..%d", kVirtualMaxRanks);
  HIPCHK(hipSetDevice(device));
  VirtualGroup* g = new VirtualGroup();
  g->P = nranks;
  g->device = device;
  g->alive = nranks;
  g->timeout_s = kVirtualTimeoutS;
  for (int r = 0; r < nranks; ++r) {
    krcn_comm* c = new krcn_comm();
    c->nranks = nranks;
    c->rank = r;
    c->device = device;
    c->vg = g;
    out[r] = c;
  }
  return KRCN_OK;
}

extern "C" krcn_status krcn_comm_destroy(krcn_comm* c) {
  if (!c) return KRCN_OK;
  if (c->comm) ncclCommDestroy(c->comm);
  if (c->vg) {
    bool last;
    {
      std::lock_guard<std::mutex> lk(c->vg->mu);
      last = --c->vg->alive == 0;
    }
    if (last) delete c->vg;
  }
  delete c;
  return KRCN_OK;
}

extern "C" krcn_status krcn_comm_allreduce(krcn_comm* c, int dtype, void* buf, int64_t n, void* stream) {
  if (!c || (!buf && n)) return fail(KRCN_ERR_INVALID, "krcn_comm_allreduce: null argument");
  if (n == 0 || c->nranks == 1) return KRCN_OK;
  HIPCHK(hipSetDevice(c->device));
  if (c->vg) return virtual_allreduce(c, buf, n, dtype, S(stream));
  ncclDataType_t t;
  nccl_dtype(dtype, &t);
  NCCLCHK(ncclAllReduce(buf, buf, size_t(n), t, ncclSum, c->comm, S(stream)));
  return KRCN_OK;
}

// ------------------------------------------------------------- profiling
extern "C" krcn_status krcn_prof_enable(krcn_csr* h, int on) {
  if (!h) return fail(KRCN_ERR_INVALID, "krcn_prof_enable: null handle");
  h->prof = on != 0;
  h->prof_used = 0;
  return KRCN_OK;
}

extern "C" krcn_status krcn_prof_read(krcn_csr* h, double* out8_host) {
  if (!h || !out8_host) return fail(KRCN_ERR_INVALID, "krcn_prof_read: null argument");
  CHK(set_device(h));
  double p1 = 0, p2 = 0, tot = 0, k1 = 0, cb = 0;
  for (size_t i = 0; i < h->prof_used; ++i) {
    ProfRec& r = h->prof_pool[i];
    HIPCHK(hipEventSynchronize(r.e2));
    float a = 0, b = 0;
    HIPCHK(hipEventElapsedTime(&a, r.e0, r.e1));
    HIPCHK(hipEventElapsedTime(&b, r.e1, r.e2));
    p1 += a;
    p2 += b;
    tot += double(a) + double(b);
    if (r.mid) {
      float x = 0, y = 0;
      HIPCHK(hipEventElapsedTime(&x, r.e0, r.em));
      HIPCHK(hipEventElapsedTime(&y, r.em, r.e1));
      k1 += x;
      cb += y;
    } else {
      k1 += a;
    }
  }
  const double c = double(h->prof_used);
  out8_host[0] = c; out8_host[1] = p1;
  out8_host[2] = c; out8_host[3] = p2;
  out8_host[4] = c; out8_host[5] = tot;
  out8_host[6] = k1; out8_host[7] = cb;
  h->prof_used = 0;
  return KRCN_OK;
}

#ifdef KRCN_TUNING
// Placement diagnostics (tools/placement_rounds.py; not in krcn.h): move one
// of the handle's scratch buffers to a fresh allocation (allocated before the
// old one is freed, so it lands elsewhere).  which: 1 w, 2 u, 3 pass-1 slice
// partials, 4 td (rows-shard scratch d-vector), 5 the small partial buffers.
extern "C" int krcn_debug_realloc(krcn_csr* h, int which) {
  auto mv = [&](void** p, size_t bytes) -> int {
    if (!*p || bytes == 0) return 0;
    void* q = nullptr;
    if (hipMalloc(&q, bytes) != hipSuccess) return 1;
    if (hipFree(*p) != hipSuccess) return 1;
    *p = q;
    return 0;
  };
  if (!h || ensure_plans(h) != KRCN_OK) return 1;
  const size_t vs = size_t(h->vs);
  switch (which) {
    case 1: return mv(&h->W, size_t(h->d) * vs);
    case 2: return mv(&h->u, size_t(h->n + 2) * vs);
    case 3: return mv(&h->p1.part, size_t(h->p1.S) * size_t(std::max<int64_t>(h->p1.rows, 1)) * vs);
    case 4: return mv(&h->td, size_t(h->d + kMaxPartials) * vs);
    case 5: {
      void* a = h->pa; void* b = h->pb; void* z = h->pz;
      int r = mv(&a, size_t(h->pcap) * 8) | mv(&b, size_t(h->pcap) * 8) | mv(&z, size_t(h->pcap) * 8);
      h->pa = static_cast<double*>(a); h->pb = static_cast<double*>(b); h->pz = static_cast<double*>(z);
      return r;
    }
    default: return 1;
  }
}
#endif

#ifdef KRCN_WIN_TIMING
// Debug builds only: read (and optionally clear) the window-pass stamps.
extern "C" int krcn_debug_win_stamps_ops(unsigned long long* out, int n, int reset);
extern "C" int krcn_debug_win_stamps_lz64(unsigned long long* out, int n, int reset);
extern "C" int krcn_debug_win_stamps_lz32(unsigned long long* out, int n, int reset);
extern "C" int krcn_debug_win_stamps(unsigned long long* out, int n, int reset) {
  std::vector<unsigned long long> t(size_t(n), 0);
  std::fill(out, out + n, 0ull);
  int (*rd[])(unsigned long long*, int, int) = {krcn_debug_win_stamps_ops, krcn_debug_win_stamps_lz64,
                                                 krcn_debug_win_stamps_lz32};
  for (auto f : rd) {
    if (f(t.data(), n, reset)) return 1;
    for (int i = 0; i < n; ++i) out[i] = std::max(out[i], t[i]);
  }
  return 0;
}
#endif

#ifdef KRCN_SORT_TIMING
// Debug builds only: read (and optionally clear) the phase cycles of k_sorted_pass.
extern "C" int krcn_debug_cycles(unsigned long long* out, int n, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(krcn::krcn_dbg_cycles), sizeof(unsigned long long) * n) != hipSuccess)
    return 1;
  if (reset) {
    std::vector<unsigned long long> z(1024 * 16 * 8, 0);
    if (hipMemcpyToSymbol(HIP_SYMBOL(krcn::krcn_dbg_cycles), z.data(), sizeof(unsigned long long) * z.size()) !=
        hipSuccess)
      return 1;
  }
  return 0;
}
#endif
