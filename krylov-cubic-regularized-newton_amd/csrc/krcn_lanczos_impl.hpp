// krcn_lanczos_impl.hpp — the device Lanczos recurrence of cubic.py:77-111
// (included once per dtype by krcn_lanczos_f64.hip / krcn_lanczos_f32.hip).
#pragma once
#include "krcn_internal.hpp"

// ------------------------------------------------------------- Lanczos
// The recurrence allocates nothing: the alphas | betas | state block and the
// CGS2 coefficients exist from krcn_csr_create (m <= kLzMaxM), the CGS2 dot
// partials from krcn_csr_reserve (reserve_reorth, krcn_plan.hip).  An
// unsharded handle reserves them on its first reorthogonalised call; a handle
// of a multi-rank communicator must have reserved them before the collectives.
static krcn_status check_lanczos_ws(krcn_csr* h, int m, int reorth) {
  if (m > h->mcap) return fail(KRCN_ERR_UNSUPPORTED, "krcn_lanczos: m = %d exceeds %d", m, h->mcap);
  if (!reorth || m <= h->reorth_m) return KRCN_OK;
  if (h->comm && h->comm->nranks > 1)
    return fail(KRCN_ERR_INVALID, "krcn_lanczos: reorthogonalisation workspace reserved for m <= %d, not %d: call "
                "krcn_csr_reserve(h, m, 1) before the recurrence on a sharded handle", h->reorth_m, m);
  return reserve_reorth(h, m);
}

// CGS2 of z against V[0..k) (krcn_cgs2.hpp): three sweeps over V, four
// launches; the ||z||^2 partials land in h->pb, their count in *Pnorm.
template <typename T, int U>
static void cgs_updates(krcn_csr* h, const T* V, int k, T* z, int C, bool cached, hipStream_t s) {
  const int64_t d = h->d;
  const int n3 = int((d + kCgsUpdCols - 1) / kCgsUpdCols);
  const size_t lds = cgs_upd_lds<T>(k, U, C, cached);
  if (cached)
    hipLaunchKernelGGL((k_cgs_update_dots<T, true, U>), dim3(n3), dim3(kCgsUpdNT), lds, s, d, k, V,
                       static_cast<const double*>(h->pr), C, z, h->pr2, h->st);
  else
    hipLaunchKernelGGL((k_cgs_update_dots<T, false, U>), dim3(n3), dim3(kCgsUpdNT), lds, s, d, k, V,
                       static_cast<const double*>(h->pr), C, z, h->pr2, h->st);
}

template <typename T, int U>
static void cgs_norm(krcn_csr* h, const T* V, int k, T* z, int gn, hipStream_t s) {
  hipLaunchKernelGGL((k_cgs_update_norm<T, U>), dim3(gn), dim3(kCgsUpdNT), 0, s, h->d, k, V,
                     static_cast<const double*>(h->hcoef), z, h->pb, h->st);
}

// step B operands for the fused first sweep (k_cgs_rowdots_vb)
template <typename T> struct CgsStepB {
  const T* W; const double* pa; int Pa;
};

// The 1 KiB-piece CGS2 path applies: unsharded, rows of whole 16-byte
// vectors, aligned, at most pcap column groups, the k_cgs_rowdots_v chunk
// partials of a k-row sweep within pr and its row ranges within cy (both
// sized by reserve_reorth; tuning knob KRCN_CGS_1K=0 keeps the batched
// round-3 kernels for A/B).
template <typename T>
static bool cgs_vec_ok(const krcn_csr* h, const T* V, const T* z, bool over_ranks, int k) {
  static const bool env = [] {
    const char* e = tuning_env("KRCN_CGS_1K");
    return !(e && e[0] == '0');
  }();
  constexpr int E = Vec16<T>::E;
  const int64_t d = h->d;
  const int64_t ncg = (d / E + 63) / 64;
  if (!env || over_ranks || d % E != 0 || ncg > h->pcap) return false;
  if (int64_t(cgs_rdv_chunks_of(d / E)) * k + 4 * int64_t(k) > h->prv_cap) return false;
  const int q = cgs_col_ranges(k);
  if (q > 1 && (q > h->cy_q || !h->cy || !h->ccnt)) return false;
  return reinterpret_cast<uintptr_t>(V) % 16 == 0 && reinterpret_cast<uintptr_t>(z) % 16 == 0;
}

template <typename T, int U>
static void cgs_colsweeps(krcn_csr* h, const T* V, int k, T* z, int C, int S, int ncg, const CgsStepB<T>* sb,
                          hipStream_t s);

template <typename T, int S>
static void cgs_rowdots_v(krcn_csr* h, const T* V, int k, const T* z, int C, hipStream_t s) {
  hipLaunchKernelGGL((k_cgs_rowdots_v<T, S>), dim3(C, k), dim3(kNT), 0, s, h->d, k, V, z, h->pr, h->st);
}

template <typename T, int S>
static void cgs_rowdots_vb(krcn_csr* h, const T* V, int k, int C, const CgsStepB<T>& sb, hipStream_t s) {
  hipLaunchKernelGGL((k_cgs_rowdots_vb<T, S>), dim3(C, k), dim3(kNT), 0, s, h->d, k, const_cast<T*>(V), sb.W, sb.pa,
                     sb.Pa, h->alphas_dev, h->pr, h->st);
}

template <typename T, int U>
static void cgs_colsweeps(krcn_csr* h, const T* V, int k, T* z, int C, int S, int ncg, const CgsStepB<T>* sb,
                          hipStream_t s) {
  const int64_t d = h->d;
  // a colsweep block walks NB batches of 4 U rows (default 8 x 32 = 256-row
  // ranges: profiles/r04_cgs2_ab.txt; tuning knob KRCN_CGS_NB = 1, 2, 4, 8, 16)
  const int NB = cgs_nb();
  const int Q = (k + 4 * U * NB - 1) / (4 * U * NB);   // = cgs_col_ranges(k) (cgs_vec_ok checked cy holds them)
  auto rowdots = [&](const T* zz) {
    switch (S) {
      case 1: cgs_rowdots_v<T, 1>(h, V, k, zz, C, s); break;
      case 2: cgs_rowdots_v<T, 2>(h, V, k, zz, C, s); break;
      case 4: cgs_rowdots_v<T, 4>(h, V, k, zz, C, s); break;
      case 8: cgs_rowdots_v<T, 8>(h, V, k, zz, C, s); break;
      default: cgs_rowdots_v<T, 16>(h, V, k, zz, C, s); break;
    }
  };
  if (sb) {   // z = V[k] is formed (step B) by the first sweep itself
    switch (S) {
      case 1: cgs_rowdots_vb<T, 1>(h, V, k, C, *sb, s); break;
      case 2: cgs_rowdots_vb<T, 2>(h, V, k, C, *sb, s); break;
      case 4: cgs_rowdots_vb<T, 4>(h, V, k, C, *sb, s); break;
      case 8: cgs_rowdots_vb<T, 8>(h, V, k, C, *sb, s); break;
      default: cgs_rowdots_vb<T, 16>(h, V, k, C, *sb, s); break;
    }
  } else {
    rowdots(z);
  }
  auto colsweep = [&](auto norm) {
    constexpr bool kN = decltype(norm)::value;
    const double* hpp = static_cast<const double*>(h->pr);
    if (NB == 16)
      hipLaunchKernelGGL((k_cgs_colsweep<T, U, kN, 16>), dim3(ncg, Q), dim3(kNT), 0, s, d, k, V, hpp, C, z, h->cy,
                         h->ccnt, h->pb, h->st);
    else if (NB == 8)
      hipLaunchKernelGGL((k_cgs_colsweep<T, U, kN, 8>), dim3(ncg, Q), dim3(kNT), 0, s, d, k, V, hpp, C, z, h->cy,
                         h->ccnt, h->pb, h->st);
    else if (NB == 4)
      hipLaunchKernelGGL((k_cgs_colsweep<T, U, kN, 4>), dim3(ncg, Q), dim3(kNT), 0, s, d, k, V, hpp, C, z, h->cy,
                         h->ccnt, h->pb, h->st);
    else if (NB == 2)
      hipLaunchKernelGGL((k_cgs_colsweep<T, U, kN, 2>), dim3(ncg, Q), dim3(kNT), 0, s, d, k, V, hpp, C, z, h->cy,
                         h->ccnt, h->pb, h->st);
    else
      hipLaunchKernelGGL((k_cgs_colsweep<T, U, kN, 1>), dim3(ncg, Q), dim3(kNT), 0, s, d, k, V, hpp, C, z, h->cy,
                         h->ccnt, h->pb, h->st);
  };
  colsweep(std::false_type{});
  rowdots(z);
  colsweep(std::true_type{});
}

template <typename T>
static krcn_status reorth_cgs2(krcn_csr* h, const T* V, int k, T* z, bool over_ranks, int* Pnorm, hipStream_t s,
                               const CgsStepB<T>* sb = nullptr) {
  const int64_t d = h->d;
  const int n3 = int((d + kCgsUpdCols - 1) / kCgsUpdCols);
  const int cgrid = (k + kCgsHPad + kCgsCoefRows - 1) / kCgsCoefRows;
  if (k > kCgsKMax) return fail(KRCN_ERR_UNSUPPORTED, "CGS2: more than 2048 basis vectors");
  constexpr int E = Vec16<T>::E;
  const int64_t ncg = (d / E + 63) / 64;   // k_cgs_colsweep column groups: one ||z||^2 partial each
  const bool vec_ok = cgs_vec_ok<T>(h, V, z, over_ranks, k);
  if (sb && !vec_ok) return fail(KRCN_ERR_UNSUPPORTED, "CGS2: step B fused into a sweep the path does not run");
  if (vec_ok) {
    const int64_t nv = d / E;
    const int S = cgs_rdv_steps(nv, k);
    const int C = cgs_rdv_chunks(nv, S);
    *Pnorm = int(ncg);
    switch (cgs_col_unroll(k, cgs_umax())) {
      case 1: cgs_colsweeps<T, 1>(h, V, k, z, C, S, int(ncg), sb, s); break;
      case 2: cgs_colsweeps<T, 2>(h, V, k, z, C, S, int(ncg), sb, s); break;
      case 4: cgs_colsweeps<T, 4>(h, V, k, z, C, S, int(ncg), sb, s); break;
      case 8: cgs_colsweeps<T, 8>(h, V, k, z, C, S, int(ncg), sb, s); break;
      default: cgs_colsweeps<T, 16>(h, V, k, z, C, S, int(ncg), sb, s); break;
    }
    LAUNCHCHK();
    return KRCN_OK;
  }
  const int C = cgs_rd_chunks(d, k);
  {
    const int64_t cw = (d + C - 1) / C;
    hipLaunchKernelGGL((k_cgs_rowdots<T>), dim3(C, (k + kCgsRdRows - 1) / kCgsRdRows), dim3(kCgsRdNT), 0, s, d, k,
                       cw, V, static_cast<const T*>(z), h->pr, h->st);
  }
  LAUNCHCHK();
  if (over_ranks) {
    // the chunk partials are per rank: sum them to h1 first, all-reduce, and
    // hand the update the global h1 as a single chunk
    hipLaunchKernelGGL(k_cgs_coeffs, dim3(cgrid), dim3(kCgsCoefNT), 0, s, h->pr, C, k, h->hcoef, h->st);
    LAUNCHCHK();
    CHK(allreduce(h, h->hcoef, k, KRCN_F64, s));
    HIPCHK(hipMemcpyAsync(h->pr, h->hcoef, size_t(k) * sizeof(double), hipMemcpyDeviceToDevice, s));
  }
  const int Cu = over_ranks ? 1 : C;
  const bool cached = int64_t(k) * kCgsSlabLd * int64_t(sizeof(T)) <= kCgsCacheBytes;
  const int gn = int(std::min<int64_t>((d + kCgsNormCols - 1) / kCgsNormCols, kMaxPartials));
  const int U = cgs_unroll(k);
  *Pnorm = gn;
  switch (U) {
    case 1: cgs_updates<T, 1>(h, V, k, z, Cu, cached, s); break;
    case 2: cgs_updates<T, 2>(h, V, k, z, Cu, cached, s); break;
    case 4: cgs_updates<T, 4>(h, V, k, z, Cu, cached, s); break;
    case 8: cgs_updates<T, 8>(h, V, k, z, Cu, cached, s); break;
    default: cgs_updates<T, 16>(h, V, k, z, Cu, cached, s); break;
  }
  LAUNCHCHK();
  hipLaunchKernelGGL(k_cgs_coeffs, dim3(cgrid), dim3(kCgsCoefNT), 0, s, h->pr2, n3, k, h->hcoef, h->st);
  LAUNCHCHK();
  if (over_ranks) CHK(allreduce(h, h->hcoef, k, KRCN_F64, s));
  switch (cgs_norm_unroll(k)) {
    case 1: cgs_norm<T, 1>(h, V, k, z, gn, s); break;
    case 2: cgs_norm<T, 2>(h, V, k, z, gn, s); break;
    case 4: cgs_norm<T, 4>(h, V, k, z, gn, s); break;
    case 8: cgs_norm<T, 8>(h, V, k, z, gn, s); break;
    default: cgs_norm<T, 16>(h, V, k, z, gn, s); break;
  }
  LAUNCHCHK();
  return KRCN_OK;
}

// Make the partials `*p` (*P entries) global across ranks when the reduced
// space is sharded: collapse them to one scalar in h->scal[slot], all-reduce
// it there, and point the consumer at it (*p = that slot, *P = 1).
static krcn_status globalise(krcn_csr* h, double** p, int* P, int slot, hipStream_t s) {
  hipLaunchKernelGGL((k_finish<0>), dim3(1), dim3(kNT), 0, s, *p, *P, h->scal + slot);
  LAUNCHCHK();
  CHK(allreduce(h, h->scal + slot, 1, KRCN_F64, s));
  *p = h->scal + slot;
  *P = 1;
  return KRCN_OK;
}

// krcn_csr_set_graph(h, 1) replays repeated Lanczos calls as a hipGraph.
// Off by default: interleaved A/B on the box (profiles/
// r02_graph_ab.txt) measured rcv1 and rcv1_stress equal, w8a within its noise
// and news20 7-8 % slower under replay than the eager stream launches.

static uint64_t bits(double x) {
  uint64_t b;
  std::memcpy(&b, &x, sizeof(b));
  return b;
}

// A/B knob KRCN_PACK_NORM=0: column shards keep the separate ||z||^2 all-reduce
// (and so the two-collective step)
static bool pack_env_ok() {
  static const bool v = [] {
    const char* e = tuning_env("KRCN_PACK_NORM");
    return !(e && e[0] == '0');
  }();
  return v;
}

template <typename T>
static krcn_status lanczos_impl(krcn_csr* h, const T* w, const T* g, int m, int reorth, double tol,
                                double l2, T* V, double* alphas_host, double* betas_host,
                                krcn_lanczos_info* info, hipStream_t s_call) {
  hipStream_t s = s_call;   // the capture stream while a graph is being recorded
  const int64_t d = h->d, n = h->n;
  CHK(plans_for_compute(h));
  CHK(check_lanczos_ws(h, m, reorth));
  const bool dshard = h->shard == KRCN_SHARD_COLS;  // d-space dots need a rank sum
  const bool rows = h->shard == KRCN_SHARD_ROWS;
  const bool cols = h->shard == KRCN_SHARD_COLS;
  // Step B fused into the next pass 1: LDS-window slices plans, unsharded, no
  // reorthogonalisation.
  static const bool fuse_env = [] {
    const char* e = tuning_env("KRCN_LANCZOS_FUSE");   // A/B knob: 0 keeps the separate step B
    return !(e && e[0] == '0');
  }();
  const bool fuse_win = h->p1.win && !h->p1.accum && h->p1.grid % h->p1.S == 0;
  const bool fuse_sorted = !h->p1.win && !h->p1.jag && h->p1.sorted && h->p1.S > 1;
  const bool fuse_small = h->p1.win && h->p1.accum && h->p1.S == 1 && d <= kWinNT;
  static const bool zw_env = [] {
    const char* e = tuning_env("KRCN_ZW");   // A/B knob: 0 keeps pass 1's store of z_j
    return !(e && e[0] == '0');
  }();
  const bool fuse = fuse_env && h->shard == KRCN_SHARD_NONE && !reorth && (fuse_win || fuse_sorted || fuse_small) &&
                    h->p1.grid <= h->pcap;
  // one-piece plans with per-block X^T copies: pass 2 folds into pass 1 plus
  // the partials' combine (A/B knob KRCN_XT_SMALL=0 keeps the X^T pass)
  static const bool xt_env = [] {
    const char* e = tuning_env("KRCN_XT_SMALL");
    return !(e && e[0] == '0');
  }();
  const bool xt_small = fuse && fuse_small && h->p1.xt && xt_env && h->p1.grid <= h->pcap;
  // Two launches per step for plans whose pass 1 is unsliced sorted tiles and
  // pass 2 a single-window jagged pass: pass 1 with step B fused stores
  // u' = w (.) X z_j, and pass 2 settles beta in every block's prologue and
  // gathers u = u' / beta (SrcLzU), where the plain path would run a
  // separate step B.  No BASELINE config gets such a plan by default (the
  // plan policy that would give rcv1 one lost, krcn_plan.hip ensure_plans);
  // krcn_csr_set_pass_format reaches it.  (A/B knob KRCN_LZ2=0: off.)
  static const bool lz2_env = [] {
    const char* e = tuning_env("KRCN_LZ2");
    return !(e && e[0] == '0');
  }();
  const bool fuse_u = fuse_env && lz2_env && h->shard == KRCN_SHARD_NONE && !reorth && h->p1.sorted && !h->p1.win &&
                      !h->p1.jag && h->p1.S == 1 && h->p2.jag && h->p2.S == 1 && h->p1.grid <= h->pcap;
  // Early alpha (window-slices or sliced sorted-tile pass 1; krcn_kernels.hpp
  // EpiLz2E): the slice combine also forms the partials of (X v_j).(w X v_j),
  // pass 2 settles alpha_j from them in its prologue and runs step B in its
  // epilogue (z_{j+1} into V[j+1]), so pass 1 gathers the stored z_j alone
  // instead of forming it from w and v_{j-1}.  Pass 2 must reduce two sums
  // per block (Red2): the single-window and one-group accumulate jagged
  // passes and the accumulate window pass do.  (A/B knob KRCN_LZ_EARLY=0:
  // the fused window step of rounds 2-4.)
  static const bool early_env = [] {
    const char* e = tuning_env("KRCN_LZ_EARLY");
    return !(e && e[0] == '0');
  }();
  const bool p2_red2 = (h->p2.jag && (h->p2.S == 1 || h->p2.jG == 1)) || (h->p2.win && h->p2.accum);
  // window-slices (news20) and sliced sorted-tile (rcv1) pass-1 plans: the
  // early step replaces their fused step B (pass 1 then gathers one vector
  // instead of forming z = w - alpha v from two)
  const bool early = fuse && (fuse_win || fuse_sorted) && early_env && p2_red2 && h->pq;
  // Row shards (synth on 8 GPUs), fp64: the same early alpha with the
  // d-vector all-reduce carrying the rank's partials of (X v_j).(w X v_j)
  // past element d, so the row apply after it settles alpha_j and runs steps A and
  // B in one launch (EpiLz2E: v_j, z_{j+1}, their partials) — no k_lz_step_b
  // and no W round trip.  The z_j . v_{j-1} partials are d-space, replicated
  // on every rank.  (A/B knob KRCN_LZ_EARLY=0 as above.)
  // Every rank must issue the same collectives with the same lengths: with a
  // multi-rank communicator the gate and the packed partial count (Pc) are the
  // values the ranks agreed on after the plan build (agree_rows: the maximum
  // over ranks; a rank whose combine writes fewer zero-fills the rest).
  const bool multi = h->comm && h->comm->nranks > 1;
  const int pq_local = pass_partials(h->p1);
  const int Pc = multi ? h->rows_pq : pq_local;
  const bool rows_fit = multi ? h->rows_early != 0 : std::max(h->p1.grid, h->p1.combine_grid) <= kMaxPartials;
  if (rows && multi && h->rows_pq < 0)
    return fail(KRCN_ERR_INVALID, "krcn_lanczos: the row shards have not agreed on their plans (krcn_csr_reserve "
                "or krcn_csr_attach_comm on every rank)");
  const bool early_rows = rows && std::is_same<T, double>::value && !reorth && early_env && rows_fit &&
                          Pc >= pq_local && Pc <= kMaxPartials;
  // Column shards (news20 on 8 GPUs), fp64: one collective per step.  The row
  // sums t = X z_j are all-reduced with this rank's ||z_p||^2 and z_p . v_p
  // packed as elements n and n + 1; the row apply (replicated over n on every
  // rank) settles beta and forms u with the partials of u.q, which are then
  // the same on every rank — so pass 2 settles alpha_j in its prologue
  // (SrcLzAlpha) and runs steps A and B in its epilogue (EpiLz2E) with no
  // scalar all-reduce and no step-B launch.
  const bool early_cols = cols && std::is_same<T, double>::value && !reorth && early_env && pack_env_ok() &&
                          apply_grid(n) <= h->pcap;
  T* W = static_cast<T*>(h->W);
  T* u = static_cast<T*>(h->u);

  // The launch sequence below depends only on the arguments, the plans and
  // the handle's buffers, so unsharded, unprofiled calls replay it as one
  // hipGraph: recorded on the handle's private stream the second time the same
  // arguments arrive, launched on the caller's stream from then on (one
  // submission per call instead of 2-4 dependent launches per Lanczos step).
  const bool graph = h->graph && h->shard == KRCN_SHARD_NONE && !h->prof;
  const uint64_t key[krcn_csr::kGraphKey] = {uint64_t(uintptr_t(w)), uint64_t(uintptr_t(g)), uint64_t(uintptr_t(V)),
                                             uint64_t(uintptr_t(W)), uint64_t(m), uint64_t(reorth), bits(tol),
                                             bits(l2), h->ws_gen, uint64_t(sizeof(T))};
  bool replay = false, capture = false;
  if (graph) {
    replay = h->gexec && std::equal(key, key + krcn_csr::kGraphKey, h->gkey);
    capture = !replay && std::equal(key, key + krcn_csr::kGraphKey, h->glast);
    std::copy(key, key + krcn_csr::kGraphKey, h->glast);
  }
  auto enqueue = [&]() -> krcn_status {
  LzCtl<T> c{V, g, d, m, 0, 0, h->st, h->betas_dev, h->pb, 0, tol};

  // start (cubic.py:85): zero alphas / betas, partials of ||g||^2 (pass 1 or
  // the combine of step 0 finishes the norm)
  int Pn = vec_grid(d);
  hipLaunchKernelGGL((k_lz_begin<T>), dim3(Pn), dim3(kNT), 0, s, d, g, m, h->alphas_dev, h->betas_dev, h->pb);
  LAUNCHCHK();
  double* pn = h->pb;
  if (dshard) CHK(globalise(h, &pn, &Pn, 1, s));
  c.pnorm = pn;
  c.Pnorm = Pn;
  double* pa_g = h->pa;   // v.w partials as the consumers read them (globalise may redirect)
  const T tn = T(h->n_global), tl2 = T(l2);

  // Column shards, fp64, no reorthogonalisation: ||z_{j+1}||^2 of step B
  // travels as element n of the next row-sum all-reduce instead of an
  // all-reduce of its own (2 collectives per step instead of 3).  Pass 1 then
  // gathers z unnormalised without the beta prologue (SrcGuard), and the row
  // apply after the all-reduce runs it (SrcLzStep: beta, the breakdown test,
  // the state) from u[n].  The last loop step keeps the scalar all-reduce:
  // k_lz_final_check reads that norm.
  static const bool pack_env = [] {
    const char* e = tuning_env("KRCN_PACK_NORM");   // A/B knob: 0 keeps the separate all-reduce
    return !(e && e[0] == '0');
  }();
  const bool pack = cols && std::is_same<T, double>::value && !reorth && pack_env;
  bool packed = false;   // u[n] holds this rank's ||z_j||^2 for the coming step
  double* const unorm = static_cast<double*>(h->u) + n;

  // One HVP + step A on the step's vector; partials of v.w land in h->pa.
  auto hvp_step = [&](int mode, int* Pa) -> krcn_status {
    c.mode = mode;
    ProfRec* pr = prof_next(h);
    if (pr) HIPCHK(hipEventRecord(pr->e0, s));
    const SrcLzState<T> later{c, {}};
    if (cols && mode == 0 && packed) {
      const SrcGuard<T> zsrc{V + int64_t(c.j) * d, h->st, 0};
      CHK(run_pass<T>(h->p1, zsrc, zsrc, EpiStore<T>{u}, nullptr, nullptr, s, pr));
      CHK(allreduce(h, u, n + 1, h->dtype, s));
      LzCtl<T> cp = c;
      cp.pnorm = unorm;
      cp.Pnorm = 1;
      hipLaunchKernelGGL((k_rows_apply<T, SrcLzStep<T>, EpiLz1<T>>), dim3(apply_grid(n)), dim3(kNT), 0, s, int(n),
                         static_cast<const T*>(u), SrcLzStep<T>{cp, {}}, EpiLz1<T>{w, u, T(1)},
                         static_cast<double*>(nullptr));
      LAUNCHCHK();
    } else if (cols) {
      // raw X_p z_p, all-reduced, then u = w (t / div)
      if (mode == 0) CHK(run_pass<T>(h->p1, SrcLzStep<T>{c, {}}, later, EpiStore<T>{u}, nullptr, nullptr, s, pr));
      else CHK(run_pass<T>(h->p1, later, later, EpiStore<T>{u}, nullptr, nullptr, s, pr));
      CHK(allreduce(h, u, n, h->dtype, s));
      hipLaunchKernelGGL((k_rows_apply<T, SrcLzState<T>, EpiLz1<T>>), dim3(apply_grid(n)), dim3(kNT), 0, s, int(n),
                         static_cast<const T*>(u), later, EpiLz1<T>{w, u, T(1)}, static_cast<double*>(nullptr));
      LAUNCHCHK();
    } else if (mode == 0) {
      CHK(run_pass<T>(h->p1, SrcLzStep<T>{c, {}}, later, EpiLz1<T>{w, u, T(1)}, nullptr, nullptr, s, pr));
    } else {
      CHK(run_pass<T>(h->p1, later, later, EpiLz1<T>{w, u, T(1)}, nullptr, nullptr, s, pr));
    }
    if (pr) HIPCHK(hipEventRecord(pr->e1, s));
    const SrcGuard<T> src2{u, h->st, mode};
    EpiLz2<T> e2{};
    e2.c = c; e2.W = W; e2.n = tn; e2.l2 = tl2;
    if (rows) {
      // the raw X_p^T u_p partial is all-reduced before step A runs
      T* raw = static_cast<T*>(h->td);
      CHK(run_pass<T>(h->p2, src2, src2, EpiStore<T>{raw}, nullptr, nullptr, s));
      CHK(allreduce(h, raw, d, h->dtype, s));
      const int Pe = apply_grid(d);
      hipLaunchKernelGGL((k_rows_apply<T, SrcGuard<T>, EpiLz2<T>>), dim3(Pe), dim3(kNT), 0, s, int(d),
                         static_cast<const T*>(raw), src2, e2, h->pa);
      LAUNCHCHK();
      *Pa = Pe;
    } else {
      CHK(run_pass<T>(h->p2, src2, src2, e2, h->pa, Pa, s));
    }
    if (pr) HIPCHK(hipEventRecord(pr->e2, s));
    pa_g = h->pa;
    if (dshard) CHK(globalise(h, &pa_g, Pa, 2, s));
    return KRCN_OK;
  };

  // Step B fused into the next pass 1 (fuse, above): pass 1 of step j builds
  // z_j = w - alpha_{j-1} v_{j-1} in its windows (SrcLzZ), the slice combine
  // settles beta_{j-1}; the last loop step keeps the separate step B
  // (k_lz_final_check and the final quotient read its z_{m-1} and norm partials).
  int Pa_prev = 0;
  for (int j = 0; j + 1 < m; ++j) {
    c.j = j;
    int Pa = 0;
    if (early) {
      // pass 1 (SrcLzBeta: block 0 settles beta_{j-1} from pass 2's ||z_j||^2
      // partials, the breakdown test) over z_j, the combine (u, alpha partials), pass 2
      // (alpha_j; v_j, z_{j+1}, their partials).  The z.v partials alternate
      // between pa and pz: pass 2 of step j reads step j-1's while it writes.
      c.mode = 0;
      ProfRec* pr = prof_next(h);
      if (pr) HIPCHK(hipEventRecord(pr->e0, s));
      int Pq = 0;
#if KRCN_FOLD
      if (std::is_same<T, double>::value && fold_ok(h)) {   // the slice combine folded into pass 1
        EpiSliceFold<T> ef{static_cast<T*>(h->p1.part), int64_t(h->p1.rows), h->fcnt, h->fcnt + int64_t(h->p1.ntiles) * kFoldPad,
                           nullptr, h->p1.ntiles, h->pq, w, u, c, h->p1.S};
        CHK(run_fold_pass1<T>(h, SrcLzBeta<T>{c, {}}, ef, s));
        Pq = h->p1.ntiles;
      } else
#endif
      CHK(run_pass<T>(h->p1, SrcLzBeta<T>{c, {}}, SrcLzState<T>{c, {}}, EpiLz1A<T>{w, u, T(1)}, h->pq, &Pq, s, pr));
      if (pr) HIPCHK(hipEventRecord(pr->e1, s));
      double* zv_out = (j & 1) ? h->pz : h->pa;
      const double* zv_in = (j & 1) ? h->pa : h->pz;
      const SrcLzAlpha<T> asrc{u, h->st, h->pq, Pq, zv_in, Pa_prev, h->alphas_dev, j, double(h->n_global), l2};
      EpiLz2E<T> e2{};
      e2.c = c; e2.n = tn; e2.l2 = tl2; e2.part2 = zv_out;
      CHK(run_pass<T>(h->p2, asrc, asrc, e2, h->pb, &Pa, s));
      if (pr) HIPCHK(hipEventRecord(pr->e2, s));
      Pa_prev = Pa;
      c.pnorm = h->pb;   // ||z_{j+1}||^2: the next pass 1, or the final check
      c.Pnorm = Pa;
      continue;
    }
    if (early_cols) {
      c.mode = 0;
      ProfRec* pr = prof_next(h);
      if (pr) HIPCHK(hipEventRecord(pr->e0, s));
      // (j = 0 runs unguarded: the state still holds the previous call's
      // flag until the row apply's prologue resets it)
      const SrcGuard<T> zsrc{j == 0 ? g : V + int64_t(j) * d, h->st, j == 0 ? 1 : 0};
      if (j == 0) {
        CHK(run_pass<T>(h->p1, zsrc, zsrc, EpiStore<T>{u}, nullptr, nullptr, s, pr));
      } else {
        const SrcGuardPack<T> psrc{V + int64_t(j) * d, h->st, h->pb, h->pz, Pa_prev, unorm};
        CHK(run_pass<T>(h->p1, psrc, zsrc, EpiStore<T>{u}, nullptr, nullptr, s, pr));
      }
      // u[n] = ||z_p||^2, u[n + 1] = z_p . v_{p,j-1}: packed by pass 1's block 0
      // from the previous pass 2's partials (j = 0: ||g||^2 is already global)
      CHK(allreduce(h, u, n + (j == 0 ? 0 : 2), h->dtype, s));
      LzCtl<T> cp = c;
      if (j > 0) {
        cp.pnorm = unorm;
        cp.Pnorm = 1;
      }
      const int Pr = apply_grid(n);
      hipLaunchKernelGGL((k_rows_apply<T, SrcLzStep<T>, EpiLz1A<T>>), dim3(Pr), dim3(kNT), 0, s, int(n),
                         static_cast<const T*>(u), SrcLzStep<T>{cp, {}}, EpiLz1A<T>{w, u, T(1)}, h->pq);
      LAUNCHCHK();
      if (pr) HIPCHK(hipEventRecord(pr->e1, s));
      const SrcLzAlpha<T> asrc{u, h->st, h->pq, Pr, unorm + 1, 1, h->alphas_dev, j, double(h->n_global), l2};
      EpiLz2E<T> e2{};
      e2.c = c; e2.n = tn; e2.l2 = tl2; e2.part2 = h->pz;
      CHK(run_pass<T>(h->p2, asrc, asrc, e2, h->pb, &Pa, s));
      if (pr) HIPCHK(hipEventRecord(pr->e2, s));
      if (j + 2 < m) {   // the next pass 1 packs the next all-reduce's two d-space sums
        c.pnorm = unorm;
        c.Pnorm = 1;
      } else {   // the final check reads ||z_{m-1}||^2 as a global sum
        double* pbp = h->pb;
        int Pb = Pa;
        CHK(globalise(h, &pbp, &Pb, 3, s));
        c.pnorm = pbp;
        c.Pnorm = Pb;
      }
      Pa_prev = Pa;
      continue;
    }
    if (early_rows) {
      c.mode = 0;
      ProfRec* pr = prof_next(h);
      if (pr) HIPCHK(hipEventRecord(pr->e0, s));
      // the combine's alpha partials land past the d-vector (td holds d +
      // kMaxPartials) and travel in the same all-reduce
      T* raw = static_cast<T*>(h->td);
      double* rq = reinterpret_cast<double*>(raw + d);
      int Pq = 0;
      CHK(run_pass<T>(h->p1, SrcLzStep<T>{c, {}}, SrcLzState<T>{c, {}}, EpiLz1A<T>{w, u, T(1)}, rq, &Pq, s, pr));
      if (pr) HIPCHK(hipEventRecord(pr->e1, s));
      if (Pq != pq_local)
        return fail(KRCN_ERR_INVALID, "krcn_lanczos: pass 1 wrote %d partials, the plan promised %d", Pq, pq_local);
      // slots [Pq, Pc) hold the previous all-reduce's sums on this rank: zero them
      if (Pc > Pq) HIPCHK(hipMemsetAsync(rq + Pq, 0, sizeof(double) * size_t(Pc - Pq), s));
      const SrcGuard<T> src2{u, h->st, 0};
      CHK(run_pass<T>(h->p2, src2, src2, EpiStore<T>{raw}, nullptr, nullptr, s));
      CHK(allreduce(h, raw, d + Pc, h->dtype, s));
      double* zv_out = (j & 1) ? h->pz : h->pa;
      const double* zv_in = (j & 1) ? h->pa : h->pz;
      const SrcLzAlpha<T> asrc{u, h->st, rq, Pc, zv_in, Pa_prev, h->alphas_dev, j, double(h->n_global), l2};
      EpiLz2E<T> e2{};
      e2.c = c; e2.n = tn; e2.l2 = tl2; e2.part2 = zv_out;
      const int Pe = apply_grid(d);
      hipLaunchKernelGGL((k_rows_apply<T, SrcLzAlpha<T>, EpiLz2E<T>>), dim3(Pe), dim3(kNT), 0, s, int(d),
                         static_cast<const T*>(raw), asrc, e2, h->pb);
      LAUNCHCHK();
      if (pr) HIPCHK(hipEventRecord(pr->e2, s));
      Pa_prev = Pe;
      c.pnorm = h->pb;   // ||z_{j+1}||^2: the next pass 1, or the final check
      c.Pnorm = Pe;
      continue;
    }
    if (fuse_u) {
      c.mode = 0;
      ProfRec* pr = prof_next(h);
      if (pr) HIPCHK(hipEventRecord(pr->e0, s));
      const SrcLzZ<T> zsrc{c, static_cast<const T*>(W), h->pa, Pa_prev, h->alphas_dev, h->pz, T(0), 1};
      CHK(run_pass<T>(h->p1, zsrc, zsrc, EpiWeighted<T>{w, u}, nullptr, nullptr, s, pr));
      if (pr) HIPCHK(hipEventRecord(pr->e1, s));
      LzCtl<T> cb = c;
      if (j > 0) {   // z_j's norm partials: the pass-1 blocks that stored it
        cb.pnorm = h->pz;
        cb.Pnorm = std::min(h->p1.grid, kNT);
      }
      const SrcLzU<T> usrc{cb, u, {}};
      EpiLz2<T> e2{};
      e2.c = c; e2.W = W; e2.n = tn; e2.l2 = tl2;
      CHK(run_pass<T>(h->p2, usrc, usrc, e2, h->pa, &Pa, s));
      if (pr) HIPCHK(hipEventRecord(pr->e2, s));
    } else if (fuse) {
      c.mode = 0;
      ProfRec* pr = prof_next(h);
      if (pr) HIPCHK(hipEventRecord(pr->e0, s));
      LzCtl<T> cb = c;
      if (j > 0) {
        cb.pnorm = h->pz;
        cb.Pnorm = fuse_win ? h->p1.grid : std::min(h->p1.grid, kNT);   // z writers of the sorted pass
      }
      if (fuse_small) {
        const SrcLzSmall<T> zs{c, static_cast<const T*>(W), h->pa, Pa_prev, h->alphas_dev, {}};
        if (xt_small) {   // pass 1 also forms the blocks' shares of X^T u (EpiLz1X)
          const EpiLz1X<T> ex{w, T(1), h->p1.xcp, h->p1.xrow, static_cast<const T*>(h->p1.xval),
                              static_cast<T*>(h->p1.xpart), int(d), nullptr, 0};
          CHK(run_pass<T>(h->p1, zs, zs, ex, nullptr, nullptr, s, pr));
        } else {
          CHK(run_pass<T>(h->p1, zs, zs, EpiLz1<T>{w, u, T(1)}, nullptr, nullptr, s, pr));
        }
      } else {
        // window-slices pass 1 stores no z_j: pass 2 re-forms it (EpiLz2::zw)
        const SrcLzZ<T> zsrc{c, static_cast<const T*>(W), h->pa, Pa_prev, h->alphas_dev, h->pz, T(0),
                             fuse_win && zw_env ? 0 : 1};
        CHK(run_pass<T>(h->p1, zsrc, SrcLzStep<T>{cb, {}}, EpiLz1<T>{w, u, T(1)}, nullptr, nullptr, s, pr));
      }
      if (pr) HIPCHK(hipEventRecord(pr->e1, s));
      const SrcGuard<T> src2{u, h->st, 0};
      EpiLz2<T> e2{};
      e2.c = c; e2.W = W; e2.n = tn; e2.l2 = tl2;
      if (fuse_win && zw_env) {
        e2.alphas = h->alphas_dev;
        e2.zw = 1;
      }
      if (xt_small) {
        // pass 2 = the blocks' X^T u partials added in k_slice_combine's fixed
        // order, with step A in its epilogue
        static const bool xt_comb_env = [] {   // A/B knob: 0 uses k_slice_combine
          const char* e = tuning_env("KRCN_XT_COMB");
          return !(e && e[0] == '0');
        }();
        static const int xt_rb = [] {   // A/B knob: rows per combine block (16 / 32 / 64)
          const char* e = tuning_env("KRCN_XT_RB");
          const int v = e ? atoi(e) : kXtCombineRows;
          return v == 16 || v == 64 ? v : 32;
        }();
        if (xt_comb_env) {
          const int cg = int((d + xt_rb - 1) / xt_rb);
          const T* xp = static_cast<const T*>(h->p1.xpart);
          if (xt_rb == 16)
            hipLaunchKernelGGL((k_xt_combine<T, SrcGuard<T>, EpiLz2<T>, 16>), dim3(cg), dim3(kCombineNT), 0, s,
                               int(d), h->p1.grid, xp, src2, e2, h->pa);
          else if (xt_rb == 64)
            hipLaunchKernelGGL((k_xt_combine<T, SrcGuard<T>, EpiLz2<T>, 64>), dim3(cg), dim3(kCombineNT), 0, s,
                               int(d), h->p1.grid, xp, src2, e2, h->pa);
          else
            hipLaunchKernelGGL((k_xt_combine<T, SrcGuard<T>, EpiLz2<T>, 32>), dim3(cg), dim3(kCombineNT), 0, s,
                               int(d), h->p1.grid, xp, src2, e2, h->pa);
          Pa = cg;
        } else {
          const int cg = combine_grid(int(d));
          hipLaunchKernelGGL((k_slice_combine<T, SrcGuard<T>, EpiLz2<T>>), dim3(cg), dim3(kCombineNT), 0, s, int(d),
                             h->p1.grid, combine_rows(int(d)), static_cast<const T*>(h->p1.xpart), src2, e2, h->pa);
          Pa = cg;
        }
        LAUNCHCHK();
      } else {
        CHK(run_pass<T>(h->p2, src2, src2, e2, h->pa, &Pa, s));
      }
      if (pr) HIPCHK(hipEventRecord(pr->e2, s));
    } else {
      CHK(hvp_step(0, &Pa));
    }
    Pa_prev = Pa;
    if ((fuse || fuse_u) && j + 2 < m) continue;
    c.mode = 0;
    int Pb = vec_grid(d);
    T* zn = V + int64_t(j + 1) * d;
    // round 4: a reorthogonalised step on the 1 KiB-piece CGS2 path forms
    // step B inside its first sweep (k_cgs_rowdots_vb): no k_lz_step_b launch
    // (tuning knob KRCN_CGS_FUSEB=0 keeps the launch)
    static const bool fuseb_env = [] {
      const char* e = tuning_env("KRCN_CGS_FUSEB");
      return !(e && e[0] == '0');
    }();
    const bool fuse_b = reorth && fuseb_env && cgs_vec_ok<T>(h, V, zn, dshard, j + 1);
    if (!fuse_b) {
      hipLaunchKernelGGL((k_lz_step_b<T>), dim3(Pb), dim3(kNT), 0, s, d, static_cast<const T*>(W), c, pa_g, Pa,
                         h->alphas_dev, h->pb);
      LAUNCHCHK();
    }
    if (reorth) {
      const CgsStepB<T> sb{static_cast<const T*>(W), pa_g, Pa};
      CHK(reorth_cgs2<T>(h, V, j + 1, zn, dshard, &Pb, s, fuse_b ? &sb : nullptr));
    }
    packed = false;
    double* pbp = h->pb;
    if (pack && j + 2 < m) {
      hipLaunchKernelGGL((k_finish<0>), dim3(1), dim3(kNT), 0, s, h->pb, Pb, unorm);
      LAUNCHCHK();
      packed = true;
    } else if (dshard) {
      CHK(globalise(h, &pbp, &Pb, 3, s));
    }
    c.pnorm = pbp;
    c.Pnorm = Pb;
  }
  {
    c.mode = 1;
    hipLaunchKernelGGL((k_lz_final_check<T>), dim3(1), dim3(kNT), 0, s, c);
    LAUNCHCHK();
    int Pa = 0;
    CHK(hvp_step(1, &Pa));
    hipLaunchKernelGGL((k_lz_final<T>), dim3(vec_grid(d)), dim3(kNT), 0, s, pa_g, Pa, c, h->alphas_dev,
                       h->hostres_dev);
    LAUNCHCHK();
  }
  return KRCN_OK;
  };
  bool lzp_timed = false;
  if (replay) {
    HIPCHK(hipGraphLaunch(h->gexec, s_call));
  } else if (capture) {
    if (!h->gstream) HIPCHK(hipStreamCreateWithFlags(&h->gstream, hipStreamNonBlocking));
    HIPCHK(hipStreamBeginCapture(h->gstream, hipStreamCaptureModeThreadLocal));
    s = h->gstream;
    const krcn_status r = enqueue();
    hipGraph_t gr = nullptr;
    const hipError_t e = hipStreamEndCapture(h->gstream, &gr);
    s = s_call;
    if (r != KRCN_OK || e != hipSuccess) {
      if (gr) (void)hipGraphDestroy(gr);
      CHK(r);
      HIPCHK(e);
    }
    if (h->gexec) (void)hipGraphExecDestroy(h->gexec);
    h->gexec = nullptr;
    const hipError_t ei = hipGraphInstantiate(&h->gexec, gr, nullptr, nullptr, 0);
    (void)hipGraphDestroy(gr);
    if (ei != hipSuccess) h->gexec = nullptr;
    HIPCHK(ei);
    std::copy(key, key + krcn_csr::kGraphKey, h->gkey);
    HIPCHK(hipGraphLaunch(h->gexec, s_call));
  } else {
    bool timed = false;   // a call of the placement search (krcn_plan.hip lzp_*)
    CHK(lzp_begin(h, m, s, &timed));
    CHK(enqueue());
    CHK(lzp_end(h, s, timed));
    lzp_timed = timed;
  }
  // the recurrence results: k_lz_final packed the state, alphas[0..m) and
  // betas[0..m-1) straight into the mapped host block (no copy launch)
  const double* hb = h->hostres;
  if (2 * m + 3 > kLzOut) return fail(KRCN_ERR_UNSUPPORTED, "krcn_lanczos: m > 2044 not supported");
  HIPCHK(hipStreamSynchronize(s));
  CHK(lzp_done(h, lzp_timed));
  LanczosState stc;
  std::memcpy(&stc, hb, sizeof(LanczosState));
  const bool trunc = stc.done && stc.j_break < m - 2;
  const int m_eff = trunc ? stc.j_break + 1 : m;
  for (int i = 0; i < m; ++i) alphas_host[i] = i < m_eff ? hb[4 + i] : 0.0;
  for (int i = 0; i + 1 < m; ++i) betas_host[i] = i < m_eff - 1 ? hb[4 + m + i] : 0.0;
  info->m_eff = m_eff;
  info->breakdown = stc.done;
  info->j_break = stc.done ? stc.j_break : -1;
  info->hvps = (stc.done ? stc.j_break + 1 : (m - 1)) + 1;
  info->beta_last = stc.beta_last;
  info->gnorm = stc.gnorm;
  return KRCN_OK;
}

