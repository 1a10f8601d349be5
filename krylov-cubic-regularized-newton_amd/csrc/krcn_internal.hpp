// krcn_internal.hpp — shared host-side internals of libkrcn.so (not part of the ABI).
//
// The library is split into translation units that compile in parallel:
//   krcn_plan.hip        handle lifecycle, transposed CSR, pass plans, comm, profiling
//   krcn_ops.hip         objective pieces (Ax, X^T u, weights, HVP, gradient, loss, dots)
//   krcn_lanczos_f64.hip / krcn_lanczos_f32.hip
//                        the device Lanczos recurrence (krcn_lanczos_impl.hpp), one dtype each
// This header holds the handle layout, the error macros and the pass launcher
// (run_pass) that the kernels of every unit are instantiated through.
#pragma once
#include "krcn.h"
#include "krcn_host.hpp"
#include "krcn_rendezvous.hpp"
#include "krcn_kernels.hpp"
#include "krcn_tiled.hpp"
#include "krcn_window.hpp"
#include "krcn_jag.hpp"
#include "krcn_cg.hpp"
#include "krcn_cgs2.hpp"

#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <mutex>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>
#include <type_traits>
#include <vector>

using namespace krcn;

// A/B tuning knobs (the variants of DESIGN.md's measurements) are read from
// the environment only in tuning builds (make variant EXTRA_FLAGS=-DKRCN_TUNING);
// the product library runs the measured defaults whatever the environment holds.
inline const char* tuning_env(const char* name) {
#ifdef KRCN_TUNING
  return getenv(name);
#else
  (void)name;
  return nullptr;
#endif
}

// CGS2 colsweep shape (krcn_cgs2.hpp k_cgs_colsweep): rows per wave and batch
// past k = 4 U (tuning knob KRCN_CGS_COLU) and batches per block (KRCN_CGS_NB);
// a block's row range is 4 U NB rows (default 8 x 8 x 4 = 256).  The range
// count of a sweep over k rows sizes the row-range partials (reserve_reorth).
inline int cgs_umax() {
  static const int v = [] {
    const char* e = tuning_env("KRCN_CGS_COLU");
    return e && std::atoi(e) >= 2 ? std::atoi(e) : 8;
  }();
  return v;
}
inline int cgs_nb() {
  static const int v = [] {
    const char* e = tuning_env("KRCN_CGS_NB");
    const int x = e ? std::atoi(e) : 8;
    return x == 1 || x == 2 || x == 4 || x == 16 ? x : 8;
  }();
  return v;
}
inline int cgs_col_ranges(int k) {
  const int rows = 4 * cgs_col_unroll(k, cgs_umax()) * cgs_nb();
  return (k + rows - 1) / rows;
}
// chunks of k_cgs_rowdots_v over a row of nv 16-byte vectors
inline int cgs_rdv_chunks_of(int64_t nv) { return cgs_rdv_chunks(nv, cgs_rdv_steps(nv, 0)); }

#define HIPCHK(call)                                                                    \
  do {                                                                                  \
    hipError_t e_ = (call);                                                             \
    if (e_ != hipSuccess)                                                               \
      return fail(KRCN_ERR_HIP, "%s:%d %s -> %s", __FILE__, __LINE__, #call,            \
                  hipGetErrorString(e_));                                               \
  } while (0)

#define NCCLCHK(call)                                                                   \
  do {                                                                                  \
    ncclResult_t r_ = (call);                                                           \
    if (r_ != ncclSuccess)                                                              \
      return fail(KRCN_ERR_RCCL, "%s:%d %s -> %s", __FILE__, __LINE__, #call,           \
                  ncclGetErrorString(r_));                                              \
  } while (0)

#define CHK(expr)                             \
  do {                                        \
    krcn_status s_ = (expr);                  \
    if (s_ != KRCN_OK) return s_;             \
  } while (0)

#define LAUNCHCHK() HIPCHK(hipGetLastError())

// ----------------------------------------------------------------- handles
struct VirtualGroup;   // krcn_plan.hip: the ranks of a virtual communicator
constexpr int kVirtualMaxRanks = 16;
constexpr int kVirtualTimeoutS = 90;    // a rank that never arrives breaks the group after this (under
                                        // the GPU box's 180 s silence limit: a stall fails, not hangs)
struct VirtualBufs {
  void* p[kVirtualMaxRanks];
};
struct krcn_comm {
  ncclComm_t comm = nullptr;
  int nranks = 1, rank = 0, device = 0;
  VirtualGroup* vg = nullptr;   // virtual ranks on one device (krcn_comm_create_virtual), else RCCL
  uint64_t seq = 0;             // all-reduces this rank has entered (virtual ranks: the timeout report)
};

// Largest Lanczos m: the alphas | betas | state block is allocated for it in
// krcn_csr_create, and comes back through the 4096-double pinned staging buffer.
constexpr int kLzMaxM = 2044;
// the packed results block k_lz_final writes after alphas | betas | state: the
// state (4 doubles), alphas[0..m), betas[0..m-1) — one D2H of 2 m + 3 doubles
// per call (round 4 copied the whole 2 kLzMaxM + 4: 32 KB per call, the copy
// path of a large transfer, on w8a's 10-HVP calls)
constexpr int kLzOut = 2 * kLzMaxM + 4;

// Handle construction and plan builds hold this process-wide lock: they
// allocate, free temporaries (hipFree synchronises the whole device) and sort
// with hipCUB, and a virtual-rank test builds 8 handles from 8 threads.
std::mutex& build_mutex();

// All-reduce of a virtual communicator: every rank's host thread drains its
// stream, the last to arrive sums the ranks' buffers in rank order on the
// device and writes the sum back to each of them (krcn_plan.hip).
krcn_status virtual_allreduce(krcn_comm* c, void* buf, int64_t count, int dtype, hipStream_t s);

struct ProfRec {
  hipEvent_t e0, e1, e2;
  hipEvent_t em;        // between pass 1's main launch and its slice combine
  bool mid = false;
};

// Execution plan of one SpMV direction (pass 1: X, pass 2: X^T).
struct PassPlan {
  int S = 1, groups = 1, L = 1, grid = 1, combine_grid = 1, ntiles = 0;
  int rows = 0;
  int64_t cols = 0, nnz = 0;
  const int* ptr = nullptr;   // flattened slice-major row pointers (S * rows + 1)
  const int* idx = nullptr;
  const void* val = nullptr;
  int* own_ptr = nullptr;     // owned copies when sliced
  int* own_idx = nullptr;
  void* own_val = nullptr;
  TileDesc* tiles = nullptr;
  int* tbeg = nullptr;        // groups + 1 tile offsets
  void* part = nullptr;       // S * rows partial row sums (sliced)
  int sorted = 0;             // sorted block tiles (k_sorted_pass) instead of wave tiles
  int sort_nt = 256;          // sorted tiles: threads per block (tile = kSortPerThread x sort_nt nonzeros)
  int* tmid = nullptr;        // sorted tiles: first single-long-row tile of each group
  unsigned* gword = nullptr;  // sorted tiles: (column - tile base) << kSortSlotBits | CSR slot
  void* gval = nullptr;       //               value, same (tile-sorted) order
  int win = 0;                // LDS-window format (k_window_pass)
  int accum = 0;              //   1: every block walks all slices of its tile range (no partials)
  int R = 64;                 //   rows per tile (one lane per row)
  int W = 0;                  //   slice width (window entries)
  int stride = 1;             //   segment slots per block
  int kpb = 0;                //   slices mode: blocks per slice when not a power of two (0: block = slice + S chunk)
  int nseg = 0;
  unsigned short* widx = nullptr;  // slice-local 16-bit column offsets (slice-major CSR order)
  WinSeg* segs = nullptr;     // per-block segment lists: block b runs segs[b * stride + i]
  int* tb = nullptr;          // compact row pointers: tile bases (S x (ntiles + 1))
  unsigned short* ro = nullptr;   //   row ends relative to the tile base (S x rows)
  int jag = 0;                // jagged lane-per-row format (k_jag_pass; S, W, widx, own_val, grid)
  int jK = 0;                 //   groups per wave (units per wave and slice)
  int jG = 1, jSg = 1;        //   accumulate: slice groups, slices per group
  int* jgcut = nullptr;       //   group cuts per block (grid + 1)
  int* jumeta = nullptr;      //   per (block, slice, wave): K unit bases, K unit sizes
  unsigned char* jcnt = nullptr;  // per unit: lane counts
  int jlong = 0, jlpiece = 0;     //   single window: long rows (JagArgs), LDS piece of their partials
  int* jlcut = nullptr;       //     per block: long rows, then tasks (2 x (grid + 1))
  int* jlrow = nullptr;       //     per long row: row id
  int* jltask = nullptr;      //     per long row: first task (+ 1 end entry)
  int* jtask = nullptr;       //     per task: element start, element count
  unsigned short* jlidx = nullptr;
  void* jlval = nullptr;
  int xt = 0;                 // one-piece window-accum X: per-block X^T copies (EpiLz1X)
  int* xcp = nullptr;         //   per block: cols + 1 absolute column offsets
  unsigned short* xrow = nullptr;  //   row offsets in the block's rows, column-major per block
  void* xval = nullptr;
  void* xpart = nullptr;      //   per block X^T u partials (grid x cols)
  size_t owned = 0;
  int64_t pcap = 0;           // entries of the handle's partials buffers (ensure_plans)
};

struct krcn_csr {
  int device = 0, dtype = KRCN_F64, shard = KRCN_SHARD_NONE;
  size_t vs = 8;
  int64_t n = 0, d = 0, nnz = 0, n_global = 0;
  const int* ptr = nullptr;
  const int* idx = nullptr;
  const void* val = nullptr;
  int* tptr = nullptr;
  int* tidx = nullptr;
  void* tval = nullptr;
  int lanes_x = KRCN_LANES_AUTO, lanes_xt = KRCN_LANES_AUTO;
  int slicing = KRCN_SLICING_AUTO;
  int format = KRCN_FORMAT_AUTO;
  int format_pass[2] = {-1, -1};   // krcn_csr_set_pass_format (-1: the handle's format)
  int sort_nt = 0;            // sorted-tile block size; 0 = by matrix size
  bool plans_ready = false;
  bool p1_unsliced = false;   // pass 2 took a single-window jagged plan: pass 1's sorted tiles go
                              // unsliced (the two-launch Lanczos step, krcn_lanczos_impl.hpp)
  PassPlan p1, p2;            // pass 1 over X, pass 2 over X^T
  // workspace
  double* pa = nullptr;   // partials of reducing launches (pcap entries)
  double* pb = nullptr;   // second partials buffer
  double* scal = nullptr; // 16 device scalars (all-reduced dots, results)
  LanczosState* st = nullptr;
  void* u = nullptr;      // n-vector (w (.) Xv)
  void* tn = nullptr;     // n-vector scratch (raw partials, residual)
  void* W = nullptr;      // d-vector (Lanczos w)
  void* td = nullptr;     // d-vector scratch (raw partial X^T u)
  double* hostbuf = nullptr;  // pinned host staging
  double* hostres = nullptr;  // pinned host results block k_lz_final writes directly (no D2H copy)
  double* hostres_dev = nullptr;   //   its device-side address
  int mcap = 0;               // Lanczos m the alphas block holds (kLzMaxM, from krcn_csr_create)
  double* alphas_dev = nullptr;
  double* betas_dev = nullptr;
  double* hcoef = nullptr;    // reorth coefficients (mcap)
  double* pz = nullptr;       // per-slice partials of ||z||^2 (fused step B, pcap entries)
  double* pq = nullptr;       // early-alpha step: the combine's partials of (X v).(w (X v)) (pcap entries)
  int* fcnt = nullptr;        // slice-combine fold (KRCN_FOLD builds): per pass-1 tile, tickets drawn
  int64_t pcap = kMaxPartials;   // entries of pa / pb / pz: >= every reducing launch's grid
  double* pr = nullptr;       // CGS2 h1 partials (k_cgs_rowdots: column chunks x rows)
  double* pr2 = nullptr;      // CGS2 h2 partials (k_cgs_update_dots: column slabs x rows)
  double* cy = nullptr;       // CGS2 row-range partials of V^T h (k_cgs_colsweep: ranges x d)
  int* ccnt = nullptr;        //   its per column group arrival counters (zero between launches)
  int64_t pr_cap = 0;
  int64_t prv_cap = 0;        // entries of pr (the 1 KiB-piece path checks its C k chunk partials fit)
  int cy_q = 0;               // row ranges cy holds (0: not allocated; one range needs none)
  int reorth_m = 0;           // CGS2 workspace reserved for Lanczos m <= this (krcn_csr_reserve)
  void* cg_r = nullptr;       // CG vectors r | p | q (3 d-vectors, krcn_cg_solve)
  struct krcn::CgState* cg_st = nullptr;
  size_t owned = 0;
  krcn_comm* comm = nullptr;
  bool prof = false;
  std::vector<ProfRec> prof_pool;
  ProfRec* prof_cur = nullptr;   // run_pass records its em when set
  size_t prof_used = 0;
  // hipGraph of the Lanczos launch sequence (lanczos_impl): keyed by the call's
  // arguments and ws_gen, which every plan rebuild / workspace realloc bumps
  static constexpr int kGraphKey = 10;
  uint64_t ws_gen = 0;
  bool graph = false;          // krcn_csr_set_graph
  hipStream_t gstream = nullptr;
  hipGraphExec_t gexec = nullptr;
  uint64_t gkey[kGraphKey] = {};    // arguments gexec was recorded with
  uint64_t glast[kGraphKey] = {};   // arguments of the previous call
  // row shards of a multi-rank communicator: what every rank's early-alpha
  // Lanczos step must agree on (krcn_plan.hip agree_rows, after each plan build)
  int rows_pq = -1;            // packed alpha partials = max over ranks of pass_partials(p1); -1: not agreed
  int rows_early = 0;          // every rank's pass-1 grids fit kMaxPartials
  // placement probe of the hot buffers (ensure_plans, krcn_csr_set_placement_trials)
  static constexpr int kPlaceMax = 8;
  int place_trials = -1;       // -1 auto, 0 off, k: k placements probed
  int place_ran = 0;           // placements probed at the last plan build (0: none)
  int place_best = -1;         // the one kept
  float place_us[kPlaceMax] = {};   // probe HVP time of each (us)
  double place_hot_mb = 0.0;   // hot bytes the auto rule saw
  // the placement search over the first Lanczos calls (krcn_plan.hip lzp_*)
  int lzp_stage = 0;           // 0: not started; s >= 1: the next call times placement s - 1; -1: done
  int lzp_m = 0;               // the m the timed calls share
  int lzp_ran = 0, lzp_best = -1;
  float lzp_ms[kPlaceMax] = {};
  std::vector<std::vector<void*>> lzp_cand;   // the placements (slot values), [0] the one found
  hipEvent_t lzp_e0 = nullptr, lzp_e1 = nullptr;
};

void free_plan(PassPlan& P);
krcn_status ensure_plans(krcn_csr* h);
// `reps` back-to-back local HVPs (pass 1 and pass 2 of the handle's plans, no
// collective) on the handle's scratch vectors: *us = microseconds per HVP
// (krcn_ops.hip; the placement probe of ensure_plans).
krcn_status placement_probe(krcn_csr* h, hipStream_t s, int reps, float* us);
// The placement search over Lanczos calls (krcn_plan.hip): lzp_begin before
// a call's launches (may relocate the hot buffers on stream s and start the
// timing), lzp_end after them, lzp_done after the call's synchronisation.
krcn_status lzp_begin(krcn_csr* h, int m, hipStream_t s, bool* timed);
krcn_status lzp_end(krcn_csr* h, hipStream_t s, bool timed);
krcn_status lzp_done(krcn_csr* h, bool timed);
void lzp_abort(krcn_csr* h);
// CGS2 dot partials for Lanczos m <= m (krcn_plan.hip; frees and reallocates).
krcn_status reserve_reorth(krcn_csr* h, int m);

// A handle whose communicator spans several ranks joins collectives in every
// compute call, so it must not build plans (allocations, device-wide syncs)
// inside one: krcn_csr_attach_comm / krcn_csr_reserve build them up front, and
// a compute call on such a handle without them fails instead.  Other handles
// build their plans on first use.
inline krcn_status plans_for_compute(krcn_csr* h) {
  if (h->plans_ready) return KRCN_OK;
  if (h->comm && h->comm->nranks > 1)
    return fail(KRCN_ERR_INVALID, "a sharded handle with a %d-rank communicator has no plans: call krcn_csr_reserve "
                "(or krcn_csr_attach_comm) after changing its policies, before the collectives", h->comm->nranks);
  return ensure_plans(h);
}

// ---------------------------------------------------------------- helpers
inline hipStream_t S(void* s) { return reinterpret_cast<hipStream_t>(s); }

inline int vec_grid(int64_t len) {
  int64_t b = (len + kNT - 1) / kNT;
  if (b < 1) b = 1;
  if (b > 1024) b = 1024;
  return int(b);
}

// Lanes per row: the largest power of two <= mean row length / 8, in [1, 64]
// (measured on news20 / rcv1 shapes: 6.7 nnz/row -> 1, 57 -> 4, 74 -> 8).
inline int auto_lanes(int64_t rows, int64_t nnz) {
  const double mean = rows > 0 ? double(nnz) / double(rows) : 0.0;
  int L = 1;
  while (L < 64 && double(L * 2) * 8.0 <= mean) L *= 2;
  return L;
}

inline int resolve_lanes(int policy, int64_t rows, int64_t nnz) {
  if (policy == KRCN_LANES_AUTO) return auto_lanes(rows, nnz);
  if (policy == KRCN_LANES_SEQUENTIAL) return 1;
  return policy;
}

template <typename F>
inline void with_lanes(int L, F&& f) {
  switch (L) {
    case 1: f(std::integral_constant<int, 1>{}); break;
    case 2: f(std::integral_constant<int, 2>{}); break;
    case 4: f(std::integral_constant<int, 4>{}); break;
    case 8: f(std::integral_constant<int, 8>{}); break;
    case 16: f(std::integral_constant<int, 16>{}); break;
    case 32: f(std::integral_constant<int, 32>{}); break;
    default: f(std::integral_constant<int, 64>{}); break;
  }
}

template <class F>
inline void with_sort_nt(int nt, F&& f) {
  switch (nt) {
    case 512: f(std::integral_constant<int, 512>{}); break;
    case 1024: f(std::integral_constant<int, 1024>{}); break;
    default: f(std::integral_constant<int, 256>{}); break;
  }
}

inline krcn_status set_device(const krcn_csr* h) {
  HIPCHK(hipSetDevice(h->device));
  return KRCN_OK;
}

template <typename T>
inline krcn_status dalloc(krcn_csr* h, T** p, size_t count) {
  if (count == 0) count = 1;
  HIPCHK(hipMalloc(reinterpret_cast<void**>(p), count * sizeof(T)));
  h->owned += count * sizeof(T);
  return KRCN_OK;
}

inline krcn_status nccl_dtype(int dtype, ncclDataType_t* t) {
  *t = dtype == KRCN_F64 ? ncclDouble : ncclFloat;
  return KRCN_OK;
}

// (an RCCL communicator of one rank still runs the collective: the
// rehearsals of bench.py --rehearse-shard time its launch and stream cost)
inline krcn_status allreduce(krcn_csr* h, void* buf, int64_t count, int dtype, hipStream_t s) {
  if (!h->comm || count == 0) return KRCN_OK;
  if (h->comm->vg) return h->comm->nranks == 1 ? KRCN_OK : virtual_allreduce(h->comm, buf, count, dtype, s);
  ncclDataType_t t;
  nccl_dtype(dtype, &t);
  NCCLCHK(ncclAllReduce(buf, buf, size_t(count), t, ncclSum, h->comm->comm, s));
  return KRCN_OK;
}

// ------------------------------------------------------------- profiling
inline ProfRec* prof_next(krcn_csr* h) {
  if (!h->prof) return nullptr;
  if (h->prof_used == h->prof_pool.size()) {
    ProfRec r;
    // timing-only events without the system-scope release fence a default
    // event record carries (they sit between kernels of the timed region)
    const unsigned fl = hipEventDisableSystemFence;
    if (hipEventCreateWithFlags(&r.e0, fl) != hipSuccess || hipEventCreateWithFlags(&r.e1, fl) != hipSuccess ||
        hipEventCreateWithFlags(&r.e2, fl) != hipSuccess || hipEventCreateWithFlags(&r.em, fl) != hipSuccess)
      return nullptr;
    h->prof_pool.push_back(r);
  }
  ProfRec* r = &h->prof_pool[h->prof_used++];
  r->mid = false;
  return r;
}

// A/B knob KRCN_COMBINE_W=1: slices combine with 16-byte loads (k_slice_combine_w).
inline bool combine_w_env() {
  static const bool v = [] {
    const char* e = tuning_env("KRCN_COMBINE_W");
    return e && e[0] == '1';
  }();
  return v;
}

// The slice combine of a sliced pass over its S partial arrays (P.part).
template <typename T, class Src2, class Epi>
inline krcn_status run_combine(PassPlan& P, int S, const Src2& rest, const Epi& epi, double* partials, int* Pout,
                               hipStream_t s) {
  int grid = P.combine_grid;
  if (S <= kCombineSmallS) {
    grid = combine_small_grid(P.rows);
    const int nt = combine_small_nt(P.rows);
    const T* pp = static_cast<const T*>(P.part);
    auto go = [&](auto sm, auto ntc) {
      hipLaunchKernelGGL((k_slice_combine_small<T, Src2, Epi, decltype(sm)::value, decltype(ntc)::value>), dim3(grid),
                         dim3(decltype(ntc)::value), 0, s, P.rows, S, pp, rest, epi, partials);
    };
    auto by_s = [&](auto ntc) {
      if (S <= 2) go(std::integral_constant<int, 2>{}, ntc);
      else if (S <= 4) go(std::integral_constant<int, 4>{}, ntc);
      else if (S <= 8) go(std::integral_constant<int, 8>{}, ntc);
      else go(std::integral_constant<int, 16>{}, ntc);
    };
    if (nt == 256) by_s(std::integral_constant<int, 256>{});
    else by_s(std::integral_constant<int, kCombineNT>{});
  } else if (combine_w_env() && S >= 32 && P.rows % CombW<T>::VW == 0 &&
             combine_w_grid(P.rows, CombW<T>::VW) <= P.pcap) {
    grid = combine_w_grid(P.rows, CombW<T>::VW);
    hipLaunchKernelGGL((k_slice_combine_w<T, Src2, Epi>), dim3(grid), dim3(kCombineNT), 0, s, P.rows, S,
                       static_cast<const T*>(P.part), rest, epi, partials);
  } else {
    hipLaunchKernelGGL((k_slice_combine<T, Src2, Epi>), dim3(grid), dim3(kCombineNT), 0, s, P.rows, S,
                       combine_rows(P.rows), static_cast<const T*>(P.part), rest, epi, partials);
  }
  LAUNCHCHK();
  if (Pout) *Pout = grid;
  return KRCN_OK;
}

// One SpMV pass: `first` is the source of the tiled launch, `rest` of the
// slice-combine launch (sliced plans); partial sums of a reducing epilogue land
// in `partials` (*Pout entries).
// `mid` (profiling): its em event is recorded between the main launch and
// the slice combine.
template <typename T, class Src, class Src2, class Epi>
inline krcn_status run_pass(PassPlan& P, const Src& first, const Src2& rest, const Epi& epi, double* partials,
                            int* Pout, hipStream_t s, ProfRec* mid = nullptr) {
  // a reducing launch writes one partial per block: the buffer must hold them
  const int reducer_grid = P.jag ? (P.jG > 1 ? P.combine_grid : P.grid)
                                 : (P.win ? !P.accum : P.S > 1) ? P.combine_grid : P.grid;
  if (partials && reducer_grid > P.pcap)
    return fail(KRCN_ERR_INVALID, "run_pass: %d partials exceed the %lld-entry buffer", reducer_grid,
                (long long)P.pcap);
  if constexpr (IsLzSmall<Src>::value) {   // one-piece window-accum plans only
    if (!P.win || !P.accum || P.S != 1 || P.cols > kWinNT)
      return fail(KRCN_ERR_UNSUPPORTED, "fused small-vector Lanczos pass 1 needs a one-piece window-accum plan");
    WinArgs wa{P.rows, P.W, P.stride, P.S, 1, P.ntiles, P.cols, P.tb, P.ro, P.widx, P.val, P.segs};
    wa.kpb = P.kpb;
    if (P.R == 16)
      hipLaunchKernelGGL((k_window_pass<T, 16, Src, Epi, true>), dim3(P.grid), dim3(kWinNT), 0, s, wa, first, epi,
                         partials);
    else if (P.R == 32)
      hipLaunchKernelGGL((k_window_pass<T, 32, Src, Epi, true>), dim3(P.grid), dim3(kWinNT), 0, s, wa, first, epi,
                         partials);
    else
      hipLaunchKernelGGL((k_window_pass<T, 64, Src, Epi, true>), dim3(P.grid), dim3(kWinNT), 0, s, wa, first, epi,
                         partials);
    LAUNCHCHK();
    if (Pout) *Pout = P.grid;
    return KRCN_OK;
  } else {
  if constexpr (IsLzU<Src>::value) {
    if (!P.jag || P.S != 1)
      return fail(KRCN_ERR_UNSUPPORTED, "the two-launch Lanczos pass 2 needs a single-window jagged plan");
  }
  if (P.jag) {
    if constexpr (IsLzZ<Src>::value) {
      return fail(KRCN_ERR_UNSUPPORTED, "fused Lanczos pass 1 needs an LDS-window slices plan");
    } else {
      JagArgs ja{P.rows, P.S == 1 ? 1 : P.jSg, P.W, P.jG, P.cols, P.jgcut, P.jumeta, P.jcnt, P.widx, P.val};
      ja.xmap = P.S == 1 && KRCN_JAG_XMAP;
      if (P.jlong > 0) {
        ja.nlong = P.jlong;
        ja.lpiece = P.jlpiece;
        ja.lcut = P.jlcut;
        ja.tcut = P.jlcut + P.grid + 1;
        ja.lrow = P.jlrow;
        ja.ltask = P.jltask;
        ja.task = P.jtask;
        ja.lidx = P.jlidx;
        ja.lval = P.jlval;
      }
      // accumulate over G slice groups: per-group partial row sums, combined
      // in group order by k_slice_combine (which runs the epilogue)
      auto acc = [&](const auto& ep, double* parts) {
        using E = std::decay_t<decltype(ep)>;
        if (P.jK == 4)
          hipLaunchKernelGGL((k_jag_acc<T, 4, Src, E>), dim3(P.grid), dim3(kJagNT), 0, s, ja, first, ep, parts);
        else
          hipLaunchKernelGGL((k_jag_acc<T, kJagK2, Src, E>), dim3(P.grid), dim3(kJagNT), 0, s, ja, first, ep, parts);
      };
      if (P.S == 1) {
        auto one = [&](auto kc) {
          hipLaunchKernelGGL((k_jag_pass<T, decltype(kc)::value, jag_cpg(decltype(kc)::value), 8, Src, Epi>), dim3(P.grid), dim3(kJagNT),
                             0, s, ja, first, epi, partials);
        };
        if (P.jK == 1) one(std::integral_constant<int, 1>{});
        else if (P.jK == 2) one(std::integral_constant<int, 2>{});
        else if (P.jK == 3) one(std::integral_constant<int, 3>{});
        else one(std::integral_constant<int, kJagK1>{});
      }
      else if (P.jG > 1)
        acc(EpiSlicePart<T>{static_cast<T*>(P.part), int64_t(P.rows)}, static_cast<double*>(nullptr));
      else
        acc(epi, partials);
      LAUNCHCHK();
      if (mid && P.S > 1 && P.jG > 1) {   // (events only where a combine launch follows)
        HIPCHK(hipEventRecord(mid->em, s));
        mid->mid = true;
      }
      if (P.S > 1 && P.jG > 1) {
        CHK(run_combine<T>(P, P.jG, rest, epi, partials, Pout, s));
      } else if (Pout) {
        *Pout = P.grid;
      }
      return KRCN_OK;
    }
  }
  if (P.win) {
    WinArgs wa{P.rows, P.W, P.stride, P.S, IsLzZ<Src>::value ? 2 : (P.accum ? 1 : 0), P.ntiles, P.cols,
                     P.tb, P.ro, P.widx, P.val, P.segs};
    wa.kpb = P.kpb;
    auto launch = [&](auto rc) {
      constexpr int RR = decltype(rc)::value;
      if constexpr (IsLzZ<Src>::value) {   // fused step B: slices-mode plans only
        EpiSlicePart<T> ep{static_cast<T*>(P.part), int64_t(P.rows)};
        hipLaunchKernelGGL((k_window_pass<T, RR, Src, EpiSlicePart<T>, false>), dim3(P.grid), dim3(kWinNT), 0, s,
                           wa, first, ep, static_cast<double*>(nullptr));
      } else if (P.accum) {
        hipLaunchKernelGGL((k_window_pass<T, RR, Src, Epi, true>), dim3(P.grid), dim3(kWinNT), 0, s, wa, first, epi,
                           partials);
      } else {
        EpiSlicePart<T> ep{static_cast<T*>(P.part), int64_t(P.rows)};
        hipLaunchKernelGGL((k_window_pass<T, RR, Src, EpiSlicePart<T>, false>), dim3(P.grid), dim3(kWinNT), 0, s,
                           wa, first, ep, static_cast<double*>(nullptr));
      }
    };
    if (P.R == 16) launch(std::integral_constant<int, 16>{});
    else if (P.R == 32) launch(std::integral_constant<int, 32>{});
    else launch(std::integral_constant<int, 64>{});
    LAUNCHCHK();
    if (mid && !P.accum) {
      HIPCHK(hipEventRecord(mid->em, s));
      mid->mid = true;
    }
    if (!P.accum) {
      CHK(run_combine<T>(P, P.S, rest, epi, partials, Pout, s));
    } else if (Pout) {
      *Pout = P.grid;
    }
    return KRCN_OK;
  }
  if constexpr (IsLzZ<Src>::value) {
    if constexpr (std::is_same<Epi, EpiWeighted<T>>::value) {
    if (!P.sorted || P.S != 1)
      return fail(KRCN_ERR_UNSUPPORTED, "the two-launch Lanczos pass 1 needs an unsliced sorted-tile plan");
    {
      // unsliced: the two-launch step (pass 2's SrcLzU settles beta); epi is
      // the caller's (EpiWeighted: u' = w (.) X z_j)
      with_lanes(P.L, [&](auto lc) {
        constexpr int LL = decltype(lc)::value;
        with_sort_nt(P.sort_nt, [&](auto nc) {
          constexpr int NT = decltype(nc)::value;
          hipLaunchKernelGGL((k_sorted_pass<T, LL, NT, Src, Epi>), dim3(P.grid), dim3(NT), 0, s, P.rows, 1, P.ptr,
                             P.gword, static_cast<const T*>(P.gval), P.tiles, P.tbeg, P.tmid, first, epi, partials);
        });
      });
      LAUNCHCHK();
      if (Pout) *Pout = P.grid;
      return KRCN_OK;
    }
    } else {
    // fused step B over sorted tiles, sliced: the combine settles beta
    if (!P.sorted)
      return fail(KRCN_ERR_UNSUPPORTED, "fused Lanczos pass 1 needs an LDS-window or sorted-tile plan");
    with_lanes(P.L, [&](auto lc) {
      constexpr int LL = decltype(lc)::value;
      with_sort_nt(P.sort_nt, [&](auto nc) {
        constexpr int NT = decltype(nc)::value;
        EpiSlicePart<T> ep{static_cast<T*>(P.part), int64_t(P.rows)};
        hipLaunchKernelGGL((k_sorted_pass<T, LL, NT, Src, EpiSlicePart<T>>), dim3(P.grid), dim3(NT), 0, s, P.rows,
                           P.groups, P.ptr, P.gword, static_cast<const T*>(P.gval), P.tiles, P.tbeg, P.tmid, first,
                           ep, static_cast<double*>(nullptr));
      });
    });
    LAUNCHCHK();
    if (mid) {
      HIPCHK(hipEventRecord(mid->em, s));
      mid->mid = true;
    }
    return run_combine<T>(P, P.S, rest, epi, partials, Pout, s);
    }
  } else {
  with_lanes(P.L, [&](auto lc) {
    constexpr int LL = decltype(lc)::value;
    if (P.sorted) {
      with_sort_nt(P.sort_nt, [&](auto nc) {
        constexpr int NT = decltype(nc)::value;
        if (P.S == 1) {
          hipLaunchKernelGGL((k_sorted_pass<T, LL, NT, Src, Epi>), dim3(P.grid), dim3(NT), 0, s, P.rows, 1, P.ptr,
                             P.gword, static_cast<const T*>(P.gval), P.tiles, P.tbeg, P.tmid, first, epi,
                             partials);
        } else {
          EpiSlicePart<T> ep{static_cast<T*>(P.part), int64_t(P.rows)};
          hipLaunchKernelGGL((k_sorted_pass<T, LL, NT, Src, EpiSlicePart<T>>), dim3(P.grid), dim3(NT), 0, s,
                             P.rows, P.groups, P.ptr, P.gword, static_cast<const T*>(P.gval), P.tiles, P.tbeg,
                             P.tmid, first, ep, static_cast<double*>(nullptr));
        }
      });
    } else if (P.S == 1) {
      hipLaunchKernelGGL((k_tiled_pass<T, LL, Src, Epi>), dim3(P.grid), dim3(kNT), 0, s, P.rows, 1, P.ptr, P.idx,
                         static_cast<const T*>(P.val), P.tiles, P.tbeg, first, epi, partials);
    } else {
      EpiSlicePart<T> ep{static_cast<T*>(P.part), int64_t(P.rows)};
      hipLaunchKernelGGL((k_tiled_pass<T, LL, Src, EpiSlicePart<T>>), dim3(P.grid), dim3(kNT), 0, s, P.rows,
                         P.groups, P.ptr, P.idx, static_cast<const T*>(P.val), P.tiles, P.tbeg, first, ep,
                         static_cast<double*>(nullptr));
    }
  });
  LAUNCHCHK();
  if (mid && P.S > 1) {
    HIPCHK(hipEventRecord(mid->em, s));
    mid->mid = true;
  }
  if (P.S > 1) {
    CHK(run_combine<T>(P, P.S, rest, epi, partials, Pout, s));
  } else if (Pout) {
    *Pout = P.grid;
  }
  return KRCN_OK;
  }
  }
}

// The number of partials run_pass writes for plan P when its epilogue
// reduces (the *Pout of a non-fused launch): the combine's grid for sliced
// plans, the main launch's otherwise.  Row shards agree on its maximum over
// ranks before the collectives (krcn_plan.hip agree_rows).
inline int pass_partials(const PassPlan& P) {
  auto combine = [&](int S) {
    if (S <= kCombineSmallS) return combine_small_grid(P.rows);
    if (combine_w_env() && S >= 32 && P.rows % 2 == 0 && combine_w_grid(P.rows, 2) <= P.pcap)
      return combine_w_grid(P.rows, 2);   // (fp64 rows: CombW<double>::VW = 2; row shards are fp64)
    return P.combine_grid;
  };
  if (P.jag) return (P.S > 1 && P.jG > 1) ? combine(P.jG) : P.grid;
  if (P.win) return P.accum ? P.grid : combine(P.S);
  return P.S > 1 ? combine(P.S) : P.grid;
}

#if KRCN_FOLD
// The early-alpha pass 1 of a window-slices plan with its slice combine
// folded in (krcn_window.hpp EpiSliceFold; tuning builds).
inline bool fold_ok(const krcn_csr* h) {
  const PassPlan& P = h->p1;
  return h->fcnt && P.win && !P.accum && P.R == 32 && P.S <= 96 && P.ntiles <= h->pcap;
}
template <typename T>
inline krcn_status run_fold_pass1(krcn_csr* h, const SrcLzBeta<T>& src, const EpiSliceFold<T>& epi, hipStream_t s) {
  PassPlan& P = h->p1;
  WinArgs wa{P.rows, P.W, P.stride, P.S, 0, P.ntiles, P.cols, P.tb, P.ro, P.widx, P.val, P.segs};
  wa.kpb = P.kpb;
  hipLaunchKernelGGL((k_window_pass<T, 32, SrcLzBeta<T>, EpiSliceFold<T>, false>), dim3(P.grid), dim3(kWinNT), 0, s,
                     wa, src, epi, static_cast<double*>(nullptr));
  LAUNCHCHK();
  return KRCN_OK;
}
#endif

// Pass over X (rows) / X^T with a plain gathered vector.
template <typename T, class Epi>
inline krcn_status launch_rows_x(krcn_csr* h, const T* x, const Epi& epi, double* partials, int* P,
                                 hipStream_t s) {
  CHK(plans_for_compute(h));
  return run_pass<T>(h->p1, SrcPlain<T>{x}, SrcPlain<T>{x}, epi, partials, P, s);
}

template <typename T, class Epi>
inline krcn_status launch_rows_xt(krcn_csr* h, const T* u, const Epi& epi, double* partials, int* P,
                                  hipStream_t s) {
  CHK(plans_for_compute(h));
  return run_pass<T>(h->p2, SrcPlain<T>{u}, SrcPlain<T>{u}, epi, partials, P, s);
}

// Lanczos recurrences, one translation unit per dtype (krcn_lanczos_impl.hpp).
krcn_status lanczos_f64(krcn_csr* h, const double* w, const double* g, int m, int reorth, double tol, double l2,
                        double* V, double* alphas_host, double* betas_host, krcn_lanczos_info* info, hipStream_t s);
krcn_status lanczos_f32(krcn_csr* h, const float* w, const float* g, int m, int reorth, double tol, double l2,
                        float* V, double* alphas_host, double* betas_host, krcn_lanczos_info* info, hipStream_t s);


