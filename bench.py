"""Benchmark of the Krylov-CRN hot path: Hessian-vector products / s on MI355X.

Workload (BASELINE.json metric: "HVP/s + achieved HBM GB/s, news20 CSR"):
news20-shaped synthetic CSR (n 19,996, d 1,355,191, nnz 9,097,916, fp64,
krcn.synth, seed 20240117), Krylov subspace m = 100 (configs[2]).  One step =
one full device Lanczos recurrence (cubic.py:77-111) from the gradient at
x = 0.5*1: m HVPs (loss.py:289-302) plus the Lanczos vector work, alphas/betas
returned to the host.  value = HVPs executed by the whole job / wall time.

Multi-GPU (one process per GPU: under torchrun, or `--gpus N`, which starts
the N ranks itself via krcn.launch and refuses N > visible GPUs): the matrix is sharded across ranks
(columns when n < d — news20 — rows otherwise) and the recurrence all-reduces
through RCCL; total work is fixed, so scaling is "strong".

Also reported: roofline of the dominant kernel (per-launch HIP-event times of
pass 1 (X v) and pass 2 (X^T u) inside the timed region, algorithmic bytes of
SURVEY.md §8d), the whole-HVP GB/s, a cold-cache single-HVP time, and the CPU
baseline (the oracle's scipy restatement of loss.py:299-302, timed on this
host on a bounded sample, rank 0 at N = 1 only).
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "krylov-cubic-regularized-newton_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import krcn  # noqa: E402
from krcn import dist as kdist  # noqa: E402
from krcn import launch  # noqa: E402
from krcn import synth  # noqa: E402

HBM_PEAK_GBPS = 8000.0   # MI355X_MICROARCH.md: 8.0 TB/s spec


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=None,
                   help="GPUs (one rank each); without a torchrun environment N > 1 starts N ranks itself")
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=8)
    p.add_argument("--config", default="news20", choices=sorted(synth.CONFIGS))
    p.add_argument("--m", type=int, default=None, help="Krylov dimension (default: the config's)")
    p.add_argument("--libsvm", default=None, metavar="PATH",
                   help="bench a local LIBSVM file instead of the synthetic matrix (m / dtype from --config)")
    p.add_argument("--rehearse-shard", type=int, default=0, metavar="N",
                   help="one GPU runs rank 0's block of an N-way partition through the sharded path "
                        "(1-rank RCCL communicator); value = that rank's HVP/s, not a whole-job number")
    p.add_argument("--partition", default="auto", choices=["auto", "rows", "cols"])
    p.add_argument("--skew", action="store_true",
                   help="skewed synthetic pattern: lognormal row lengths, power-law column popularity")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--rank-timeout", type=float, default=1500.0,
                   help="--gpus N: seconds after which hung ranks are killed (exit 124)")
    p.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline budget")
    p.add_argument("--no-cold", action="store_true")
    p.add_argument("--placement-trials", type=int, default=None,
                   help="hot-buffer placements probed at the plan build (-1 auto = the library default, 0 off)")
    p.add_argument("--traffic-json", default=os.path.join(REPO, "profiles", "traffic.json"))
    return p.parse_args()


def cpu_baseline(A, b, budget_s, label):
    """The oracle's scipy HVP (csr_matvec + expit reweight + csc_matvec), 1 thread."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import krcn_oracle as O
    x = np.full(A.shape[1], 0.5)
    v = np.random.default_rng(0).standard_normal(A.shape[1])
    O.hess_vec_prod(A, x, v)
    count, t0 = 0, time.perf_counter()
    while True:
        O.hess_vec_prod(A, x, v)
        count += 1
        el = time.perf_counter() - t0
        if el >= budget_s:
            break
    try:
        cpu = open("/proc/cpuinfo").read().split("model name")[1].split("\n")[0].strip(" :\t")
    except Exception:
        cpu = "unknown"
    out = {"value": count / el, "unit": "HVP/s", "cores": 1, "kind": "port",
           "sample": f"{count} HVPs of the {label} problem ({A.shape[0]} x {A.shape[1]}, {A.nnz} nnz) at x=0.5 "
                     f"(scipy csr_matvec/csc_matvec, "
                     f"expit; oracle/krcn_oracle.hess_vec_prod) in {el:.1f} s; host CPU {cpu}; "
                     f"{len(os.sched_getaffinity(0))} cores visible, 1 used"}
    # strong CPU line: the OpenMP C restatement, bitwise scipy's
    # result (tests/test_oracle_omp.py), HVPs from fixed weights like the device path
    try:
        import krcn_oracle_omp
        # the GPU box gives each GPU a 16-core share of its host (the harness
        # sets OMP_NUM_THREADS=16 and asks worker pools to stay within it),
        # however many cores sched_getaffinity shows; the strong line uses that share
        visible = len(os.sched_getaffinity(0))
        threads = min(int(os.environ.get("OMP_NUM_THREADS", "16") or 16), visible)
        h = krcn_oracle_omp.HVP(A, threads=threads)
        w = O.hessian_weights(A, x)
        h(w, v)
        count, t0 = 0, time.perf_counter()
        while True:
            h(w, v)
            count += 1
            el = time.perf_counter() - t0
            if el >= budget_s / 3:
                break
        out["strong"] = {"value": count / el, "unit": "HVP/s", "cores": threads, "kind": "port",
                         "sample": f"{count} HVPs of the {label} problem from fixed weights "
                                   f"(oracle/krcn_hvp_omp.c, OpenMP, {threads} threads = the box's per-GPU "
                                   f"core share; {visible} cores visible) in {el:.1f} s"}
    except (OSError, ImportError) as e:   # the C restatement is not built: report without it
        out["strong"] = {"error": str(e)}
    return out


class HipEvents:
    """hipEvents on torch's current stream without the system-scope release
    fence that a default event record carries (hipEventDisableSystemFence,
    the flag libkrcn's own per-pass events use): the fence writes the L2 back
    at every record, a cost the HVP itself never pays between calls."""
    FLAG = 0x20000000   # hipEventDisableSystemFence (hip_runtime_api.h)

    def __init__(self, count):
        import ctypes
        self.ct = ctypes
        self.lib = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
        self.ev = []
        for _ in range(count):
            e = ctypes.c_void_p()
            if self.lib.hipEventCreateWithFlags(ctypes.byref(e), ctypes.c_uint(self.FLAG)) != 0:
                raise RuntimeError("hipEventCreateWithFlags failed")
            self.ev.append(e)

    def record(self, i):
        s = self.ct.c_void_p(torch.cuda.current_stream().cuda_stream)
        if self.lib.hipEventRecord(self.ev[i], s) != 0:
            raise RuntimeError("hipEventRecord failed")

    def elapsed_us(self, i, j):
        ms = self.ct.c_float()
        if self.lib.hipEventElapsedTime(self.ct.byref(ms), self.ev[i], self.ev[j]) != 0:
            raise RuntimeError("hipEventElapsedTime failed")
        return 1e3 * ms.value

    def close(self):
        for e in self.ev:
            self.lib.hipEventDestroy(e)


def flush_caches(buf):
    buf.add_(1.0)   # 512 MiB read+write evicts L2 and the 256 MiB Infinity Cache


def main():
    args = parse()
    if not launch.in_launched_rank():
        if (args.gpus or 1) > 1:
            # N fresh rank processes, started before anything touches the GPU here
            have = launch.visible_gpus()
            if have < args.gpus:
                sys.exit(f"bench: --gpus {args.gpus} requested but only {have} GPU(s) are visible")
            sys.exit(launch.launch_ranks(args.gpus, [os.path.abspath(__file__), *sys.argv[1:]],
                                         timeout=args.rank_timeout))
    elif args.gpus is not None:
        launch.require_world(args.gpus)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())
    cfg = synth.CONFIGS[args.config]
    m = args.m or cfg["m"]
    dtype = torch.float64 if cfg["dtype"] == "f64" else torch.float32
    reorth = bool(cfg.get("reorth", False))

    if args.libsvm:
        from krcn import libsvm
        A, b = libsvm.load(args.libsvm)
        label = "libsvm:" + os.path.basename(args.libsvm)
    else:
        A, b = synth.make_problem(args.config, skew=args.skew)
        label = args.config + ("-skew" if args.skew else "")
    n, d = A.shape
    nnz = A.nnz
    problem = kdist.ShardedProblem(A, b, dtype=dtype, partition=args.partition, device=dev,
                                   rehearse=args.rehearse_shard)
    X = problem.X
    if args.placement_trials is not None:
        X.set_placement_trials(args.placement_trials)
    x = problem.full_d(0.5)
    Ax = X.matvec(x)
    w = X.weights(Ax)
    g = X.gradient(Ax, problem.b_dev)
    V = torch.empty((m, X.d), dtype=dtype, device=dev)

    def step():
        return X.lanczos(w, g, m, reorth=reorth, V=V)

    for _ in range(args.warmup):
        step()
    problem.barrier()
    torch.cuda.synchronize()
    hvps = 0
    t0 = time.perf_counter()
    for _ in range(args.steps):
        _, _, _, info = step()
        hvps += info.hvps
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    problem.barrier()
    elapsed = problem.max_over_ranks(t1 - t0)
    # per-pass HIP-event times on the library's stream, in separate steps so the
    # events do not perturb the headline number above
    X.prof_enable(True)
    for _ in range(max(1, min(args.steps, 5))):
        step()
    torch.cuda.synchronize()
    prof = X.prof_read()
    X.prof_enable(False)

    s_val = 8 if dtype == torch.float64 else 4
    b_hvp = synth.hvp_bytes(n, d, nnz, s_val=s_val)
    fmt = X.plan_format()
    plan = X.plan_info()
    # step B runs inside pass 1 on window-slice, sliced sorted-tile and
    # one-piece window plans (krcn_lanczos_impl.hpp: fuse_win / _sorted / _small)
    fused = ((fmt["pass1"] == "window-slices" or (fmt["pass1"] == "sorted" and plan["pass1"][0] < -1)
              or (fmt["pass1"] == "window-accum" and plan["pass1"][0] == 1 and X.d <= 1024))
             and problem.spec.mode_name == "none" and not reorth)
    kb = synth.lanczos_kernel_bytes(X.n, X.d, X.nnz, fused, s_val=s_val,
                                    z_store=fmt["pass1"] != "window-slices")
    # one-piece fused plans also fold X^T u into pass 1 (per-block column-major
    # copies, EpiLz1X): pass 1 reads both orders of X and w, and
    # "pass 2" is k_xt_combine of the block partials with step A (no matrix)
    xt = fused and fmt["pass1"] == "window-accum" and X.d <= 1024
    if xt:
        kb["pass1"] += X.nnz * (s_val + 4) + 4 * (X.d + 1) + s_val * X.n
        kb["pass2"] = s_val * 4 * X.d
    cnt = max(prof["count"], 1)
    launches = {   # this rank's average launch times (us) and algorithmic bytes
        "pass1": (1e3 * prof["pass1_kernel_ms"] / cnt, kb["pass1"]),
        "combine": (1e3 * prof["combine_ms"] / cnt, kb["combine"]),
        "pass2": (1e3 * prof["pass2_ms"] / cnt, kb["pass2"]),
    }
    if prof["combine_ms"] <= 0.0:   # the plan has no slice-combine launch (no events were recorded)
        del launches["combine"]
    if xt and launches["pass2"][0] < 0.5:
        # the blocks' X^T u partials are combined and step A runs inside pass
        # 1's launch (EpiLz1X::fold_run): nothing is launched between pass 1's
        # events and pass 2's, so pass 1 carries pass 2's bytes too
        launches["pass1"] = (launches["pass1"][0], kb["pass1"] + kb["pass2"])
        del launches["pass2"]
    names = {
        "pass1": "pass 1: X z (k_window_pass" + (", step B of the previous step fused" if fused else "") + ")",
        "combine": "slice combine: u = w (t / beta) (k_slice_combine)",
        "pass2": "pass 2: X^T u fused with Lanczos step A (k_window_pass / EpiLz2)",
    }
    if not fmt["pass1"].startswith("window"):
        names["pass1"] = f"pass 1: X z ({fmt['pass1']} tiles" + (", step B fused" if fused else "") + ")"
    if not fmt["pass2"].startswith("window"):
        names["pass2"] = f"pass 2: X^T u fused with Lanczos step A ({fmt['pass2']} tiles)"
    if xt:
        names["pass1"] = ("pass 1: X z with step B fused and the blocks' X^T u partials (k_window_pass, EpiLz1X)"
                          + ("; their combine and step A in the same launch" if "pass2" not in launches else ""))
        names["pass2"] = "pass 2: the blocks' X^T u partials combined with Lanczos step A (k_xt_combine)"
    dom_key = max(launches, key=lambda k: launches[k][0])
    dom_us, dom_bytes = launches[dom_key]
    dom = names[dom_key]
    achieved = dom_bytes / (dom_us * 1e-6) / 1e9 if dom_us > 0 else 0.0
    p1_us = 1e3 * prof["pass1_ms"] / cnt
    p2_us = 1e3 * prof["pass2_ms"] / cnt
    traffic = None
    traffic_src = "no counter measurement for this configuration"
    # counter traffic is keyed by what a launch processes: the whole problem on
    # `world` GPUs, or (--rehearse-shard N) rank 0's block of an N-way partition
    tkey = f"{label}:rehearse{args.rehearse_shard}" if args.rehearse_shard > 1 else f"{label}:{world}"
    if os.path.exists(args.traffic_json):
        try:
            ent = json.load(open(args.traffic_json)).get(tkey, {})
            traffic = ent.get(dom_key)
            if traffic is not None:
                traffic_src = (f"profiles/traffic.json['{tkey}'] from {ent.get('source', '?')}, measured on "
                               f"tree {ent.get('head', 'unknown')} (rocprofv3 PMC, 2 x FETCH_SIZE + WRITE_SIZE, "
                               "per launch; not measured in this run)")
        except Exception:
            traffic = None

    reorth_info = None
    if reorth:
        # CGS2 cost: the same recurrence without reorthogonalisation, timed on
        # the same handle; the difference is the reorth time per step.  Its
        # algorithmic bytes: three sweeps over V_{0..j} per step j (CGS2 with
        # the second dot sweep fused into the first update, krcn_cgs2.hpp) plus
        # z read and written by each update sweep.
        for _ in range(2):
            X.lanczos(w, g, m, reorth=False, V=V)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        for _ in range(args.steps):
            X.lanczos(w, g, m, reorth=False, V=V)
        torch.cuda.synchronize()
        plain_ms = 1e3 * (time.perf_counter() - t2) / args.steps
        step_ms = 1e3 * elapsed / args.steps
        s_v = 8 if dtype == torch.float64 else 4
        rbytes = sum(3 * (j + 1) * X.d * s_v + 4 * X.d * s_v for j in range(m - 1))
        reorth_ms = step_ms - plain_ms
        reorth_info = {"ms_per_step": reorth_ms, "lanczos_without_reorth_ms": plain_ms,
                       "algorithmic_bytes_per_step": rbytes,
                       "achieved_gbps": rbytes / (reorth_ms * 1e-3) / 1e9 if reorth_ms > 0 else None,
                       "method": "step time minus the same Lanczos without reorth, same handle"}

    hvp_per_s = hvps / elapsed
    out = {
        "metric": "Hessian-vector products/sec + achieved HBM GB/s, news20 CSR, 1/2/4/8 MI355X",
        "value": hvp_per_s,
        "unit": "HVP/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": 1e3 * elapsed / args.steps,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64" if dtype == torch.float64 else "f32",
        "data": (f"LIBSVM file {args.libsvm}" if args.libsvm else
                 "synthetic (krcn.synth, shape-matched to LIBSVM " + args.config + ", seed 20240117)"),
        "config": {"workload": f"{label}: one device Lanczos (cubic.py:77-111) of m={m} HVPs per step"
                               + (" with CGS2 reorth" if reorth else ""),
                   "n": n, "d": d, "nnz": nnz, "m": m, "partition": problem.partition,
                   "parallelism": (f"{problem.partition}-sharded x{world}" if world > 1 else
                                   f"rank 0 of {problem.partition}-sharded x{args.rehearse_shard} "
                                   "(1-rank RCCL rehearsal)" if args.rehearse_shard > 1 else "single GPU")},
        "achieved_hbm_gbps_hvp": b_hvp * hvp_per_s / 1e9,
        "hvp_bytes_algorithmic": b_hvp,
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": achieved, "peak": HBM_PEAK_GBPS,
                     "unit": "GB/s", "frac": achieved / HBM_PEAK_GBPS, "traffic": traffic,
                     "algorithmic_bytes_per_launch": dom_bytes, "avg_launch_us": dom_us,
                     "launches": {k: {"avg_us": round(v[0], 3), "algorithmic_bytes": v[1],
                                      "achieved_gbps": round(v[1] / (v[0] * 1e-6) / 1e9, 1) if v[0] > 0 else None}
                                  for k, v in launches.items()},
                     "pass1_with_combine_us": p1_us, "pass2_us": p2_us, "launches_timed": prof["count"],
                     "fused_step_b": fused, "fused_xt": xt, "formats": fmt,
                     "plan": {"pass1": list(plan["pass1"]), "pass2": list(plan["pass2"]),
                              "fields": "(slices, <0: sorted tiles), lanes, tiles, grid"},
                     "traffic_source": traffic_src},
        "placement": dict(X.placement_info(),
                          note="hot-buffer placements probed at the plan build, fastest kept "
                               "(krcn_csr_set_placement_trials; DESIGN.md §5 Placement)"),
        "cpu_baseline": None,
    }
    if reorth_info is not None:
        out["reorth"] = reorth_info
    solo = world == 1 and args.rehearse_shard <= 1   # whole-problem single-GPU lines
    if not args.no_cold and solo:
        flush = torch.zeros(64 * 1024 * 1024, dtype=torch.float64, device=dev)
        v = (g / X.diff_norm(g)).contiguous()
        ts = []
        for _ in range(5):
            flush_caches(flush)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            X.hvp(w, v)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3)
        out["hvp_cold_us"] = float(np.median(ts))
        out["hvp_cold_gbps"] = b_hvp / (np.median(ts) * 1e-6) / 1e9
        del flush
    if solo:
        # SURVEY.md §8d protocol: 200 back-to-back warm HVPs timed with hipEvents
        # on the stream the library launches on (torch's current stream)
        v = (g / X.diff_norm(g)).contiguous()
        y = X.empty_d()
        for _ in range(5):
            X.hvp(w, v, out=y)
        # 200 back-to-back HVPs in 20 batches of 10, one fence-free hipEvent
        # (HipEvents) between batches: an event record between two launches
        # holds the next dispatch until the previous kernels have completed
        # (rocprofv3 trace: a 4-5 us idle gap in front of every event-bracketed
        # HVP, 0.1-0.3 us between launches without one), so per-HVP events
        # would time that gap 200 times.  Per-HVP time = batch time / 10.
        nb, per = 20, 10
        he = HipEvents(nb + 1)
        he.record(0)
        for i in range(nb):
            for _ in range(per):
                X.hvp(w, v, out=y)
            he.record(i + 1)
        torch.cuda.synchronize()
        us = np.array([he.elapsed_us(i, i + 1) / per for i in range(nb)])
        # the same HVPs each bracketed by a pair of torch events (default flags),
        # as rounds 1-4 reported them: kept for continuity
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(200)]
        for e0, e1 in evs:
            e0.record()
            X.hvp(w, v, out=y)
            e1.record()
        torch.cuda.synchronize()
        us_t = np.array([e0.elapsed_time(e1) * 1e3 for e0, e1 in evs])
        he.close()
        med = float(np.median(us))
        out["hvp_warm_us"] = {"median": med, "p10": float(np.percentile(us, 10)), "p90": float(np.percentile(us, 90)),
                              "events": "200 HVPs in 20 batches of 10 back to back, a hipEventDisableSystemFence "
                                        "event between batches; per HVP = batch / 10"}
        out["hvp_warm_gbps"] = b_hvp / (med * 1e-6) / 1e9
        out["hvp_warm_frac"] = {"of_8.0_TBps": out["hvp_warm_gbps"] / HBM_PEAK_GBPS,
                                "of_6.29_TBps_copy": out["hvp_warm_gbps"] / 6290.0}
        med_t = float(np.median(us_t))
        out["hvp_warm_us_bracketed"] = {"median": med_t, "p10": float(np.percentile(us_t, 10)),
                                        "p90": float(np.percentile(us_t, 90)),
                                        "frac_of_8.0_TBps": b_hvp / (med_t * 1e-6) / 1e9 / HBM_PEAK_GBPS,
                                        "events": "torch.cuda.Event pair around each HVP (rounds 1-4)"}
    if rank == 0 and solo and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(A, b, args.cpu_seconds, label)
    if rank == 0:
        print(json.dumps(out), flush=True)
    problem.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
