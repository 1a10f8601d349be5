"""Benchmark of the Krylov-CRN hot path: Hessian-vector products / s on MI355X.

Workload (BASELINE.json metric: "HVP/s + achieved HBM GB/s, news20 CSR"):
news20-shaped synthetic CSR (n 19,996, d 1,355,191, nnz 9,097,916, fp64,
krcn.synth, seed 20240117), Krylov subspace m = 100 (configs[2]).  One step =
one full device Lanczos recurrence (cubic.py:77-111) from the gradient at
x = 0.5*1: m HVPs (loss.py:289-302) plus the Lanczos vector work, alphas/betas
returned to the host.  value = HVPs executed by the whole job / wall time.

Multi-GPU (torchrun, one process per GPU): the matrix is sharded across ranks
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
from krcn import synth  # noqa: E402

HBM_PEAK_GBPS = 8000.0   # MI355X_MICROARCH.md: 8.0 TB/s spec


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--config", default="news20", choices=sorted(synth.CONFIGS))
    p.add_argument("--m", type=int, default=None, help="Krylov dimension (default: the config's)")
    p.add_argument("--partition", default="auto", choices=["auto", "rows", "cols"])
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline budget")
    p.add_argument("--no-cold", action="store_true")
    p.add_argument("--traffic-json", default=os.path.join(REPO, "profiles", "traffic.json"))
    return p.parse_args()


def cpu_baseline(A, b, budget_s):
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
    return {"value": count / el, "unit": "HVP/s", "cores": 1, "kind": "port",
            "sample": f"{count} HVPs of the news20-shaped problem at x=0.5 (scipy csr_matvec/csc_matvec, "
                      f"expit; oracle/krcn_oracle.hess_vec_prod) in {el:.1f} s; host CPU {cpu}; "
                      f"{len(os.sched_getaffinity(0))} cores visible, 1 used"}


def flush_caches(buf):
    buf.add_(1.0)   # 512 MiB read+write evicts L2 and the 256 MiB Infinity Cache


def main():
    args = parse()
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

    A, b = synth.make_problem(args.config)
    n, d = A.shape
    nnz = A.nnz
    problem = kdist.ShardedProblem(A, b, dtype=dtype, partition=args.partition, device=dev)
    X = problem.X
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
    # this rank's launches; pass 2 is fused with Lanczos step A
    p1_bytes, p2_bytes = synth.lanczos_pass_bytes(X.n, X.d, X.nnz, s_val=s_val)
    p1_us = 1e3 * prof["pass1_ms"] / max(prof["count"], 1)
    p2_us = 1e3 * prof["pass2_ms"] / max(prof["count"], 1)
    plan = X.plan_info()

    def kname(key):
        S = plan[key][0]
        k = "k_sorted_pass" if S < 0 else "k_tiled_pass"
        return k + (f" over {abs(S)} column slices + k_slice_combine" if abs(S) > 1 else "")
    if p1_us > p2_us:
        dom, dom_key, dom_bytes, dom_us = (f"pass 1: X z + weights ({kname('pass1')}, SrcLzStep)",
                                           "pass1", p1_bytes, p1_us)
    else:
        dom, dom_key, dom_bytes, dom_us = (f"pass 2: X^T u fused with Lanczos step A ({kname('pass2')}, EpiLz2)",
                                           "pass2", p2_bytes, p2_us)
    achieved = dom_bytes / (dom_us * 1e-6) / 1e9
    traffic = None
    if os.path.exists(args.traffic_json):
        try:
            tj = json.load(open(args.traffic_json))
            traffic = tj.get(f"{args.config}:{world}", {}).get(dom_key)
        except Exception:
            traffic = None

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
        "data": "synthetic (krcn.synth, shape-matched to LIBSVM " + args.config + ", seed 20240117)",
        "config": {"workload": f"{args.config}: one device Lanczos (cubic.py:77-111) of m={m} HVPs per step"
                               + (" with CGS2 reorth" if reorth else ""),
                   "n": n, "d": d, "nnz": nnz, "m": m, "partition": problem.partition,
                   "parallelism": f"{problem.partition}-sharded x{world}" if world > 1 else "single GPU"},
        "achieved_hbm_gbps_hvp": b_hvp * hvp_per_s / 1e9,
        "hvp_bytes_algorithmic": b_hvp,
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": achieved, "peak": HBM_PEAK_GBPS,
                     "unit": "GB/s", "frac": achieved / HBM_PEAK_GBPS, "traffic": traffic,
                     "algorithmic_bytes_per_launch": dom_bytes, "avg_launch_us": dom_us,
                     "pass1_us": p1_us, "pass2_us": p2_us, "launches_timed": prof["count"],
                     "plan": {"pass1": list(plan["pass1"]), "pass2": list(plan["pass2"]),
                              "fields": "(slices, <0: sorted tiles), lanes, tiles, grid"},
                     "traffic_source": "profiles/traffic.json (rocprofv3 PMC, 2 x FETCH_SIZE + WRITE_SIZE)"},
        "cpu_baseline": None,
    }
    if not args.no_cold and world == 1:
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
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(A, b, args.cpu_seconds)
    if rank == 0:
        print(json.dumps(out), flush=True)
    problem.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
