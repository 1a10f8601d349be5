"""Plan A/B for one config: µs per HVP of a device Lanczos under several
(format, slicing) choices.  python3 tools/lz_fmt.py <config> <m> [fmt,slicing ...]"""
import sys, time, itertools
import numpy as np, torch
sys.path.insert(0, '/root/repo/krylov-cubic-regularized-newton_amd')
import krcn
from krcn import synth
cfg = sys.argv[1]; m = int(sys.argv[2])
A, b = synth.make_problem(cfg)
x = np.random.default_rng(0).uniform(-0.2, 0.2, A.shape[1])
import scipy.special as ss
t = A @ x
wts = ss.expit(-b * t) * ss.expit(b * t) if b is not None else np.full(A.shape[0], 0.25)
W = torch.from_numpy(wts).cuda()
g = torch.from_numpy(np.random.default_rng(1).standard_normal(A.shape[1])).cuda()
combos = [(0, 0)] + [tuple(int(v) for v in s.split(',')) for s in sys.argv[3:]]
for fmt, sl in combos:
    try:
        X = krcn.DeviceCSR(A, fmt=fmt, slicing=sl)
        pf, pi = X.plan_format(), X.plan_info()
    except Exception as e:
        print(fmt, sl, 'ERR', str(e)[:100]); continue
    for _ in range(3): X.lanczos(W, g, m)
    torch.cuda.synchronize()
    ts = []
    for _ in range(7):
        t0 = time.perf_counter(); X.lanczos(W, g, m); torch.cuda.synchronize(); ts.append(time.perf_counter() - t0)
    us = 1e6 * np.median(ts) / m
    print(f'fmt={fmt} sl={sl} {pf} {pi} {us:.2f} us/HVP {1e6/us:.0f} HVP/s', flush=True)
