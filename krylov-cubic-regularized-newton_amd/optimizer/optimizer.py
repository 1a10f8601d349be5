"""Optimizer run loop (same API as the reference's optimizer/optimizer.py:17-172).

The outer loop stays on the host, as north_star asks: `run` repeats
`step()` + `save_checkpoint()` until the iteration budget, the time budget or
the ||x_k - x_{k-1}|| < tolerance test fires.  The iterate itself stays on the
GPU (a torch tensor owned by the loss's device handle); it crosses PCIe only
when the trace stores a checkpoint, which is what the reference's deep copies
of numpy iterates amount to; those copies are asynchronous (pinned memory,
`loss.to_host_async`) and `run` waits for them before it returns.
"""
from __future__ import annotations

import time

import numpy as np

from .opt_trace import Trace


class Optimizer:
    """Base class of the optimizers (optimizer.py:17-62).

    loss: an Oracle (here a device LogisticRegression).  trace_len,
    save_first_iterations: checkpoint schedule.  tolerance: stationarity level
    on ||x_k - x_{k-1}||.  seeds: RNG seeds, one run each.  tqdm: progress bar.
    """

    def __init__(self, loss, trace_len=200, use_prox=True, tolerance=0, line_search=None,
                 save_first_iterations=5, label=None, seeds=None, tqdm=True):
        self.loss = loss
        self.trace_len = trace_len
        self.use_prox = use_prox and (getattr(loss, "regularizer", None) is not None)
        self.tolerance = tolerance
        self.line_search = line_search
        self.save_first_iterations = save_first_iterations
        self.label = label
        self.tqdm = tqdm
        self.initialized = False
        self.x_old_tol = None
        self.trace = Trace(loss=loss, label=label)
        self.seeds = [42] if seeds is None else list(seeds)
        self.finished_seeds = []

    # ------------------------------------------------------------------ run
    def run(self, x0, t_max=np.inf, it_max=np.inf, ls_it_max=None):
        """Run every seed until convergence (optimizer.py:63-102); returns the trace."""
        if t_max is np.inf and it_max is np.inf:
            it_max = 100
            print(f"{self.label}: The number of iterations is set to {it_max}.")
        self.t_max, self.it_max = t_max, it_max
        for seed in self.seeds:
            if seed in self.finished_seeds:
                continue
            if len(self.seeds) > 1:
                print(f"{self.label}: Running seed {seed}")
            self.rng = np.random.default_rng(seed)
            if ls_it_max is None:
                self.ls_it_max = it_max
            if not self.initialized:
                self.init_run(x0)
                self.initialized = True
            self._loop()
            sync = getattr(self.loss, "sync", None)
            if sync is not None:   # async checkpoint copies (update_trace) land
                sync()
            self.finished_seeds.append(seed)
            self.initialized = False
        return self.trace

    def _progress_value(self, by_iterations):
        if by_iterations and self.line_search is not None:
            return self.ls_it
        return self.it if by_iterations else self.t

    def _loop(self):
        by_iterations = self.ls_it_max is not np.inf
        bar = None
        if self.tqdm:
            from tqdm import tqdm
            bar = tqdm(total=self.ls_it_max if by_iterations else self.t_max)
        shown = 0
        try:
            while not self.check_convergence():
                if self.tolerance > 0:
                    self.x_old_tol = self.loss.copy_vector(self.x)
                self.step()
                self.save_checkpoint()
                now = self._progress_value(by_iterations)
                if bar is not None:
                    bar.update(now - shown)
                shown = now
        finally:
            if bar is not None:
                bar.close()

    def check_convergence(self):
        """Stop on iterations, wall time or ||x - x_old|| < tolerance (optimizer.py:104-113).
        In a distributed run every rank adopts rank-wide agreement (any rank stops)."""
        done = self.it >= self.it_max
        if self.line_search is not None:
            done = done or self.line_search.it >= self.ls_it_max
        done = done or (time.perf_counter() - self.t_start >= self.t_max)
        if self.tolerance > 0 and self.x_old_tol is not None:
            done = done or self.loss.norm_diff(self.x, self.x_old_tol) < self.tolerance
        agree = getattr(self.loss, "any_rank", None)
        return agree(done) if agree is not None else done

    def step(self):
        pass

    # ----------------------------------------------------------- checkpoints
    def init_run(self, x0):
        """optimizer.py:118-134; x0 is copied onto the loss's device."""
        self.dim = x0.shape[0]
        self.x = self.loss.to_device(x0, copy=True)
        self.trace.xs = [self.loss.to_host(self.x)]
        self._keep_device_iterate()
        self.trace.its = [0]
        self.trace.ts = [0]
        if self.line_search is not None:
            self.trace.ls_its = [0]
            self.trace.lrs = [self.line_search.lr]
        self.it = 0
        self.t = 0
        self.t_start = time.perf_counter()
        self.time_progress = 0
        self.iterations_progress = 0
        self.max_progress = 0
        if self.line_search is not None:
            self.line_search.reset(self)

    def should_update_trace(self):
        """First `save_first_iterations` steps, then about trace_len evenly spread
        checkpoints in time or iterations (optimizer.py:136-145)."""
        if self.it <= self.save_first_iterations:
            return True
        budget = self.trace_len - self.save_first_iterations
        self.time_progress = int(budget * self.t / self.t_max)
        self.iterations_progress = int(budget * (self.it / self.it_max))
        if self.line_search is not None:
            self.iterations_progress = max(self.iterations_progress,
                                           int(budget * (self.line_search.it / self.it_max)))
        return max(self.time_progress, self.iterations_progress) > self.max_progress

    def save_checkpoint(self):
        self.it += 1
        if self.line_search is not None:
            self.ls_it = self.line_search.it
        self.t = time.perf_counter() - self.t_start
        if self.should_update_trace():
            self.update_trace()
        self.max_progress = max(self.time_progress, self.iterations_progress)

    def update_trace(self):
        # an async D2H into pinned memory when the loss offers one: the copy
        # overlaps the next step, and run() waits for it before returning
        to_host = getattr(self.loss, "to_host_async", self.loss.to_host)
        self.trace.xs.append(to_host(self.x))
        self._keep_device_iterate()
        self.trace.ts.append(self.t)
        self.trace.its.append(self.it)
        if self.line_search is not None:
            self.trace.ls_its.append(self.line_search.it)
            self.trace.lrs.append(self.line_search.lr)

    def _keep_device_iterate(self):
        """A device copy of the iterate just stored (the loss decides within its
        memory budget): compute_loss_of_iterates then evaluates it in place."""
        keep = getattr(self.loss, "keep_device_iterate", None)
        if keep is not None and hasattr(self.trace, "keep_device"):
            self.trace.keep_device(self.trace.xs[-1], keep(self.x))

    def compute_loss_of_iterates(self):
        self.loss.reset()
        self.trace.compute_loss_of_iterates()

    def reset(self, loss):
        self.initialized = False
        self.x_old_tol = None
        self.trace = Trace(loss=loss, label=self.label)
        self.finished_seeds = []
