"""Run log of an optimizer (same API as the reference's optimizer/opt_trace.py:19-119).

Iterates are stored as host numpy copies, exactly like the reference's
deep-copied numpy xs, so `compute_loss_of_iterates`, plotting and pickling work
unchanged.  In a column-sharded distributed run each rank stores its own shard.

Provenance: the reference's Trace (optimizer/opt_trace.py:1-8) incorporates
code from "opt_methods" by Konstantin Mishchenko
(https://github.com/konstmish/opt_methods, optmethods/opt_trace.py), MIT
License; this class keeps that API (attribute and method names), so the same
attribution applies to its interface.
"""
from __future__ import annotations

import os
import pickle
import warnings
from pathlib import Path

import numpy as np


class Trace:
    """xs / ts / its / loss_vals of one run (opt_trace.py:19-37)."""

    def __init__(self, loss, label=None):
        self.loss = loss
        self.label = label
        self.xs = []
        self.ts = []
        self.its = []
        self.loss_vals = []
        self.its_converted_to_epochs = False
        self.ls_its = None
        self._dev = {}   # id(host iterate) -> (host iterate, its device copy)

    def keep_device(self, x_host, x_dev):
        """Remember the device copy of a stored iterate (Optimizer.update_trace),
        so compute_loss_of_iterates can evaluate it without an upload."""
        if x_dev is not None:
            self._dev[id(x_host)] = (x_host, x_dev)

    def compute_loss_of_iterates(self):
        """loss.value at every stored iterate (opt_trace.py:39-43).  With a
        device loss the iterates whose device copies were kept are evaluated
        in one batched submission (loss.values_of_iterates); values, their
        order and the best-iterate tracking are those of the per-iterate loop."""
        if len(self.loss_vals) != 0:
            warnings.warn("Loss values have already been computed. Set .loss_vals = [] to recompute.")
            return
        batch = getattr(self.loss, "values_of_iterates", None)
        if batch is not None:
            self.loss_vals = np.asarray(batch(self.xs, getattr(self, "_dev", {})))
        else:
            self.loss_vals = np.asarray([self.loss.value(x) for x in self.xs])

    def convert_its_to_epochs(self, batch_size=1):
        if self.its_converted_to_epochs:
            warnings.warn("The iteration count has already been converted to epochs.")
            return
        self.its = np.asarray(self.its) / (self.loss.n / batch_size)
        self.its_converted_to_epochs = True

    def _axis(self, its, use_ls_its, time):
        if its is not None:
            return its
        if use_ls_its and self.ls_its is not None:
            return self.ls_its
        return self.ts if time else self.its

    def plot_losses(self, its=None, f_opt=None, label=None, markevery=None, use_ls_its=True,
                    time=False, *args, **kwargs):
        import matplotlib.pyplot as plt
        label = self.label if label is None else label
        its = self._axis(its, use_ls_its, time)
        if len(self.loss_vals) == 0:
            self.compute_loss_of_iterates()
        f_opt = self.loss.f_opt if f_opt is None else f_opt
        markevery = max(1, len(self.loss_vals) // 20) if markevery is None else markevery
        plt.plot(its, self.loss_vals - f_opt, label=label, markevery=markevery, *args, **kwargs)
        plt.ylabel(r"$f(x)-f^*$")

    def plot_distances(self, its=None, x_opt=None, label=None, markevery=None, use_ls_its=True,
                       time=False, *args, **kwargs):
        import matplotlib.pyplot as plt
        its = self._axis(its, use_ls_its, time)
        if x_opt is None:
            x_opt = self.xs[-1] if self.loss.x_opt is None else self.loss.x_opt
            if hasattr(x_opt, "cpu"):
                x_opt = x_opt.cpu().numpy()
        label = self.label if label is None else label
        markevery = max(1, len(self.xs) // 20) if markevery is None else markevery
        dists = [float(np.linalg.norm(x - x_opt)) ** 2 for x in self.xs]
        plt.plot(its, dists, label=label, markevery=markevery, *args, **kwargs)
        plt.ylabel(r"$\Vert x-x^*\Vert^2$")

    @property
    def best_loss_value(self):
        if len(self.loss_vals) == 0:
            self.compute_loss_of_iterates()
        return np.min(self.loss_vals)

    def save(self, file_name, path="./results/"):
        """Pickle the trace without its loss object (opt_trace.py:102-108)."""
        keep, self.loss = self.loss, None
        keep_dev, self._dev = getattr(self, "_dev", {}), {}   # device copies do not travel
        try:
            Path(path).mkdir(parents=True, exist_ok=True)
            with open(os.path.join(path, file_name), "wb") as f:
                pickle.dump(self, f)
        finally:
            self.loss = keep
            self._dev = keep_dev

    @classmethod
    def from_pickle(cls, path, loss=None):
        """Load a trace this package saved (only the caller's own files)."""
        if not os.path.isfile(path):
            return None
        with open(path, "rb") as f:
            trace = pickle.load(f)
        trace.loss = loss
        if loss is not None and len(trace.loss_vals):
            loss.f_opt = min(np.min(trace.loss_vals), loss.f_opt)
        return trace
