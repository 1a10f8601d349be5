"""Batched compute_loss_of_iterates (opt_trace.py:39-41).

The optimizer keeps a device copy of every stored iterate next to its pinned
host copy; Trace.compute_loss_of_iterates then evaluates all of them in one
krcn_loss_values submission instead of one upload + X x + loss reduction +
sync per iterate.  The values, their order and the best-iterate tracking
(f_opt / x_opt, loss.py:66-73) must be BITWISE those of the per-iterate loop.
"""
import numpy as np
import pytest
import torch

from krcn import synth
from optimizer.cubic import Cubic_Krylov_LS
from optimizer.loss import LogisticRegression

pytestmark = pytest.mark.gpu


def host(x):
    return x.detach().cpu().numpy() if isinstance(x, torch.Tensor) else np.array(x)


def run(A, b, steps, m, l2=0.0):
    loss = LogisticRegression(A, b, l1=0, l2=l2, store_mat_vec_prod=True)
    opt = Cubic_Krylov_LS(loss=loss, reg_coef=1e-3, label="k", subspace_dim=m, tolerance=1e-9, tqdm=False)
    tr = opt.run(x0=np.full(A.shape[1], 0.5), it_max=steps)
    return loss, opt, tr


@pytest.mark.parametrize("l2", [0.0, 1e-3])
def test_batched_values_bitwise_per_iterate(l2):
    A, b = synth.make_problem("rcv1")
    loss, opt, tr = run(A, b, 6, 20, l2)
    assert len(tr._dev) == len(tr.xs) == 7
    opt.compute_loss_of_iterates()
    batched = np.array(tr.loss_vals)
    f_opt, x_opt = loss.f_opt, host(loss.x_opt)
    # the same iterates through the per-iterate loop (no device copies)
    loss.f_opt, loss.x_opt = np.inf, None
    tr.loss_vals, tr._dev = [], {}
    opt.compute_loss_of_iterates()
    np.testing.assert_array_equal(batched, np.array(tr.loss_vals))
    assert loss.f_opt == f_opt
    np.testing.assert_array_equal(host(loss.x_opt), x_opt)


def test_partial_device_copies_and_pickle(tmp_path):
    """Iterates without a device copy (past the budget) go through the loop in
    place; a saved trace carries no device tensors."""
    A, b = synth.make_problem("rcv1")
    loss, opt, tr = run(A, b, 4, 10)
    keys = list(tr._dev)
    del tr._dev[keys[1]], tr._dev[keys[3]]
    opt.compute_loss_of_iterates()
    mixed = np.array(tr.loss_vals)
    tr.loss_vals, tr._dev = [], {}
    opt.compute_loss_of_iterates()
    np.testing.assert_array_equal(mixed, np.array(tr.loss_vals))
    tr.save("t.pkl", path=str(tmp_path))
    import pickle
    back = pickle.load(open(tmp_path / "t.pkl", "rb"))
    assert back._dev == {} and len(back.xs) == len(tr.xs)
