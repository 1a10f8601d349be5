"""Host-side logic of the drop-in package (no GPU): the m x m cubic subproblem,
label mapping, the optimizer's checkpoint schedule and the trace."""
import numpy as np
import pytest

from optimizer import cubic as C
from optimizer import loss as L
from optimizer.optimizer import Optimizer


def test_cubic_solver_root_matches_reference(f3):
    """The product's host subproblem is bit-identical to the reference's
    (same expression order, same LAPACK calls)."""
    for m in (3, 10, 50):
        for k in range(3):
            key = f"m{m}_k{k}"
            s, its, r, dec = C.cubic_solver_root(f3[f"{key}_g"], f3[f"{key}_T"], float(f3[f"{key}_M"]),
                                                 epsilon=1e-8, r0=float(f3[f"{key}_r0"]))
            np.testing.assert_array_equal(s, f3[f"{key}_s"])
            assert its == f3[f"{key}_its"]
            assert r == f3[f"{key}_r"]
            assert dec == f3[f"{key}_dec"]


@pytest.mark.parametrize("b,expect", [
    ([-1, 1, 1, -1], [0, 1, 1, 0]),
    ([1, 2, 2], [0, 1, 1]),
    ([0, 1, 0], [0, 1, 0]),
    ([3, 7, 3], [1, 0, 1]),
])
def test_label_mapping(b, expect):
    np.testing.assert_array_equal(L._labels01(np.array(b)), expect)


def test_label_mapping_rejects_multiclass():
    with pytest.raises(ValueError):
        L._labels01(np.array([0, 1, 2]))


class _HostLoss:
    """Minimal stand-in with the device-loss vector hooks (host numpy)."""
    regularizer = None
    f_opt = np.inf
    x_opt = None
    n = 10

    def to_device(self, x, copy=False):
        return np.array(x, copy=True)

    def to_host(self, x):
        return np.array(x, copy=True)

    def copy_vector(self, x):
        return np.array(x, copy=True)

    def norm_diff(self, a, b=None):
        return float(np.linalg.norm(a - (0 if b is None else b)))

    def reset(self):
        pass

    def value(self, x):
        return float(np.sum(x ** 2))


class _Halving(Optimizer):
    def step(self):
        self.x = self.x / 2


def test_checkpoint_schedule_and_tolerance():
    opt = _Halving(loss=_HostLoss(), trace_len=20, tolerance=1e-3, tqdm=False)
    tr = opt.run(np.ones(4), it_max=1000)
    # stops once ||x_k - x_{k-1}|| < tol:  ||x_k - x_{k-1}|| = 2 * 2^-k
    assert opt.it == 11
    assert tr.its == [0, 1, 2, 3, 4, 5]   # x0 + the first save_first_iterations (5) steps
    assert len(tr.xs) == len(tr.its) == len(tr.ts)
    opt.compute_loss_of_iterates()
    np.testing.assert_allclose(tr.loss_vals, [float(np.sum(x ** 2)) for x in tr.xs])


def test_iteration_budget_default():
    opt = _Halving(loss=_HostLoss(), tqdm=False)
    opt.run(np.ones(2))          # neither t_max nor it_max: 100 iterations
    assert opt.it == 100


def test_lanczos_without_gpu_fails_loudly():
    """A callable operator runs the recurrence on the device; without a GPU
    there is no CPU path to fall back to."""
    with pytest.raises(RuntimeError):
        C.Lanczos(lambda v: v, np.ones(3), 2)
    with pytest.raises(TypeError):
        C.Lanczos(np.eye(3), np.ones(3), 2)


def test_comparison_methods_construct_like_the_reference():
    """Cubic_LS / SSCN keep the reference's constructor (cubic.py:128-150,
    335-347): solver selection, the unrecognised-solver message, SSCN's
    tolerance = 0."""
    opt = C.Cubic_LS(loss=_HostLoss(), reg_coef=1e-3, cubic_solver="full", tqdm=False)
    assert opt.cubic_solver == opt.cubic_solver_root_full
    opt = C.Cubic_LS(loss=_HostLoss(), reg_coef=1e-3, tqdm=False)
    assert opt.cubic_solver == opt.cubic_solver_root_CG
    opt = C.SSCN(loss=_HostLoss(), reg_coef=1e-3, subspace_dim=7, tolerance=1e-3, tqdm=False)
    assert opt.tolerance == 0 and opt.subspace_dim == 7 and opt.r0 == 0.1


def test_tridiagonal_subproblem_matches_dense_reference(f3):
    """cubic_solver_root_tridiag (O(m) LDL^T solves) against the reference's
    dense cubic_solver_root outputs: same Newton iteration count, s / lam /
    model decrease to rounding (measured <= 7e-16 relative)."""
    for m in (3, 10, 50):
        for k in range(3):
            key = f"m{m}_k{k}"
            T = f3[f"{key}_T"]
            s, its, r, dec = C.cubic_solver_root_tridiag(f3[f"{key}_g"], np.diag(T), np.diag(T, 1),
                                                         float(f3[f"{key}_M"]), epsilon=1e-8,
                                                         r0=float(f3[f"{key}_r0"]))
            assert its == f3[f"{key}_its"]
            ref = f3[f"{key}_s"]
            assert np.abs(s - ref).max() <= 1e-13 * np.abs(ref).max()
            assert abs(r - f3[f"{key}_r"]) <= 1e-13 * abs(f3[f"{key}_r"])
            assert abs(dec - f3[f"{key}_dec"]) <= 1e-13 * abs(f3[f"{key}_dec"])


def test_tridiagonal_subproblem_indefinite_raises():
    import numpy.linalg as la
    import pytest
    g = np.array([1.0, 0.0, 0.0])
    with pytest.raises(la.LinAlgError):
        C.cubic_solver_root_tridiag(g, np.array([-5.0, 1.0, 1.0]), np.array([0.1, 0.1]), 1e-3, r0=0.1)
