"""Pseudo-Huber dynamics cost (IRLS) and variable bounds (projected Newton with an
Armijo search along the projection arc) on the GPU vs the CPU oracle (oracle/gn.py:
same iteration -- cost_functions.py:25-31, nlp/nlp.py:314-317).

Tolerances as tests/test_gpu_parity.py: assembled H, g <= 1e-12 relative; iterates
<= 1e-9 (1 + max|X|) after the same number of iterations; converged <= 1e-8;
bound satisfaction exact (the projection clips to the bound value).
"""

import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

from mhe import configs, solver  # noqa: E402
from oracle import gn  # noqa: E402

DELTA = 0.02


def _pb(w, **kw):
    return gn.Problem(w.N, w.T, w.n, w.m, w.dyn, w.meas, w.cpm.D, (w.T / 2) * w.cpm.w,
                      w.cpm.lagrange_matrix(w.t_meas), w.Qw, w.Rw, Pw=w.Pw, meas_static=w.meas_static, **kw)


def _U(w):
    return np.broadcast_to(w.U, (w.B,) + w.U.shape[1:])


def _np(ts):
    return [t.cpu().numpy() for t in ts]


def test_huber_assembly_matches_oracle():
    w = configs.make_c2(B=3, N=20)
    s = solver.from_workload(w, dyn_cost="huber", huber_delta=DELTA)
    H, g, cost = _np(s.assemble(w.X_init, w.U, w.Y))
    Hr, gr, cr = gn.normal_equations(_pb(w, dyn_cost="huber", delta=DELTA), w.X_init, _U(w), w.Y)
    d = Hr.shape[1]
    assert np.abs(H[:, :d, :d] - Hr).max() <= 1e-12 * np.abs(Hr).max()
    assert np.abs(g[:, :d] - gr).max() <= 1e-12 * np.abs(gr).max()
    assert np.allclose(cost, cr, rtol=1e-12)


@pytest.mark.parametrize("max_iter,tol", [(5, 0.0), (400, 1e-10)])
def test_huber_iterates_match_oracle(max_iter, tol):
    w = configs.make_c2(B=4, N=20)
    s = solver.from_workload(w, dyn_cost="huber", huber_delta=DELTA)
    X, cost, iters, status = _np(s.solve(w.X_init, w.U, w.Y, max_iter=max_iter, tol=tol))
    Xr, cr, ir, sr = gn.gauss_newton(_pb(w, dyn_cost="huber", delta=DELTA), w.X_init, _U(w), w.Y,
                                     max_iter=max_iter, tol=tol)
    assert status.tolist() == sr.tolist()
    assert np.all(np.abs(iters - ir) <= (0 if tol == 0 else 1))
    lim = 1e-9 if tol == 0 else 1e-8
    assert np.abs(X - Xr).max() <= lim * (1 + np.abs(Xr).max())
    assert np.allclose(cost, cr, rtol=lim)


def _bounds_case():
    w = configs.make_c2(B=4, N=20)
    bounds = [(1, 0.5, np.inf), (0, -np.inf, 1.5)]
    pb = _pb(w, lb=[-np.inf, 0.5], ub=[1.5, np.inf])
    return w, bounds, pb


def _check_bounds(w, X, cost, iters, status, pb):
    Xr, cr, ir, sr = gn.gauss_newton(pb, w.X_init, _U(w), w.Y, max_iter=30, tol=1e-10)
    assert (X[:, :, 1] >= 0.5).all() and (X[:, :, 0] <= 1.5).all()
    assert (X[:, :, 1] == 0.5).any(), "the test bound should be active"
    assert status.tolist() == sr.tolist() == [gn.OK] * w.B and np.all(np.abs(iters - ir) <= 1)
    assert np.abs(X - Xr).max() <= 1e-8 * (1 + np.abs(Xr).max())
    assert np.allclose(cost, cr, rtol=1e-8)
    # a KKT point of the bound-constrained problem, not just the oracle's iterate
    lo, hi = gn.box(pb, X.shape)
    _, g0, _ = gn.normal_equations(pb, np.clip(w.X_init, lo, hi), _U(w), w.Y)
    assert np.all(gn.kkt_residual(pb, X, _U(w), w.Y) <= 1e-9 * np.abs(2 * g0).max(axis=1))


def test_bounds_iterates_match_oracle_fixed_count():
    """Same active sets and line-search decisions: iterates after 6 steps (tol 0)."""
    w, bounds, pb = _bounds_case()
    s = solver.from_workload(w, bounds=bounds)
    X, cost, iters, status = _np(s.solve(w.X_init, w.U, w.Y, max_iter=6, tol=0.0))
    Xr, cr, ir, sr = gn.gauss_newton(pb, w.X_init, _U(w), w.Y, max_iter=6, tol=0.0)
    assert iters.tolist() == ir.tolist() == [6] * w.B and status.tolist() == sr.tolist()
    assert np.abs(X - Xr).max() <= 1e-9 * (1 + np.abs(Xr).max())
    assert np.allclose(cost, cr, rtol=1e-10)


def test_bounds_projected_newton_register_path():
    w, bounds, pb = _bounds_case()
    s = solver.from_workload(w, bounds=bounds)
    _check_bounds(w, *_np(s.solve(w.X_init, w.U, w.Y, max_iter=30, tol=1e-10)), pb)


def test_bounds_projected_newton_large_system_path():
    w, bounds, pb = _bounds_case()
    s = solver.from_workload(w, bounds=bounds, force_large=True)
    assert s.large_system
    _check_bounds(w, *_np(s.solve(w.X_init, w.U, w.Y, max_iter=30, tol=1e-10)), pb)


def test_bounds_iterates_match_oracle_fixed_count_large_system_path():
    w, bounds, pb = _bounds_case()
    s = solver.from_workload(w, bounds=bounds, force_large=True)
    X, cost, iters, status = _np(s.solve(w.X_init, w.U, w.Y, max_iter=6, tol=0.0))
    Xr, cr, ir, sr = gn.gauss_newton(pb, w.X_init, _U(w), w.Y, max_iter=6, tol=0.0)
    assert iters.tolist() == ir.tolist() == [6] * w.B and status.tolist() == sr.tolist()
    assert np.abs(X - Xr).max() <= 1e-9 * (1 + np.abs(Xr).max())
    assert np.allclose(cost, cr, rtol=1e-10)


def _backtracking_case():
    """A far start (4 X_init) under the same bounds: the oracle's Armijo search
    halves the step several times (6 of the 8 x B steps, one of them twice) (the line search must use the gradient
    at the iterate, not the forward-substituted right-hand side)."""
    w, bounds, pb = _bounds_case()
    X0 = 4.0 * w.X_init
    trace = []
    Xr, cr, ir, sr = gn.gauss_newton(pb, X0, _U(w), w.Y, max_iter=8, tol=0.0, trace=trace)
    assert sum(a < 1.0 for _, _, a in trace) >= 4, "the case should backtrack"
    return w, bounds, pb, X0, (Xr, cr, ir, sr)


@pytest.mark.parametrize("force_large", [False, True])
def test_bounds_line_search_backtracking_matches_oracle(force_large):
    """Same accept / backtrack decisions as the oracle: iterates after 8 steps (tol 0)
    with several halvings, on the register-resident and the large-system path."""
    w, bounds, pb, X0, (Xr, cr, ir, sr) = _backtracking_case()
    s = solver.from_workload(w, bounds=bounds, force_large=force_large)
    assert s.large_system == force_large
    X, cost, iters, status = _np(s.solve(X0, w.U, w.Y, max_iter=8, tol=0.0))
    err = np.abs(X - Xr).max()
    print(f"backtracking case (force_large={force_large}): max |X - X_oracle| = {err:.3e}")
    assert iters.tolist() == ir.tolist() == [8] * w.B and status.tolist() == sr.tolist()
    assert err <= 1e-9 * (1 + np.abs(Xr).max())
    assert np.allclose(cost, cr, rtol=1e-10)


@pytest.mark.parametrize("max_iter,tol", [(5, 0.0), (400, 1e-10)])
def test_huber_large_system_path_matches_oracle(max_iter, tol):
    """pseudo-Huber on the large-system path (d = 302 > 208 by size):
    IRLS weights in k_big_resid, a^2 D^T diag(c lambda) D blocks in k_big_assemble."""
    w = configs.make_c2(B=3, N=150)
    s = solver.from_workload(w, dyn_cost="huber", huber_delta=DELTA)
    assert s.large_system
    X, cost, iters, status = _np(s.solve(w.X_init, w.U, w.Y, max_iter=max_iter, tol=tol))
    Xr, cr, ir, sr = gn.gauss_newton(_pb(w, dyn_cost="huber", delta=DELTA), w.X_init, _U(w), w.Y,
                                     max_iter=max_iter, tol=tol)
    assert status.tolist() == sr.tolist()
    assert np.all(np.abs(iters - ir) <= (0 if tol == 0 else 1))
    lim = 1e-10 if tol == 0 else 1e-8
    err = np.abs(X - Xr).max()
    print(f"huber large path ({max_iter}, {tol}): max err {err:.3e}")
    assert err <= lim * (1 + np.abs(Xr).max())
    assert np.allclose(cost, cr, rtol=lim)


def test_huber_large_and_register_paths_agree():
    w = configs.make_c2(B=4, N=20)
    sr_ = solver.from_workload(w, dyn_cost="huber", huber_delta=DELTA)
    sb = solver.from_workload(w, dyn_cost="huber", huber_delta=DELTA, force_large=True)
    a = _np(sr_.solve(w.X_init, w.U, w.Y, max_iter=6, tol=0.0))
    b = _np(sb.solve(w.X_init, w.U, w.Y, max_iter=6, tol=0.0))
    assert np.abs(a[0] - b[0]).max() <= 1e-10 * (1 + np.abs(a[0]).max())
    assert np.allclose(a[1], b[1], rtol=1e-10)


def test_facade_huber_and_bounds_match_oracle():
    """nlp.NLP path: addDynamicsCost(pseudo_huber_loss) + addVarBounds, as autonomous-car.py."""
    import nlp.cost_functions as cost_functions
    import nlp.dynamics as dynamics
    import nlp.measurements as measurements
    import nlp.nlp as nlp
    w = configs.make_c2(B=1, N=20)
    Q = np.linalg.inv(w.Qw)
    problem = nlp.fixedTimeOptimalEstimationNLP(w.N, w.T, w.n, w.m)
    X = problem.addVariables(w.N + 1, w.n, name="x")
    t_nodes = w.cpm.tau2t(w.cpm.tau)
    problem.addDynamics(dynamics.van_der_pol, X, t_nodes, np.zeros((1, w.N + 1)))
    problem.addDynamicsCost(cost_functions.pseudo_huber_loss, None, {"Q": np.linalg.inv(Q), "delta": DELTA})
    problem.addResidualCost(measurements.full_state, X, w.t_meas, w.Y[0].T, w.Rw[0])
    problem.addVarBounds(X, 1, 0.5, np.inf)
    problem.initializeEstimate(X, t_nodes, w.X_init[0].T)
    problem.max_iter, problem.tol = 40, 0.0  # same iteration count on both sides (projected Newton, IRLS)
    problem.solve()
    Xg = np.stack([problem.extractVariableValue("x", k) for k in range(w.N + 1)])
    pb = _pb(w, dyn_cost="huber", delta=DELTA, lb=[-np.inf, 0.5], ub=[np.inf, np.inf])
    Xr, cr, ir, sr = gn.gauss_newton(pb, w.X_init, _U(w), w.Y, max_iter=40, tol=0.0)
    assert problem.solver["iter_count"] == ir[0] == 40
    assert (Xg[:, 1] >= 0.5).all() and not problem.solver["bounds_violated"]
    assert np.abs(Xg - Xr[0]).max() <= 1e-8 * (1 + np.abs(Xr).max())
    assert np.isclose(problem.solver["objective"], cr[0], rtol=1e-8)
