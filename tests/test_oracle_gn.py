"""The GN oracle itself: structured vs explicit normal equations, and the GN
optimum vs an independent optimiser (scipy least_squares on the same objective)."""
import numpy as np
import pytest
from scipy.optimize import least_squares

from mhe import configs
from oracle import gn


def _problem(w):
    return gn.Problem(w.N, w.T, w.n, w.m, w.dyn, w.meas, w.cpm.D, (w.T / 2) * w.cpm.w,
                      w.cpm.lagrange_matrix(w.t_meas), w.Qw, w.Rw, Pw=w.Pw, meas_static=w.meas_static)


@pytest.mark.parametrize("make,kw", [(configs.make_c1, {}), (configs.make_c2, {"B": 2, "N": 20})])
def test_structured_equals_explicit(make, kw):
    w = make(**kw)
    pb = _problem(w)
    U = np.broadcast_to(w.U, (w.B,) + w.U.shape[1:])
    H1, g1, c1 = gn.normal_equations(pb, w.X_init, U, w.Y)
    H2, g2, c2 = gn.normal_equations_explicit(pb, w.X_init, U, w.Y)
    assert np.abs(H1 - H2).max() <= 1e-13 * np.abs(H2).max()
    assert np.abs(g1 - g2).max() <= 1e-12 * np.abs(g2).max()
    assert np.allclose(c1, c2, rtol=1e-13)


def test_gn_optimum_matches_least_squares():
    w = configs.make_c2(B=1, N=30)
    pb = _problem(w)
    U = np.broadcast_to(w.U, (1,) + w.U.shape[1:])
    X, cost, iters, status = gn.gauss_newton(pb, w.X_init, U, w.Y, max_iter=40, tol=1e-13)
    assert status[0] == gn.OK

    def resid(xf):
        Wd, _, e, _ = gn.residuals(pb, xf.reshape(1, w.P, w.n), U, w.Y)
        rd = (np.sqrt(pb.c)[:, None] * Wd[0] * np.sqrt(np.diag(pb.Qw))[None, :]).ravel()
        rm = (e[0] * np.sqrt(np.array([np.diag(r) for r in pb.Rw]))).ravel()
        return np.concatenate([rd, rm])

    sol = least_squares(resid, w.X_init[0].ravel(), jac="3-point", xtol=1e-15, ftol=1e-15, gtol=1e-15,
                        method="lm")
    # LM with a finite-difference Jacobian terminates on its own ftol: loose
    assert np.abs(sol.x.reshape(w.P, w.n) - X[0]).max() <= 2e-6 * (1 + np.abs(X[0]).max())
    assert abs(2 * sol.cost - cost[0]) <= 1e-10 * cost[0]
    assert 2 * sol.cost >= cost[0] * (1 - 1e-14)  # GN is at least as good


def test_gn_optimum_is_stationary_fd():
    """Independent of every Jacobian formula: central-difference gradient of the
    reference objective at the GN optimum is ~0 (relative to the initial gradient)."""
    w = configs.make_c2(B=1, N=20)
    pb = _problem(w)
    U = np.broadcast_to(w.U, (1,) + w.U.shape[1:])
    X, cost, iters, status = gn.gauss_newton(pb, w.X_init, U, w.Y, max_iter=40, tol=1e-13)

    def J(x):
        return gn.residuals(pb, x.reshape(1, w.P, w.n), U, w.Y)[3][0]

    def fd_grad(x, h=1e-6):
        g = np.zeros_like(x)
        for i in range(x.size):
            e = np.zeros_like(x); e[i] = h
            g[i] = (J(x + e) - J(x - e)) / (2 * h)
        return g

    g0 = fd_grad(w.X_init[0].ravel())
    gs = fd_grad(X[0].ravel())
    assert np.abs(gs).max() <= 1e-6 * np.abs(g0).max()


def _huber_problem(w, delta=0.05, lb=None, ub=None):
    return gn.Problem(w.N, w.T, w.n, w.m, w.dyn, w.meas, w.cpm.D, (w.T / 2) * w.cpm.w,
                      w.cpm.lagrange_matrix(w.t_meas), w.Qw, w.Rw, Pw=w.Pw, meas_static=w.meas_static,
                      dyn_cost="huber", delta=delta, lb=lb, ub=ub)


def test_huber_structured_equals_explicit():
    w = configs.make_c2(B=2, N=20)
    pb = _huber_problem(w)
    U = np.broadcast_to(w.U, (w.B,) + w.U.shape[1:])
    H1, g1, c1 = gn.normal_equations(pb, w.X_init, U, w.Y)
    H2, g2, c2 = gn.normal_equations_explicit(pb, w.X_init, U, w.Y)
    assert np.abs(H1 - H2).max() <= 1e-13 * np.abs(H2).max()
    assert np.abs(g1 - g2).max() <= 1e-12 * np.abs(g2).max()
    assert np.allclose(c1, c2, rtol=1e-13)


def test_huber_gn_optimum_is_stationary_fd():
    """The IRLS fixed point is a stationary point of the pseudo-Huber objective
    (cost_functions.py:25-31): central-difference gradient ~ 0."""
    w = configs.make_c2(B=1, N=15)
    pb = _huber_problem(w, delta=0.02)
    U = np.broadcast_to(w.U, (1,) + w.U.shape[1:])
    X, cost, iters, status = gn.gauss_newton(pb, w.X_init, U, w.Y, max_iter=400, tol=1e-10)
    assert status[0] == gn.OK  # IRLS: linear convergence (~110 iterations here)
    x = X.ravel()
    grad = np.zeros_like(x)
    h = 1e-6
    for i in range(x.size):
        xp, xm = x.copy(), x.copy()
        xp[i] += h
        xm[i] -= h
        grad[i] = (gn.residuals(pb, xp.reshape(X.shape), U, w.Y)[3][0] -
                   gn.residuals(pb, xm.reshape(X.shape), U, w.Y)[3][0]) / (2 * h)
    _, g, _ = gn.normal_equations(pb, X, U, w.Y)
    assert np.abs(grad).max() <= 1e-5 * max(1.0, cost[0])
    assert np.abs(2 * g[0]).max() <= 1e-7 * max(1.0, cost[0])


def _bounded(w, lb, ub):
    return gn.Problem(w.N, w.T, w.n, w.m, w.dyn, w.meas, w.cpm.D, (w.T / 2) * w.cpm.w,
                      w.cpm.lagrange_matrix(w.t_meas), w.Qw, w.Rw, Pw=w.Pw, meas_static=w.meas_static,
                      lb=lb, ub=ub)


def test_inactive_bounds_change_nothing():
    w = configs.make_c2(B=2, N=20)
    U = np.broadcast_to(w.U, (w.B,) + w.U.shape[1:])
    Xf, cf, itf, sf = gn.gauss_newton(_problem(w), w.X_init, U, w.Y, max_iter=30, tol=1e-10)
    Xl, cl, itl, sl = gn.gauss_newton(_bounded(w, [-10, -10], [10, 10]), w.X_init, U, w.Y, max_iter=30, tol=1e-10)
    assert sl.tolist() == sf.tolist() == [gn.OK] * 2 and np.all(np.abs(itl - itf) <= 1)
    assert np.abs(Xl - Xf).max() <= 1e-10 * (1 + np.abs(Xf).max())


BOXES = [([-np.inf, 0.5], [np.inf, np.inf]),     # the advisor's case: lb x[1] >= 0.5
         ([-np.inf, 0.5], [1.5, np.inf]),
         ([-0.5, -1.0], [0.5, 1.0])]             # both components boxed, many active entries


@pytest.mark.parametrize("lb,ub", BOXES)
def test_bounded_optimum_is_kkt_and_matches_lbfgsb(lb, ub):
    """The projected Newton limit is a KKT point of the bound-constrained problem
    (stationary on the free entries, gradient pointing out of the box on the active
    ones) and reaches the cost an independent bound-constrained optimiser
    (scipy L-BFGS-B on the same objective and analytic gradient) reaches.  Plain
    step clipping stopped at a non-KKT point up to 4x costlier."""
    from scipy.optimize import minimize
    w = configs.make_c2(B=3, N=20)
    U = np.broadcast_to(w.U, (w.B,) + w.U.shape[1:])
    pb = _bounded(w, lb, ub)
    X, cost, iters, status = gn.gauss_newton(pb, w.X_init, U, w.Y, max_iter=60, tol=1e-10)
    assert status.tolist() == [gn.OK] * w.B
    lo, hi = gn.box(pb, X.shape)
    assert np.all(X >= lo) and np.all(X <= hi) and np.any((X == lo) | (X == hi))
    _, g0, _ = gn.normal_equations(pb, np.clip(w.X_init, lo, hi), U, w.Y)
    kkt = gn.kkt_residual(pb, X, U, w.Y)
    assert np.all(kkt <= 1e-9 * np.abs(2 * g0).max(axis=1))
    for b in range(w.B):
        def f(x):
            return gn.residuals(pb, x.reshape(1, w.P, w.n), U[b:b + 1], w.Y[b:b + 1])[3][0]

        def grad(x):
            return 2 * gn.normal_equations(pb, x.reshape(1, w.P, w.n), U[b:b + 1], w.Y[b:b + 1])[1][0]
        r = minimize(f, np.clip(w.X_init[b], lo[b], hi[b]).ravel(), jac=grad, method="L-BFGS-B",
                     bounds=list(zip(lo[b].ravel(), hi[b].ravel())),
                     options=dict(maxiter=20000, ftol=1e-15, gtol=1e-12, maxcor=50))
        assert cost[b] <= r.fun * (1 + 1e-12)
        assert np.abs(X[b] - r.x.reshape(w.P, w.n)).max() <= 1e-5 * (1 + np.abs(X[b]).max())


def test_bounded_status_and_start_projection():
    """The initial iterate is projected onto the box; max_iter = 0 returns it."""
    w = configs.make_c2(B=2, N=20)
    U = np.broadcast_to(w.U, (w.B,) + w.U.shape[1:])
    pb = _bounded(w, [-np.inf, 0.5], [np.inf, np.inf])
    X, cost, iters, status = gn.gauss_newton(pb, w.X_init, U, w.Y, max_iter=0, tol=1e-10)
    assert np.array_equal(X[..., 1], np.maximum(w.X_init[..., 1], 0.5)) and iters.tolist() == [0, 0]
    assert status.tolist() == [gn.MAXITER] * 2
    assert np.allclose(cost, gn.residuals(pb, X, U, w.Y)[3], rtol=1e-14)
