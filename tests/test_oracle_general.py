"""Oracle for general problems (oracle/gn_general.py): mixed rows, extra variables,
equality constraints.

Pinning: every mixed-row encoding reproduces the reference plug-ins
(tests/golden/plugins.npz: values and complex-step / central-difference Jacobians
of nlp/measurements.py run by gen_golden.py); the GN solution of a constrained
problem satisfies the constraints and the KKT stationarity of the reference
objective (gradient checked against central differences of the cost).
"""
import numpy as np
import pytest

from oracle import gn
from oracle import gn_general as gg

from general_problems import multi_receiver_problem, row, two_receiver_problem


def _check(plugins, key, mk_row, n_x, H_tol=1e-9):
    xs, ys, Hs = plugins[f"meas_{key}_x"], plugins[f"meas_{key}_y"], plugins[f"meas_{key}_H"]
    for t in range(xs.shape[0]):
        par = plugins[f"meas_{key}_par"][t] if f"meas_{key}_par" in plugins.files else None
        h, G = gg.mixed_row(mk_row(par), xs[t])
        assert abs(h - float(np.ravel(ys[t])[0])) <= 1e-12 * max(1.0, abs(h)), (key, t)
        np.testing.assert_allclose(G[:n_x], np.ravel(Hs[t]), rtol=H_tol, atol=H_tol, err_msg=key)


def test_mixed_rows_match_reference_plugins(golden):
    p = golden["plugins"]
    _check(p, "pseudorange", lambda s: row(gg.ROW_PR, [0, 1, 2, 3], s[:3]), 5)
    _check(p, "vehicle_pseudorange", lambda s: row(gg.ROW_PR, [0, 1, 8, 6], s[:3]), 9)
    _check(p, "pseudorange_rate", lambda s: row(gg.ROW_PRR, [0, 1, 2, 4, 5, 6, 7], s[:6]), 8)
    _check(p, "multi_receiver_range_3d", lambda s: row(gg.ROW_R3, [0, 1, 2], s[:3]), 10)
    _check(p, "multi_receiver_range_2d", lambda s: row(gg.ROW_R2, [0, 1], s[:2]), 4)
    # "y" form: r_x = y0 - x[0], r_y = y1 - x[1]  (central differences in the fixture)
    _check(p, "multi_receiver_heading_2d", lambda s: row(gg.ROW_HEAD, [-1, 0, -1, 1], s[:2]), 4, H_tol=1e-7)
    _check(p, "range3d_AB", lambda s: row(gg.ROW_R3, [0, 1, 2, 5, 6, 7]), 10)
    _check(p, "range2d_AB", lambda s: row(gg.ROW_R2, [0, 1, 5, 6]), 10)
    # idxA/idxB form: r_x = x[5] - x[0] + 1e-5, r_y = x[6] - x[1]
    _check(p, "heading2d_AB", lambda s: row(gg.ROW_HEAD, [5, 0, 6, 1], [1e-5, 0.0]), 10, H_tol=1e-7)


def test_gradient_matches_cost_differences():
    pb, X0, U, Y, PAR, x0, _ = two_receiver_problem(N=4, B=1, seed=3)
    H, g, c0 = gg.normal_equations_full(pb, X0, None, U, Y, PAR, x0)
    rng = np.random.default_rng(0)
    v = X0[0].ravel()
    for _ in range(6):
        k = rng.integers(0, v.size)
        h = 1e-4
        Xp, Xm = X0.copy(), X0.copy()
        Xp.reshape(1, -1)[0, k] += h
        Xm.reshape(1, -1)[0, k] -= h
        fd = (gg.cost_full(pb, Xp, None, U, Y, PAR, x0)[0] - gg.cost_full(pb, Xm, None, U, Y, PAR, x0)[0]) / (2 * h)
        assert abs(fd - 2 * g[0, k]) <= 1e-5 * max(1.0, abs(fd)), (k, fd, 2 * g[0, k])


def _nullspace(C):
    u, s, vt = np.linalg.svd(C)
    r = int(np.sum(s > 1e-12 * s.max()))
    return vt[r:].T


def test_constrained_solution_is_kkt_point():
    pb, X0, U, Y, PAR, x0, _ = two_receiver_problem(B=2)
    X, Z, cost, iters, st = gg.gauss_newton_general(pb, X0, None, U, Y, PAR, x0, max_iter=30, tol=1e-12)
    assert (st == gn.OK).all(), st
    d = X.shape[1] * X.shape[2]
    C = gg.constraint_rows(pb, d, 0)
    Nz = _nullspace(C)
    for b in range(2):
        v = X[b].ravel()
        assert np.abs(C @ v).max() <= 1e-9
        _, g, _ = gg.normal_equations_full(pb, X[b:b + 1], None, U[b:b + 1], Y[b:b + 1], PAR[b:b + 1], x0[b:b + 1])
        assert np.abs(Nz.T @ g[0]).max() <= 1e-7 * max(1.0, np.abs(g[0]).max())


def test_constraint_met_after_first_step():
    pb, X0, U, Y, PAR, x0, _ = two_receiver_problem(B=1)
    X, _, _, _, _ = gg.gauss_newton_general(pb, X0, None, U, Y, PAR, x0, max_iter=1, tol=0.0)
    assert np.abs(X[0, :, 2] - X[0, :, 7]).max() <= 1e-9


def test_extra_variables_solution():
    pb, X0, Z0, U, Y, PAR, xt, zt = multi_receiver_problem()
    X, Z, cost, iters, st = gg.gauss_newton_general(pb, X0, Z0, U, Y, PAR, None, max_iter=30, tol=1e-12)
    assert (st == gn.OK).all(), st
    assert np.all(Z[:, 2] == 7.0)                      # held: no row depends on it
    assert np.abs(Z[:, :2] - zt[:, :2]).max() < 0.5     # recovered the static receiver
    for b in range(2):
        _, g, _ = gg.normal_equations_full(pb, X[b:b + 1], Z[b:b + 1], None, Y[b:b + 1], PAR[b:b + 1])
        assert np.abs(g[0]).max() <= 1e-6 * max(1.0, np.abs(Y).max())
