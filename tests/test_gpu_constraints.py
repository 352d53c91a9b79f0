"""Inequality constraints (nlp/nlp.py:49-50) and state bounds together with equality
rows (:52-53, :314-317) through the facade's active set over device GN solves.

Checks, at the device answer X*:
  * feasibility of every row and the multiplier signs mu >= 0 reported by the device;
  * the KKT conditions with the ORACLE's gradient of the reference objective
    (oracle/gn_general.normal_equations_full): grad J + C_A^T lambda = 0 over the
    equality rows and the active set, mu = s lambda >= 0 -- independent of the device's
    multipliers;
  * X* against the oracle's dense-KKT Gauss-Newton solve with the same rows held at
    equality: |dX| <= 1e-9 (1 + |X|) (the §8(c) iterate tolerance, a converged solve).
"""
import numpy as np
import pytest

import nlp.constraints as constraints
import nlp.cost_functions as cost_functions
import nlp.dynamics as dynamics
import nlp.measurements as measurements
import nlp.nlp as nlp
from mhe import configs
from oracle import gn_general as gg
from general_problems import row


def _problem(w):
    problem = nlp.fixedTimeOptimalEstimationNLP(w.N, w.T, w.n, w.m)
    X = problem.addVariables(w.N + 1, w.n, name="x")
    t_nodes = w.cpm.tau2t(w.cpm.tau)
    problem.addDynamics(dynamics.van_der_pol, X, t_nodes, np.zeros((1, w.N + 1)))
    problem.addDynamicsCost(cost_functions.weighted_l2_norm, None, {"Q": w.Qw})
    problem.addResidualCost(measurements.full_state, X, w.t_meas, w.Y[0].T, w.Rw[0])
    problem.initializeEstimate(X, t_nodes, w.X_init[0].T)
    problem.max_iter, problem.tol = 60, 1e-12
    return problem, X


def _oracle(w, eq, rhs):
    """The same objective as COMPONENT rows of the general oracle (dense KKT steps)."""
    n = w.n
    Phi = w.cpm.lagrange_matrix(w.t_meas)
    rows = np.array([row(gg.ROW_COMP, [a]) for i in range(Phi.shape[0]) for a in range(n)])
    Rw = np.array([w.Rw[i][a, a] for i in range(Phi.shape[0]) for a in range(n)])
    pb = gg.GeneralProblem(w.N, w.T, n, w.m, w.dyn, "mixed", w.cpm.D, (w.T / 2.0) * w.cpm.w,
                           np.repeat(Phi, n, axis=0), w.Qw, Rw, Pw=None, eq=eq, eq_rhs=rhs)
    U = np.broadcast_to(w.U, (1,) + w.U.shape[1:])
    return pb, U, w.Y[:1].reshape(1, -1, 1), rows[None]


def _solution(problem, w):
    return np.stack([problem.extractVariableValue("x", k) for k in range(w.N + 1)])


def _check(problem, w, eq_rows, ineq_rows):
    Xg = _solution(problem, w)
    v = Xg.ravel()
    assert problem.solver["success"], problem.solver
    gv = np.array([s * (v[a] - (v[b] if b >= 0 else 0.0) - r) for a, b, r, s in ineq_rows])
    scale = 1.0 + np.abs(v).max()
    assert gv.max() <= 1e-9 * scale, gv.max()
    act = problem.solver["active_set"]
    assert len(act) >= 1
    assert np.all(problem.solver["multipliers"] >= -1e-9 * (1 + np.abs(problem.solver["multipliers"]).max()))
    # KKT with the oracle's gradient
    allrows = [(a, b, r, 1.0) for a, b, r in eq_rows] + list(act)
    pb, U, Y, PAR = _oracle(w, None, None)
    _, g, _ = gg.normal_equations_full(pb, Xg[None], None, U, Y, PAR)
    g = g[0]
    C = np.zeros((len(allrows), v.size))
    for k, (a, b, r, s) in enumerate(allrows):
        C[k, a] += 1.0
        if b >= 0:
            C[k, b] -= 1.0
    lam, *_ = np.linalg.lstsq(C.T, -g, rcond=None)
    res = np.abs(g + C.T @ lam).max()
    mu = np.array([s for *_, s in act]) * lam[len(eq_rows):]
    print(f"KKT: |grad + C^T lam| = {res:.2e} (|grad| {np.abs(g).max():.2e}), min mu {mu.min():.3e}, "
          f"active {len(act)} of {len(ineq_rows)}")
    assert res <= 1e-6 * (1.0 + np.abs(g).max())
    assert mu.min() >= -1e-6 * (1.0 + np.abs(mu).max())
    # the oracle's solve with the same rows held at equality
    eq = np.array([(a, b) for a, b, *_ in allrows])
    rhs = np.array([r for _, _, r, _ in allrows])
    pb, U, Y, PAR = _oracle(w, eq, rhs)
    Xr, _, _, _, sr = gg.gauss_newton_general(pb, w.X_init[:1], None, U, Y, PAR, max_iter=60, tol=1e-12)
    err = np.abs(Xg - Xr[0]).max()
    print(f"X vs oracle (same active set): {err:.2e}")
    assert sr[0] == 0 and err <= 1e-9 * (1 + np.abs(Xr).max())
    return Xg


def test_ineq_rows_from_arguments():
    """Row encoding: element - element, element - constant, constant - element; bounds
    become rows only next to constraint rows."""
    w = configs.make_c2(B=1, N=6)
    problem, X = _problem(w)
    problem.addIneqConstraint(constraints.equality_constaint, [X[1][0], X[2][1]])
    problem.addIneqConstraint(constraints.equality_constaint, [X[3][0], 1.5])
    problem.addIneqConstraint(constraints.equality_constaint, [-0.5, X[4][1]])
    rows = problem._ineq_rows()
    assert rows == [(2, 5, 0.0, 1.0), (6, -1, 1.5, 1.0), (9, -1, -0.5, -1.0)]
    problem.addVarBounds(X, 1, -2.0, 3.0)
    assert len(problem._ineq_rows()) == 3 + 2 * (w.N + 1)
    with pytest.raises(nlp.UnsupportedFeature):
        problem.addIneqConstraint(constraints.equality_constaint, [1.0, 2.0])


@pytest.mark.gpu
def test_inequality_constraints_active_set_matches_oracle():
    w = configs.make_c2(B=1, N=16)
    base, _ = _problem(w)
    base.solve()
    X_free = _solution(base, w)
    cap = 0.8 * X_free[:, 0].max()          # active near the peaks of x_0
    problem, X = _problem(w)
    for j in range(w.N + 1):
        problem.addIneqConstraint(constraints.equality_constaint, [X[j][0], cap])
    problem.solve()
    rows = problem._ineq_rows()
    Xg = _check(problem, w, [], rows)
    assert Xg[:, 0].max() <= cap + 1e-9
    assert problem.solver["objective"] >= base.solver["objective"]


@pytest.mark.gpu
def test_bounds_with_equality_constraints_match_oracle():
    """addVarBounds next to addEqConstraint (the device's projected Newton takes bounds
    alone): the bounds become active-set rows."""
    w = configs.make_c2(B=1, N=16)

    def with_eq():
        problem, X = _problem(w)
        for j in (0, 5, 9):
            problem.addEqConstraint(constraints.equality_constaint, [X[j][0], X[j][1]])
        return problem, X

    base, _ = with_eq()
    base.solve()
    ub = 0.7 * _solution(base, w)[:, 1].max()   # active near the peaks of x_1 of the eq-constrained answer
    problem, X = with_eq()
    problem.addVarBounds(X, 1, -np.inf, ub)
    problem.solve()
    eq_rows = [problem._row(a, b)[:3] for a, b in problem._eq]
    Xg = _check(problem, w, eq_rows, problem._ineq_rows())
    assert Xg[:, 1].max() <= ub + 1e-9
    assert np.abs(Xg[[0, 5, 9], 0] - Xg[[0, 5, 9], 1]).max() <= 1e-9 * (1 + np.abs(Xg).max())


@pytest.mark.gpu
def test_constants_stamp_covers_equality_rows():
    """mhe_dims.eq_idx / eq_rhs are copied into the constants buffer at build time and
    stamped into its layout tag: a caller that changes the rows in place and solves
    without rebuilding gets MHE_STATUS_BAD_CONSTANTS, not the old rows."""
    from mhe import solver
    w = configs.make_c2(B=2, N=20)
    s = solver.BatchSolver(w.N, w.T, w.dyn, w.meas, w.cpm.D, (w.T / 2) * w.cpm.w, w.cpm.lagrange_matrix(w.t_meas),
                           w.Qw, w.Rw, eq=[[0, 2]], eq_rhs=[0.0])
    X, cost, iters, status = s.solve(w.X_init, w.U, w.Y, max_iter=3, tol=0.0)
    assert (status.cpu().numpy() != solver.STATUS_BAD_CONSTANTS).all()
    s._eq_rhs[0] = 0.5        # dims.eq_rhs points at this array: the stale-row case
    X, cost, iters, status = s.solve(w.X_init, w.U, w.Y, max_iter=3, tol=0.0)
    assert (status.cpu().numpy() == solver.STATUS_BAD_CONSTANTS).all()
    s._eq_rhs[0] = 0.0
    s._eq[0] = 1              # other row indices, same count
    X, cost, iters, status = s.solve(w.X_init, w.U, w.Y, max_iter=3, tol=0.0)
    assert (status.cpu().numpy() == solver.STATUS_BAD_CONSTANTS).all()
