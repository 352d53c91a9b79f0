"""Moving-horizon re-solve loop through the nlp facade (the pattern of
autonomous-car.py:228-288): per window setControl, setParameter(prior), setMeasurement,
solve(warmstart=True) (previous solution as the initial iterate, nlp/nlp.py:77-79),
extractSolution at DT for the next prior.  Every window is checked against the oracle
GN started from the same iterate with the same prior (tolerance 1e-8 (1 + max|X|))."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

import nlp.cost_functions as cost_functions  # noqa: E402
import nlp.dynamics as dynamics  # noqa: E402
import nlp.measurements as measurements  # noqa: E402
import nlp.nlp as nlp  # noqa: E402
from mhe import configs  # noqa: E402
from oracle import gn  # noqa: E402


def test_moving_horizon_windows_match_oracle():
    N, T, n, m = 8, 2.0, 2, 1
    DT, windows = 0.5, 6
    rng = np.random.default_rng(21)
    t_all = np.linspace(0.0, DT * windows + T, 81)
    x_true = configs._rk4(configs.vdp_rhs, np.array([[0.2, 1.0]]), t_all)[0]
    y_all = x_true + rng.normal(size=x_true.shape) * np.array([0.1, 0.14])
    R = np.linalg.inv(np.diag([0.01, 0.02]))
    Q = np.diag([1e-3, 1e-3])
    Pprior = np.diag([0.1, 0.1])
    problem = nlp.fixedTimeOptimalEstimationNLP(N, T, n, m)
    X = problem.addVariables(N + 1, n, name="x")
    U, W = problem.addDynamics(dynamics.van_der_pol, X, None, None)
    problem.addDynamicsCost(cost_functions.weighted_l2_norm, W, {"Q": np.linalg.inv(Q)})
    X0 = problem.addInitialCost(cost_functions.weighted_l2_norm, X[0], {"Q": np.linalg.inv(Pprior)})
    t_meas = np.linspace(0.0, T, 9)
    Y = problem.addResidualCost(measurements.full_state, X, t_meas, np.zeros((n, t_meas.shape[0])), R)
    cpm = problem.CPM
    t_nodes = cpm.tau2t(cpm.tau)
    xhat0 = y_all[0]
    problem.initializeEstimate(X, t_all[:20], y_all[:20].T)
    X_prev = None
    for step in range(windows):
        t0 = step * DT
        problem.setControl(U, np.array([0.0, T]), np.zeros((m, 2)))
        problem.setParameter(X0, xhat0)
        y_w = np.stack([np.interp(t0 + t_meas, t_all, y_all[:, c]) for c in range(n)])
        problem.setMeasurement(Y, t_meas, y_w)
        X_init = np.stack([x.value if (step > 0) else x.init for x in X])[None]
        problem.solve(warmstart=True)
        Xg = np.stack([problem.extractVariableValue("x", k) for k in range(N + 1)])
        pb = gn.Problem(N, T, n, m, "van_der_pol", "full_state", cpm.D, (T / 2) * cpm.w,
                        cpm.lagrange_matrix(t_meas), np.linalg.inv(Q), np.broadcast_to(R, (9, n, n)),
                        Pw=np.linalg.inv(Pprior))
        Xr, cr, ir, sr = gn.gauss_newton(pb, X_init, np.zeros((1, N + 1, m)), y_w.T[None], x0=xhat0[None],
                                         max_iter=problem.max_iter, tol=problem.tol)
        assert problem.solver["success"] and sr[0] == gn.OK
        assert np.abs(Xg - Xr[0]).max() <= 1e-8 * (1 + np.abs(Xr).max()), step
        assert abs(problem.solver["iter_count"] - ir[0]) <= 1
        # next prior = the estimate at t = DT (autonomous-car.py:270)
        xhat0 = problem.extractSolution("x", [DT])[0]
        assert np.allclose(xhat0, cpm.evaluateSolution(DT, list(Xg)))
        X_prev = Xg
    assert X_prev is not None
