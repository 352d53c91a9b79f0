"""The nlp.nlp facade records the reference's problem the way nlp/nlp.py does
(CPU part), and solves it on the GPU to the oracle's optimum (gpu part)."""
import numpy as np
import pytest

import nlp.cost_functions as cost_functions
import nlp.dynamics as dynamics
import nlp.measurements as measurements
import nlp.nlp as nlp
from mhe import configs
from oracle import gn


def _c1_problem(w):
    problem = nlp.fixedTimeOptimalEstimationNLP(w.N, w.T, w.n, w.m)
    X = problem.addVariables(w.N + 1, w.n, name='x')
    t = w.t_meas
    _, W = problem.addDynamics(dynamics.single_integrator, X, t, np.sin(t)[None, :])
    problem.addDynamicsCost(cost_functions.weighted_l2_norm, W, {"Q": w.Qw})
    problem.addResidualCost(measurements.full_state, X, t, w.Y[0].T, w.Rw[0])
    problem.initializeEstimate(X, t, w.Y[0].T)
    return problem, X


def test_spec_records_reference_objective():
    w = configs.make_c1()
    problem, X = _c1_problem(w)
    mname, t_meas, Rw, PAR, idx = problem._spec()
    assert mname == "full_state" and PAR is None
    assert np.array_equal(t_meas, w.t_meas)
    assert Rw.shape == (w.M, 1, 1)
    U = np.stack([u.get() for u in problem._dyn[2]])
    assert np.allclose(U, w.U[0])  # setControl = interp1d at tau2t(tau) (nlp/nlp.py:304-308)
    X0 = np.stack([x.init for x in X])
    assert np.allclose(X0, w.X_init[0])  # initializeEstimate (nlp/nlp.py:288-302)


def test_soft_errors_and_unsupported():
    w = configs.make_c1()
    problem, X = _c1_problem(w)
    assert problem.extractVariableValue('x', 0) is None      # before solve: print + None
    assert problem.extractVariableValue('nope', 0) is None   # unknown name: print + None
    with pytest.raises(nlp.UnsupportedFeature):
        problem.addEqConstraint(lambda a, p: a[0] - a[1], [X[0], X[1]])
    with pytest.raises(nlp.UnsupportedFeature):
        problem.addDynamicsCost(lambda x, params=None: x, None, {"Q": np.eye(1)})  # not a registered cost
    with pytest.raises(nlp.UnsupportedFeature):
        nlp.fixedTimeOptimalControlNLP(10, 1.0, 2, 1)


def test_plugins_match_reference_values(golden):
    g = golden["plugins"]
    for name in ("van_der_pol", "single_integrator_2D", "gnss_pos_and_bias", "kinematic_bycicle_and_bias"):
        f = getattr(dynamics, name)
        for x, u, fr in zip(g[f"dyn_{name}_x"][:8], g[f"dyn_{name}_u"][:8], g[f"dyn_{name}_f"][:8]):
            assert np.allclose(f(x, u, None), fr, rtol=1e-14, atol=1e-14)
    for x, par, yr in zip(g["meas_pseudorange_x"][:8], g["meas_pseudorange_par"][:8], g["meas_pseudorange_y"][:8]):
        assert np.allclose(measurements.pseudorange(x, {"sat_pos": par}), yr, rtol=1e-14)


@pytest.mark.gpu
def test_facade_solve_c1_matches_oracle():
    w = configs.make_c1()
    problem, X = _c1_problem(w)
    problem.build()
    problem.solve()
    pb = gn.Problem(w.N, w.T, w.n, w.m, w.dyn, w.meas, w.cpm.D, (w.T / 2) * w.cpm.w,
                    w.cpm.lagrange_matrix(w.t_meas), w.Qw, w.Rw)
    Xr, cr, ir, sr = gn.gauss_newton(pb, w.X_init, w.U, w.Y, max_iter=50, tol=1e-10)
    Xs = np.stack([problem.extractVariableValue('x', k) for k in range(w.N + 1)])
    assert problem.solver["return_status"] == "Solve_Succeeded"
    assert np.abs(Xs - Xr[0]).max() <= 1e-8 * (1 + np.abs(Xr).max())
    assert abs(problem.solver["objective"] - cr[0]) <= 1e-9 * cr[0]
    # W is eliminated but extractable (nlp/nlp.py:222,235)
    Wr, _, _, _ = gn.residuals(pb, Xr, w.U, w.Y)
    Ws = np.stack([problem.extractVariableValue('w', k) for k in range(w.N + 1)])
    assert np.abs(Ws - Wr[0]).max() <= 1e-7 * (1 + np.abs(Wr).max())
    xs = problem.extractSolution('x', w.t_meas)
    assert xs.shape == (w.M, 1)
    problem.solve(warmstart=True)
    assert problem.solver["iter_count"] <= 2


@pytest.mark.gpu
def test_facade_gnss_per_row_residual_costs():
    """gnss_stationary.py:121-128 pattern: one addResidualCost per pseudorange."""
    w = configs.make_gnss_small(B=1, n_sat=6, epochs=21, T=20.0)
    problem = nlp.fixedTimeOptimalEstimationNLP(w.N, w.T, 5, 3)
    X = problem.addVariables(w.N + 1, 5, name='x')
    t_nodes = problem.CPM.tau2t(problem.CPM.tau)
    for k, x in enumerate(X):
        problem.initialGuess(x, w.X_init[0, k])
    _, W = problem.addDynamics(dynamics.gnss_pos_and_bias, X, np.array([0.0, w.T]), np.zeros((3, 2)))
    problem.addDynamicsCost(cost_functions.weighted_l2_norm, W, {"Q": w.Qw})
    for i, t in enumerate(w.t_meas):
        problem.addResidualCost(measurements.pseudorange, X, np.array([[t]]), np.array([[w.Y[0, i, 0]]]),
                                np.array([[w.Rw[i, 0, 0]]]), {"sat_pos": w.PAR[0, i]})
    problem.build()
    problem.solve()
    pb = gn.Problem(w.N, w.T, 5, 3, w.dyn, w.meas, w.cpm.D, (w.T / 2) * w.cpm.w,
                    w.cpm.lagrange_matrix(w.t_meas), w.Qw, w.Rw, meas_static={"idx": [0, 1, 2, 3]})
    Xr, cr, ir, sr = gn.gauss_newton(pb, w.X_init, w.U, w.Y, w.PAR, max_iter=50, tol=1e-10)
    Xs = np.stack([problem.extractVariableValue('x', k) for k in range(w.N + 1)])
    assert sr[0] == 0 and problem.solver["success"]
    assert np.abs(Xs - Xr[0]).max() <= 1e-6 * (1 + np.abs(Xr).max())


def test_build_before_set_parameter_is_deferred():
    """gnss-multi-receiver.py calls problem.build() before any setParameter()/
    setMeasurement(); build() must defer the parameter-dependent constants to solve()."""
    w = configs.make_c1()
    problem = nlp.fixedTimeOptimalEstimationNLP(w.N, w.T, w.n, w.m)
    X = problem.addVariables(w.N + 1, w.n, name='x')
    _, W = problem.addDynamics(dynamics.single_integrator, X, w.t_meas, np.sin(w.t_meas)[None, :])
    problem.addDynamicsCost(cost_functions.weighted_l2_norm, W, {"Q": w.Qw})
    Rp = problem.addParameter(1, 1)[0]
    problem.addResidualCost(measurements.full_state, X, w.t_meas[:3], None, Rp, {"p": 1})
    problem.build()                       # no error, nothing built yet
    assert problem._engine is None and problem._engine_key is None
    with pytest.raises(nlp.ParameterNotSet):
        problem._build()                  # what solve() would hit with the parameter still unset
