"""The oracle's composite objective pinned to the reference's OWN problem builder.

tests/golden/objective.npz holds J and the collocation-constraint residuals of the
reference's ``fixedTimeOptimalEstimationNLP`` (/root/reference/nlp/nlp.py:189-317),
built by the reference code itself on a recording CasADi stand-in and evaluated at
seeded points (tests/golden/gen_objective.py).  Here the oracle (oracle/gn.py,
oracle/gn_general.py -- the checker every GPU parity test uses) evaluates the same
quantities from the same inputs.  What this pins beyond the plug-in fixtures:

  * the (T/2) w_k weighting of the dynamics cost (nlp.py:244-245), for an arbitrary W;
  * the W defect W_k + f(X_k, U_k) - (2/T) sum_j D_kj X_j (nlp.py:225-235) at
    arbitrary (X, W), i.e. the (2/T) D collocation operator and W's elimination;
  * R entering as an information matrix in r^T R r (nlp.py:258, 273), per-row
    parameters (satellite positions, R, y set through setParameter / setMeasurement),
    empty satellite slots with R = 0;
  * the prior (nlp.py:279-286), pseudo-Huber (cost_functions.py:25-31), the controls
    as the reference's setControl interpolates them (nlp.py:304-308);
  * gnss-multi-receiver.py's window-0 objective, and the stored IPOPT fixes
    (NLP_{A,B}.csv) measured on the REFERENCE's J (not on the replica).

Tolerance: full-state problems 1e-13 relative.  Pseudorange problems carry the
rounding of e = y - h at |y| ~ 2e7 m in any evaluation order (oracle.gn.cost_noise),
so J agrees to that floor plus 1e-13 relative.  Parity unpinned against IPOPT itself
(absent): these are objective values, not solver iterates.
"""
import os

import numpy as np
import pytest

from oracle import collocation as oc
from oracle import gn
from oracle import gn_general as gg

FIX = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "objective.npz")


@pytest.fixture(scope="module")
def z():
    return np.load(FIX)


def _consts(N, T, t_meas):
    N = int(N)
    return oc.diff_matrix(N), (float(T) / 2.0) * oc.quad_weights(N), oc.interp_matrix(N, float(T), t_meas, mode="poly1d")


def _dyn_cost(pb, W):
    return float(np.einsum("k,ka,ac,kc->", pb.c, W, pb.Qw, W))


@pytest.mark.parametrize("tag,dyn", [("c1", "single_integrator"), ("c2", "van_der_pol")])
def test_linear_objective_matches_reference_builder(z, tag, dyn):
    g = {k[len(tag) + 1:]: z[k] for k in z.files if k.startswith(tag + "_")}
    N, T = int(g["N"]), float(g["T"])
    D, c, Phi = _consts(N, T, g["t_meas"])
    n = g["X"].shape[1]
    M = g["Y"].shape[0]
    pb = gn.Problem(N, T, n, 1, dyn, "full_state", D, c, Phi, g["Qw"], np.broadcast_to(g["Rw"], (M, n, n)).copy())
    X, U, Y = g["X"][None], g["U"][None], g["Y"][None]
    W, _, _, cost = gn.residuals(pb, X, U, Y)
    # the defect at an arbitrary W is W - W(X): pins (2/T) D and f at the nodes
    scale = np.abs(g["W_elim"]).max()
    assert np.abs(g["defects"] - (g["W"] - W[0])).max() <= 1e-13 * scale
    assert np.abs(g["W_elim"] - W[0]).max() <= 1e-13 * scale
    # J with W eliminated, and J at the arbitrary W (the (T/2) w_k weighting alone)
    assert abs(cost[0] - g["J_elim"]) <= 1e-13 * abs(g["J_elim"]), (cost[0], g["J_elim"])
    meas = cost[0] - _dyn_cost(pb, W[0])
    assert abs(_dyn_cost(pb, g["W"]) + meas - g["J"]) <= 1e-13 * abs(g["J_elim"])
    print(f"{tag}: J_ref = {float(g['J_elim']):.15e}, oracle rel err {abs(cost[0] / g['J_elim'] - 1):.1e}")


def test_controls_interpolated_as_reference_setcontrol(z):
    """nlp.py:304-308 (interp1d with extrapolation at tau2t(tau_k)): the reference's own
    parameter values equal what the oracle's host side computes from the same u."""
    from scipy.interpolate import interp1d
    g = {k[3:]: z[k] for k in z.files if k.startswith("c1_")}
    t_nodes = oc.tau2t(oc.nodes(int(g["N"])), 0.0, float(g["T"]))
    U = interp1d(g["t_meas"], g["u_in"], fill_value="extrapolate")(t_nodes).T
    assert np.array_equal(U, g["U"])


def test_pseudorange_objective_matches_reference_builder(z):
    g = {k[5:]: z[k] for k in z.files if k.startswith("gnss_")}
    N, T = int(g["N"]), float(g["T"])
    D, c, Phi = _consts(N, T, g["t_meas"])
    pb = gn.Problem(N, T, 5, 3, "gnss_pos_and_bias", "pseudorange", D, c, Phi, g["Qw"], g["Rw"],
                    meas_static={"idx": [0, 1, 2, 3]})
    X, Y, PAR = g["X"][None], g["Y"][None], g["PAR"][None]
    U = np.zeros((1, N + 1, 3))
    W, _, _, cost = gn.residuals(pb, X, U, Y, PAR)
    noise = gn.cost_noise(pb, X, U, Y, PAR)[0]
    scale = np.abs(g["W_elim"]).max()
    assert np.abs(g["defects"] - (g["W"] - W[0])).max() <= 1e-13 * scale
    tol = noise + 1e-13 * abs(g["J_elim"])
    assert abs(cost[0] - g["J_elim"]) <= tol, (cost[0], g["J_elim"], tol)
    meas = cost[0] - _dyn_cost(pb, W[0])
    assert abs(_dyn_cost(pb, g["W"]) + meas - g["J"]) <= tol
    print(f"gnss_small: |J_oracle - J_ref| = {abs(cost[0] - g['J_elim']):.2e} (bound {tol:.2e}, J = {float(g['J_elim']):.6e})")


@pytest.mark.parametrize("tag", ["autocar", "autocar_huber"])
def test_autocar_window_objective_matches_reference_builder(z, tag):
    """autonomous-car.py window 0: vehicle_dynamics_and_gnss with the car constants,
    vehicle_pseudorange rows whose sat_pos and R are PARAMETERS (empty slots R = 0),
    prior, L2 or pseudo-Huber dynamics cost, bounds recorded as constraints."""
    import autocar as ac
    g = {k[len(tag) + 1:]: z[k] for k in z.files if k.startswith(tag + "_")}
    huber = tag.endswith("huber")
    N, T, n = ac.N, ac.T, ac.n
    Rw, Yv, sat = g["Rw"], g["Y"], g["sat"]          # (N_gnss+1, N_SAT)
    t_meas = np.repeat(np.linspace(0, T, Rw.shape[0]), Rw.shape[1])
    D, c, Phi = _consts(N, T, t_meas)
    car = dict(zip(("C_AF", "C_AR", "M", "D_F", "D_R", "I_Z"), g["car"]))
    pb = gn.Problem(N, T, n, 2, "vehicle_dynamics_and_gnss", "vehicle_pseudorange", D, c, Phi,
                    np.linalg.inv(ac.Q_NLP), Rw.reshape(-1, 1, 1), Pw=np.linalg.inv(ac.P_NLP),
                    dyn_cost="huber" if huber else "l2", delta=5.0 if huber else None, dyn_par=car)
    X, U = g["X"][None], g["U"][None]
    Y, PAR, x0 = Yv.reshape(1, -1, 1), sat.reshape(1, -1, 3), g["x0"][None]
    W, _, _, cost = gn.residuals(pb, X, U, Y, PAR, x0)
    noise = gn.cost_noise(pb, X, U, Y, PAR, x0)[0]
    scale = np.abs(g["W_elim"]).max()
    assert np.abs(g["defects"] - (g["W"] - W[0])).max() <= 1e-12 * scale
    tol = noise + 1e-13 * abs(g["J_elim"])
    assert abs(cost[0] - g["J_elim"]) <= tol, (cost[0], g["J_elim"], tol)
    # the bounds the script adds (:194-195) are recorded constraints: x[2] in [-pi, pi],
    # x[3] >= 0 -- residuals evaluated by the reference at X
    kinds, vals = g["cons_kind"], g["cons_val"]
    assert kinds.size == 4 * (N + 1)
    exp = []   # addVarBounds(X, 2, ...) over every node, then addVarBounds(X, 3, ...) (nlp.py:314-317)
    for k in range(N + 1):
        exp += [X[0, k, 2] - np.pi, X[0, k, 2] + np.pi]
    for k in range(N + 1):
        exp += [X[0, k, 3] - np.inf, X[0, k, 3] - 0.0]
    assert np.array_equal(vals, np.array(exp))
    print(f"{tag}: |J_oracle - J_ref| = {abs(cost[0] - g['J_elim']):.2e} (bound {tol:.2e}, J = {float(g['J_elim']):.6e})")


def _tworx_problem(g):
    import general_problems as gp
    c = gp.TWO_RX
    N, T, n = c["N"], c["T"], c["n"]
    satA = [g["satA"][i, :g["cntA"][i]] for i in range(g["cntA"].size)]
    prA = [g["prA"][i, :g["cntA"][i]] for i in range(g["cntA"].size)]
    satB = [g["satB"][i, :g["cntB"][i]] for i in range(g["cntB"].size)]
    prB = [g["prB"][i, :g["cntB"][i]] for i in range(g["cntB"].size)]
    t, rows, Rw, Y = gp.two_rx_window_rows(c, satA, prA, satB, prB)
    o = np.argsort(t, kind="stable")
    t, rows, Rw, Y = t[o], rows[o], Rw[o], Y[o]
    Qw, Pw = gp.two_rx_weights()
    D, cw, Phi = _consts(N, T, t)
    eq = np.array([[k * n + 2, k * n + 7] for k in range(N + 1)])
    pb = gg.GeneralProblem(N, T, n, 6, "gnss_two_receiver", "mixed", D, cw, Phi, Qw, Rw, Pw=Pw, eq=eq)
    return pb, Y.reshape(1, -1, 1), rows[None]


def _tworx_cost(pb, X, g, Y, PAR):
    return float(gg.cost_full(pb, X[None], None, g["U"][None], Y, PAR, g["x0"][None])[0])


def _tworx_noise(pb, X, Y, PAR):
    """Rounding floor of the pseudorange rows (as oracle.gn.cost_noise): 4 eps |R e| (|y| + |h|)."""
    xi = np.einsum("ij,ja->ia", pb.Phi, X)
    h = np.array([gg.mixed_row(PAR[0, i], xi[i])[0] for i in range(xi.shape[0])])
    e = Y[0, :, 0] - h
    return float(4 * np.finfo(float).eps * np.sum(np.abs(pb.Rw * e) * (np.abs(Y[0, :, 0]) + np.abs(h))))


def test_two_receiver_window_objective_matches_reference_builder(z):
    """gnss-multi-receiver.py window 0 on the reference's own logs: the replica
    (tests/general_problems.py, the oracle of tests/test_multi_receiver.py) evaluates
    the reference's J at a seeded point and at the optimum X*, and its zA = zB rows."""
    g = {k[6:]: z[k] for k in z.files if k.startswith("tworx_")}
    pb, Y, PAR = _tworx_problem(g)
    for X, J in ((g["X"], g["J_elim"]), (g["Xs"], g["Js_ref"])):
        Jo = _tworx_cost(pb, X, g, Y, PAR)
        tol = _tworx_noise(pb, X, Y, PAR) + 1e-13 * abs(J)
        print(f"two receivers: J_ref = {float(J):.9e}, |J_oracle - J_ref| = {abs(Jo - J):.2e} (bound {tol:.2e})")
        assert abs(Jo - J) <= tol
    assert np.abs(g["eq_at_Xs"]).max() <= 1e-9   # zA = zB, as the reference states it


def test_stored_ipopt_fixes_not_stationary_on_reference_objective(z):
    """The stored IPOPT fixes of window 0 (NLP_{A,B}.csv) measured on the REFERENCE's
    objective (not the replica's): holding A's and B's horizontal positions at t = T at
    the stored values, the best the reference J allows is J_c, far above J* at the
    oracle's optimum; and the reference J's gradient in the held coordinates there
    (central differences, W eliminated through the reference's own constraints) is far
    from zero -- no stationary point of the script's objective has those positions."""
    g = {k[6:]: z[k] for k in z.files if k.startswith("tworx_")}
    Js, Jc, grad = float(g["Js_ref"]), float(g["Jc_ref"]), g["grad_ref"]
    gap = Jc - Js
    print(f"window 0 on the reference J: J* = {Js:.6f}, J_c = {Jc:.6f}, J_c - J* = {gap:.4f}; "
          f"dJ/d(xA, yA, xB, yB) at the stored fixes = {np.array2string(grad, precision=1)} per m")
    # rounding of J at ~1e6 is ~1e-9 J; a tol-converged interior point leaves second-order excess
    assert gap > 1e-5 * Js
    # central-difference error at h = 1e-3 m: rounding eps J / h ~ 1e-6 per m; the gradient is ~1e2 per m
    assert np.abs(grad).max() > 10.0
    # the replica agrees with the reference J at X_c too (same objective, two evaluations)
    pb, Y, PAR = _tworx_problem(g)
    Jo = _tworx_cost(pb, g["Xc"], g, Y, PAR)
    assert abs(Jo - Jc) <= _tworx_noise(pb, g["Xc"], Y, PAR) + 1e-13 * Jc
