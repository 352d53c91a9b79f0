"""Seeded test problems for the general path, shared by the
oracle tests and the GPU parity tests: mixed scalar rows (include/mhe.h
encoding), extra variables, equality constraints."""
import numpy as np

from oracle import collocation as oc
from oracle import gn_general as gg

Q = gg.MIXED_Q


def row(code, idx, vals=()):
    r = np.full(Q, -1.0)
    r[0] = code
    r[8:] = 0.0
    for k, i in enumerate(idx):
        r[1 + k] = i
    for k, v in enumerate(vals):
        r[8 + k] = v
    return r


def two_receiver_problem(N=6, T=5.0, B=2, seed=0, with_eq=True, M_range=11):
    """Small gnss-multi-receiver-shaped problem (gnss-multi-receiver.py:50-140):
    gnss_two_receiver dynamics, range_3d / heading_2d between the receivers,
    pseudoranges of A and B at 1 Hz, prior, zA = zB at every node."""
    rng = np.random.default_rng(seed)
    n, m, P = 10, 6, N + 1
    D = oc.diff_matrix(N)
    c = (T / 2.0) * oc.quad_weights(N)
    t_nodes = oc.tau2t(oc.nodes(N), 0.0, T)
    t_rng = np.linspace(0, T, M_range)
    t_gnss = np.linspace(0, T, 6)
    rows, times, Rw = [], [], []
    for t in t_rng:
        rows.append(row(gg.ROW_R3, [0, 1, 2, 5, 6, 7])); times.append(t); Rw.append(10.0)
    for t in t_rng:
        rows.append(row(gg.ROW_HEAD, [5, 0, 6, 1], [1e-5, 0.0])); times.append(t); Rw.append(1.0)
    sats = rng.normal(size=(6, 8, 3)) * 1.5e7 + np.array([0, 0, 2e7])
    for i, t in enumerate(t_gnss):
        for j in range(8):
            for base, w in ((0, 0.1), (5, 1.0)):
                rows.append(row(gg.ROW_PR, [base, base + 1, base + 2, base + 3], sats[i, j]))
                times.append(t); Rw.append(w if j < 7 else 0.0)   # slot 7 masked (R = 0)
    rows, times, Rw = np.array(rows), np.array(times), np.array(Rw)
    order = np.argsort(times, kind="stable")
    rows, times, Rw = rows[order], times[order], Rw[order]
    Phi = oc.interp_matrix(N, T, times)
    M = len(times)
    # truth: two receivers ~45 m apart at equal height, moving; clock biases
    xt = np.zeros((B, P, n))
    for b in range(B):
        pa = rng.normal(size=3) * 30
        va = rng.normal(size=3)
        off = np.array([30.0, -33.0, 0.0])
        for k, t in enumerate(t_nodes):
            xt[b, k, 0:3] = pa + va * t
            xt[b, k, 5:8] = pa + off + va * t
            xt[b, k, 2] = xt[b, k, 7]
            xt[b, k, 3], xt[b, k, 4] = 1e3 + 0.5 * t, 0.5
            xt[b, k, 8], xt[b, k, 9] = -2e3 + 0.2 * t, 0.2
    U = np.zeros((B, P, m))
    U[:, :, 0:3] = xt[:, :1, 0:3] * 0 + np.array([1.0, 0.5, 0.0])
    U[:, :, 3:6] = np.array([1.0, 0.5, 0.0])
    PAR = np.tile(rows[None], (B, 1, 1))
    Y = np.zeros((B, M, 1))
    for b in range(B):
        for i in range(M):
            xi = Phi[i] @ xt[b]
            Y[b, i, 0] = gg.mixed_row(rows[i], xi)[0] + rng.normal() * (0.01 if rows[i, 0] != gg.ROW_PR else 1.0)
    Qw = np.linalg.inv(np.diag([.01, .01, .01, 0.01, 0.01, .01, .01, .01, 0.01, 0.01]))
    Pw = np.linalg.inv(0.01 * np.diag([1, 1, 1, 0.1, 0.1, 1, 1, 1, 0.1, 0.1]))
    eq = np.array([[k * n + 2, k * n + 7] for k in range(P)]) if with_eq else None
    pb = gg.GeneralProblem(N, T, n, m, "gnss_two_receiver", "mixed", D, c, Phi, Qw, Rw, Pw=Pw, eq=eq)
    x0 = xt[:, 0] + rng.normal(size=(B, n)) * 0.5
    X0 = xt + rng.normal(size=xt.shape) * 2.0
    return pb, X0, U, Y, PAR, x0, xt


def multi_receiver_problem(N=7, T=6.0, B=2, seed=1):
    """multi-receiver.py-shaped problem: multi_receiver dynamics (n=8, m=0),
    pseudorange + pseudorange_rate rows, range_2d to the static receiver XA = z
    (3 extra variables; z[2] enters no row, as XA[2] in the reference)."""
    rng = np.random.default_rng(seed)
    n, P = 8, N + 1
    t_ep = np.linspace(0, T, 7)
    sats = rng.normal(size=(7, 6, 3)) * 1.5e7 + np.array([0, 0, 2e7])
    svel = rng.normal(size=(7, 6, 3)) * 2e3
    rows, times, Rw = [], [], []
    for i, t in enumerate(t_ep):
        for j in range(6):
            rows.append(row(gg.ROW_PR, [0, 1, 2, 3], sats[i, j])); times.append(t); Rw.append(0.01)
            rows.append(row(gg.ROW_PRR, [0, 1, 2, 4, 5, 6, 7], np.concatenate([sats[i, j], svel[i, j]])))
            times.append(t); Rw.append(10.0)
        rows.append(row(gg.ROW_R2, [0, 1, n + 0, n + 1])); times.append(t); Rw.append(100.0)
    rows, times, Rw = np.array(rows), np.array(times), np.array(Rw)
    Phi = oc.interp_matrix(N, T, times)
    t_nodes = oc.tau2t(oc.nodes(N), 0.0, T)
    xt = np.zeros((B, P, n))
    zt = np.zeros((B, 3))
    for b in range(B):
        p0, v = rng.normal(size=3) * 10, rng.normal(size=3) * 0.3
        for k, t in enumerate(t_nodes):
            xt[b, k, 0:3], xt[b, k, 4:7] = p0 + v * t, v
            xt[b, k, 3], xt[b, k, 7] = 500 + 0.3 * t, 0.3
        zt[b, :2] = p0[:2] + np.array([2.0, 1.0])
    M = len(times)
    Y = np.zeros((B, M, 1))
    for b in range(B):
        for i in range(M):
            Y[b, i, 0] = gg.mixed_row(rows[i], np.concatenate([Phi[i] @ xt[b], zt[b]]))[0] + rng.normal() * 0.01
    Qw = np.linalg.inv(np.diag([0.01, 0.01, 0.01, 0.01, 1., 1., 0.01, 0.01]))
    pb = gg.GeneralProblem(N, T, n, 0, "multi_receiver", "mixed", oc.diff_matrix(N), (T / 2.0) * oc.quad_weights(N),
                           Phi, Qw, Rw,
                           n_extra=3)
    X0 = xt + rng.normal(size=xt.shape) * 0.5
    Z0 = zt + rng.normal(size=zt.shape) * 0.5
    Z0[:, 2] = 7.0   # unobservable: must stay where it starts
    return pb, X0, Z0, None, Y, np.tile(rows[None], (B, 1, 1)), xt, zt


# ---------------------------------------------------------------------------
# gnss-multi-receiver.py (two receivers, 96 MHE windows) restated on the oracle
TWO_RX = dict(T=5.0, N=10, n=10, m=6, r_pr_A=10.0, r_pr_B=1.0, r_range=0.01, r_heading=0.1,
              distance=0.5 * 91.44, heading=-44.0, dt_range=0.1, dt_heading=0.1, dt_gnss=1.0, N_sat=10, DT=1.0)


def two_rx_weights():
    """gnss-multi-receiver.py:44-50"""
    Q = np.diag([.01, .01, .01, 0.01, 0.01, .01, .01, .01, 0.01, 0.01])
    P = 0.01 * np.diag([1, 1, 1, 0.1, 0.1, 1, 1, 1, 0.1, 0.1])
    return np.linalg.inv(Q), np.linalg.inv(P)


def two_rx_window_rows(c, satA, prA, satB, prB):
    """Rows of one window in the script's addResidualCost order (:63-123): range_3d at
    t_range, heading_2d at t_heading, then per GNSS epoch i and slot j < N_sat the
    pseudoranges of A and B (R = 0 and zero inputs for empty slots, :186-204).
    satX[i] (k_i, 3) ENU satellite positions and prX[i] (k_i,) of the window's epochs.
    Returns (t, rows (M,14), Rw (M,), Y (M,))."""
    T = c["T"]
    t_range = np.linspace(0, T, int(np.floor(T / c["dt_range"])) + 1)
    t_head = np.linspace(0, T, int(np.floor(T / c["dt_heading"])) + 1)
    t_gnss = np.linspace(0, T, int(np.floor(T / c["dt_gnss"])) + 1)
    t, rows, Rw, Y = [], [], [], []
    for tt in t_range:
        t.append(tt); rows.append(row(gg.ROW_R3, [0, 1, 2, 5, 6, 7]))
        Rw.append(c["dt_range"] * (1.0 / c["r_range"])); Y.append(c["distance"])
    for tt in t_head:
        t.append(tt); rows.append(row(gg.ROW_HEAD, [5, 0, 6, 1], [1e-5, 0.0]))
        Rw.append(c["dt_heading"] * (1.0 / c["r_heading"])); Y.append(np.deg2rad(c["heading"]))
    for i, tt in enumerate(t_gnss):
        for j in range(c["N_sat"]):
            for sat, pr, base, r in ((satA, prA, 0, c["r_pr_A"]), (satB, prB, 5, c["r_pr_B"])):
                if j < sat[i].shape[0]:
                    t.append(tt); rows.append(row(gg.ROW_PR, [base, base + 1, base + 2, base + 3], sat[i][j]))
                    Rw.append(c["dt_gnss"] * (1.0 / r)); Y.append(pr[i][j])
                else:
                    t.append(tt); rows.append(row(gg.ROW_PR, [base, base + 1, base + 2, base + 3], np.zeros(3)))
                    Rw.append(0.0); Y.append(0.0)
    return np.array(t), np.array(rows), np.array(Rw), np.array(Y)


def two_rx_mhe_oracle(dA, dB, lsA, lsB, p_ref, n_windows, enu, max_iter=50, tol=1e-10, overrides=None, with_eq=True):
    """gnss-multi-receiver.py:142-244 on the oracle.  dA/dB: load_gnss_logs dicts,
    lsA/lsB: runLeastSquares-style dicts with x/y/z_ENU, xd/yd/zd_ENU, bias;
    enu(p_ecef) -> ENU at p_ref.  Returns per window the state at t = T (x_opt[49])
    and at t = DT, plus per-window GN status."""
    from scipy.interpolate import interp1d
    c = dict(TWO_RX, **(overrides or {}))
    T, N, n, DT = c["T"], c["N"], c["n"], c["DT"]
    P = N + 1
    Qw, Pw = two_rx_weights()
    D, cw = oc.diff_matrix(N), (T / 2.0) * oc.quad_weights(N)
    t_nodes = oc.tau2t(oc.nodes(N), 0.0, T)
    eq = np.array([[k * n + 2, k * n + 7] for k in range(P)])
    xhat0 = np.array([lsA["x_ENU"][0], lsA["y_ENU"][0], lsA["z_ENU"][0], lsA["bias"][0], 0.0,
                      lsB["x_ENU"][0], lsB["y_ENU"][0], lsB["z_ENU"][0], lsB["bias"][0], 0.0])
    tA, tB = np.asarray(dA["t"], dtype=np.float64), np.asarray(dB["t"], dtype=np.float64)
    t_off = tB[0] - tA[0]
    X = np.zeros((1, P, n))
    out_T, out_DT, status = [], [], []
    for step, t0 in enumerate(np.linspace(0, n_windows - 1, n_windows) * DT):
        iA = np.nonzero((tA >= t0) & (tA <= t0 + T))[0]
        iB = np.nonzero((tB >= t0 + t_off) & (tB <= t0 + t_off + T))[0]
        sA, sB = tA[iA] - t0, tB[iB] - t0 - t_off
        uA = np.vstack([lsA[k][iA] for k in ("xd_ENU", "yd_ENU", "zd_ENU")])
        uB = np.vstack([lsB[k][iB] for k in ("xd_ENU", "yd_ENU", "zd_ENU")])
        uB = interp1d(sB, uB, fill_value="extrapolate")(sA)
        U = interp1d(sA, np.vstack((uA, uB)), fill_value="extrapolate")(t_nodes).T[None]
        satA = [np.array([enu(s) for s in dA["sat_pos"][k]]).reshape(-1, 3) for k in iA]
        satB = [np.array([enu(s) for s in dB["sat_pos"][k]]).reshape(-1, 3) for k in iB]
        t, rows, Rw, Y = two_rx_window_rows(c, satA, [dA["pr"][k] for k in iA], satB, [dB["pr"][k] for k in iB])
        order = np.argsort(t, kind="stable")
        t, rows, Rw, Y = t[order], rows[order], Rw[order], Y[order]
        pb = gg.GeneralProblem(N, T, n, 6, "gnss_two_receiver", "mixed", D, cw, oc.interp_matrix(N, T, t), Qw, Rw,
                               Pw=Pw, eq=eq if with_eq else None)
        X, _, _, _, st = gg.gauss_newton_general(pb, X, None, U, Y.reshape(1, -1, 1), rows[None], xhat0[None],
                                                 max_iter=max_iter, tol=tol)
        status.append(int(st[0]))
        out_T.append(oc.interp_matrix(N, T, [T])[0] @ X[0])
        xhat0 = oc.interp_matrix(N, T, [DT])[0] @ X[0]
        out_DT.append(xhat0)
    return np.array(out_T), np.array(out_DT), np.array(status)


def two_rx_mhe_facade(dA, dB, lsA, lsB, p_ref, n_windows, overrides=None):
    """gnss-multi-receiver.py:38-244 written against THIS package's facade (nlp.nlp,
    its plug-in modules, utils.utils) -- the same calls in the same order.  Returns
    per window x_opt at t = T and xhat0 at t = DT, plus the GN status string."""
    from nlp import constraints, cost_functions, dynamics, measurements
    from nlp import nlp as nlpmod
    from utils import utils as gu
    c = dict(TWO_RX, **(overrides or {}))
    Qi, Pi = two_rx_weights()
    T, N, n, m = c["T"], c["N"], c["n"], c["m"]
    problem = nlpmod.fixedTimeOptimalEstimationNLP(N, T, n, m)
    X = problem.addVariables(N + 1, n, name='x')
    U, W = problem.addDynamics(dynamics.gnss_two_receiver, X, None, None)
    problem.addDynamicsCost(cost_functions.weighted_l2_norm, W, {"Q": Qi})
    X0 = problem.addInitialCost(cost_functions.weighted_l2_norm, X[0], {"Q": Pi})
    t_range = np.linspace(0, T, int(np.floor(T / c["dt_range"])) + 1)
    problem.addResidualCost(measurements.multi_receiver_range_3d, X, t_range,
                            c["distance"] * np.ones((1, t_range.shape[0])),
                            c["dt_range"] * np.array([1. / c["r_range"]]), {"idxA": [0, 1, 2], "idxB": [5, 6, 7]})
    for i in range(N + 1):
        problem.addEqConstraint(constraints.equality_constaint, [X[i][2], X[i][7]])
    t_heading = np.linspace(0, T, int(np.floor(T / c["dt_heading"])) + 1)
    problem.addResidualCost(measurements.multi_receiver_heading_2d, X, t_heading,
                            np.deg2rad(c["heading"]) * np.ones((1, t_heading.shape[0])),
                            c["dt_heading"] * np.array([1. / c["r_heading"]]), {"idxA": [0, 1], "idxB": [5, 6]})
    N_gnss = int(np.floor(T / c["dt_gnss"]))
    t_gnss = np.linspace(0, T, N_gnss + 1)
    R_A, Y_A, S_A, R_B, Y_B, S_B = [], [], [], [], [], []
    for i in range(N_gnss + 1):
        t_i = np.array([[t_gnss[i]]])
        rows = ([], [], [], [], [], [])
        for j in range(c["N_sat"]):
            for base, (Ys, Rs, Ss) in ((0, rows[0:3]), (5, rows[3:6])):
                sp = problem.addParameter(1, 3)[0]
                Rp = problem.addParameter(1, 1)[0]
                Yp = problem.addResidualCost(measurements.pseudorange, X, t_i, None, Rp,
                                             {"p": 1, "sat_pos": sp, "idx": [base, base + 1, base + 2, base + 3]})[0]
                Ys.append(Yp); Rs.append(Rp); Ss.append(sp)
        Y_A.append(rows[0]); R_A.append(rows[1]); S_A.append(rows[2])
        Y_B.append(rows[3]); R_B.append(rows[4]); S_B.append(rows[5])
    problem.build()
    xhat0 = np.array([lsA["x_ENU"][0], lsA["y_ENU"][0], lsA["z_ENU"][0], lsA["bias"][0], 0.0,
                      lsB["x_ENU"][0], lsB["y_ENU"][0], lsB["z_ENU"][0], lsB["bias"][0], 0.0])
    DT = c["DT"]
    tA, tB = np.asarray(dA["t"], dtype=np.float64), np.asarray(dB["t"], dtype=np.float64)
    t_offset = tB[0] - tA[0]
    out_T, out_DT, status = [], [], []
    from scipy.interpolate import interp1d
    for step, t0 in enumerate(np.linspace(0, (n_windows - 1) * DT, n_windows)):
        iA = gu.get_time_indices(tA, t0, t0 + T)
        iB = gu.get_time_indices(tB, t0 + t_offset, t0 + t_offset + T)
        sA, sB = tA[iA] - t0, tB[iB] - t0 - t_offset
        uA = np.vstack([lsA[k][iA].reshape(1, -1) for k in ("xd_ENU", "yd_ENU", "zd_ENU")])
        uB = np.vstack([lsB[k][iB].reshape(1, -1) for k in ("xd_ENU", "yd_ENU", "zd_ENU")])
        uB = interp1d(sB, uB, fill_value="extrapolate")(sA)
        problem.setControl(U, sA, np.vstack((uA, uB)))
        problem.setParameter(X0, xhat0)
        for d, idxs, Ys, Rs, Ss, r in ((dA, iA, Y_A, R_A, S_A, c["r_pr_A"]), (dB, iB, Y_B, R_B, S_B, c["r_pr_B"])):
            for i in range(N_gnss + 1):
                k = idxs[i]
                t_i = np.array([[t_gnss[i]]])
                ns = d["sat_pos"][k].shape[0]
                for j in range(c["N_sat"]):
                    if j < ns:
                        problem.setParameter(Rs[i][j], c["dt_gnss"] * np.linalg.inv(np.diag([r])))
                        problem.setParameter(Ss[i][j], gu.ecef2enu(d["sat_pos"][k][j, :], p_ref))
                        problem.setMeasurement(Ys[i][j], t_i, np.array([[d["pr"][k][j]]]))
                    else:
                        problem.setParameter(Rs[i][j], 0.0)
                        problem.setParameter(Ss[i][j], np.zeros(3))
                        problem.setMeasurement(Ys[i][j], t_i, np.array([[0.0]]))
        problem.solve(warmstart=True)
        x_opt = problem.extractSolution('x', np.linspace(0, T, 50))
        xhat0 = problem.extractSolution('x', [DT])[0]
        out_T.append(x_opt[-1])
        out_DT.append(xhat0)
        status.append(problem.solver["return_status"])
    return np.array(out_T), np.array(out_DT), status
