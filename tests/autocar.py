"""autonomous-car.py's moving-horizon NLP (autonomous-car.py:184-389) on seeded
synthetic data, written twice: against THIS package's facade (nlp.nlp, same calls
in the same order as the reference script) and on the oracle (oracle/gn.py), for
window-by-window GPU parity.

Why synthetic: the script's inputs (data/autonomous-car/sim/{sensor,traj}_data.pkl)
and its stored IPOPT results (filtering/nlp-{l2,huber}.pkl) are Python-2 pickles;
the only loader this environment permits for files shipped inside the reference,
torch.load(weights_only=True), refuses them (protocol-2 BINSTRING opcodes / non-UTF-8
bytes, even with numpy's reconstructors allow-listed), so they are not read.  The data
here has the same shape: a 100 Hz dynamic-bicycle trajectory (utils/vehicle_sim.py
constants, linear tyres), 10 Hz pseudoranges of up to 11 satellites (some epochs with
fewer: R = 0 slot masks), clock bias b0 + alpha t with alpha = 200 m/s and R = 10 m^2
(utils/vehicle_sim.py:119-136).
"""
import numpy as np
from scipy.interpolate import interp1d

from oracle import collocation as oc
from oracle import gn, models

CAR = {"C_AF": 1.1441e5, "C_AR": 1.3388e5, "MU": 0.75, "M": 2009, "D_F": 1.53, "D_R": 1.23, "I_Z": 2000,
       "H": 0.25, "G": 9.81}                       # utils/vehicle_sim.py:10-23
Q_NLP = np.diag([0.01, 0.01, 0.01, 100, 500, 500, .001, .001, .001])   # autonomous-car.py:114
P_NLP = np.diag(np.ones(9))                                              # :117
T, N, n, m, N_SAT, DT = 2.0, 5, 9, 2, 11, 1.0                            # :184-189, :228
P_REF = np.array([-2700404.0, -4292605.0, 3855137.0])                    # ~Hoover Tower, ECEF (m)


def _rhs(x, u):
    f, _ = models.dyn_eval("vehicle_dynamics_and_gnss", np.concatenate([x, np.zeros(3)])[None], u[None], CAR)
    return f[0, :6]


def synth(seed=0, duration=16.0, dt=0.01, dt_gnss=0.1, vary=True):
    """(traj, gnss) dicts shaped like autonomous-car.py's sensor/traj data.  vary=False:
    10 satellites at every epoch (the Huber loop reads the satellite count at the
    window-relative index i, autonomous-car.py:350 -- with varying counts the
    reference script itself would index past an epoch's list)."""
    from utils import utils as gu
    rng = np.random.default_rng(seed)
    t = np.round(np.arange(0.0, duration + dt / 2, dt), 10)
    u = np.stack([1500.0 + 800.0 * np.sin(0.35 * t), 0.04 * np.sin(0.5 * t + 0.3)])      # [F_xr, delta]
    x = np.zeros((6, t.size))
    x[:, 0] = [0.0, 0.0, 0.3, 8.0, 0.0, 0.0]
    for k in range(t.size - 1):   # RK4
        xk, uk = x[:, k], u[:, k]
        k1 = _rhs(xk, uk)
        k2 = _rhs(xk + dt / 2 * k1, uk)
        k3 = _rhs(xk + dt / 2 * k2, uk)
        k4 = _rhs(xk + dt * k3, uk)
        x[:, k + 1] = xk + dt / 6 * (k1 + 2 * k2 + 2 * k3 + k4)
    R, alpha, b0 = 10.0, 200.0, 0.0
    up = np.array([0.0, 0.0, 1.0])
    dirs = rng.normal(size=(N_SAT, 3))
    dirs /= np.linalg.norm(dirs, axis=1, keepdims=True)
    dirs = np.where((dirs @ up)[:, None] < 0.2, -dirs, dirs) + 0.4 * up
    dirs /= np.linalg.norm(dirs, axis=1, keepdims=True)
    sats_enu = 2.0e7 * dirs
    sats_ecef = np.stack([gu.enu2ecef(s, P_REF) for s in sats_enu])
    tg, sp, pr = [], [], []
    for k in range(0, t.size, int(round(dt_gnss / dt))):
        c = (N_SAT if rng.uniform() > 0.3 else int(rng.integers(7, N_SAT))) if vary else N_SAT - 1
        p = np.array([x[0, k], x[1, k], 0.0])
        tg.append(t[k])
        sp.append(sats_ecef[:c].copy())
        pr.append(np.linalg.norm(sats_enu[:c] - p, axis=1) + b0 + alpha * t[k] + np.sqrt(R) * rng.normal(size=c))
    traj = {"t": t, "x": x, "u": u, "x0": x[:, 0].copy(), "dt": dt}
    gnss = {"t": np.array(tg), "sat_pos": sp, "pr": pr, "R": R, "alpha": alpha, "b0": b0}
    return traj, gnss


def facade_mhe(traj, gnss, n_windows, huber=False, device="cuda"):
    """autonomous-car.py:184-289 (L2) / :290-389 (pseudo-Huber) against this package's
    facade, the same calls in the same order (including the Huber loop's use of ``i``
    for the satellite count, autonomous-car.py:350).  Returns per window the
    10-point trajectory x_opt and the GN status; plus the problem (engine counters)."""
    import nlp.cost_functions as cost_functions
    import nlp.dynamics as dynamics
    import nlp.measurements as measurements
    import nlp.nlp as nlp
    from utils import utils
    dt_gnss = gnss["t"][1] - gnss["t"][0]
    problem = nlp.fixedTimeOptimalEstimationNLP(N, T, n, m, device=device)
    X = problem.addVariables(N + 1, n, name='x')
    U, W = problem.addDynamics(dynamics.vehicle_dynamics_and_gnss, X, None, None, {"car_params": CAR})
    if huber:
        problem.addDynamicsCost(cost_functions.pseudo_huber_loss, W, {"Q": np.linalg.inv(Q_NLP), "delta": 5.0})
    else:
        problem.addDynamicsCost(cost_functions.weighted_l2_norm, W, {"Q": np.linalg.inv(Q_NLP)})
    problem.addVarBounds(X, 2, -np.pi, np.pi)
    problem.addVarBounds(X, 3, 0, np.inf)
    X0 = problem.addInitialCost(cost_functions.weighted_l2_norm, X[0], {"Q": np.linalg.inv(P_NLP)})
    N_gnss = int(np.floor(T / dt_gnss))
    t_gnss = np.linspace(0, T, N_gnss + 1)
    Y, R, sat_pos = [], [], []
    for i in range(N_gnss + 1):
        t_i = np.array([[t_gnss[i]]])
        Y_i, R_i, sat_pos_i = [], [], []
        for j in range(N_SAT):
            sat_pos_ij = problem.addParameter(1, 3)[0]
            R_ij = problem.addParameter(1, 1)[0]
            Y_ij = problem.addResidualCost(measurements.vehicle_pseudorange, X, t_i, None,
                                           R_ij, {"p": 1, "sat_pos": sat_pos_ij})[0]
            Y_i.append(Y_ij); R_i.append(R_ij); sat_pos_i.append(sat_pos_ij)
        Y.append(Y_i); R.append(R_i); sat_pos.append(sat_pos_i)
    problem.build()
    r_pr = float(gnss["R"])
    xhat0 = np.hstack((traj["x0"], np.array([gnss["b0"], gnss["alpha"], 0.0])))
    out, status = [], []
    for step, t0 in enumerate(np.linspace(0, n_windows - 1, n_windows) * DT):
        traj_indices = utils.get_time_indices(traj["t"], t0, t0 + T)
        gnss_indices = utils.get_time_indices(gnss["t"], t0, t0 + T)
        problem.setControl(U, traj["t"][traj_indices] - t0, traj["u"][:, traj_indices])
        problem.setParameter(X0, xhat0)
        for i in range(N_gnss + 1):
            i_gnss = gnss_indices[i]
            t_i = np.array([[t_gnss[i]]])
            N_sat_i = gnss["sat_pos"][i if huber else i_gnss].shape[0]
            for j in range(N_SAT):
                if j < N_sat_i:
                    problem.setParameter(R[i][j], dt_gnss * np.linalg.inv(np.diag([r_pr])))
                    problem.setParameter(sat_pos[i][j], utils.ecef2enu(gnss["sat_pos"][i_gnss][j, :], P_REF))
                    problem.setMeasurement(Y[i][j], t_i, np.array([[gnss["pr"][i_gnss][j]]]))
                else:
                    problem.setParameter(R[i][j], 0.0)
                    problem.setParameter(sat_pos[i][j], np.zeros(3))
                    problem.setMeasurement(Y[i][j], t_i, np.array([[0.0]]))
        problem.solve(warmstart=True)
        out.append(problem.extractSolution('x', np.linspace(0, T, 10)))
        xhat0 = problem.extractSolution('x', [DT])
        status.append(problem.solver["return_status"])
    return np.array(out), status, problem


def oracle_mhe(traj, gnss, n_windows, huber=False, max_iter=50, tol=1e-10, pr_scale=None):
    """The same loop on the oracle: per window the structured GN problem (W
    eliminated), projected Newton for the two bounds, IRLS for the Huber cost; warm
    start = the previous window's node values, prior = its value at t = DT.
    ``pr_scale`` multiplies every pseudorange (tests/tolerance.py's perturbation)."""
    from utils import utils
    dt_gnss = gnss["t"][1] - gnss["t"][0]
    N_gnss = int(np.floor(T / dt_gnss))
    t_gnss = np.linspace(0, T, N_gnss + 1)
    P = N + 1
    D, cw = oc.diff_matrix(N), (T / 2.0) * oc.quad_weights(N)
    t_nodes = oc.tau2t(oc.nodes(N), 0.0, T)
    t_meas = np.repeat(t_gnss, N_SAT)
    Phi = oc.interp_matrix(N, T, t_meas)
    E10, E1 = oc.interp_matrix(N, T, np.linspace(0, T, 10)), oc.interp_matrix(N, T, [DT])
    r_pr = float(gnss["R"])
    xhat0 = np.hstack((traj["x0"], np.array([gnss["b0"], gnss["alpha"], 0.0])))
    X = np.zeros((1, P, n))
    out, status = [], []
    for step, t0 in enumerate(np.linspace(0, n_windows - 1, n_windows) * DT):
        ti = utils.get_time_indices(traj["t"], t0, t0 + T)
        gi = utils.get_time_indices(gnss["t"], t0, t0 + T)
        Uk = interp1d(traj["t"][ti] - t0, traj["u"][:, ti], fill_value="extrapolate")(t_nodes).T[None]
        Rw, Yv, PAR = np.zeros((N_gnss + 1, N_SAT)), np.zeros((N_gnss + 1, N_SAT)), np.zeros((N_gnss + 1, N_SAT, 3))
        for i in range(N_gnss + 1):
            k = gi[i]
            ns = gnss["sat_pos"][i if huber else k].shape[0]
            for j in range(min(ns, N_SAT)):
                Rw[i, j] = dt_gnss / r_pr
                PAR[i, j] = utils.ecef2enu(gnss["sat_pos"][k][j, :], P_REF)
                Yv[i, j] = gnss["pr"][k][j] * (1.0 if pr_scale is None else pr_scale[k][j])
        pb = gn.Problem(N, T, n, m, "vehicle_dynamics_and_gnss", "vehicle_pseudorange", D, cw, Phi,
                        np.linalg.inv(Q_NLP), Rw.reshape(-1, 1, 1), Pw=np.linalg.inv(P_NLP),
                        dyn_cost="huber" if huber else "l2", delta=5.0 if huber else None,
                        lb=[-np.inf, -np.inf, -np.pi, 0.0] + [-np.inf] * 5,
                        ub=[np.inf, np.inf, np.pi] + [np.inf] * 6, dyn_par=CAR)
        X, cost, it, st = gn.gauss_newton(pb, X, Uk, Yv.reshape(1, -1, 1), PAR.reshape(1, -1, 3), xhat0[None],
                                          max_iter=max_iter, tol=tol)
        status.append(int(st[0]))
        out.append(E10 @ X[0])
        xhat0 = (E1 @ X[0])[0]
    return np.array(out), np.array(status)
