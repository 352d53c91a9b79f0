"""Pin the composite objective to the reference's OWN problem builder (build container
only).  Run:  python tests/golden/gen_objective.py   -> tests/golden/objective.npz

The reference's ``fixedTimeOptimalEstimationNLP`` (/root/reference/nlp/nlp.py:189-317)
runs unmodified on top of ``casadi_lazy`` (a recording stand-in for CasADi's Opti /
MX / Function, this directory): its addDynamics / addDynamicsCost / addResidualCost /
addInitialCost / addEqConstraint / addVarBounds / setControl / setMeasurement /
setParameter calls build the objective J and the collocation constraints
``W_k + f(X_k, U_k) == (2/T) sum_j D_kj X_j`` (:235) exactly as the scripts call them.
Then J and the constraint residuals are EVALUATED at seeded points -- no IPOPT (there
is none here).  Stored per problem (numbers only):

  * the inputs as the reference set them (parameter values after its own setControl /
    setMeasurement / setParameter: controls at the nodes, measurements, weights,
    satellite positions, prior mean);
  * X, W (seeded), J(X, W), the dynamics-constraint residuals at (X, W) and
    J_elim(X) = J(X, W(X)) with W(X) = -residual(X, 0) -- W eliminated by the
    reference's own constraint expression;
  * every other recorded constraint's residual at X (zA = zB rows, variable bounds).

Problems: C1 (single_integrator, estimation_example.py shape), C2 at N = 20 (van der
Pol; the reference's poly1d basis is invalid beyond N ~ 30),
gnss_small (gnss_stationary.py's one-addResidualCost-per-pseudorange form),
autonomous-car.py's MHE window 0 (L2 and pseudo-Huber, R / sat_pos as parameters,
bounds, prior; tests/autocar.synth data -- the script's pickles are refused) and
gnss-multi-receiver.py's window 0 on the reference's own logs.  For the last one the
generator also evaluates the reference J at the oracle's optimum X* and at X_c, the
optimum with A's and B's horizontal positions at t = T held at the stored IPOPT fixes
(data/gnss-multi-receiver/NLP_{A,B}.csv), and central differences of the reference J
(W eliminated through its own constraints) with respect to those held coordinates:
the non-stationarity of the stored fixes measured on the reference's objective.
Consumed by tests/test_objective_pin.py.
"""
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [HERE, os.path.join(ROOT, "nlp-filter_amd"), ROOT, os.path.join(ROOT, "tests")]

import casadi_lazy as cl  # noqa: E402

REF = "/root/reference"


def load_reference_nlp():
    """nlp/nlp.py and its plug-in modules with casadi_lazy as `casadi`; utils/* through
    gen_golden's loader (flat imports, numeric only)."""
    import gen_golden as g0
    sys.modules["casadi"] = cl
    ref = types.SimpleNamespace()
    ref.collocation = g0._load("refobj_collocation", f"{REF}/nlp/collocation.py", {"range": g0._py2_range})
    ref.constraints = g0._load("refobj_constraints", f"{REF}/nlp/constraints.py")
    sys.modules["collocation"], sys.modules["constraints"] = ref.collocation, ref.constraints
    ref.nlp = g0._load("refobj_nlp", f"{REF}/nlp/nlp.py")
    ref.dynamics = g0._load("refobj_dynamics", f"{REF}/nlp/dynamics.py")
    ref.measurements = g0._load("refobj_measurements", f"{REF}/nlp/measurements.py")
    ref.cost_functions = g0._load("refobj_cost_functions", f"{REF}/nlp/cost_functions.py")
    sys.path.insert(0, f"{REF}/utils")
    saved = {k: sys.modules.get(k) for k in ("gnss", "utils")}  # before any load that may fail
    try:
        ref.gutils = g0._load("refobj_gutils", f"{REF}/utils/utils.py")
        ref.data = g0._load("refobj_data", f"{REF}/utils/data.py")
        ref.gnss = g0._load("refobj_gnss", f"{REF}/utils/gnss.py")
        sys.modules["gnss"], sys.modules["utils"] = ref.gnss, ref.gutils   # leastsquares.py's flat imports
        ref.ls = g0._load("refobj_leastsquares", f"{REF}/utils/leastsquares.py")
        ref.vehicle_sim = g0._load("refobj_vehicle_sim", f"{REF}/utils/vehicle_sim.py")
    finally:
        sys.path.pop(0)
        for k, v in saved.items():   # this package's `utils` must stay importable
            if v is None:
                sys.modules.pop(k, None)
            else:
                sys.modules[k] = v
    return ref


class Recorded:
    """A reference problem plus the index range of its dynamics constraints."""

    def __init__(self, problem, dyn_slice):
        self.p, self.dyn = problem, dyn_slice

    def bindings(self, X, W):
        b = dict(self.p.opti.values)
        for k in range(self.p.N + 1):
            b[self.p.w[f"x_{k}"]] = X[k]
            b[self.p.w[f"w_{k}"]] = W[k]
        return b

    def defects(self, X, W):
        b = self.bindings(X, W)
        return np.stack([cl.evaluate(c.residual(), b).ravel() for c in self.p.opti.constraints[self.dyn]])

    def W_of(self, X):
        """W eliminated by the reference's own constraints: residual = W + f - (2/T) D X is
        W plus a function of X, so W(X) = -residual(X, 0)."""
        return -self.defects(X, np.zeros((self.p.N + 1, self.p.n)))

    def J(self, X, W):
        return float(cl.evaluate(self.p.opti.objective, self.bindings(X, W))[0, 0])

    def J_elim(self, X):
        return self.J(X, self.W_of(X))

    def other_constraints(self, X):
        b = self.bindings(X, self.W_of(X))
        out = []
        for i, c in enumerate(self.p.opti.constraints):
            if self.dyn.start <= i < self.dyn.stop:
                continue
            out.append((c.kind, cl.evaluate(c.residual(), b).ravel()))
        return out

    def value(self, sym):
        return self.p.opti.values[sym]


def _new_problem(ref, N, T, n, m):
    problem = ref.nlp.fixedTimeOptimalEstimationNLP(N, T, n, m)
    X = problem.addVariables(N + 1, n, name="x")
    return problem, X


def _dynamics(problem, *args, **kw):
    c0 = len(problem.opti.constraints)
    U, W = problem.addDynamics(*args, **kw)
    return U, W, slice(c0, len(problem.opti.constraints))


def _pack(out, tag, rec, X, W, extra=None):
    out[f"{tag}_X"] = X
    out[f"{tag}_W"] = W
    out[f"{tag}_J"] = np.array(rec.J(X, W))
    out[f"{tag}_defects"] = rec.defects(X, W)
    out[f"{tag}_J_elim"] = np.array(rec.J_elim(X))
    out[f"{tag}_W_elim"] = rec.W_of(X)
    oc = rec.other_constraints(X)
    if oc:
        out[f"{tag}_cons_kind"] = np.array([{"==": 0, "<=": 1, ">=": 2}[k] for k, _ in oc], dtype=np.int32)
        out[f"{tag}_cons_val"] = np.array([v[0] for _, v in oc])
    for k, v in (extra or {}).items():
        out[f"{tag}_{k}"] = np.asarray(v)


def gen_linear(ref, out):
    """C1 and C2 (N = 20): the estimation_example.py call sequence."""
    from mhe import configs
    rng = np.random.default_rng(77)
    for tag, w, dyn in (("c1", configs.make_c1(B=1), ref.dynamics.single_integrator),
                        ("c2", configs.make_c2(B=1, N=20), ref.dynamics.van_der_pol)):
        problem, X = _new_problem(ref, w.N, w.T, w.n, w.m)
        u = np.sin(w.t_meas)[None] if tag == "c1" else np.zeros((1, w.M))
        U, W, dsl = _dynamics(problem, dyn, X, w.t_meas, u)
        problem.addDynamicsCost(ref.cost_functions.weighted_l2_norm, W, {"Q": w.Qw})
        problem.addResidualCost(ref.measurements.full_state, X, w.t_meas, w.Y[0].T, w.Rw[0])
        problem.build()
        rec = Recorded(problem, dsl)
        Xe = w.X_init[0] + rng.normal(size=w.X_init[0].shape) * 0.1
        We = rng.normal(size=Xe.shape) * 0.05
        Un = np.stack([rec.value(Uk).ravel() for Uk in U])
        _pack(out, tag, rec, Xe, We, {"N": w.N, "T": w.T, "t_meas": w.t_meas, "Y": w.Y[0], "U": Un, "Qw": w.Qw,
                                      "Rw": w.Rw[0], "u_in": u})


def gen_gnss_small(ref, out):
    """gnss_stationary.py:105-128: one addResidualCost per pseudorange, sat_pos numeric."""
    from mhe import configs
    w = configs.make_gnss_small(B=1)
    rng = np.random.default_rng(78)
    problem, X = _new_problem(ref, w.N, w.T, w.n, w.m)
    t_ep = np.unique(w.t_meas)
    U, W, dsl = _dynamics(problem, ref.dynamics.gnss_pos_and_bias, X, t_ep, np.zeros((3, t_ep.size)))
    problem.addDynamicsCost(ref.cost_functions.weighted_l2_norm, W, {"Q": w.Qw})
    for i in range(w.M):
        problem.addResidualCost(ref.measurements.pseudorange, X, np.array([[w.t_meas[i]]]), np.array([[w.Y[0, i, 0]]]),
                                np.array([[w.Rw[i, 0, 0]]]), {"sat_pos": w.PAR[0, i]})
    problem.build()
    rec = Recorded(problem, dsl)
    Xe = w.X_init[0] + rng.normal(size=w.X_init[0].shape) * 2.0
    We = rng.normal(size=Xe.shape) * 0.05
    _pack(out, "gnss", rec, Xe, We, {"N": w.N, "T": w.T, "t_meas": w.t_meas, "Y": w.Y[0], "PAR": w.PAR[0],
                                     "Qw": w.Qw, "Rw": w.Rw})


def gen_autocar(ref, out):
    """autonomous-car.py:184-263 (L2) and :295-363 (pseudo-Huber), window 0, with
    tests/autocar.synth data (the script's pickled inputs are refused)."""
    import autocar as ac
    traj, gnss = ac.synth(0)
    car = ref.vehicle_sim.get_parameters()
    p_ref = ac.P_REF
    for tag, huber in (("autocar", False), ("autocar_huber", True)):
        T, N, n, m, N_sat = ac.T, ac.N, ac.n, ac.m, ac.N_SAT
        dt_gnss = gnss["t"][1] - gnss["t"][0]
        problem, X = _new_problem(ref, N, T, n, m)
        U, W, dsl = _dynamics(problem, ref.dynamics.vehicle_dynamics_and_gnss, X, None, None, {"car_params": car})
        if huber:
            problem.addDynamicsCost(ref.cost_functions.pseudo_huber_loss, W, {"Q": np.linalg.inv(ac.Q_NLP), "delta": 5.0})
        else:
            problem.addDynamicsCost(ref.cost_functions.weighted_l2_norm, W, {"Q": np.linalg.inv(ac.Q_NLP)})
        problem.addVarBounds(X, 2, -np.pi, np.pi)
        problem.addVarBounds(X, 3, 0, np.inf)
        X0 = problem.addInitialCost(ref.cost_functions.weighted_l2_norm, X[0], {"Q": np.linalg.inv(ac.P_NLP)})
        N_gnss = int(np.floor(T / dt_gnss))
        t_gnss = np.linspace(0, T, N_gnss + 1)
        Y, R, sat_pos = [], [], []
        for i in range(N_gnss + 1):
            t_i = np.array([[t_gnss[i]]])
            Yi, Ri, Si = [], [], []
            for j in range(N_sat):
                s = problem.addParameter(1, 3)[0]
                r = problem.addParameter(1, 1)[0]
                Yi.append(problem.addResidualCost(ref.measurements.vehicle_pseudorange, X, t_i, None, r,
                                                  {"p": 1, "sat_pos": s})[0])
                Ri.append(r); Si.append(s)
            Y.append(Yi); R.append(Ri); sat_pos.append(Si)
        problem.build()
        # window 0 (:232-263): controls, prior, measurements
        t0 = 0.0
        r_pr = float(gnss["R"])
        xhat0 = np.hstack((traj["x0"], np.array([gnss["b0"], gnss["alpha"], 0.0])))
        ti = ref.gutils.get_time_indices(traj["t"], t0, t0 + T)
        gi = ref.gutils.get_time_indices(gnss["t"], t0, t0 + T)
        problem.setControl(U, traj["t"][ti] - t0, traj["u"][:, ti])
        problem.setParameter(X0, xhat0)
        for i in range(N_gnss + 1):
            k = gi[i]
            t_i = np.array([[t_gnss[i]]])
            ns = gnss["sat_pos"][i if huber else k].shape[0]   # :350 uses i in the Huber loop
            for j in range(N_sat):
                if j < ns:
                    problem.setParameter(R[i][j], dt_gnss * np.linalg.inv(np.diag([r_pr])))
                    problem.setParameter(sat_pos[i][j], ref.gutils.ecef2enu(gnss["sat_pos"][k][j, :], p_ref))
                    problem.setMeasurement(Y[i][j], t_i, np.array([[gnss["pr"][k][j]]]))
                else:
                    problem.setParameter(R[i][j], 0.0)
                    problem.setParameter(sat_pos[i][j], np.zeros(3))
                    problem.setMeasurement(Y[i][j], t_i, np.array([[0.0]]))
        rec = Recorded(problem, dsl)
        rng = np.random.default_rng(79 + int(huber))
        t_nodes = np.asarray(problem.CPM.tau2t(problem.CPM.tau), dtype=np.float64)
        from scipy.interpolate import interp1d
        xt = interp1d(traj["t"], traj["x"])(t_nodes).T
        Xe = np.zeros((N + 1, n))
        Xe[:, :6] = xt
        Xe[:, 6] = gnss["b0"] + gnss["alpha"] * t_nodes
        Xe[:, 7] = gnss["alpha"]
        Xe += rng.normal(size=Xe.shape) * np.array([0.5, 0.5, 0.02, 0.2, 0.05, 0.02, 1.0, 0.1, 0.2])
        We = rng.normal(size=Xe.shape) * 0.1
        val = lambda lst: np.array([[rec.value(s).ravel() for s in row] for row in lst])  # noqa: E731
        _pack(out, tag, rec, Xe, We, {
            "U": np.stack([rec.value(Uk).ravel() for Uk in U]), "x0": rec.value(X0).ravel(),
            "Rw": val(R)[..., 0], "Y": val(Y)[..., 0], "sat": val(sat_pos), "car": np.array(
                [car[k] for k in ("C_AF", "C_AR", "M", "D_F", "D_R", "I_Z")])})


def gen_two_rx(ref, out):
    """gnss-multi-receiver.py:19-131 (problem) and :141-208 (window 0) on the reference's
    own logs and least-squares fixes; then J of the reference at the oracle optimum,
    at the optimum with the stored IPOPT fixes held, and its gradient there."""
    import general_problems as gp
    from oracle import collocation as oc
    from oracle import gn_general as gg
    data_path = f"{REF}/data/gnss-multi-receiver"
    dataA = ref.data.load_gnss_logs(data_path + "/rec1/rec1_gnss_log_50y_moving_")
    dataB = ref.data.load_gnss_logs(data_path + "/rec2/rec2_gnss_log_50y_moving_")
    p_ref = ref.gutils.lla2ecef(np.array([37.4276, -122.1670, 0]))
    t0 = np.min(np.hstack((dataA["t"], dataB["t"])))
    dataA["t"] -= t0
    dataB["t"] -= t0
    LS_A = ref.ls.runLeastSquares(dataA["t"], dataA["sat_pos"], dataA["pr"], dataA["sat_vel"], dataA["pr_rate"], p_ref)
    LS_B = ref.ls.runLeastSquares(dataB["t"], dataB["sat_pos"], dataB["pr"], dataB["sat_vel"], dataB["pr_rate"], p_ref)
    c = gp.TWO_RX
    Q = np.diag([.01, .01, .01, 0.01, 0.01, .01, .01, .01, 0.01, 0.01])
    P = 0.01 * np.diag([1, 1, 1, 0.1, 0.1, 1, 1, 1, 0.1, 0.1])
    T, N, n, m = 5, 10, 10, 6
    problem, X = _new_problem(ref, N, T, n, m)
    U, W, dsl = _dynamics(problem, ref.dynamics.gnss_two_receiver, X, None, None)
    problem.addDynamicsCost(ref.cost_functions.weighted_l2_norm, W, {"Q": np.linalg.inv(Q)})
    X0 = problem.addInitialCost(ref.cost_functions.weighted_l2_norm, X[0], {"Q": np.linalg.inv(P)})
    t_range = np.linspace(0, T, int(np.floor(T / 0.1)) + 1)
    problem.addResidualCost(ref.measurements.multi_receiver_range_3d, X, t_range, 0.5 * 91.44 * np.ones((1, t_range.size)),
                            0.1 * np.array([1. / 0.01]), {"idxA": [0, 1, 2], "idxB": [5, 6, 7]})
    for i in range(N + 1):
        problem.addEqConstraint(ref.constraints.equality_constaint, [X[i][2], X[i][7]])
    t_heading = np.linspace(0, T, int(np.floor(T / 0.1)) + 1)
    problem.addResidualCost(ref.measurements.multi_receiver_heading_2d, X, t_heading,
                            np.deg2rad(-44) * np.ones((1, t_heading.size)), 0.1 * np.array([1. / 0.1]),
                            {"idxA": [0, 1], "idxB": [5, 6]})
    N_sat, N_gnss = 10, int(np.floor(T / 1))
    t_gnss = np.linspace(0, T, N_gnss + 1)
    par = {"A": ([], [], []), "B": ([], [], [])}
    for i in range(N_gnss + 1):
        t_i = np.array([[t_gnss[i]]])
        rows = {"A": ([], [], []), "B": ([], [], [])}
        for j in range(N_sat):
            for tag, idx in (("A", [0, 1, 2, 3]), ("B", [5, 6, 7, 8])):
                s = problem.addParameter(1, 3)[0]
                r = problem.addParameter(1, 1)[0]
                y = problem.addResidualCost(ref.measurements.pseudorange, X, t_i, None, r,
                                            {"p": 1, "sat_pos": s, "idx": idx})[0]
                rows[tag][0].append(y); rows[tag][1].append(r); rows[tag][2].append(s)
        for tag in ("A", "B"):
            for q in range(3):
                par[tag][q].append(rows[tag][q])
    problem.build()
    xhat0 = np.array([LS_A["x_ENU"][0], LS_A["y_ENU"][0], LS_A["z_ENU"][0], LS_A["bias"][0], 0.0,
                      LS_B["x_ENU"][0], LS_B["y_ENU"][0], LS_B["z_ENU"][0], LS_B["bias"][0], 0.0])
    t_offset = dataB["t"][0] - dataA["t"][0]
    tw = 0.0   # window 0
    iA = ref.gutils.get_time_indices(dataA["t"], tw, tw + T)
    iB = ref.gutils.get_time_indices(dataB["t"], tw + t_offset, tw + t_offset + T)
    sA, sB = dataA["t"][iA] - tw, dataB["t"][iB] - tw - t_offset
    from scipy.interpolate import interp1d
    uA = np.vstack([LS_A[k][iA].reshape(1, -1) for k in ("xd_ENU", "yd_ENU", "zd_ENU")])
    uB = np.vstack([LS_B[k][iB].reshape(1, -1) for k in ("xd_ENU", "yd_ENU", "zd_ENU")])
    uB = interp1d(sB, uB, fill_value="extrapolate")(sA)
    problem.setControl(U, sA, np.vstack((uA, uB)))
    problem.setParameter(X0, xhat0)
    lists = {}
    for tag, data, idxs, r_pr in (("A", dataA, iA, 10), ("B", dataB, iB, 1)):
        Ys, Rs, Ss = par[tag]
        sats, prs = [], []
        for i in range(N_gnss + 1):
            k = idxs[i]
            t_i = np.array([[t_gnss[i]]])
            ns = data["sat_pos"][k].shape[0]
            for j in range(N_sat):
                if j < ns:
                    problem.setParameter(Rs[i][j], 1 * np.linalg.inv(np.diag([r_pr])))
                    problem.setParameter(Ss[i][j], ref.gutils.ecef2enu(data["sat_pos"][k][j, :], p_ref))
                    problem.setMeasurement(Ys[i][j], t_i, np.array([[data["pr"][k][j]]]))
                else:
                    problem.setParameter(Rs[i][j], 0.0)
                    problem.setParameter(Ss[i][j], np.zeros(3))
                    problem.setMeasurement(Ys[i][j], t_i, np.array([[0.0]]))
            # the replica's inputs, read back from the reference's parameter values
            live = [j for j in range(N_sat) if problem.opti.values[Rs[i][j]][0, 0] != 0.0]
            sats.append(np.array([problem.opti.values[Ss[i][j]].ravel() for j in live]).reshape(-1, 3))
            prs.append(np.array([problem.opti.values[Ys[i][j]][0, 0] for j in live]))
        lists[tag] = (sats, prs)
    rec = Recorded(problem, dsl)
    Un = np.stack([rec.value(Uk).ravel() for Uk in U])
    x0v = rec.value(X0).ravel()

    # the oracle (the replica of the script, W eliminated) on exactly these inputs
    t, rows, Rw, Yv = gp.two_rx_window_rows(c, lists["A"][0], lists["A"][1], lists["B"][0], lists["B"][1])
    o = np.argsort(t, kind="stable")
    t, rows, Rw, Yv = t[o], rows[o], Rw[o], Yv[o]
    Qw, Pw = gp.two_rx_weights()
    D, cw = oc.diff_matrix(N), (T / 2.0) * oc.quad_weights(N)
    eq = np.array([[k * n + 2, k * n + 7] for k in range(N + 1)])

    def solve(extra_t, extra_rows, extra_R, extra_Y, Xstart):
        tt, rr, RR, YY = (np.concatenate([t, extra_t]), np.concatenate([rows, extra_rows]),
                          np.concatenate([Rw, extra_R]), np.concatenate([Yv, extra_Y]))
        oo = np.argsort(tt, kind="stable")
        pb = gg.GeneralProblem(N, T, n, m, "gnss_two_receiver", "mixed", D, cw, oc.interp_matrix(N, T, tt[oo]),
                               Qw, RR[oo], Pw=Pw, eq=eq)
        Xs, _, _, _, st = gg.gauss_newton_general(pb, Xstart, None, Un[None], YY[oo].reshape(1, -1, 1), rr[oo][None],
                                                  x0v[None], max_iter=100, tol=1e-12)
        assert int(st[0]) == 0
        return Xs[0]

    Xs = solve(np.zeros(0), np.zeros((0, rows.shape[1])), np.zeros(0), np.zeros(0), np.zeros((1, N + 1, n)))
    refA = np.loadtxt(f"{data_path}/NLP_A.csv", delimiter=",")
    refB = np.loadtxt(f"{data_path}/NLP_B.csv", delimiter=",")
    eA = ref.gutils.ecef2enu(ref.gutils.lla2ecef(np.array([refA[0, 0], refA[0, 1], 0.0])), p_ref)
    eB = ref.gutils.ecef2enu(ref.gutils.lla2ecef(np.array([refB[0, 0], refB[0, 1], 0.0])), p_ref)
    held = np.array([eA[0], eA[1], eB[0], eB[1]])
    pen = np.array([gp.row(gg.ROW_COMP, [k]) for k in (0, 1, 5, 6)])
    Xc = solve(np.full(4, float(T)), pen, np.full(4, 1e8), held, Xs[None])
    # the held coordinates exactly at the stored fixes (the penalty leaves ~1e-6 m)
    Xc[N, [0, 1, 5, 6]] = held
    # central differences of the REFERENCE J (W eliminated by its own constraints)
    h = 1e-3
    grad = np.zeros(4)
    for q, comp in enumerate((0, 1, 5, 6)):
        Xp, Xm = Xc.copy(), Xc.copy()
        Xp[N, comp] += h
        Xm[N, comp] -= h
        grad[q] = (rec.J_elim(Xp) - rec.J_elim(Xm)) / (2 * h)
    rng = np.random.default_rng(80)
    Xe = Xs + rng.normal(size=Xs.shape) * 0.5
    We = rng.normal(size=Xs.shape) * 0.05
    satA = np.zeros((N_gnss + 1, N_sat, 3)); prA = np.zeros((N_gnss + 1, N_sat))
    satB = np.zeros((N_gnss + 1, N_sat, 3)); prB = np.zeros((N_gnss + 1, N_sat))
    cntA = np.array([len(p) for p in lists["A"][1]]); cntB = np.array([len(p) for p in lists["B"][1]])
    for i in range(N_gnss + 1):
        satA[i, :cntA[i]], prA[i, :cntA[i]] = lists["A"][0][i], lists["A"][1][i]
        satB[i, :cntB[i]], prB[i, :cntB[i]] = lists["B"][0][i], lists["B"][1][i]
    _pack(out, "tworx", rec, Xe, We, {
        "U": Un, "x0": x0v, "satA": satA, "prA": prA, "cntA": cntA, "satB": satB, "prB": prB, "cntB": cntB,
        "Xs": Xs, "Js_ref": rec.J_elim(Xs), "Xc": Xc, "Jc_ref": rec.J_elim(Xc), "held": held, "grad_ref": grad,
        "grad_h": h, "eq_at_Xs": np.array([v[0] for k, v in rec.other_constraints(Xs)])})


def main(which=None):
    ref = load_reference_nlp()
    out = {}
    gens = {"linear": gen_linear, "gnss": gen_gnss_small, "autocar": gen_autocar, "tworx": gen_two_rx}
    for name, fn in gens.items():
        if not which or name in which:
            fn(ref, out)
            print(name, "done", flush=True)
    np.savez_compressed(os.path.join(HERE, "objective.npz"), **out)
    print("wrote", os.path.join(HERE, "objective.npz"))


if __name__ == "__main__":
    main(sys.argv[1:])
