"""Oracle for general estimation problems -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline may import this
module; the product path (libmhe.so) never does.

Covers SURVEY.md §8 f4 on top of ``oracle.gn``:
  * several scalar measurement plug-ins in one problem (one addResidualCost call
    each, nlp/nlp.py:258-277), rows encoded as in include/mhe.h (MHE_MEAS_MIXED:
    PAR row = [code, i0..i6, v0..v5], indices into [x(t_i) ; z]);
  * extra decision variables z (addVariables beyond the state, nlp/nlp.py:30-45;
    XA in multi-receiver.py:73,99) entering measurement rows;
  * linear equality constraints v[a] - v[b] = 0 (addEqConstraint with
    nlp/constraints.py equality_constaint, nlp/nlp.py:52-53,
    gnss-multi-receiver.py:76-78), met by every Gauss-Newton step.

Each GN step solves the full KKT system densely,
    [H  C^T] [d ]   [-g]
    [C  0  ] [l ] = [-c],
with H = J^T W J and g = J^T W r over the unknowns [vec(X) node-major ; z] --
independent of the kernel's bordered Schur-complement algorithm.  A z component
that no residual depends on (zero row and column of H) is held fixed.
Stopping rule as the kernels: max|(dX, dz)| <= tol (1 + max|(X, z)|).
"""
import numpy as np

from . import gn

ROW_NONE, ROW_PR, ROW_PRR, ROW_R2, ROW_R3, ROW_HEAD, ROW_COMP = 0, 1, 2, 3, 4, 5, 6
MIXED_Q = 14


def mixed_row(par, xt):
    """h and dh/d[x ; z] of one mixed row (reference nlp/measurements.py)."""
    code = int(par[0])
    idx = [int(v) for v in par[1:8]]
    idx = [i if 0 <= i < xt.shape[0] else -1 for i in idx]
    v = np.asarray(par[8:14], dtype=np.float64)
    G = np.zeros(xt.shape[0])

    def X(k):
        return xt[idx[k]] if idx[k] >= 0 else 0.0

    def add(k, g):
        if idx[k] >= 0:
            G[idx[k]] += g

    if code == ROW_PR:      # :56-70
        d = np.array([X(0) - v[0], X(1) - v[1], X(2) - v[2]])
        rho = np.sqrt(d[0] ** 2 + d[1] ** 2 + d[2] ** 2)
        h = rho + X(3)
        for k in range(3):
            add(k, d[k] / rho)
        add(3, 1.0)
    elif code == ROW_PRR:   # :72-79  dot(sat_vel - x[4:7], LoS) + x[7], LoS = (sat_pos - x[:3]) / |.|
        r = np.array([v[0] - X(0), v[1] - X(1), v[2] - X(2)])
        nr = np.linalg.norm(r)
        los = r / nr
        w = np.array([v[3] - X(3), v[4] - X(4), v[5] - X(5)])
        wl = w @ los
        h = wl + X(6)
        gp = -(w - wl * los) / nr
        for k in range(3):
            add(k, gp[k])
            add(3 + k, -los[k])
        add(6, 1.0)
    elif code in (ROW_R2, ROW_R3):  # :7-20, :39-54
        K = 2 if code == ROW_R2 else 3
        d = np.array([X(k) - X(k + K) - v[k] for k in range(K)])
        r = np.sqrt(np.sum(d ** 2) + .000001)
        h = r
        for k in range(K):
            add(k, d[k] / r)
            add(k + K, -d[k] / r)
    elif code == ROW_HEAD:  # :22-37  atan2(r_x, r_y)
        rx = X(0) - X(1) + v[0]
        ry = X(2) - X(3) + v[1]
        q2 = rx * rx + ry * ry
        h = np.arctan2(rx, ry)
        add(0, ry / q2)
        add(1, -ry / q2)
        add(2, -rx / q2)
        add(3, rx / q2)
    elif code == ROW_COMP:  # :4-5 (one component)
        h = X(0)
        add(0, 1.0)
    else:
        h = 0.0
    return float(h), G


class GeneralProblem(gn.Problem):
    """gn.Problem with meas = "mixed" rows (Rw (M,) scalar weights or (B, M)),
    ``n_extra`` extra variables and ``eq`` (K, 2) constraint index pairs into the
    node-major state vector: v[a] - v[b] = eq_rhs (second index -1: v[a] = eq_rhs;
    eq_rhs None: 0)."""

    def __init__(self, *args, n_extra=0, eq=None, eq_rhs=None, **kw):
        super().__init__(*args, **kw)
        self.n_extra = int(n_extra)
        self.eq = np.zeros((0, 2), dtype=np.int64) if eq is None else np.asarray(eq, dtype=np.int64).reshape(-1, 2)
        self.eq_rhs = np.zeros(self.eq.shape[0]) if eq_rhs is None else np.asarray(eq_rhs, dtype=np.float64).ravel()


def _dynamics_part(pb, X, U, x0):
    """J^T W J, J^T W r and cost of the dynamics + prior terms (oracle.gn's
    verified structured assembly with the measurement set emptied)."""
    q = gn.Problem.__new__(gn.Problem)
    q.__dict__.update(pb.__dict__)
    q.meas = "full_state"
    q.Phi = np.zeros((0, pb.P))
    q.Rw = np.zeros((0, pb.n, pb.n))
    q.M = 0
    Y0 = np.zeros((X.shape[0], 0, pb.n))
    return gn.normal_equations(q, X, U, Y0, None, x0)


def normal_equations_full(pb, X, Z, U, Y, PAR, x0=None):
    """H (B, d+nz, d+nz), g (B, d+nz), cost (B,) over [vec(X) node-major ; z]."""
    X = np.asarray(X, dtype=np.float64)
    B, P, n = X.shape
    d, nz = P * n, pb.n_extra
    Hd, gd, cost = _dynamics_part(pb, X, U, x0)
    H = np.zeros((B, d + nz, d + nz))
    g = np.zeros((B, d + nz))
    H[:, :d, :d] = Hd
    g[:, :d] = gd
    cost = cost.copy()
    Z = np.zeros((B, 0)) if Z is None else np.asarray(Z, dtype=np.float64).reshape(B, nz)
    for b in range(B):
        Rw = pb.Rw[b] if pb.Rw.ndim == 2 else pb.Rw
        for i in range(pb.M):
            if float(np.ravel(Rw[i])[0]) == 0.0:
                continue  # R = 0 masks the row (gnss-multi-receiver.py:196-204)
            xi = pb.Phi[i] @ X[b]
            xt = np.concatenate([xi, Z[b]])
            par = PAR[min(b, PAR.shape[0] - 1), i]
            h, Gr = mixed_row(par, xt)
            e = float(np.ravel(Y[b, i])[0]) - h
            A = np.zeros(d + nz)  # d r / d unknowns, r = y - h
            A[:d] = -np.kron(pb.Phi[i], Gr[:n])
            A[d:] = -Gr[n:n + nz]
            R = float(np.ravel(Rw[i])[0])
            H[b] += R * np.outer(A, A)
            g[b] += A * (R * e)
            cost[b] += R * e * e
    return H, g, cost


def cost_full(pb, X, Z, U, Y, PAR, x0=None):
    return normal_equations_full(pb, X, Z, U, Y, PAR, x0)[2]


def constraint_rows(pb, d, nz):
    C = np.zeros((pb.eq.shape[0], d + nz))
    for k, (ia, ib) in enumerate(pb.eq):
        C[k, ia] += 1.0
        if ib >= 0:
            C[k, ib] -= 1.0
    return C


def kkt_step(H, g, C, cval):
    """Dense KKT solve; variables with an all-zero row of H (and no constraint) held."""
    D = H.shape[0]
    free = ~((np.abs(H).sum(1) == 0.0) & (np.abs(C).sum(0) == 0.0))
    Hf, gf, Cf = H[np.ix_(free, free)], g[free], C[:, free]
    K = C.shape[0]
    A = np.zeros((Hf.shape[0] + K, Hf.shape[0] + K))
    A[:Hf.shape[0], :Hf.shape[0]] = Hf
    A[:Hf.shape[0], Hf.shape[0]:] = Cf.T
    A[Hf.shape[0]:, :Hf.shape[0]] = Cf
    sol = np.linalg.solve(A, np.concatenate([-gf, -cval]))
    step = np.zeros(D)
    step[free] = sol[:Hf.shape[0]]
    return step, sol[Hf.shape[0]:]


def gauss_newton_general(pb, X0, Z0, U, Y, PAR, x0=None, max_iter=20, tol=1e-10, perturb=None):
    """Returns X, Z, cost, iters, status (same stopping rule / status codes as the kernels).
    ``perturb`` (a seed): H and g moved by eps of every entry's magnitude each iteration
    (gn.perturb_rel -- the conditioning floor of tests/tolerance.py)."""
    X = np.array(X0, dtype=np.float64, copy=True)
    B, P, n = X.shape
    nz = pb.n_extra
    Z = np.zeros((B, nz)) if Z0 is None else np.array(Z0, dtype=np.float64, copy=True).reshape(B, nz)
    d = P * n
    C = constraint_rows(pb, d, nz)
    iters = np.zeros(B, dtype=np.int32)
    status = np.full(B, gn.MAXITER, dtype=np.int32)
    for b in range(B):
        sl = slice(b, b + 1)
        pbb = pb
        if pb.Rw.ndim == 2:
            pbb = GeneralProblem.__new__(GeneralProblem)
            pbb.__dict__.update(pb.__dict__)
            pbb.Rw = pb.Rw[b]
        for _ in range(max_iter):
            Ub = None if U is None else U[min(b, U.shape[0] - 1)][None]
            H, g, _ = normal_equations_full(pbb, X[sl], Z[sl], Ub, Y[sl], PAR[min(b, PAR.shape[0] - 1)][None],
                                            None if x0 is None else x0[sl])
            if perturb is not None:
                H, g = gn.perturb_rel(H, perturb), gn.perturb_rel(g, perturb + 1)
            v = np.concatenate([X[b].ravel(), Z[b]])
            cval = C @ v - pb.eq_rhs
            try:
                L = np.linalg.cholesky(H[0][:d, :d])
            except np.linalg.LinAlgError:
                status[b] = gn.NOT_SPD
                break
            del L
            step, _ = kkt_step(H[0], g[0], C, cval)
            if not np.all(np.isfinite(step)):
                status[b] = gn.NONFINITE
                break
            X[b] += step[:d].reshape(P, n)
            Z[b] += step[d:]
            iters[b] += 1
            vmax = max(np.max(np.abs(X[b])), np.max(np.abs(Z[b])) if nz else 0.0)
            if np.max(np.abs(step)) <= tol * (1.0 + vmax):
                status[b] = gn.OK
                break
    cost = np.array([cost_full(pb if pb.Rw.ndim != 2 else _rw(pb, b), X[b:b + 1], Z[b:b + 1],
                               None if U is None else U[min(b, U.shape[0] - 1)][None], Y[b:b + 1],
                               PAR[min(b, PAR.shape[0] - 1)][None], None if x0 is None else x0[b:b + 1])[0]
                     for b in range(B)])
    return X, Z, cost, iters, status


def _rw(pb, b):
    q = GeneralProblem.__new__(GeneralProblem)
    q.__dict__.update(pb.__dict__)
    q.Rw = pb.Rw[b]
    return q
