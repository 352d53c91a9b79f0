"""Oracle: the estimation objective and a batched Gauss-Newton solver -- TEST INFRASTRUCTURE ONLY.

Restates the objective that ``fixedTimeOptimalEstimationNLP`` hands to IPOPT,
with the process-noise variables W eliminated through the collocation equality:

  W_k(X) = (2/T) sum_j D_kj X_j - f(X_k, U_k)            nlp/nlp.py:225-235
  J_dyn  = sum_k (T/2) w_k  W_k^T Qw W_k                  nlp/nlp.py:242-245, cost_functions.py:20-22
  J_meas = sum_i e_i^T Rw_i e_i,  e_i = y_i - h(X(t_i))   nlp/nlp.py:264-273 (R passed as information)
           X(t_i) = sum_j phi_j(t_i) X_j                  nlp/nlp.py:266-269
  J_0    = (X_0 - x0)^T Pw (X_0 - x0)                     nlp/nlp.py:279-286

Gauss-Newton on J (the same stationary point IPOPT returns for this
unconstrained problem): H delta = -g with H = sum A^T W A, g = sum A^T W r.
With the pseudo-Huber dynamics cost (cost_functions.py:25-31) the step is IRLS:
per defect component W r -> rho'(r)/2 and W -> diag(rho'(r)/(2r)).
With addVarBounds (nlp/nlp.py:314-317) the iteration is a projected Newton method
on the GN model (epsilon-active set, reduced system on the free entries, Armijo
search along the projection arc; ``gauss_newton_bounded``): its limit points are
KKT points of the bound-constrained problem, the point IPOPT's interior-point
method converges to.

Two independent forms are provided:
  * ``normal_equations``          structured (Kronecker) form, vectorised over the batch
                                  -- also the CPU-baseline workload of bench.py;
  * ``normal_equations_explicit`` builds the stacked Jacobian row by row from the
                                  reference's per-node / per-measurement expressions.
"""
import numpy as np

from . import models

OK, MAXITER, NOT_SPD, NONFINITE = 0, 1, 2, 3


class Problem:
    """Structure shared by every trajectory of a batch (plain container)."""

    def __init__(self, N, T, n, m, dyn, meas, D, c, Phi, Qw, Rw, Pw=None, meas_static=None,
                 dyn_cost="l2", delta=None, lb=None, ub=None, dyn_par=None):
        self.N, self.T, self.n, self.m = N, float(T), n, m
        # dynamics cost: "l2" = weighted_l2_norm, "huber" = pseudo_huber_loss with params
        # {"Q": Qw, "delta": delta} (cost_functions.py:20-31; only diag(Qw) enters the Huber)
        self.dyn_cost, self.delta = dyn_cost, None if delta is None else float(delta)
        # addVarBounds (nlp/nlp.py:314-317) per state component: (n,) arrays, +-inf = free
        self.lb = None if lb is None else np.asarray(lb, dtype=np.float64)
        self.ub = None if ub is None else np.asarray(ub, dtype=np.float64)
        self.P = N + 1
        self.d = self.P * n
        self.alpha = 2.0 / float(T)
        self.dyn, self.meas = dyn, meas
        self.dyn_par = dyn_par                            # the dynamics plug-in's params (car_params)
        self.meas_static = meas_static or {}
        self.D = np.asarray(D, dtype=np.float64)
        self.c = np.asarray(c, dtype=np.float64)          # (T/2) w_k
        self.Phi = np.asarray(Phi, dtype=np.float64)      # (M, P)
        self.Qw = np.asarray(Qw, dtype=np.float64)        # (n, n)
        self.Rw = np.asarray(Rw, dtype=np.float64)        # (M, p, p) or (B, M, p, p)
        self.Pw = None if Pw is None else np.asarray(Pw, dtype=np.float64)
        self.M = self.Phi.shape[0]


def residuals(pb, X, U, Y, PAR=None, x0=None):
    """Return W (B,P,n), xi (B,M,n), e (B,M,p), cost (B,)."""
    X = np.asarray(X, dtype=np.float64)
    DX = np.einsum("kj,bja->bka", pb.D, X)
    f, _ = models.dyn_eval(pb.dyn, X, U, pb.dyn_par)
    W = pb.alpha * DX - f
    if pb.dyn_cost == "huber":  # sum_i 2 Q_ii delta^2 (sqrt(1 + W_i^2/delta^2) - 1), cost_functions.py:25-31
        q, dl = np.diag(pb.Qw), pb.delta
        cost = np.einsum("k,bka->b", pb.c, 2.0 * q * dl ** 2 * (np.sqrt(1.0 + W ** 2 / dl ** 2) - 1.0))
    else:
        cost = np.einsum("k,bka,ac,bkc->b", pb.c, W, pb.Qw, W)
    xi = np.einsum("ij,bja->bia", pb.Phi, X)
    h, _ = models.meas_eval(pb.meas, xi, PAR, pb.meas_static)
    Rw = pb.Rw if pb.Rw.ndim == 4 else pb.Rw[None]
    with np.errstate(invalid="ignore"):
        e = np.where(masked_rows(Rw)[..., None], 0.0, Y - h)
    cost = cost + np.einsum("bip,bipq,biq->b", e, np.broadcast_to(Rw, e.shape + (e.shape[-1],)), e)
    if pb.Pw is not None:
        r0 = X[:, 0] - x0
        cost = cost + np.einsum("ba,ac,bc->b", r0, pb.Pw, r0)
    return W, xi, e, cost


def cost_noise(pb, X, U, Y, PAR=None, x0=None):
    """Rounding level of the cost at X (B,): e = y - h(x) carries eps (|y| + |h|) of
    rounding in any evaluation order, so cost = sum e^T R e carries up to
    2 |R e| eps (|y| + |h|) per row -- with pseudoranges (|y| ~ 2e7 m) far above
    1e-12 |cost|.  Twice that bound (COST_NOISE) enters the Armijo test of the
    projected Newton method: a decrease below the rounding level cannot be resolved,
    so it must not be demanded (else the search shrinks the step to zero there)."""
    X = np.asarray(X, dtype=np.float64)
    xi = np.einsum("ij,bja->bia", pb.Phi, X)
    h, _ = models.meas_eval(pb.meas, xi, PAR, pb.meas_static)
    Rw = pb.Rw if pb.Rw.ndim == 4 else pb.Rw[None]
    mask = masked_rows(Rw)[..., None]
    with np.errstate(invalid="ignore"):
        e = np.where(mask, 0.0, Y - h)
        mag = np.where(mask, 0.0, np.abs(Y) + np.abs(h))
    Re = np.einsum("bipq,biq->bip", np.broadcast_to(Rw, e.shape + (e.shape[-1],)), e)
    return COST_NOISE * np.finfo(np.float64).eps * np.einsum("bip,bip->b", np.abs(Re), mag)


def masked_rows(Rw):
    """(B|1, M) True where a row's weight matrix is all zero: the reference masks empty
    satellite slots with R = 0 (autonomous-car.py:260-263, gnss-multi-receiver.py:196-204),
    so such a row contributes nothing -- even where h or its Jacobian is singular there."""
    return np.all(Rw.reshape(Rw.shape[:2] + (int(np.prod(Rw.shape[2:])),)) == 0.0, axis=-1)


def _meas_block(Phi, G):
    """sum_i Phi_ij Phi_il G_i[a, c] -> (B, P, n, P, n).  Rows with bitwise-equal Phi rows
    (one measurement epoch) are summed first -- the same sum, regrouped -- so the
    contraction is E x P^2 n^2 instead of M x P^2 n^2 (C4: 501 instead of 6012)."""
    B, M, n, _ = G.shape
    P = Phi.shape[1]
    uq, inv = np.unique(Phi, axis=0, return_inverse=True)
    Ge = np.zeros((B, uq.shape[0], n, n))
    np.add.at(Ge, (slice(None), inv.ravel()), G)
    A = (uq[:, :, None] * Ge.reshape(B, uq.shape[0], 1, n * n)[:, :, :, :])     # (B, E, P, n*n)
    out = np.einsum("bejq,el->bjlq", A, uq, optimize=True).reshape(B, P, P, n, n)
    return out.transpose(0, 1, 3, 2, 4)


def normal_equations(pb, X, U, Y, PAR=None, x0=None):
    """Structured GN normal equations. Returns H (B,d,d), g (B,d), cost (B,)."""
    X = np.asarray(X, dtype=np.float64)
    B, P, n = X.shape
    W, xi, e, cost = residuals(pb, X, U, Y, PAR, x0)
    _, F = models.dyn_eval(pb.dyn, X, U, pb.dyn_par)
    a = pb.alpha
    # dynamics: block(j,l) = a^2 (D^T C D)_jl Qw - a D_lj E_l - a D_jl E_j^T + delta_jl F_j^T E_j
    if pb.dyn_cost == "huber":
        # IRLS: the half-gradient Qw W -> rho'(W)/2, the weight Qw -> diag(rho'(W)/(2W))
        Lam, Vh = huber_weights(pb, W)                           # (B,P,n) each
        E = pb.c[None, :, None, None] * Lam[..., None] * F        # c_k diag(Lam_k) F_k
        H4 = (a * a) * np.einsum("kj,k,kl,zka,ae->zjale", pb.D, pb.c, pb.D, Lam, np.eye(n))
    else:
        E = np.einsum("k,ac,zkce->zkae", pb.c, pb.Qw, F)          # c_k Qw F_k
        DCD = np.einsum("kj,k,kl->jl", pb.D, pb.c, pb.D)
        H4 = np.broadcast_to((a * a) * np.einsum("jl,ae->jale", DCD, pb.Qw), (B, P, n, P, n)).copy()
    H4 -= a * np.einsum("lj,zlae->zjale", pb.D, E)
    H4 -= a * np.einsum("jl,zjea->zjale", pb.D, E)
    FtE = np.einsum("zjca,zjce->zjae", F, E)
    for j in range(P):
        H4[:, j, :, j, :] += FtE[:, j]
    if pb.dyn_cost == "huber":
        V = pb.c[None, :, None] * Vh                              # c_k rho'(W_k)/2
    else:
        V = np.einsum("k,ac,zkc->zka", pb.c, pb.Qw, W)            # c_k Qw W_k
    g = a * np.einsum("kj,zka->zja", pb.D, V) - np.einsum("zjca,zjc->zja", F, V)
    # measurements
    _, Hm = models.meas_eval(pb.meas, xi, PAR, pb.meas_static)    # (B,M,p,n)
    Rw = pb.Rw if pb.Rw.ndim == 4 else np.broadcast_to(pb.Rw[None], (B,) + pb.Rw.shape)
    Hm = np.where(masked_rows(Rw)[..., None, None], 0.0, Hm)
    G = np.einsum("zipa,zipq,ziqc->ziac", Hm, Rw, Hm)              # (B,M,n,n)
    H4 += _meas_block(pb.Phi, G)
    ge = np.einsum("zipa,zipq,ziq->zia", Hm, Rw, e)
    g -= np.einsum("ij,zia->zja", pb.Phi, ge)
    if pb.Pw is not None:
        H4[:, 0, :, 0, :] += pb.Pw
        g[:, 0] += (X[:, 0] - x0) @ pb.Pw.T
    d = P * n
    return H4.reshape(B, d, d), g.reshape(B, d), cost


def huber_weights(pb, W):
    """Per-component pseudo-Huber IRLS weights at the defects W (B,P,n):
    Lam = rho'(W) / (2 W) = q / sqrt(1 + W^2/delta^2),  Vh = rho'/2 = Lam W.
    (IRLS majorises the loss, so undamped steps decrease it monotonically; the
    fixed point is the stationary point of the pseudo-Huber objective.)"""
    q, dl = np.diag(pb.Qw), pb.delta
    lam = q / np.sqrt(1.0 + W ** 2 / dl ** 2)
    return lam, lam * W


def normal_equations_explicit(pb, X, U, Y, PAR=None, x0=None):
    """Row-by-row stacked Jacobian (independent restatement; small problems only)."""
    X = np.asarray(X, dtype=np.float64)
    B, P, n = X.shape
    d = P * n
    Hs, gs, cs = [], [], []
    for b in range(B):
        rows, Ws, rs = [], [], []
        for k in range(P):  # dynamics defect rows, nlp/nlp.py:225-235
            fk, Fk = models.dyn_eval(pb.dyn, X[b, k], None if U is None else U[b, k], pb.dyn_par)
            Wk = pb.alpha * (pb.D[k] @ X[b]) - fk
            A = np.zeros((n, d))
            for j in range(P):
                A[:, j * n:(j + 1) * n] += pb.alpha * pb.D[k, j] * np.eye(n)
            A[:, k * n:(k + 1) * n] -= Fk
            if pb.dyn_cost == "huber":  # IRLS: H += A^T diag(c rho'/(2W)) A, g += A^T (c rho'/2)
                q, dl = np.diag(pb.Qw), pb.delta
                sk = 1.0 + Wk ** 2 / dl ** 2
                lam = pb.c[k] * q / np.sqrt(sk)
                rows.append(A); Ws.append(np.diag(lam)); rs.append(("g", lam * Wk,
                                                                    pb.c[k] * np.sum(2 * q * dl ** 2 * (np.sqrt(sk) - 1))))
                continue
            rows.append(A); Ws.append(pb.c[k] * pb.Qw); rs.append(Wk)
        Rw = pb.Rw[b] if pb.Rw.ndim == 4 else pb.Rw
        for i in range(pb.M):  # measurement rows, nlp/nlp.py:264-273
            xi = pb.Phi[i] @ X[b]
            par = None if PAR is None else PAR[min(b, PAR.shape[0] - 1), i]
            if not np.any(Rw[i]):
                continue  # R = 0 masks the row (autonomous-car.py:260-263)
            hi, Hi = models.meas_eval(pb.meas, xi, par, pb.meas_static)
            A = np.zeros((Hi.shape[0], d))
            for j in range(P):
                A[:, j * n:(j + 1) * n] = -pb.Phi[i, j] * Hi
            rows.append(A); Ws.append(Rw[i]); rs.append(Y[b, i] - hi)
        if pb.Pw is not None:  # prior, nlp/nlp.py:279-286
            A = np.zeros((n, d)); A[:, :n] = np.eye(n)
            rows.append(A); Ws.append(pb.Pw); rs.append(X[b, 0] - x0[b])
        H = np.zeros((d, d)); g = np.zeros(d); c = 0.0
        for A, Wm, r in zip(rows, Ws, rs):
            H += A.T @ Wm @ A
            if isinstance(r, tuple):  # (tag, weighted half-gradient, cost) for non-quadratic costs
                g += A.T @ r[1]
                c += r[2]
                continue
            g += A.T @ (Wm @ r)
            c += r @ Wm @ r
        Hs.append(H); gs.append(g); cs.append(c)
    return np.stack(Hs), np.stack(gs), np.array(cs)


def perturb_rel(A, seed):
    """A with every entry moved by eps |A_ij| (random sign; symmetric for square A):
    the backward error of ANY evaluation order of A's sums (tests/tolerance.py)."""
    rng = np.random.default_rng(seed)
    S = rng.choice([-1.0, 1.0], size=A.shape)
    if A.ndim >= 2 and A.shape[-1] == A.shape[-2]:
        S = np.triu(S) + np.swapaxes(np.triu(S, 1), -1, -2)
    return A * (1.0 + np.finfo(np.float64).eps * S)


def gauss_newton(pb, X0, U, Y, PAR=None, x0=None, max_iter=20, tol=1e-10, trace=None, perturb=None):
    """Batched GN with the same stopping rule as the HIP kernel.

    Per trajectory: solve H delta = -g (Cholesky), X += delta, iters += 1;
    converged when max|delta| <= tol * (1 + max|X|). Converged trajectories are
    frozen. Returns X, cost (at the returned X), iters, status.
    With bounds (pb.lb / pb.ub) the iteration is the projected Newton method of
    ``gauss_newton_bounded``.  ``perturb`` (a seed) moves every entry of H and g by
    eps of its magnitude each iteration -- the conditioning floor of tests/tolerance.py.
    """
    if pb.lb is not None or pb.ub is not None:
        return gauss_newton_bounded(pb, X0, U, Y, PAR, x0, max_iter, tol, trace)
    X = np.array(X0, dtype=np.float64, copy=True)
    B = X.shape[0]
    iters = np.zeros(B, dtype=np.int32)
    status = np.full(B, MAXITER, dtype=np.int32)
    active = np.ones(B, dtype=bool)
    for _ in range(max_iter):
        idx = np.nonzero(active)[0]
        if idx.size == 0:
            break
        sub = lambda A: None if A is None else (A[idx] if A.shape[0] == B else A)
        pbs = pb
        if pb.Rw.ndim == 4:
            pbs = _with_rw(pb, pb.Rw[idx])
        H, g, _ = normal_equations(pbs, X[idx], sub(U), Y[idx], sub(PAR), sub(x0))
        if perturb is not None:  # rounding-level perturbation of the normal equations
            H, g = perturb_rel(H, perturb), perturb_rel(g, perturb + 1)
        for t, b in enumerate(idx):
            try:
                L = np.linalg.cholesky(H[t])
            except np.linalg.LinAlgError:
                status[b] = NOT_SPD
                active[b] = False
                continue
            delta = -np.linalg.solve(L.T, np.linalg.solve(L, g[t]))
            if not np.all(np.isfinite(delta)):
                status[b] = NONFINITE
                active[b] = False
                continue
            step = delta.reshape(X.shape[1:])
            X[b] = X[b] + step
            iters[b] += 1
            if np.max(np.abs(step)) <= tol * (1.0 + np.max(np.abs(X[b]))):
                status[b] = OK
                active[b] = False
    _, _, _, cost = residuals(pb, X, U, Y, PAR, x0)
    return X, cost, iters, status


# Projected Newton (Bertsekas 1982, "Projected Newton methods for optimization
# problems with simple constraints") on the Gauss-Newton model, for addVarBounds
# (nlp/nlp.py:314-317: lb <= x[idx] <= ub at every node).  Constants shared with
# the HIP kernels (k_gn_bounded, k_big_linesearch):
EPS_ACT = 1e-6       # epsilon-active set: eps = min(EPS_ACT (1 + max|X|), w)
ARMIJO_SIGMA = 1e-4  # sufficient decrease along the projection arc
LS_MAX = 30          # step halvings; the last trial is taken if none is accepted
COST_SLACK = 1e-12   # relative cost slack of the Armijo test: near a solution the decrease
                     # falls below the cost's rounding error and full steps must pass
COST_NOISE = 4.0     # cost_noise: 2 (d cost / d e) x 2 (margin) eps |R e| (|y| + |h|) per row


def box(pb, shape):
    """(lo, hi) arrays of `shape` (..., n) from the per-component bounds."""
    lo = np.broadcast_to(-np.inf if pb.lb is None else pb.lb, shape)
    hi = np.broadcast_to(np.inf if pb.ub is None else pb.ub, shape)
    return lo, hi


def active_set(pb, X, g):
    """epsilon-active set of the projected Newton method at X with half-gradient g
    (both (P, n)): bounded entries within eps of a bound whose gradient points out of
    the box.  w = max |X - P(X - g)| over the bounded entries (0 at a KKT point), so
    eps -> 0 at a solution and the set becomes the exact binding set."""
    lo, hi = box(pb, X.shape)
    bounded = np.isfinite(lo) | np.isfinite(hi)
    w = np.max(np.abs(X - np.clip(X - g, lo, hi)), where=bounded, initial=0.0)
    eps = min(EPS_ACT * (1.0 + np.max(np.abs(X))), w)
    return bounded & (((X <= lo + eps) & (g > 0)) | ((X >= hi - eps) & (g < 0)))


def gauss_newton_bounded(pb, X0, U, Y, PAR=None, x0=None, max_iter=20, tol=1e-10, trace=None):
    """Gauss-Newton with bounds as a projected Newton method (per trajectory):

      X <- P(X0)                                   (P: projection onto the box)
      repeat:  H, g at X   (g = J^T W r = half the gradient of the cost)
        A  = active_set(X, g)
        Ht = H with the rows / columns of A replaced by their diagonal entries
        d  = -Ht^-1 g                               (reduced GN step on the free set,
                                                     diagonally scaled gradient on A)
        s  = P(X + d) - X                           (stationarity: s = 0 at a KKT point)
        a = 1, 1/2, ... (LS_MAX trials): X(a) = P(X + a d) until
          cost(X(a)) <= cost(X) + 2 sigma [sum_free a g.d + sum_A g.(X(a) - X)]
                         + noise(X) + noise(X(a)) + COST_SLACK |cost(X)|
        (noise: cost_noise, the rounding level of the cost at that point)
        X <- X(a);  converged when max|s| <= tol (1 + max|X|).
    Limit points are KKT points of the bound-constrained least-squares problem (the
    fixed point of plain step clipping is not).  Returns X, cost, iters, status.
    ``trace`` (a list) receives (trajectory, iteration, accepted alpha) per step."""
    X = np.array(X0, dtype=np.float64, copy=True)
    B = X.shape[0]
    lo, hi = box(pb, X.shape[1:])
    X = np.clip(X, lo, hi)
    iters = np.zeros(B, dtype=np.int32)
    status = np.full(B, MAXITER, dtype=np.int32)
    cost_out = np.zeros(B)

    def one(A, b):
        return None if A is None else A[b:b + 1] if A.shape[0] == B else A

    for b in range(B):
        pbs = _with_rw(pb, pb.Rw[b:b + 1]) if pb.Rw.ndim == 4 else pb
        args = (one(U, b), Y[b:b + 1], one(PAR, b), one(x0, b))
        Xb = X[b:b + 1].copy()
        while True:
            H, g, J = normal_equations(pbs, Xb, *args)
            if iters[b] >= max_iter:
                break
            H, g, J = H[0], g[0], J[0]
            act = active_set(pb, Xb[0], g.reshape(Xb.shape[1:])).ravel()
            dH = np.diag(H).copy()
            H[act, :] = 0.0
            H[:, act] = 0.0
            H[act, act] = dH[act]
            try:
                L = np.linalg.cholesky(H)
            except np.linalg.LinAlgError:
                status[b] = NOT_SPD
                break
            d = -np.linalg.solve(L.T, np.linalg.solve(L, g))
            if not np.all(np.isfinite(d)):
                status[b] = NONFINITE
                break
            d = d.reshape(Xb.shape[1:])
            x = Xb[0]
            s = np.clip(x + d, lo, hi) - x
            actr = act.reshape(x.shape)
            gr = g.reshape(x.shape)
            alpha = 1.0
            nz0 = cost_noise(pbs, Xb, *args)[0]
            for _ in range(LS_MAX):
                xt = np.clip(x + alpha * d, lo, hi)
                pred = alpha * np.sum(np.where(actr, 0.0, gr * d)) + np.sum(np.where(actr, gr * (xt - x), 0.0))
                Jt = residuals(pbs, xt[None], *args)[3][0]
                nzt = cost_noise(pbs, xt[None], *args)[0]
                if Jt <= J + 2.0 * ARMIJO_SIGMA * pred + nz0 + nzt + COST_SLACK * abs(J):
                    break
                alpha *= 0.5
            Xb = xt[None]
            if trace is not None:
                trace.append((b, int(iters[b]), alpha))
            iters[b] += 1
            if np.max(np.abs(s)) <= tol * (1.0 + np.max(np.abs(xt))):
                status[b] = OK
                H, g, J = normal_equations(pbs, Xb, *args)
                break
        X[b] = Xb[0]
        cost_out[b] = np.asarray(J).reshape(-1)[0]
    return X, cost_out, iters, status


def kkt_residual(pb, X, U, Y, PAR=None, x0=None):
    """Bound-constrained stationarity at X (B, P, n): max over entries of
    |X - P(X - grad)| with grad = 2 g the cost gradient -- zero exactly at KKT points
    (free entries: grad = 0; at a lower bound grad >= 0; at an upper bound grad <= 0)."""
    _, g, _ = normal_equations(pb, X, U, Y, PAR, x0)
    lo, hi = box(pb, X.shape)
    grad = 2.0 * g.reshape(X.shape)
    return np.max(np.abs(X - np.clip(X - grad, lo, hi)).reshape(X.shape[0], -1), axis=1)


def gn_step_batched(pb, X, U, Y, PAR=None, x0=None):
    """One vectorised GN iteration over the whole batch (CPU-baseline workload)."""
    H, g, cost = normal_equations(pb, X, U, Y, PAR, x0)
    L = np.linalg.cholesky(H)
    z = np.linalg.solve(L, -g[..., None])
    delta = np.linalg.solve(np.swapaxes(L, -1, -2), z)[..., 0]
    return X + delta.reshape(X.shape), cost


def _with_rw(pb, Rw):
    q = Problem.__new__(Problem)
    q.__dict__.update(pb.__dict__)
    q.Rw = Rw
    return q


# --------------------------------------------------------------------------
# CPU port of the per-iteration algorithm (bench.py cpu_baseline leg).
# Same split as the HIP kernel: the X-independent part of J^T W J (dynamics
# a^2 (D^T C D) (x) Qw, linear-measurement information, prior) is built once;
# every iteration adds the X-dependent dynamics terms, factors with batched
# LAPACK Cholesky and does two triangular solves per trajectory.
class CpuPort:
    def __init__(self, pb):
        if pb.meas != "full_state" or pb.Rw.ndim != 3:
            raise NotImplementedError("CpuPort covers the linear-measurement configs (C1, C2)")
        P, n, a = pb.P, pb.n, pb.alpha
        DCD = np.einsum("kj,k,kl->jl", pb.D, pb.c, pb.D)
        H4 = (a * a) * np.einsum("jl,ae->jale", DCD, pb.Qw)
        PR = pb.Phi[:, :, None] * pb.Phi[:, None, :]                   # (M,P,P)
        H4 += np.einsum("ijl,iae->jale", PR, pb.Rw)
        if pb.Pw is not None:
            H4[0, :, 0, :] += pb.Pw
        self.pb = pb
        self.Hc = H4.reshape(P * n, P * n)

    def iteration(self, X, U, Y, x0=None):
        """One GN iteration for the whole batch; returns X + delta."""
        import scipy.linalg as sla
        pb = self.pb
        B, P, n = X.shape
        d = P * n
        W, xi, e, cost = residuals(pb, X, U, Y, None, x0)
        _, F = models.dyn_eval(pb.dyn, X, U, pb.dyn_par)
        E = np.einsum("k,ac,zkce->zkae", pb.c, pb.Qw, F)
        # M[(j,a),(l,e)] = D_lj E_l[a,e];  H = Hc - a (M + M^T) + blkdiag(F^T E)
        Mx = (pb.D.T[None, :, None, :, None] * E.transpose(0, 2, 1, 3)[:, None]).reshape(B, d, d)
        H = self.Hc[None] - pb.alpha * (Mx + np.swapaxes(Mx, 1, 2))
        FtE = np.einsum("zjca,zjce->zjae", F, E)
        for k in range(P):
            H[:, k * n:(k + 1) * n, k * n:(k + 1) * n] += FtE[:, k]
        V = np.einsum("k,ac,zkc->zka", pb.c, pb.Qw, W)
        g = pb.alpha * np.einsum("kj,zka->zja", pb.D, V) - np.einsum("zjca,zjc->zja", F, V)
        ge = np.einsum("ipq,ziq->zip", pb.Rw, e)
        g -= np.einsum("ij,zia->zja", pb.Phi, ge)
        if pb.Pw is not None:
            g[:, 0] += (X[:, 0] - x0) @ pb.Pw.T
        g = g.reshape(B, d)
        L = np.linalg.cholesky(H)
        out = np.empty_like(X)
        for b in range(B):
            y = sla.solve_triangular(L[b], -g[b], lower=True, check_finite=False)
            delta = sla.solve_triangular(L[b], y, lower=True, trans="T", check_finite=False)
            out[b] = X[b] + delta.reshape(P, n)
        return out
