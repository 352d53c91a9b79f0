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
