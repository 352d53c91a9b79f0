"""Seeded synthetic workloads for the BASELINE.json configs.

Host-side data generation only (truth by fixed-step RK4, noise by
``numpy.random.default_rng(seed)``, draws in batch order).  Nothing here is on
the timed path.

C1  single_integrator: n=1, m=1, full_state, N=20, T=10, M=50, B=1
    (estimation_example.py:13,20,24,33 scales; u = sin t)
C2  van_der_pol:       n=2, m=1 (u = 0), full_state, N=100, T=10, M=101, B=1024
    (van_der_pol.py:10,33 scales; R, Q from estimation_example.py:20,33)
C3  gnss_stationary:   n=5, m=3, pseudorange, N=200, T=200, 201 epochs x 12 sats, B=4096
    (large-system path: d = 1005)
C4  rc-car:            kinematic_bycicle_and_bias (n=6, m=2) + pseudorange, N=500, T=100 s
    of the reference's rc-car logs (px4 controls, 101 GNSS epochs x 12 slots), B=8192
    over 8 GPUs (d = 3006; rc-car.py:21-47,89-113 at N=500)
C5  multi-receiver:    multi_receiver (n=8, m=0) + pseudorange + pseudorange_rate per
    satellite and a 2-D range to the extra variable XA (n_extra=3) per epoch -- mixed
    rows, N=200, T=200, 201 epochs x (12 + 12 + 1) rows, B=16384 over 8 GPUs
    (multi-receiver.py:62-100 at N=200; d = 1608 + 3).  BASELINE.json calls it an
    "N-receiver joint state (~4N dims, N=8)": the reference's own multi-receiver
    problem has the 8-dim state of receiver B plus receiver A's position XA, and
    that is the structure used here.
"""
import numpy as np
from scipy.interpolate import interp1d

from nlp.collocation import ChebyshevPseudospectralMethod


class Workload:
    """Everything one batched estimation solve needs (numpy, host)."""

    def __init__(self, **kw):
        self.__dict__.update(kw)

    @property
    def P(self):
        return self.N + 1


def _rk4(f, x0, t, substeps=20):
    """Fixed-step RK4 over sample times t for a batch x0 (B, n)."""
    out = np.zeros((x0.shape[0], t.shape[0], x0.shape[1]))
    x = x0.copy()
    out[:, 0] = x
    for i in range(1, t.shape[0]):
        h = (t[i] - t[i - 1]) / substeps
        tt = t[i - 1]
        for _ in range(substeps):
            k1 = f(tt, x)
            k2 = f(tt + h / 2, x + h / 2 * k1)
            k3 = f(tt + h / 2, x + h / 2 * k2)
            k4 = f(tt + h, x + h * k3)
            x = x + h / 6 * (k1 + 2 * k2 + 2 * k3 + k4)
            tt += h
        out[:, i] = x
    return out


def _init_from_measurements(cpm, t_meas, Y):
    """initializeEstimate (nlp/nlp.py:288-302) applied to y for every trajectory."""
    t_nodes = cpm.tau2t(cpm.tau)
    X = np.zeros((Y.shape[0], t_nodes.shape[0], Y.shape[2]))
    for b in range(Y.shape[0]):
        X[b] = interp1d(t_meas, Y[b].T, fill_value="extrapolate")(t_nodes).T
    return X


def make_c1(seed=0, B=1, N=20):
    T, M = 10.0, 50
    rng = np.random.default_rng(seed)
    t = np.linspace(0, T, M)
    u = np.sin(t)
    cpm = ChebyshevPseudospectralMethod(N, 0, T)
    x0 = np.zeros((B, 1))
    # single integrator: x(t) = int_0^t sin = 1 - cos t
    xt = x0[:, None, :] + (1 - np.cos(t))[None, :, None]
    R = np.array([[0.01]])
    Y = xt + rng.normal(size=xt.shape) * np.sqrt(R[0, 0])
    t_nodes = cpm.tau2t(cpm.tau)
    U = interp1d(t, u[None, :], fill_value="extrapolate")(t_nodes).T[None]  # (1, P, 1)
    Q = np.array([[1e-4]])
    return Workload(name="C1_single_integrator", N=N, T=T, n=1, m=1, p=1, M=M, B=B,
                    dyn="single_integrator", meas="full_state", meas_static={},
                    t_meas=t, Y=Y, U=U, PAR=None, Qw=np.linalg.inv(Q),
                    Rw=np.broadcast_to(np.linalg.inv(R), (M, 1, 1)).copy(), Pw=None, x0=None,
                    X_init=_init_from_measurements(cpm, t, Y), X_true=xt, cpm=cpm)


def vdp_rhs(t, x):
    return np.stack([(1 - x[:, 1] ** 2) * x[:, 0] - x[:, 1], x[:, 0]], axis=1)


def make_c2(B=1024, seed=1, N=100, shard=None):
    """C2.  ``shard=(lo, hi)``: only trajectories [lo, hi) of the seeded batch of B --
    bitwise the same arrays as slicing the full batch (the random draws are made for
    all B, in batch order, which costs microseconds; the RK4 truth and the initial
    iterates, the expensive part, only for the shard).  The strong-scaling bench
    gives every rank its own shard this way (mhe.dist.shard_range)."""
    T, M = 10.0, 101
    lo, hi = (0, B) if shard is None else (int(shard[0]), int(shard[1]))
    if not 0 <= lo <= hi <= B:
        raise ValueError(f"shard {shard} outside [0, {B}]")
    rng = np.random.default_rng(seed)
    x0 = (np.array([0.0, 1.0])[None, :] + rng.normal(size=(B, 2)) * 0.1)[lo:hi]
    t = np.linspace(0, T, M)
    xt = _rk4(vdp_rhs, x0, t)
    R = np.diag([0.01, 0.02])
    noise = rng.normal(size=(B, M, 2))[lo:hi]
    Y = xt + noise * np.sqrt(np.diag(R))[None, None, :]
    cpm = ChebyshevPseudospectralMethod(N, 0, T)
    Q = np.diag([1e-4, 1e-4])
    B = hi - lo
    return Workload(name="C2_van_der_pol", N=N, T=T, n=2, m=1, p=2, M=M, B=B, shard=(lo, hi),
                    dyn="van_der_pol", meas="full_state", meas_static={},
                    t_meas=t, Y=Y, U=np.zeros((1, N + 1, 1)), PAR=None, Qw=np.linalg.inv(Q),
                    Rw=np.broadcast_to(np.linalg.inv(R), (M, 2, 2)).copy(), Pw=None, x0=None,
                    X_init=_init_from_measurements(cpm, t, Y), X_true=xt, cpm=cpm)




def make_gnss_small(B=4, seed=2, N=10, T=50.0, n_sat=8, epochs=51, sat=None, count=None):
    """Small gnss_stationary-shaped problem (pseudorange, n=5) for parity tests.

    Satellite ENU positions: ``sat`` (epochs, n_sat, 3) when given (time-varying; slots
    j >= count[e] are empty: R = 0 and a zero position, as the reference masks them,
    autonomous-car.py:260-263), else synthetic ones at ~2e7 m fixed per slot, shared by
    the batch.  Truth = stationary receiver + drifting clock; Q, r_pr as
    gnss_stationary.py:18-19.
    """
    rng = np.random.default_rng(seed)
    t_ep = np.linspace(0, T, epochs)
    if sat is None:
        az = rng.uniform(0, 2 * np.pi, n_sat)
        el = rng.uniform(0.3, 1.3, n_sat)
        s0 = 2.2e7 * np.stack([np.cos(el) * np.cos(az), np.cos(el) * np.sin(az), np.sin(el)], axis=1)
        sat = np.broadcast_to(s0, (epochs, n_sat, 3)).copy()
    sat = np.asarray(sat, dtype=np.float64)[:epochs]
    n_sat = sat.shape[1]
    live = np.ones((epochs, n_sat), dtype=bool) if count is None else (np.arange(n_sat)[None, :] < np.asarray(count)[:epochs, None])
    sat = np.where(live[..., None], sat, 0.0)
    t_meas = np.repeat(t_ep, n_sat)
    PAR = sat.reshape(1, -1, 3)  # (1, M, 3)
    M = t_meas.shape[0]
    pos = rng.normal(size=(B, 3)) * 10.0
    b0 = rng.normal(size=B) * 100.0
    bd = rng.normal(size=B) * 0.5
    r_pr = 100.0
    xt = np.zeros((B, epochs, 5))
    xt[:, :, :3] = pos[:, None, :]
    xt[:, :, 3] = b0[:, None] + bd[:, None] * t_ep[None, :]
    xt[:, :, 4] = bd[:, None]
    rho = np.linalg.norm(xt[:, :, None, :3] - sat[None, :, :, :], axis=-1) + xt[:, :, None, 3]
    Y = np.where(live[None], rho + rng.normal(size=rho.shape) * np.sqrt(r_pr), 0.0).reshape(B, M, 1)
    cpm = ChebyshevPseudospectralMethod(N, 0, T)
    t_nodes = cpm.tau2t(cpm.tau)
    X_init = np.zeros((B, N + 1, 5))
    X_init[:, :, :3] = pos[:, None, :] + rng.normal(size=(B, 1, 3)) * 3.0
    X_init[:, :, 3] = (b0[:, None] + bd[:, None] * t_nodes[None, :]) + rng.normal(size=(B, 1)) * 3.0
    X_init[:, :, 4] = bd[:, None]
    Q = np.diag([0.0001, 0.0001, 0.0001, 0.1, 0.001])
    Rw = np.where(live.reshape(-1), 1.0 / r_pr, 0.0)[:, None, None]
    return Workload(name="gnss_small", N=N, T=T, n=5, m=3, p=1, M=M, B=B,
                    dyn="gnss_pos_and_bias", meas="pseudorange", meas_static={"idx": [0, 1, 2, 3]},
                    t_meas=t_meas, Y=Y, U=np.zeros((1, N + 1, 3)), PAR=PAR, Qw=np.linalg.inv(Q),
                    Rw=Rw, Pw=None, x0=None, X_init=X_init, X_true=xt, cpm=cpm)


def c3_geometry():
    """The satellite geometry of the reference's gnss_stationary log (201 epochs x 12
    slots, ENU; tests/golden/gnss_stationary_c3.npz, generated by the reference's own
    load_gnss_logs / ecef2enu in tests/golden/gen_golden.py)."""
    import os
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "tests", "golden", "gnss_stationary_c3.npz")
    z = np.load(path)
    return z["sat_enu"], z["count"]


def make_c3(B=4096, seed=2, N=200):
    """C3 gnss_stationary shape: gnss_pos_and_bias (n=5, m=3, u=0) +
    pseudorange, N=200, T=200 s, 201 epochs x 12 satellite slots (M=2412), d=1005, with
    the satellite positions of data/gnss_stationary's log (empty slots: R = 0)."""
    sat, cnt = c3_geometry()
    w = make_gnss_small(B=B, seed=seed, N=N, T=200.0, epochs=201, sat=sat, count=cnt)
    w.name = "C3_gnss_stationary"
    return w


CONFIGS = {"C1": make_c1, "C2": make_c2, "C3": make_c3}


def _sky(rng, n_sat, r=2.2e7):
    az = rng.uniform(0, 2 * np.pi, n_sat)
    el = rng.uniform(0.3, 1.3, n_sat)
    return r * np.stack([np.cos(el) * np.cos(az), np.cos(el) * np.sin(az), np.sin(el)], axis=1)


def bicycle_rhs(x, u):
    """dynamics.kinematic_bycicle_and_bias (nlp/dynamics.py:117-136), batch form;
    x[2] is used as the heading exactly as the reference does."""
    L = 0.28
    v = 8.72649116358 * u[:, 0] - 0.856053299155
    delta = np.deg2rad(28) * u[:, 1]
    return np.stack([v * np.cos(x[:, 2]), v * np.sin(x[:, 2]), np.zeros_like(v), x[:, 4], np.zeros_like(v),
                     (v / L) * np.tan(delta)], axis=1)


def rc_car_inputs():
    """The reference's rc-car inputs (tests/golden/rc_car_c4.npz, written by
    tests/golden/gen_golden.py gen_rc_car_c4 from data/rc-car/px4/log_164_*.ulg and
    data/rc-car/gnss/gnss_log_2020_02_27_10_02_20*.mat exactly as px4/convert.py and
    rc-car.py:21-38 process them): px4 times t_u (s, from 0) and controls u (2, T')
    [throttle, steer]; GNSS epoch times t_gnss, ENU satellite positions sat_enu
    (E, 12, 3), slot counts, pseudoranges."""
    import os
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "tests", "golden", "rc_car_c4.npz")
    return np.load(path)


def make_c4(B=1024, seed=3, N=500, T=100.0):
    """C4 rc-car: kinematic_bycicle_and_bias (n=6, m=2) + pseudorange,
    N=500 (d = 3006), on the reference's own rc-car data over the first T = 100 s: the
    throttle / steering of data/rc-car/px4/log_164 (250 Hz; setControl interpolates them
    at the nodes, nlp/nlp.py:304-308) and the satellite epochs of
    data/rc-car/gnss/gnss_log_2020_02_27_10_02_20 (101 epochs x 12 slots, 9-12 live:
    empty slots R = 0, as the scripts mask them) -- rc_car_inputs().  Per trajectory:
    a seeded initial state (position, heading, clock bias and drift), the truth
    integrated from those controls (RK4, 25 sub-steps a second), pseudoranges at the
    real satellite positions with r_pr = 10 (rc-car.py:47); Q as rc-car.py:46.  No
    heading rows: rc-car.py:89-114 adds pseudoranges only."""
    z = rc_car_inputs()
    ep = np.nonzero(z["t_gnss"] <= T + 1e-9)[0]
    t_ep, sat, cnt = z["t_gnss"][ep], z["sat_enu"][ep], z["count"][ep]
    epochs, n_sat = t_ep.size, sat.shape[1]
    live = np.arange(n_sat)[None, :] < cnt[:, None]
    rng = np.random.default_rng(seed)
    uf = interp1d(z["t_u"], z["u"], fill_value="extrapolate")

    def ctrl(t):
        return np.broadcast_to(uf(np.atleast_1d(t)).T[None], (B, np.size(t), 2))

    x0 = np.zeros((B, 6))
    x0[:, :2] = rng.normal(size=(B, 2)) * 10.0
    x0[:, 2] = rng.uniform(-np.pi, np.pi, B)
    x0[:, 3] = rng.normal(size=B) * 100.0
    x0[:, 4] = rng.normal(size=B) * 0.5
    xt = _rk4(lambda tt, x: bicycle_rhs(x, ctrl(tt)[:, 0]), x0, t_ep, substeps=25)
    r_pr = 10.0
    rho = np.linalg.norm(xt[:, :, None, :3] - sat[None], axis=-1) + xt[:, :, None, 3]
    M = epochs * n_sat
    Y = np.where(live[None], rho + rng.normal(size=rho.shape) * np.sqrt(r_pr), 0.0).reshape(B, M, 1)
    cpm = ChebyshevPseudospectralMethod(N, 0, T)
    t_nodes = cpm.tau2t(cpm.tau)
    U = interp1d(z["t_u"], z["u"], fill_value="extrapolate")(t_nodes).T[None]   # setControl
    X_init = interp1d(t_ep, xt, axis=1)(t_nodes) + rng.normal(size=(B, 1, 6)) * np.array([2.0, 2.0, 0.02, 2.0, 0.05, 0.1])
    Q = np.diag([1, 1, 0.001, .01, .01, 1])
    Rw = np.where(live.reshape(-1), 1.0 / r_pr, 0.0)[:, None, None]
    return Workload(name="C4_rc_car", N=N, T=T, n=6, m=2, p=1, M=M, B=B,
                    dyn="kinematic_bycicle_and_bias", meas="pseudorange", meas_static={"idx": [0, 1, 2, 3]},
                    t_meas=np.repeat(t_ep, n_sat), Y=Y, U=U, PAR=sat.reshape(1, M, 3),
                    Qw=np.linalg.inv(Q), Rw=Rw, Pw=None, x0=None, X_init=X_init, X_true=xt, cpm=cpm)


def pr_row(idx, sat):
    """MHE_MEAS_MIXED PSEUDORANGE row (include/mhe.h): [1, i0..i3, -1 x 3, sat, 0 x 3]."""
    return [1.0] + [float(i) for i in idx] + [-1.0] * 3 + list(np.asarray(sat, dtype=np.float64)) + [0.0] * 3


def range3d_row(idx):
    """MHE_MEAS_MIXED RANGE_3D row between x[idx[0:3]] and x[idx[3:6]], offset 0."""
    return [4.0] + [float(i) for i in idx] + [-1.0] + [0.0] * 6


def make_c5_small(B=2048, seed=4, N=200, epochs=None, n_sat=12):
    """C5s (an extra config, NOT SURVEY §8(d)'s C5): the reference's own multi-receiver.py
    structure -- multi_receiver dynamics (x = [p, b, v, alpha], n=8, m=0),
    per epoch 12 pseudoranges + 12 pseudorange rates (sat_pos, sat_vel) and one 2-D range
    to XA (extra decision variable, 3 components; multi-receiver.py:73,99), mixed rows
    (include/mhe.h).  Weights as multi-receiver.py:77-88 (the script passes inv(Q))."""
    T = float(N)
    epochs = N + 1 if epochs is None else epochs
    rng = np.random.default_rng(seed)
    t_ep = np.linspace(0, T, epochs)
    sat0 = _sky(rng, n_sat)
    svel = rng.normal(size=(n_sat, 3))
    svel = 3000.0 * svel / np.linalg.norm(svel, axis=1, keepdims=True)
    p0 = rng.normal(size=(B, 3)) * 10.0
    hd = rng.uniform(0, 2 * np.pi, B)
    vel = np.stack([np.cos(hd), np.sin(hd), np.zeros(B)], axis=1) * rng.uniform(0.5, 1.5, (B, 1))
    b0 = rng.normal(size=B) * 100.0
    al = rng.normal(size=B) * 0.5
    # receiver A (truth of XA) 2.4384 m (multi-receiver.py:98) beside the middle of B's track
    side = np.stack([-np.sin(hd), np.cos(hd), np.zeros(B)], axis=1)
    xa = p0 + vel * (T / 2) + 2.4384 * side + np.concatenate([np.zeros((B, 2)), rng.normal(size=(B, 1))], 1)
    r_pr, r_prr, r_range = 100.0, 0.1, 0.01
    rows, t_rows, Rw = [], [], []
    Yl = []
    for k, tk in enumerate(t_ep):
        sp = sat0 + svel * tk
        pos = p0 + vel * tk
        bias = b0 + al * tk
        for j in range(n_sat):
            d = pos - sp[j]
            rho = np.linalg.norm(d, axis=1)
            rows.append([1, 0, 1, 2, 3, -1, -1, -1] + list(sp[j]) + [0.0, 0.0, 0.0])
            t_rows.append(tk); Rw.append(1.0 / r_pr)
            Yl.append(rho + bias + rng.normal(size=B) * np.sqrt(r_pr))
            los = -d / rho[:, None]
            rows.append([2, 0, 1, 2, 4, 5, 6, 7] + list(sp[j]) + list(svel[j]))
            t_rows.append(tk); Rw.append(1.0 / r_prr)
            Yl.append(np.sum((svel[j][None] - vel) * los, axis=1) + al + rng.normal(size=B) * np.sqrt(r_prr))
        rows.append([3, 0, 1, 8, 9, -1, -1, -1, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0])
        t_rows.append(tk); Rw.append(1.0 / r_range)
        Yl.append(np.sqrt(np.sum((pos[:, :2] - xa[:, :2]) ** 2, axis=1) + 1e-6) + rng.normal(size=B) * np.sqrt(r_range))
    M = len(rows)
    cpm = ChebyshevPseudospectralMethod(N, 0, T)
    t_nodes = cpm.tau2t(cpm.tau)
    xt = np.zeros((B, t_nodes.shape[0], 8))
    xt[:, :, :3] = p0[:, None] + vel[:, None] * t_nodes[None, :, None]
    xt[:, :, 3] = b0[:, None] + al[:, None] * t_nodes[None]
    xt[:, :, 4:7] = vel[:, None]
    xt[:, :, 7] = al[:, None]
    X_init = xt + rng.normal(size=(B, 1, 8)) * np.array([2.0, 2.0, 2.0, 2.0, 0.05, 0.05, 0.05, 0.05])
    Q = np.diag([0.01, 0.01, 0.01, 0.01, 1., 1., 0.01, 0.01])
    return Workload(name="C5s_multi_receiver_n8", N=N, T=T, n=8, m=0, p=1, M=M, B=B,
                    dyn="multi_receiver", meas="mixed", meas_static={}, n_extra=3,
                    t_meas=np.asarray(t_rows), Y=np.stack(Yl, axis=1)[:, :, None], U=None,
                    PAR=np.asarray(rows, dtype=np.float64)[None], Qw=np.linalg.inv(Q), Rw=np.asarray(Rw),
                    Pw=None, x0=None, X_init=X_init, Z_init=xa + rng.normal(size=(B, 3)) * 0.5,
                    X_true=xt, Z_true=xa, cpm=cpm)


def make_c5(B=2048, seed=4, N=200, R=8, r_pr=1.0, r_range=0.01, spacing=0.5 * 91.44):
    """C5 as SURVEY.md §8(d) defines it: 8 receivers, each the per-receiver block of
    gnss_two_receiver [x, y, z, b, alpha] (nlp/dynamics.py:98-115) -> n = 40, m = 24
    (each receiver's velocity as its control, as gnss-multi-receiver.py:156-165 feeds
    LS velocities); per epoch 12 pseudoranges per receiver (idx offsets 5r, the
    satellite epochs of data/gnss_stationary's log, empty slots R = 0) and one
    multi_receiver_range_3d row between each adjacent pair (nlp/measurements.py:39-54),
    mixed rows (include/mhe.h).  N = 200, T = 200 s, 201 epochs x (96 + 7) rows, d = 8040.
    Weights as gnss-multi-receiver.py:43-48 (Q per receiver block, r_pr = 1 (B's),
    r_range = 0.01, dt = 1 s).  Receivers in a line `spacing` m apart, moving together
    (default the script's 50-yard baseline, gnss-multi-receiver.py:68).  Gauss-Newton's
    local rate here is set by the range rows' dropped curvature R e (I - u u^T) / |d|:
    at a 5 m baseline it exceeds the Gauss-Newton curvature of the receivers' relative
    position and the iteration oscillates (IPOPT's exact Hessian would not)."""
    T = float(N)
    epochs = N + 1
    rng = np.random.default_rng(seed)
    sat_all, cnt = c3_geometry()
    sat_all, cnt = sat_all[:epochs], cnt[:epochs]
    t_ep = np.linspace(0, T, epochs)
    n, m = 5 * R, 3 * R
    p0 = rng.normal(size=(B, 3)) * 10.0
    hd = rng.uniform(0, 2 * np.pi, B)
    vel = np.stack([np.cos(hd), np.sin(hd), np.zeros(B)], axis=1) * rng.uniform(0.5, 1.5, (B, 1))
    side = np.stack([-np.sin(hd), np.cos(hd), np.zeros(B)], axis=1)
    b0 = rng.normal(size=(B, R)) * 100.0
    al = rng.normal(size=(B, R)) * 0.5
    offs = (np.arange(R) - (R - 1) / 2.0) * spacing                     # positions along the line
    rows, t_rows, Rw, Yl = [], [], [], []
    for k, tk in enumerate(t_ep):
        base = p0 + vel * tk                                             # (B, 3)
        pos = base[:, None, :] + offs[None, :, None] * side[:, None, :]  # (B, R, 3)
        for r in range(R):
            for j in range(sat_all.shape[1]):
                live = j < cnt[k]
                sp = sat_all[k, j] if live else np.zeros(3)
                rows.append(pr_row([5 * r, 5 * r + 1, 5 * r + 2, 5 * r + 3], sp))
                t_rows.append(tk); Rw.append(1.0 / r_pr if live else 0.0)
                rho = np.linalg.norm(pos[:, r] - sp, axis=1) + b0[:, r] + al[:, r] * tk
                Yl.append(np.where(live, rho + rng.normal(size=B) * np.sqrt(r_pr), 0.0))
        for r in range(R - 1):
            rows.append(range3d_row([5 * r, 5 * r + 1, 5 * r + 2, 5 * r + 5, 5 * r + 6, 5 * r + 7]))
            t_rows.append(tk); Rw.append(1.0 / r_range)
            d = np.sqrt(np.sum((pos[:, r] - pos[:, r + 1]) ** 2, axis=1) + 1e-6)
            Yl.append(d + rng.normal(size=B) * np.sqrt(r_range))
    M = len(rows)
    cpm = ChebyshevPseudospectralMethod(N, 0, T)
    t_nodes = cpm.tau2t(cpm.tau)
    xt = np.zeros((B, t_nodes.shape[0], n))
    for r in range(R):
        pr_ = (p0[:, None] + vel[:, None] * t_nodes[None, :, None]) + offs[r] * side[:, None]
        xt[:, :, 5 * r:5 * r + 3] = pr_
        xt[:, :, 5 * r + 3] = b0[:, r:r + 1] + al[:, r:r + 1] * t_nodes[None]
        xt[:, :, 5 * r + 4] = al[:, r:r + 1]
    U = np.repeat(np.tile(vel, (1, R))[:, None, :], t_nodes.shape[0], axis=1) + rng.normal(size=(B, 1, m)) * 0.05
    X_init = xt + rng.normal(size=(B, 1, n)) * np.tile([2.0, 2.0, 2.0, 2.0, 0.05], R)
    Qd = np.tile([.01, .01, .01, 0.01, 0.01], R)                         # gnss-multi-receiver.py:43
    return Workload(name="C5_eight_receivers", N=N, T=T, n=n, m=m, p=1, M=M, B=B,
                    dyn="gnss_eight_receivers", meas="mixed", meas_static={}, n_extra=0,
                    t_meas=np.asarray(t_rows), Y=np.stack(Yl, axis=1)[:, :, None], U=U,
                    PAR=np.asarray(rows, dtype=np.float64)[None], Qw=np.diag(1.0 / Qd), Rw=np.asarray(Rw),
                    Pw=None, x0=None, X_init=X_init, X_true=xt, cpm=cpm)


CONFIGS.update({"C4": make_c4, "C5": make_c5, "C5s": make_c5_small})
