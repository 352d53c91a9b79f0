"""CPU restatement of the reference EKF -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline may import
this module; the product path (utils.ekf -> libmhe.so) never does.

Follows kingdwd/nlp-filter:
  utils/ekf.py:20-38  EKF.update   (predict; correct only when z is given)
  utils/ekf.py:40-45  predict      S- = G S G^T + Q
  utils/ekf.py:47-61  correct      P = H S- H^T + R, K = S- H^T inv(P) (explicit
                                   inverse, as the reference), mu += K (z - h),
                                   S += -K H S-
  utils/gnss.py:79-90 gnss_pos_and_bias  (in-place x update; G = I, G[3,4] = dt)
  utils/gnss.py:4-24  pseudorange, :27-45 multi_pseudorange,
  utils/gnss.py:48-61 multi_pseudorange_and_bias (bias row of J left zero)
  autonomous-car.py:18-52 discrete_vehicle_dynamics (Euler on utils/vehicle_sim.py:
                      72-85 with linear tyres :58-66; Jacobian at the UPDATED state,
                      since the reference updates x in place first)
  autonomous-car.py:54-77 vehicle_sensors_model (multi_pseudorange on x[0,1,8,6,7])
Pinned by tests/golden/ekf_gnss_stationary.npz (the reference EKF run on the
gnss_stationary log) and tests/golden/ekf_autocar.npz (the reference EKF with the
autonomous-car script's own plug-ins on seeded data of the script's shape), both
written by tests/golden/gen_golden.py.
"""
import numpy as np


def gnss_pos_and_bias(x, u, params=None, jac=False):
    x = np.array(x, dtype=np.float64)
    x += params["dt"] * np.array([u[0], u[1], u[2], x[4], 0.0])
    if jac:
        J = np.eye(5)
        J[3, 4] = params["dt"]
        return x, J
    return x


def pseudorange(x, params=None, jac=False):
    s = params["sat_pos"]
    y = np.sqrt((x[0] - s[0]) ** 2 + (x[1] - s[1]) ** 2 + (x[2] - s[2]) ** 2) + x[3]
    if jac:
        J = np.zeros(5)
        los = s - x[:3]
        J[:3] = -los / np.linalg.norm(los)
        J[3] = 1.0
        return y, J
    return y


def multi_pseudorange(x, params=None, jac=False):
    S = params["sat_pos"]
    y = np.zeros(S.shape[0])
    J = np.zeros((S.shape[0], 5))
    for i in range(S.shape[0]):
        y[i], J[i] = pseudorange(x, {"sat_pos": S[i]}, jac=True)
    return (y, J) if jac else y


def multi_pseudorange_and_bias(x, params=None, jac=False):
    S = params["sat_pos"]
    y = np.zeros(S.shape[0] + 1)
    J = np.zeros((S.shape[0] + 1, 5))
    y[-1] = x[3]
    y[:-1], J[:-1] = multi_pseudorange(x, {"sat_pos": S}, jac=True)
    return (y, J) if jac else y


def discrete_vehicle_dynamics(x, u, params=None, jac=False):
    dt, C = params["dt"], params["car_params"]
    x = np.array(x, dtype=np.float64)
    vx, vy, r, psi = x[3], x[4], x[5], x[2]
    Fr = -C["C_AR"] * ((vy - C["D_R"] * r) / vx)
    Ff = -C["C_AF"] * ((vy + C["D_F"] * r) / vx - u[1])
    xd = np.zeros(9)
    xd[0] = vx * np.cos(psi) - vy * np.sin(psi)
    xd[1] = vx * np.sin(psi) + vy * np.cos(psi)
    xd[2] = r
    xd[3] = (-Ff * np.sin(u[1]) + u[0]) / C["M"] + r * vy
    xd[4] = (Ff * np.cos(u[1]) + Fr) / C["M"] - r * vx
    xd[5] = (C["D_F"] * Ff * np.cos(u[1]) - C["D_R"] * Fr) / C["I_Z"]
    xd[6] = x[7]
    x = x + dt * xd
    if not jac:
        return x
    vx, vy, r, psi = x[3], x[4], x[5], x[2]          # the Jacobian sees the updated state
    M, I, DF, DR = C["M"], C["I_Z"], C["D_F"], C["D_R"]
    dFf = np.array([C["C_AF"] * (vy + DF * r) / vx ** 2, -C["C_AF"] / vx, -C["C_AF"] * DF / vx])   # d/d(vx, vy, r)
    dFr = np.array([C["C_AR"] * (vy - DR * r) / vx ** 2, -C["C_AR"] / vx, C["C_AR"] * DR / vx])
    su, cu = np.sin(u[1]), np.cos(u[1])
    J = np.eye(9)
    J[0, 2] += dt * (-vx * np.sin(psi) - vy * np.cos(psi))
    J[0, 3] += dt * np.cos(psi)
    J[0, 4] += -dt * np.sin(psi)
    J[1, 2] += dt * (vx * np.cos(psi) - vy * np.sin(psi))
    J[1, 3] += dt * np.sin(psi)
    J[1, 4] += dt * np.cos(psi)
    J[2, 5] += dt
    J[3, 3] += -(dt / M) * su * dFf[0]
    J[3, 4] += dt * (r - su * dFf[1] / M)
    J[3, 5] += dt * (vy - su * dFf[2] / M)
    J[4, 3] += dt * ((cu * dFf[0] + dFr[0]) / M - r)
    J[4, 4] += (dt / M) * (cu * dFf[1] + dFr[1])
    J[4, 5] += dt * ((cu * dFf[2] + dFr[2]) / M - vx)
    J[5, 3:6] += (dt / I) * (DF * cu * dFf - DR * dFr)
    J[6, 7] += dt
    return x, J


def vehicle_sensors_model(x, params=None, jac=False):
    S = params["sat_pos"]
    p = np.array([x[0], x[1], x[8]])
    d = p[None, :] - S
    rng = np.sqrt((d ** 2).sum(axis=1))
    y = rng + x[6]
    if not jac:
        return y
    J = np.zeros((S.shape[0], 9))
    J[:, [0, 1, 8]] = d / rng[:, None]
    J[:, 6] = 1.0
    return y, J


class EKF:
    def __init__(self, dyn_func, meas_func, mu0, S0):
        self.mu = np.array(mu0, dtype=np.float64)
        self.S = np.array(S0, dtype=np.float64)
        self.dynamics = dyn_func
        self.measurement = meas_func

    def update(self, u, z, Q, R, dyn_func_params=None, meas_func=None, meas_func_params=None):
        mu_pred, G = self.dynamics(self.mu, u, params=dyn_func_params, jac=True)
        S_pred = G @ (self.S @ G.T) + Q
        if z is not None:
            h = meas_func if meas_func is not None else self.measurement
            z_pred, H = h(mu_pred, params=meas_func_params, jac=True)
            P = H @ (S_pred @ H.T) + R
            K = S_pred @ (H.T @ np.linalg.inv(P))
            self.mu = mu_pred + K @ (z - z_pred)
            self.S = S_pred + (-(K @ (H @ S_pred)))
        else:
            self.mu, self.S = mu_pred, S_pred


def run_fixture(fx, meas=multi_pseudorange):
    """Replay the gnss_stationary fixture recipe; returns (mu (T,5), S (T,5,5))."""
    f = EKF(gnss_pos_and_bias, meas, fx["mu0"], fx["S0"])
    mus, Ss = [], []
    for k in range(fx["pr"].shape[0]):
        ns = int(fx["nsat"][k])
        R = np.diag(float(fx["r_pr"]) * np.ones(ns))
        f.update(np.zeros(3), fx["pr"][k, :ns], fx["Q"], R, {"dt": float(fx["dt"])}, None,
                 {"sat_pos": fx["sat_pos"][k, :ns]})
        mus.append(f.mu.copy())
        Ss.append(f.S.copy())
    return np.stack(mus), np.stack(Ss)
