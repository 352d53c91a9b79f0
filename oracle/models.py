"""Oracle: plug-in models with analytic Jacobians -- TEST INFRASTRUCTURE ONLY.

Batched NumPy restatements of the reference plug-ins.  Every function takes
arrays with arbitrary leading batch dims and returns (value, Jacobian).

Dynamics  f(x, u) -> (f (..., n), F = df/dx (..., n, n))
  single_integrator            nlp/dynamics.py:4-8
  single_integrator_2D / _3D   nlp/dynamics.py:10-27
  double_integrator            nlp/dynamics.py:29-38
  van_der_pol                  nlp/dynamics.py:61-66
  gnss_pos_and_bias            nlp/dynamics.py:68-79
  multi_receiver (m = 0)       nlp/dynamics.py:81-96
  gnss_two_receiver            nlp/dynamics.py:98-115
  kinematic_bycicle_and_bias   nlp/dynamics.py:117-136 (uses x[2] as the heading,
                               exactly as the reference code does)
  gnss_eight_receivers         8 x the receiver block of nlp/dynamics.py:98-115 (C5, n=40)
  vehicle_dynamics_and_gnss    nlp/dynamics.py:148-174 (static = params["car_params"]:
                               a dict with C_AF, C_AR, M, D_F, D_R, I_Z as
                               utils/vehicle_sim.py:10-23, or that 6-vector)

Measurements  h(x, par) -> (h (..., p), H = dh/dx (..., p, n))
  full_state                   nlp/measurements.py:4-5
  pseudorange                  nlp/measurements.py:56-70  (par = sat_pos[3], static idx)
  vehicle_pseudorange          nlp/measurements.py:81-88  (idx = [0, 1, 8, 6])
  multi_receiver_range_3d      nlp/measurements.py:39-54  ("y" point form, par = y[3];
                                                           "idxA/idxB" form, no par)
"""
import numpy as np

VDP = "van_der_pol"


def _zeros_like_F(x):
    n = x.shape[-1]
    return np.zeros(x.shape + (n,))


def dyn_eval(name, x, u, static=None):
    x = np.asarray(x, dtype=np.float64)
    u = np.asarray(u, dtype=np.float64) if u is not None else None
    F = _zeros_like_F(x)
    if name == "single_integrator":
        f = u[..., :1].copy()
    elif name in ("single_integrator_2D", "single_integrator_3D"):
        f = u.copy()
    elif name == "double_integrator":
        f = np.stack([x[..., 2], x[..., 3], u[..., 0], u[..., 1]], axis=-1)
        F[..., 0, 2] = 1.0
        F[..., 1, 3] = 1.0
    elif name == VDP:
        x0, x1 = x[..., 0], x[..., 1]
        f = np.stack([(1 - x1 ** 2) * x0 - x1 + u[..., 0], x0], axis=-1)
        F[..., 0, 0] = 1 - x1 ** 2
        F[..., 0, 1] = -2 * x1 * x0 - 1
        F[..., 1, 0] = 1.0
    elif name == "gnss_pos_and_bias":
        z = np.zeros_like(x[..., 0])
        f = np.stack([u[..., 0], u[..., 1], u[..., 2], x[..., 4], z], axis=-1)
        F[..., 3, 4] = 1.0
    elif name == "multi_receiver":
        z = np.zeros_like(x[..., 0])
        f = np.stack([x[..., 4], x[..., 5], x[..., 6], x[..., 7], z, z, z, z], axis=-1)
        for a in range(4):
            F[..., a, a + 4] = 1.0
    elif name == "gnss_two_receiver":
        z = np.zeros_like(x[..., 0])
        f = np.stack([u[..., 0], u[..., 1], u[..., 2], x[..., 4], z,
                      u[..., 3], u[..., 4], u[..., 5], x[..., 9], z], axis=-1)
        F[..., 3, 4] = 1.0
        F[..., 8, 9] = 1.0
    elif name == "kinematic_bycicle_and_bias":
        L = 0.28
        v = 8.72649116358 * u[..., 0] - 0.856053299155
        delta = np.deg2rad(28) * u[..., 1]
        z = np.zeros_like(x[..., 0])
        f = np.stack([v * np.cos(x[..., 2]), v * np.sin(x[..., 2]), z, x[..., 4], z,
                      (v / L) * np.tan(delta)], axis=-1)
        F[..., 0, 2] = -v * np.sin(x[..., 2])
        F[..., 1, 2] = v * np.cos(x[..., 2])
        F[..., 3, 4] = 1.0
    elif name == "gnss_eight_receivers":
        # 8 x the per-receiver block of gnss_two_receiver (nlp/dynamics.py:98-115)
        z = np.zeros_like(x[..., 0])
        cols = []
        for r in range(8):
            cols += [u[..., 3 * r], u[..., 3 * r + 1], u[..., 3 * r + 2], x[..., 5 * r + 4], z]
            F[..., 5 * r + 3, 5 * r + 4] = 1.0
        f = np.stack(cols, axis=-1)
    elif name == "vehicle_dynamics_and_gnss":
        C = static
        if isinstance(C, dict):
            C = C.get("car_params", C)
            C = [C["C_AF"], C["C_AR"], C["M"], C["D_F"], C["D_R"], C["I_Z"]]
        caf, car, mass, df, dr, iz = (float(c) for c in np.asarray(C, dtype=np.float64)[:6])
        px, py, psi, vx, vy, r = (x[..., k] for k in range(6))
        d = u[..., 1]
        den = vx + 0.001                                  # nlp/dynamics.py:153
        fyr = -car * (vy - dr * r) / den
        fyf = -caf * ((vy + df * r) / den - d)
        z = np.zeros_like(px)
        f = np.stack([vx * np.cos(psi) - vy * np.sin(psi), vx * np.sin(psi) + vy * np.cos(psi), r,
                      (-fyf * np.sin(d) + u[..., 0]) / mass + r * vy,
                      (fyf * np.cos(d) + fyr) / mass - r * vx,
                      (df * fyf * np.cos(d) - dr * fyr) / iz, x[..., 7], z, z], axis=-1)
        # d(F_yf, F_yr)/d(vx, vy, r)
        dfyf = [caf * (vy + df * r) / den ** 2, -caf / den, -caf * df / den]
        dfyr = [car * (vy - dr * r) / den ** 2, -car / den, car * dr / den]
        F[..., 0, 2] = -vx * np.sin(psi) - vy * np.cos(psi)
        F[..., 0, 3] = np.cos(psi)
        F[..., 0, 4] = -np.sin(psi)
        F[..., 1, 2] = vx * np.cos(psi) - vy * np.sin(psi)
        F[..., 1, 3] = np.sin(psi)
        F[..., 1, 4] = np.cos(psi)
        F[..., 2, 5] = 1.0
        for k, c in enumerate((3, 4, 5)):
            F[..., 3, c] = -np.sin(d) * dfyf[k] / mass
            F[..., 4, c] = (np.cos(d) * dfyf[k] + dfyr[k]) / mass
            F[..., 5, c] = (df * np.cos(d) * dfyf[k] - dr * dfyr[k]) / iz
        F[..., 3, 4] += r
        F[..., 3, 5] += vy
        F[..., 4, 3] -= r
        F[..., 4, 5] -= vx
        F[..., 6, 7] = 1.0
    else:
        raise KeyError(f"oracle has no dynamics model {name!r}")
    return f, F


def meas_eval(name, x, par=None, static=None):
    x = np.asarray(x, dtype=np.float64)
    static = static or {}
    n = x.shape[-1]
    if name == "full_state":
        h = x.copy()
        H = np.broadcast_to(np.eye(n), x.shape + (n,)).copy()
        return h, H
    if name in ("pseudorange", "vehicle_pseudorange"):
        idx = list(static.get("idx", [0, 1, 2, 3])) if name == "pseudorange" else [0, 1, 8, 6]
        s = np.asarray(par, dtype=np.float64)[..., :3]
        d = np.stack([x[..., idx[0]] - s[..., 0], x[..., idx[1]] - s[..., 1],
                      x[..., idx[2]] - s[..., 2]], axis=-1)
        rho = np.sqrt(d[..., 0] ** 2 + d[..., 1] ** 2 + d[..., 2] ** 2)
        h = (rho + x[..., idx[3]])[..., None]
        H = np.zeros(x.shape[:-1] + (1, n))
        # rho = 0 only at a placeholder satellite slot (position 0, weight 0: the rows
        # the solves mask, autonomous-car.py:260-263): its line-of-sight row is left 0
        # instead of 0/0 = NaN, so the checker never relies on masking a NaN away
        live = rho > 0.0
        inv = np.divide(1.0, rho, out=np.zeros_like(rho), where=live)
        for a in range(3):
            H[..., 0, idx[a]] += d[..., a] * inv
        H[..., 0, idx[3]] += 1.0
        return h, H
    if name == "multi_receiver_range_3d":
        if "idxA" in static:
            ia, ib = static["idxA"], static["idxB"]
            d = np.stack([x[..., ia[k]] - x[..., ib[k]] for k in range(3)], axis=-1)
            r = np.sqrt(d[..., 0] ** 2 + d[..., 1] ** 2 + d[..., 2] ** 2 + 1e-6)
            H = np.zeros(x.shape[:-1] + (1, n))
            for k in range(3):
                H[..., 0, ia[k]] += d[..., k] / r
                H[..., 0, ib[k]] -= d[..., k] / r
            return r[..., None], H
        idx = list(static.get("idx", [0, 1, 2]))
        y = np.asarray(par, dtype=np.float64)[..., :3]
        d = np.stack([x[..., idx[k]] - y[..., k] for k in range(3)], axis=-1)
        r = np.sqrt(d[..., 0] ** 2 + d[..., 1] ** 2 + d[..., 2] ** 2 + 1e-6)
        H = np.zeros(x.shape[:-1] + (1, n))
        for k in range(3):
            H[..., 0, idx[k]] += d[..., k] / r
        return r[..., None], H
    raise KeyError(f"oracle has no measurement model {name!r}")
