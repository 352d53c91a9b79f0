"""The autonomous-car EKF plug-ins -- kingdwd/nlp-filter autonomous-car.py:18-77 and
the car model of utils/vehicle_sim.py:10-85 they are built on.

The reference defines ``discrete_vehicle_dynamics`` and ``vehicle_sensors_model``
inside its script; a user of this package keeps passing their own script functions to
``utils.ekf.EKF``.  These host NumPy definitions are the twins the device functors
(csrc/mhe_ekf.hip ``EkfDiscreteVehicle`` / ``EkfVehicleSensors``) are checked against:
``utils.ekf`` evaluates the user's callable at seeded points and refuses it
(``UnsupportedPlugin``) when its values differ from these.  They are never on the
filter path itself.
"""
import numpy as np

from . import gnss

CAR_KEYS = ("C_AF", "C_AR", "M", "D_F", "D_R", "I_Z")


def get_parameters():
    """utils/vehicle_sim.py:10-27 -- the car constants of the simulated vehicle."""
    return {"C_AF": 1.1441e5, "C_AR": 1.3388e5, "MU": 0.75, "M": 2009, "D_F": 1.53, "D_R": 1.23, "I_Z": 2000,
            "H": 0.25, "G": 9.81}


def _xdot(x, u, C):
    """utils/vehicle_sim.py:72-85 with linear_tire_model (:58-66): x = [px, py, psi, vx, vy, r]."""
    a_r = (x[4] - C["D_R"] * x[5]) / x[3]
    a_f = (x[4] + C["D_F"] * x[5]) / x[3] - u[1]
    F_yr, F_yf = -C["C_AR"] * a_r, -C["C_AF"] * a_f
    return np.array([x[3] * np.cos(x[2]) - x[4] * np.sin(x[2]),
                     x[3] * np.sin(x[2]) + x[4] * np.cos(x[2]),
                     x[5],
                     (-F_yf * np.sin(u[1]) + u[0]) / C["M"] + x[5] * x[4],
                     (F_yf * np.cos(u[1]) + F_yr) / C["M"] - x[5] * x[3],
                     (C["D_F"] * F_yf * np.cos(u[1]) - C["D_R"] * F_yr) / C["I_Z"]])


def discrete_vehicle_dynamics(x, u, params=None, jac=False):
    """autonomous-car.py:18-52: explicit Euler step of the 9-state car
    x = [px, py, psi, vx, vy, r, b, bd, pz], u = [F_xr, delta].  As the reference, x is
    updated in place and the Jacobian is formed at the UPDATED state."""
    dt, C = params["dt"], params["car_params"]
    xd = np.hstack((_xdot(x[:6], u, C), np.array([x[7], 0.0, 0.0])))
    x += dt * xd
    if not jac:
        return x
    J = np.eye(9)
    fyf_vx = C["C_AF"] * (x[4] + C["D_F"] * x[5]) * (1.0 / x[3] ** 2)
    fyf_vy, fyf_r = -C["C_AF"] / x[3], -C["C_AF"] * C["D_F"] / x[3]
    fyr_vx = C["C_AR"] * (x[4] - C["D_R"] * x[5]) * (1.0 / x[3] ** 2)
    fyr_vy, fyr_r = -C["C_AR"] / x[3], C["C_AR"] * C["D_R"] / x[3]
    s, c, su, cu = np.sin(x[2]), np.cos(x[2]), np.sin(u[1]), np.cos(u[1])
    J[0, 2:5] += dt * np.array([-x[3] * s - x[4] * c, c, -s])
    J[1, 2:5] += dt * np.array([x[3] * c - x[4] * s, s, c])
    J[2, 5] += dt
    J[3, 3] += -(dt / C["M"]) * (su * fyf_vx)
    J[3, 4] += dt * (x[5] - su * fyf_vy / C["M"])
    J[3, 5] += dt * (x[4] - su * fyf_r / C["M"])
    J[4, 3] += dt * ((cu * fyf_vx + fyr_vx) / C["M"] - x[5])
    J[4, 4] += (dt / C["M"]) * (cu * fyf_vy + fyr_vy)
    J[4, 5] += dt * ((cu * fyf_r + fyr_r) / C["M"] - x[3])
    J[5, 3:6] += (dt / C["I_Z"]) * np.array([C["D_F"] * cu * fyf_vx - C["D_R"] * fyr_vx,
                                              C["D_F"] * cu * fyf_vy - C["D_R"] * fyr_vy,
                                              C["D_F"] * cu * fyf_r - C["D_R"] * fyr_r])
    J[6, 7] += dt
    return x, J


def vehicle_sensors_model(x, params=None, jac=False):
    """autonomous-car.py:54-77: pseudoranges of x_meas = [px, py, pz, b, bd] (= x[0, 1, 8,
    6, 7]), the Jacobian's columns scattered back to the 9-state."""
    xm = np.array([x[0], x[1], x[8], x[6], x[7]])
    if not jac:
        return gnss.multi_pseudorange(xm, params=params, jac=False)
    y, Jm = gnss.multi_pseudorange(xm, params=params, jac=True)
    J = np.zeros((y.shape[0], 9))
    J[:, [0, 1, 8, 6, 7]] = Jm
    return y, J
