"""EKF plug-ins with the reference signatures ``f(x, u, params=None, jac=False)``
and ``h(x, params=None, jac=False)`` -- kingdwd/nlp-filter utils/gnss.py.

These are the user-facing plug-in definitions (host NumPy, same results as the
reference).  ``utils.ekf.EKF`` never calls them: it maps each plug-in by name to
its device functor in csrc/mhe_ekf.hip (``EKF_DYN`` / ``EKF_MEAS``) and runs the
filter on the GPU.
"""
import numpy as np


def pseudorange(x, params=None, jac=False):
    """x = [x, y, z, b, bd]; |x[:3] - sat_pos| + b  (utils/gnss.py:4-24)"""
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
    """One pseudorange per row of params["sat_pos"]  (utils/gnss.py:27-45)"""
    S = params["sat_pos"]
    y = np.zeros(S.shape[0])
    J = np.zeros((S.shape[0], 5))
    for i in range(S.shape[0]):
        y[i], J[i] = pseudorange(x, {"sat_pos": S[i]}, jac=True)
    return (y, J) if jac else y


def multi_pseudorange_and_bias(x, params=None, jac=False):
    """Pseudoranges plus a bias row (utils/gnss.py:48-61).  As in the reference the
    bias row of the Jacobian is left zero."""
    S = params["sat_pos"]
    y = np.zeros(S.shape[0] + 1)
    J = np.zeros((S.shape[0] + 1, 5))
    y[-1] = x[3]
    y[:-1], J[:-1] = multi_pseudorange(x, {"sat_pos": S}, jac=True)
    return (y, J) if jac else y


def gnss_pos_and_bias(x, u, params=None, jac=False):
    """x+ = x + dt [u0, u1, u2, bd, 0]  (utils/gnss.py:79-90; updates x in place)"""
    x += params["dt"] * np.array([u[0], u[1], u[2], x[4], 0.0])
    if jac:
        J = np.eye(5)
        J[3, 4] = params["dt"]
        return x, J
    return x


# name -> (model id, n, m) / (model id, extra rows, q); include/mhe.h MHE_EKF_*.
# discrete_vehicle_dynamics / vehicle_sensors_model are autonomous-car.py's own
# plug-ins (twins in utils/vehicle.py).
EKF_DYN = {"gnss_pos_and_bias": (1, 5, 3), "discrete_vehicle_dynamics": (2, 9, 2)}
EKF_MEAS = {"multi_pseudorange": (1, 0, 3), "multi_pseudorange_and_bias": (2, 1, 3),
            "vehicle_sensors_model": (3, 0, 3)}
# which measurement plug-ins each dynamics functor is compiled with (csrc/mhe_ekf.hip)
EKF_PAIRS = {("gnss_pos_and_bias", "multi_pseudorange"), ("gnss_pos_and_bias", "multi_pseudorange_and_bias"),
             ("discrete_vehicle_dynamics", "vehicle_sensors_model")}
