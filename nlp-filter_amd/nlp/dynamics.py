"""Dynamics plug-ins, reference signatures ``f(x, u, params=None)`` (m > 0) and
``f(x, params=None)`` (m = 0) -- kingdwd/nlp-filter nlp/dynamics.py.

Host NumPy definitions; the GPU solver maps each registered name to a device
functor with an analytic Jacobian (csrc/mhe_models.h, mhe.registry)."""
import numpy as np

from ._ops import cos, sin, tan, vertcat


def single_integrator(x, u, params=None):
    """x = [x], u = [v_x]; xdot = u  (nlp/dynamics.py:4-8)"""
    return vertcat(u[0])


def single_integrator_2D(x, u, params=None):
    """(nlp/dynamics.py:10-17)"""
    return vertcat(u[0], u[1])


def single_integrator_3D(x, u, params=None):
    """(nlp/dynamics.py:19-27)"""
    return vertcat(u[0], u[1], u[2])


def double_integrator(x, u, params=None):
    """x = [x, y, xdot, ydot], u = [a_x, a_y]  (nlp/dynamics.py:29-38)"""
    return vertcat(x[2], x[3], u[0], u[1])


def van_der_pol(x, u, params=None):
    """x = [x0, x1]  (nlp/dynamics.py:61-66)"""
    return vertcat((1 - x[1] ** 2) * x[0] - x[1] + u[0], x[0])


def gnss_pos_and_bias(x, u, params=None):
    """x = [x, y, z, b, bd]; xdot = u, bdot = bd  (nlp/dynamics.py:68-79)"""
    return vertcat(u[0], u[1], u[2], x[4], 0.0)


def multi_receiver(x, params=None):
    """x = [xB, yB, zB, bB, xdB, ydB, zdB, alphaB], m = 0  (nlp/dynamics.py:81-96)"""
    return vertcat(x[4], x[5], x[6], x[7], 0.0, 0.0, 0.0, 0.0)


def gnss_two_receiver(x, u, params=None):
    """x = [xA, yA, zA, bA, alphaA, xB, yB, zB, bB, alphaB]  (nlp/dynamics.py:98-115)"""
    return vertcat(u[0], u[1], u[2], x[4], 0.0, u[3], u[4], u[5], x[9], 0.0)


def kinematic_bycicle_and_bias(x, u, params=None):
    """Kinematic bicycle + clock bias (nlp/dynamics.py:117-136).  As in the
    reference code, x[2] is the angle inside cos/sin."""
    L = 0.28
    v = 8.72649116358 * u[0] - 0.856053299155
    delta = np.deg2rad(28) * u[1]
    return vertcat(v * cos(x[2]), v * sin(x[2]), 0.0, x[4], 0.0, (v / L) * tan(delta))


def vehicle_dynamics(x, u, params=None):
    """Dynamic bicycle with linear tyres, x = [px, py, psi, vx, vy, r],
    u = [F_xr, delta]; C = params["car_params"]  (nlp/dynamics.py:148-164)."""
    C = params["car_params"]
    epsilon = .001
    F_yr = -C["C_AR"] * (x[4] - C["D_R"] * x[5]) / (x[3] + epsilon)
    F_yf = -C["C_AF"] * ((x[4] + C["D_F"] * x[5]) / (x[3] + epsilon) - u[1])
    return vertcat(x[3] * cos(x[2]) - x[4] * sin(x[2]),
                   x[3] * sin(x[2]) + x[4] * cos(x[2]),
                   x[5],
                   (-F_yf * sin(u[1]) + u[0]) / C["M"] + x[5] * x[4],
                   (F_yf * cos(u[1]) + F_yr) / C["M"] - x[5] * x[3],
                   (C["D_F"] * F_yf * cos(u[1]) - C["D_R"] * F_yr) / C["I_Z"])


def vehicle_dynamics_and_gnss(x, u, params=None):
    """x = [px, py, psi, vx, vy, psid, b, bd, pz]: vehicle_dynamics plus bdot = bd
    (nlp/dynamics.py:166-174; autonomous-car.py:192)."""
    return vertcat(vehicle_dynamics(x[:6], u, params), x[7], 0.0, 0.0)


def gnss_eight_receivers(x, u, params=None):
    """Eight receivers, each the per-receiver block of gnss_two_receiver
    (nlp/dynamics.py:98-115): x = [x, y, z, b, alpha] x 8 (n = 40), u = the receivers'
    velocities (m = 24).  The SURVEY.md §8(d) C5 joint state ("~4N dims, N = 8")."""
    return vertcat(*[vertcat(u[3 * r], u[3 * r + 1], u[3 * r + 2], x[5 * r + 4], 0.0) for r in range(8)])
