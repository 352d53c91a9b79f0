"""Cost plug-ins -- kingdwd/nlp-filter nlp/cost_functions.py.

The estimator solves the least-squares form: ``weighted_l2_norm`` (weight
params["Q"]) and ``l2_norm`` (identity weight) are what the Gauss-Newton
solver supports; ``pseudo_huber_loss`` is defined for host evaluation but not
yet solvable on the GPU path."""
import numpy as np


def van_der_pol(x, u, params=None):
    """(nlp/cost_functions.py:5-7) -- optimal-control stage cost"""
    return x[0] ** 2 + x[1] ** 2 + float(np.sum(np.asarray(u) ** 2))


def single_integrator(x, u, params=None):
    """(nlp/cost_functions.py:10-12) -- optimal-control stage cost"""
    return x[0] ** 2 + x[1] ** 2 + u[0] ** 2 + u[1] ** 2


def l2_norm(x, params=None):
    """||x||^2 (nlp/cost_functions.py:15-17)"""
    x = np.asarray(x, dtype=float)
    return float(x @ x)


def weighted_l2_norm(x, params=None):
    """x^T Q x with Q = params["Q"] (nlp/cost_functions.py:20-22)"""
    x = np.asarray(x, dtype=float)
    return float(x @ np.asarray(params["Q"]) @ x)


def pseudo_huber_loss(x, params=None):
    """sum_i 2 Q_ii delta^2 (sqrt(1 + x_i^2/delta^2) - 1) (nlp/cost_functions.py:25-31)"""
    Q, delta = np.asarray(params["Q"]), params["delta"]
    return float(sum(2 * Q[i, i] * delta ** 2 * (np.sqrt(1 + x[i] ** 2 / delta ** 2) - 1.0) for i in range(Q.shape[0])))
