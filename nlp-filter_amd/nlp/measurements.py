"""Measurement plug-ins, reference signature ``h(x, params=None)`` --
kingdwd/nlp-filter nlp/measurements.py (host NumPy; device functors by name)."""
import numpy as np

from ._ops import atan2, dot, norm_2, sqrt


def full_state(x, params=None):
    """(nlp/measurements.py:4-5)"""
    return np.asarray(x, dtype=float)


def multi_receiver_range_2d(x, params=None):
    """(nlp/measurements.py:7-20)"""
    if "y" in params:
        idx = params.get("idx", [0, 1])
        return sqrt((x[idx[0]] - params["y"][0]) ** 2 + (x[idx[1]] - params["y"][1]) ** 2 + .000001)
    a, b = params["idxA"], params["idxB"]
    return sqrt((x[a[0]] - x[b[0]]) ** 2 + (x[a[1]] - x[b[1]]) ** 2 + .000001)


def multi_receiver_heading_2d(x, params=None):
    """(nlp/measurements.py:22-37)"""
    if "y" in params:
        idx = params.get("idx", [0, 1])
        r_y = params["y"][1] - x[idx[1]]
        r_x = params["y"][0] - x[idx[0]]
    else:
        a, b = params["idxA"], params["idxB"]
        r_y = x[b[1]] - x[a[1]]
        r_x = x[b[0]] - x[a[0]] + .00001
    return atan2(r_x, r_y)


def multi_receiver_range_3d(x, params=None):
    """(nlp/measurements.py:39-54)"""
    if "y" in params:
        idx = params.get("idx", [0, 1, 2])
        return sqrt(sum((x[idx[k]] - params["y"][k]) ** 2 for k in range(3)) + .000001)
    a, b = params["idxA"], params["idxB"]
    return sqrt(sum((x[a[k]] - x[b[k]]) ** 2 for k in range(3)) + .000001)


def pseudorange(x, params=None):
    """||x[idx0:3] - sat_pos|| + x[idx3]  (nlp/measurements.py:56-70)"""
    idx = params.get("idx", [0, 1, 2, 3])
    s = params["sat_pos"]
    return sqrt((x[idx[0]] - s[0]) ** 2 + (x[idx[1]] - s[1]) ** 2 + (x[idx[2]] - s[2]) ** 2) + x[idx[3]]


def pseudorange_rate(x, params=None):
    """(nlp/measurements.py:72-79)"""
    r = np.asarray(params["sat_pos"]) - np.asarray(x[:3])
    los = r / norm_2(r)
    return dot(np.asarray(params["sat_vel"]) - np.asarray(x[4:7]), los) + x[7]


def vehicle_pseudorange(x, params=None):
    """(nlp/measurements.py:81-88)"""
    s = params["sat_pos"]
    return sqrt((x[0] - s[0]) ** 2 + (x[1] - s[1]) ** 2 + (x[8] - s[2]) ** 2) + x[6]
