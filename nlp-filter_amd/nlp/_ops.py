"""Tiny numeric stand-ins for the CasADi operators the reference plug-ins use
(``from casadi import vertcat, sin, cos, ...``, nlp/dynamics.py:2,
nlp/measurements.py:2), so the plug-in modules evaluate on host NumPy arrays.
On the GPU path a plug-in is never evaluated in Python: it is mapped by name
to a hand-written device functor (mhe.registry)."""
import numpy as np

sin, cos, tan, sqrt = np.sin, np.cos, np.tan, np.sqrt
atan2 = np.arctan2


def vertcat(*args):
    return np.concatenate([np.atleast_1d(np.asarray(a, dtype=float)).ravel() for a in args])


def dot(a, b):
    return float(np.sum(np.asarray(a) * np.asarray(b)))


def norm_2(a):
    return float(np.sqrt(np.sum(np.asarray(a) ** 2)))


def mtimes(a, b):
    a, b = np.asarray(a), np.asarray(b)
    if a.ndim == 0 or b.ndim == 0:
        return a * b
    return a @ b
