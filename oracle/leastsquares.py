"""CPU restatement of the reference GNSS least-squares initialiser -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline may import this
module; the product path (utils.leastsquares -> libmhe.so) never does.

Follows kingdwd/nlp-filter utils/leastsquares.py:
  :6-16    buildGeometryMatrix        rows -(sat - x)/||sat - x||
  :19-42   iterativeLeastSquares      up to maxiter GN steps, dx = pinv(G) drho,
                                      stop when ||dx|| < 1e-7; x is updated IN PLACE
                                      (the default argument is a shared array, so
                                      consecutive calls warm-start from the last fix;
                                      b is an immutable 0 and restarts every call)
  :45-63   iterativeLeastSquaresVel   one linear solve at the converged position
  :97-141  runLeastSquares            per-epoch loop (ECEF/LLA/ENU outputs)
Pinned by tests/golden/multi_receiver/LS_{A,B}.csv (the reference's stored
runLeastSquares results for the gnss-multi-receiver logs).
"""
import numpy as np

_DEFAULT_X = np.zeros(3)  # the reference's mutable default (utils/leastsquares.py:19)


def geometry(sat_pos, x):
    N = sat_pos.shape[0]
    G = np.zeros((N, 3))
    for k in range(N):
        los = sat_pos[k, :] - x
        G[k, :] = -los / np.linalg.norm(los)
    return G


def iterative_least_squares(sat_pos, pr, x=_DEFAULT_X, b=0, maxiter=100):
    """Returns (x, b, iterations); x is modified in place like the reference."""
    N = sat_pos.shape[0]
    it = 0
    for it in range(1, maxiter + 1):
        G = np.hstack((geometry(sat_pos, x), np.ones((N, 1))))
        drho = np.zeros(N)
        for k in range(N):
            drho[k] = pr[k] - np.linalg.norm(sat_pos[k, :] - x) - b
        dx = np.matmul(np.linalg.pinv(G), drho)
        x += dx[0:3]
        b += dx[3]
        if np.linalg.norm(dx) < 1e-7:
            break
    return x, b, it


def iterative_least_squares_vel(sat_pos, sat_vel, pr_rate, x):
    N = sat_pos.shape[0]
    G = np.hstack((geometry(sat_pos, x), np.ones((N, 1))))
    drho = np.zeros(N)
    for k in range(N):
        drho[k] = pr_rate[k] - np.dot(sat_vel[k, :], -G[k, :3])
    sol = np.matmul(np.linalg.pinv(G), drho)
    return sol[:3], sol[3]


def run_least_squares(sat_pos, pr, sat_vel=None, pr_rate=None, x=None):
    """Per-epoch fixes in ECEF (the arithmetic of runLeastSquares without the
    coordinate conversions).  ``x`` is the shared warm-start array (default: the
    module's own, i.e. the reference's process-wide state)."""
    x = _DEFAULT_X if x is None else x
    T = len(pr)
    out = {"x": np.zeros((T, 3)), "b": np.zeros(T), "iters": np.zeros(T, dtype=np.int32),
           "v": np.zeros((T, 3)), "bd": np.zeros(T)}
    for t in range(T):
        p, b, it = iterative_least_squares(sat_pos[t], pr[t], x)
        out["x"][t], out["b"][t], out["iters"][t] = p, b, it
        if sat_vel is not None:
            v, bd = iterative_least_squares_vel(sat_pos[t], sat_vel[t], pr_rate[t], p)
            out["v"][t], out["bd"][t] = v, bd
    return out
