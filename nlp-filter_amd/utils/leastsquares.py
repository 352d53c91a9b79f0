"""GNSS least-squares fixes on the GPU -- drop-in for kingdwd/nlp-filter utils/leastsquares.py.

Same entry points and semantics as the reference:
  ``iterativeLeastSquares(sat_pos, pr, x=<shared>, b=0, maxiter=100)``  (:19-42)
      GN position + clock-bias fix; ``x`` is updated IN PLACE and the default
      argument is one shared array, so consecutive calls warm-start from the
      previous fix exactly as the reference's mutable default does;
  ``iterativeLeastSquaresVel(sat_pos, sat_vel, pr_rate, x)``            (:45-63)
  ``runLeastSquares(t, sat_pos, pr, sat_vel, pr_rate, p_ref_ECEF)``     (:97-141)
      the per-epoch loop, as ONE launch (one lane walks the epochs in order,
      carrying the warm start), same result dict;
  ``run_batch(...)``: many logs at once (one lane per log, or with
      ``warm=False`` one lane per epoch).
Every solve runs in ``mhe_ls_run`` (csrc/mhe_ls.hip); without libmhe.so the
calls raise ``MheLibraryError``.  ``buildGeometryMatrix`` is the reference's
host helper (:6-16), kept for API parity.

Numerics: the reference solves pinv(G) drho; the kernel solves the 4x4 normal
equations by Cholesky -- the same least-squares solution for a full-rank G,
equal to rounding (tests state the tolerance).  Epochs with fewer than four
independent satellites report iters = -1 (the reference's pinv would return a
minimum-norm step there); a singular velocity system leaves v and bd NaN and the
position fix's iteration count untouched.
"""
import ctypes

import numpy as np

from mhe import _lib

from . import utils as _gu

_DEFAULT_X = np.zeros(3)  # the reference's shared mutable default (utils/leastsquares.py:19)


def buildGeometryMatrix(sat_pos, x):
    """Rows -(sat - x)/||sat - x|| (utils/leastsquares.py:6-16)."""
    sat_pos = np.asarray(sat_pos, dtype=np.float64)
    los = sat_pos - np.asarray(x, dtype=np.float64)[None, :]
    return -los / np.linalg.norm(los, axis=1, keepdims=True)


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def run_batch(sat_pos, pr, nsat, x_init=None, sat_vel=None, pr_rate=None, warm=True, maxiter=100, tol=1e-7,
              device=None, stream=None):
    """Least-squares fixes for C logs of T epochs in one launch.

    sat_pos (C,T,S,3) ECEF, pr (C,T,S), nsat (C,T) valid slots per epoch,
    x_init (C,3) starting position (default zeros); sat_vel / pr_rate (C,T,S[,3])
    add the velocity solve.  NumPy or torch inputs.  Returns a dict of device
    tensors: x (C,T,3), b (C,T), iters (C,T), x_last (C,3) and, with velocities,
    v (C,T,3), bd (C,T).  stream: a torch stream to order the work on (default:
    the current one); outputs belong to it (mhe.streams)."""
    import torch

    from mhe.streams import keep_alive, launch_stream

    lib = _lib.load()
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    with launch_stream(stream, dev) as (s, cur):
        out, used = _run_batch(lib, dev, s, sat_pos, pr, nsat, x_init, sat_vel, pr_rate, warm, maxiter, tol)
        keep_alive(s, cur, *used)
    return out


def _run_batch(lib, dev, s, sat_pos, pr, nsat, x_init, sat_vel, pr_rate, warm, maxiter, tol):
    import torch

    def d(a, dt=torch.float64):
        return None if a is None else torch.as_tensor(a, dtype=dt, device=dev).contiguous()

    sp, prt, ns = d(sat_pos), d(pr), d(nsat, torch.int32)
    if sp.dim() != 4 or sp.shape[-1] != 3:
        raise ValueError("sat_pos must be (chains, epochs, slots, 3)")
    C, T, S = sp.shape[:3]
    if tuple(prt.shape) != (C, T, S) or tuple(ns.shape) != (C, T):
        raise ValueError("pr must be (chains, epochs, slots) and nsat (chains, epochs)")
    xi = d(np.zeros((C, 3)) if x_init is None else x_init)
    with_vel = sat_vel is not None
    sv, rr = d(sat_vel), d(pr_rate)
    out = {"x": torch.empty((C, T, 3), dtype=torch.float64, device=dev),
           "b": torch.empty((C, T), dtype=torch.float64, device=dev),
           "iters": torch.empty((C, T), dtype=torch.int32, device=dev),
           "x_last": xi.clone()}
    if with_vel:
        out["v"] = torch.empty((C, T, 3), dtype=torch.float64, device=dev)
        out["bd"] = torch.empty((C, T), dtype=torch.float64, device=dev)
    dims = _lib.MheLsDims(slots=S, max_iter=int(maxiter), warm=1 if warm else 0, with_vel=1 if with_vel else 0,
                          tol=float(tol))
    rc = lib.mhe_ls_run(ctypes.byref(dims), C, T, _ptr(sp), _ptr(prt), _ptr(ns), _ptr(sv), _ptr(rr), _ptr(xi),
                        _ptr(out["x"]), _ptr(out["b"]), _ptr(out.get("v")), _ptr(out.get("bd")),
                        _ptr(out["iters"]), _ptr(out["x_last"]) if warm else None, ctypes.c_void_p(s.cuda_stream))
    _lib.check(rc, "mhe_ls_run")
    return out, [sp, prt, ns, sv, rr, xi] + list(out.values())


def _pack(sat_pos_list, values_lists, S=None):
    T = len(sat_pos_list)
    cnt = np.array([np.asarray(s).reshape(-1, 3).shape[0] for s in sat_pos_list], dtype=np.int32)
    S = max(4, int(cnt.max()) if T else 4) if S is None else S
    sp = np.zeros((1, T, S, 3))
    vals = [np.zeros((1, T, S) + np.asarray(v[0]).shape[1:]) if v is not None else None for v in values_lists]
    for k in range(T):
        c = cnt[k]
        sp[0, k, :c] = np.asarray(sat_pos_list[k]).reshape(-1, 3)
        for v, arr in zip(values_lists, vals):
            if v is not None:
                arr[0, k, :c] = np.asarray(v[k])
    return sp, vals, cnt[None]


def iterativeLeastSquares(sat_pos, pr, x=_DEFAULT_X, b=0, maxiter=100):
    """One epoch (utils/leastsquares.py:19-42); updates ``x`` in place, returns (x, b)."""
    sp, (prv,), cnt = _pack([sat_pos], [[pr]])
    if b != 0:  # the kernel starts b at 0 (the only value the reference ever passes)
        raise NotImplementedError("iterativeLeastSquares: non-zero initial bias")
    r = run_batch(sp, prv, cnt, x_init=np.asarray(x, dtype=np.float64)[None], maxiter=maxiter)
    x[:] = r["x"][0, 0].cpu().numpy()
    return x, float(r["b"][0, 0].item())


def iterativeLeastSquaresVel(sat_pos, sat_vel, pr_rate, x):
    """Velocity and bias rate at position x (utils/leastsquares.py:45-63)."""
    sp, (sv, rr), cnt = _pack([sat_pos], [[sat_vel], [pr_rate]])
    prv = np.zeros(sp.shape[:3])
    r = run_batch(sp, prv, cnt, x_init=np.asarray(x, dtype=np.float64)[None], sat_vel=sv, pr_rate=rr, maxiter=0)
    return r["v"][0, 0].cpu().numpy(), float(r["bd"][0, 0].item())


def runLeastSquares(t, sat_pos, pr, sat_vel=None, pr_rate=None, p_ref_ECEF=None):
    """Per-epoch fixes (utils/leastsquares.py:97-141), one launch; same dict."""
    T = np.asarray(t).shape[0]
    with_vel = sat_vel is not None
    sp, vals, cnt = _pack(list(sat_pos), [list(pr), list(sat_vel) if with_vel else None,
                                          list(pr_rate) if with_vel else None])
    r = run_batch(sp, vals[0], cnt, x_init=_DEFAULT_X[None], sat_vel=vals[1], pr_rate=vals[2])
    _DEFAULT_X[:] = r["x_last"][0].cpu().numpy()  # the shared default moves on, as in the reference
    X = r["x"][0].cpu().numpy()
    sol = {"t": t, "p_ref_ECEF": p_ref_ECEF, "bias": r["b"][0].cpu().numpy().copy(), "bias_rate": np.zeros(T)}
    for k in ("x_ECEF", "y_ECEF", "z_ECEF", "xd_ECEF", "yd_ECEF", "zd_ECEF", "x_ENU", "y_ENU", "z_ENU",
              "xd_ENU", "yd_ENU", "zd_ENU", "lat", "lon", "h"):
        sol[k] = np.zeros(T)
    sol["x_ECEF"], sol["y_ECEF"], sol["z_ECEF"] = X[:, 0].copy(), X[:, 1].copy(), X[:, 2].copy()
    for k in range(T):
        lla = _gu.ecef2lla(X[k])
        sol["lat"][k], sol["lon"][k], sol["h"][k] = lla[0], lla[1], lla[2]
        if p_ref_ECEF is not None:
            e = _gu.ecef2enu(X[k], p_ref_ECEF)
            sol["x_ENU"][k], sol["y_ENU"][k], sol["z_ENU"][k] = e[0], e[1], e[2]
    if with_vel:
        V = r["v"][0].cpu().numpy()
        sol["xd_ECEF"], sol["yd_ECEF"], sol["zd_ECEF"] = V[:, 0].copy(), V[:, 1].copy(), V[:, 2].copy()
        sol["bias_rate"] = r["bd"][0].cpu().numpy().copy()
        if p_ref_ECEF is not None:
            for k in range(T):
                e = _gu.ecef2enu(V[k], p_ref_ECEF, rotation_only=True)
                sol["xd_ENU"][k], sol["yd_ENU"][k], sol["zd_ENU"][k] = e[0], e[1], e[2]
    sol["iters"] = r["iters"][0].cpu().numpy()
    return sol
