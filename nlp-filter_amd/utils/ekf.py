"""Extended Kalman filter on the GPU -- drop-in for kingdwd/nlp-filter utils/ekf.py.

``EKF(dyn_func, meas_func, mu0, S0)`` and ``EKF.update(u, z, Q, R,
dyn_func_params, meas_func, meas_func_params)`` keep the reference signatures
and semantics (utils/ekf.py:11-38): ``mu`` / ``S`` are NumPy arrays replaced by
each update; ``z=None`` predicts only.  Each update is one launch of
``mhe_ekf_run`` (csrc/mhe_ekf.hip); ``run_batch`` runs many independent filter
instances over many steps in a single launch (the GPU-shaped entry point).
Plug-ins are resolved by name (``utils.gnss.EKF_DYN`` / ``EKF_MEAS``: the
utils/gnss.py models and autonomous-car.py's own ``discrete_vehicle_dynamics`` /
``vehicle_sensors_model``); a user's callable is then evaluated at seeded points
against the registered twin (``utils.gnss``, ``utils.vehicle``) and refused on any
difference.  An unregistered or mismatching plug-in raises ``UnsupportedPlugin`` --
there is no CPU path.

Numerics: the reference forms inv(P) (utils/ekf.py:55); the kernel uses a
Cholesky sweep of P, so results agree to floating-point rounding (tests state
the tolerance).
"""
import ctypes

import numpy as np

from mhe import _lib
from mhe.registry import UnsupportedPlugin

from . import gnss as _gnss
from . import vehicle as _vehicle

MAXP = 32


def _name(fn):
    return fn if isinstance(fn, str) else getattr(fn, "__name__", None)


def models(dyn_func, meas_func):
    dn, mn = _name(dyn_func), _name(meas_func)
    if dn not in _gnss.EKF_DYN:
        raise UnsupportedPlugin(f"EKF dynamics plug-in {dn!r} has no HIP functor; registered: {sorted(_gnss.EKF_DYN)}")
    if mn not in _gnss.EKF_MEAS:
        raise UnsupportedPlugin(f"EKF measurement plug-in {mn!r} has no HIP functor; registered: {sorted(_gnss.EKF_MEAS)}")
    if (dn, mn) not in _gnss.EKF_PAIRS:
        raise UnsupportedPlugin(f"EKF pair ({dn!r}, {mn!r}) is not compiled into libmhe.so; "
                                f"available: {sorted(_gnss.EKF_PAIRS)}")
    return _gnss.EKF_DYN[dn], _gnss.EKF_MEAS[mn]


def dyn_par(dyn_func, params):
    """mhe_ekf_dims.dyn_par for a dynamics plug-in and its dyn_func_params."""
    out = np.zeros(8)
    if _name(dyn_func) == "discrete_vehicle_dynamics":
        C = (params or {}).get("car_params")
        if C is None:
            raise UnsupportedPlugin("discrete_vehicle_dynamics needs dyn_func_params['car_params'] "
                                    "(autonomous-car.py:160)")
        out[:6] = [float(C[k]) for k in _vehicle.CAR_KEYS]
    return out


# ---------------------------------------------------------------- identity checks
_VERIFIED = {}


def _twin(name):
    for mod in (_gnss, _vehicle):
        if hasattr(mod, name):
            return getattr(mod, name)
    raise UnsupportedPlugin(f"EKF plug-in {name!r} has no registered twin to verify against")


def _close(a, b, rtol=1e-12):
    a, b = np.asarray(a, dtype=np.float64), np.asarray(b, dtype=np.float64)
    return a.shape == b.shape and bool(np.all(np.abs(a - b) <= rtol * (1.0 + np.abs(b))))


def _params_key(p):
    if not p:
        return ()
    return tuple(sorted((k, _params_key(v) if isinstance(v, dict) else float(v)) for k, v in p.items()
                        if isinstance(v, (dict, int, float, np.floating, np.integer))))


def verify(dyn_func, meas_func, dyn_params):
    """Refuse (UnsupportedPlugin) user callables whose values or Jacobians differ from
    the registered twins at 4 seeded points: a same-named plug-in with other math or
    other constants must not silently get the built-in device functor.  Strings and this
    package's own functions pass without evaluation; results are cached per callable
    and parameter values."""
    (_, n, m), (_, _, q) = models(dyn_func, meas_func)
    for fn, kind in ((dyn_func, "dyn"), (meas_func, "meas")):
        if isinstance(fn, str):
            continue
        twin = _twin(_name(fn))
        if fn is twin:
            continue
        key = (id(fn), kind, _params_key(dyn_params) if kind == "dyn" else ())
        if _VERIFIED.get(key) is fn:
            continue
        rng = np.random.default_rng(20262)
        for _ in range(4):
            x = rng.normal(size=n) * 3.0
            if n == 9:
                x[3] = 5.0 + abs(x[3])   # forward speed away from the tyre model's pole at vx = 0
            try:
                if kind == "dyn":
                    u = rng.normal(size=m)
                    got = fn(x.copy(), u, params=dyn_params, jac=True)
                    ref = twin(x.copy(), u, params=dyn_params, jac=True)
                else:
                    p = {"sat_pos": rng.normal(size=(4, 3)) * 2.0e4}
                    got = fn(x.copy(), params=p, jac=True)
                    ref = twin(x.copy(), params=p, jac=True)
            except UnsupportedPlugin:
                raise
            except Exception as e:
                raise UnsupportedPlugin(f"EKF plug-in {_name(fn)!r} could not be evaluated to verify it matches "
                                        f"the device functor: {type(e).__name__}: {e}") from e
            if not (_close(got[0], ref[0]) and _close(got[1], ref[1])):
                raise UnsupportedPlugin(f"EKF plug-in {_name(fn)!r} is not the registered {_name(fn)}: its values "
                                        "or Jacobian differ from the device functor's (same name, different math "
                                        "or constants)")
        _VERIFIED[key] = fn


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def run_batch(dyn_func, meas_func, mu0, S0, U, Z, nz, Q, R, dt, sat_pos, device=None, stream=None,
              keep_history=True, method="auto", inputs="batch_outer", dyn_params=None):
    """Run B independent filters for T steps in one launch.

    mu0 (B,n), S0 (B,n,n), U (B,T,m), Z (B,T,pmax), nz (B,T) valid rows per step
    (0 = predict only), Q (n,n), R (T,pmax,pmax) or (B,T,pmax,pmax), sat_pos
    (B,T,pmax,3); dt = dyn_func_params["dt"]; dyn_params = the whole dyn_func_params
    (needed for discrete_vehicle_dynamics: "car_params"; its "dt", when given, wins
    over dt).  Inputs may be NumPy or torch.
    Returns (mu_hist (B,T,n), S_hist (B,T,n,n), mu (B,n), S (B,n,n), status (B))
    as torch tensors on the device.

    method: "lane" (diagonal R: sequential scalar updates, one filter per lane),
    "wave" (any R: one wavefront per filter, augmented Cholesky sweep) or "auto"
    (lane when every R block is diagonal -- one device-side check).

    inputs="batch_inner": U, Z, nz, sat_pos are given batch-innermost instead,
    (T,m,B), (T,pmax,B), (T,B), (T,pmax,3,B) -- the device reads then coalesce.

    stream: a torch stream to order the work on (default: the current one); outputs
    belong to it (mhe.streams)."""
    import torch

    from mhe.streams import launch_stream

    (did, n, m), (mid, _, q) = models(dyn_func, meas_func)
    if dyn_params is not None and "dt" in dyn_params:
        dt = dyn_params["dt"]
    verify(dyn_func, meas_func, dict(dyn_params or {}, dt=dt))
    dp = dyn_par(dyn_func, dyn_params)
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    with launch_stream(stream, dev) as (s, cur):
        return _run_batch(did, n, m, mid, q, dev, s, cur, mu0, S0, U, Z, nz, Q, R, dt, sat_pos, keep_history,
                          method, inputs, dp)


def _run_batch(did, n, m, mid, q, dev, s, cur, mu0, S0, U, Z, nz, Q, R, dt, sat_pos, keep_history, method,
               inputs, dp):
    """run_batch on torch stream s (staging and allocation ordered on s)."""
    import torch

    from mhe.streams import keep_alive

    def d(a, dt_=torch.float64):
        return torch.as_tensor(np.asarray(a) if not torch.is_tensor(a) else a, dtype=dt_, device=dev).contiguous()

    mu = d(mu0).clone()
    S = d(S0).clone()
    B = mu.shape[0]
    Zt = d(Z)
    bi = inputs == "batch_inner"
    if inputs not in ("batch_outer", "batch_inner"):
        raise ValueError(f"unknown inputs layout {inputs!r}")
    T, pmax = (Zt.shape[0], Zt.shape[1]) if bi else (Zt.shape[1], Zt.shape[2])
    if pmax > MAXP:
        raise ValueError(f"at most {MAXP} measurement rows per step")
    Ut = d(U)
    nzt = d(nz, torch.int32)
    Pt = d(sat_pos)
    Rt = d(R)
    Qt = d(Q)
    shapes = ((T, m, B), (T, B), (T, pmax, q, B), (T, pmax, B)) if bi else \
        ((B, T, m), (B, T), (B, T, pmax, q), (B, T, pmax))
    if mu.shape != (B, n) or S.shape != (B, n, n) or Ut.shape != shapes[0] or nzt.shape != shapes[1] \
            or Pt.shape != shapes[2] or Zt.shape != shapes[3] or Qt.shape != (n, n):
        raise ValueError("run_batch: inconsistent shapes")
    if Rt.dim() == 3:
        r_b, r_s = 0, pmax * pmax
        if Rt.shape != (T, pmax, pmax):
            raise ValueError("R must be (T,pmax,pmax) or (B,T,pmax,pmax)")
    else:
        r_b, r_s = T * pmax * pmax, pmax * pmax
        if Rt.shape != (B, T, pmax, pmax):
            raise ValueError("R must be (T,pmax,pmax) or (B,T,pmax,pmax)")
    # histories are written batch-innermost (coalesced device stores) and returned as
    # (B, T, ...) views of that storage
    mh_st = torch.empty((T, n, B), dtype=torch.float64, device=dev) if keep_history else None
    Sh_st = torch.empty((T, n, n, B), dtype=torch.float64, device=dev) if keep_history else None
    st = torch.empty(B, dtype=torch.int32, device=dev)
    if method == "auto":
        offd = Rt - torch.diag_embed(torch.diagonal(Rt, dim1=-2, dim2=-1))
        r_diag = Rt.numel() == 0 or not bool((offd != 0).any().item())
    elif method in ("lane", "wave"):
        r_diag = method == "lane"
    else:
        raise ValueError(f"unknown method {method!r}")
    dims = _lib.MheEkfDims(n=n, m=m, pmax=pmax, q=q, dyn_model=did, meas_model=mid, dt=float(dt),
                           r_diag=int(r_diag), hist_batch_inner=1, in_batch_inner=int(bi))
    for i in range(8):
        dims.dyn_par[i] = float(dp[i])
    lib = _lib.load()
    rc = lib.mhe_ekf_run(ctypes.byref(dims), B, T, _ptr(mu), _ptr(S), _ptr(Ut), T * m, _ptr(Zt), T * pmax,
                         _ptr(nzt), T, _ptr(Pt), T * pmax * q, _ptr(Qt), _ptr(Rt), r_b, r_s, _ptr(mh_st),
                         _ptr(Sh_st), _ptr(st), ctypes.c_void_p(s.cuda_stream))
    _lib.check(rc, "mhe_ekf_run")
    keep_alive(s, cur, mu, S, Ut, Zt, nzt, Pt, Qt, Rt, mh_st, Sh_st, st)
    mh = mh_st.permute(2, 0, 1) if keep_history else None
    Sh = Sh_st.permute(3, 0, 1, 2) if keep_history else None
    return mh, Sh, mu, S, st


class EKF(object):
    """utils/ekf.py:4-18 -- notation of Probabilistic Robotics (Thrun et al.)."""

    def __init__(self, dyn_func, meas_func, mu0, S0):
        self.mu = mu0
        self.S = S0
        self.dynamics = dyn_func
        self.measurement = meas_func
        models(dyn_func, meas_func)  # fail at construction for unregistered plug-ins

    def update(self, u, z, Q, R, dyn_func_params=None, meas_func=None, meas_func_params=None):
        """One predict (+ correct when z is given) step, utils/ekf.py:20-38."""
        meas = meas_func if meas_func is not None else self.measurement
        (_, n, m), (_, extra, q) = models(self.dynamics, meas)
        dt = float((dyn_func_params or {})["dt"])
        mu0 = np.asarray(self.mu, dtype=np.float64).reshape(1, n)
        S0 = np.asarray(self.S, dtype=np.float64).reshape(1, n, n)
        u_ = np.asarray(u, dtype=np.float64).reshape(1, 1, m)
        if z is None:
            pmax, nz = 1, 0
            Z = np.zeros((1, 1, 1))
            P = np.zeros((1, 1, 1, q))
            Rm = np.zeros((1, 1, 1))
        else:
            zz = np.atleast_1d(np.asarray(z, dtype=np.float64))
            nz = pmax = zz.shape[0]
            Z = zz.reshape(1, 1, pmax)
            sp = np.asarray(meas_func_params["sat_pos"], dtype=np.float64).reshape(-1, q)
            if sp.shape[0] + extra != nz:
                raise ValueError("z and meas_func_params['sat_pos'] disagree in size")
            P = np.zeros((1, 1, pmax, q))
            P[0, 0, :sp.shape[0]] = sp
            Rm = np.asarray(R, dtype=np.float64).reshape(1, pmax, pmax)
        _, _, mu, S, st = run_batch(self.dynamics, meas, mu0, S0, u_, Z, np.full((1, 1), nz, np.int32),
                                    np.asarray(Q, dtype=np.float64), Rm, dt, P, keep_history=False,
                                    dyn_params=dyn_func_params)
        if int(st[0].item()) != 0:
            raise np.linalg.LinAlgError("innovation covariance is not positive definite")
        self.mu = mu[0].cpu().numpy()
        self.S = S[0].cpu().numpy()
