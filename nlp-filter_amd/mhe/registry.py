"""Plug-in registry: reference plug-in functions -> HIP model ids.

User code keeps passing plug-in *functions* with the reference signatures
(``f(x, u, params)``, ``h(x, params)``, nlp/nlp.py:212-219,258).  The GPU path
has a hand-written device functor (analytic Jacobian) for each registered
plug-in; lookup is by the function's name within a ``dynamics`` /
``measurements`` module, so both this package's ``nlp.dynamics`` and the
reference's own ``nlp/dynamics.py`` functions resolve.  An unregistered
plug-in raises ``UnsupportedPlugin`` -- there is no CPU evaluation path.

A name is not an identity: ``verify_dyn`` / ``verify_meas`` evaluate a user's
plug-in at seeded points and compare it with this package's host definition of
the registered plug-in (the twin of the device functor, pinned to the reference
by tests/golden/plugins.npz), so a function that merely shares the name --
different math, different constants -- is refused instead of silently getting
the built-in functor.
"""
import numpy as np

DYN = {
    # name: (id, n, m)                      reference nlp/dynamics.py
    "single_integrator": (1, 1, 1),         # :4-8
    "single_integrator_2D": (2, 2, 2),      # :10-17
    "single_integrator_3D": (3, 3, 3),      # :19-27
    "double_integrator": (4, 4, 2),         # :29-38
    "van_der_pol": (5, 2, 1),               # :61-66
    "gnss_pos_and_bias": (6, 5, 3),         # :68-79
    "multi_receiver": (7, 8, 0),            # :81-96
    "gnss_two_receiver": (8, 10, 6),        # :98-115
    "kinematic_bycicle_and_bias": (9, 6, 2),  # :117-136
    "vehicle_dynamics_and_gnss": (10, 9, 2),  # :148-174 (params["car_params"] -> dyn_par)
    "gnss_eight_receivers": (11, 40, 24),     # 8 x the :98-115 receiver block (C5, n = 40)
}

# Static parameters of the device functors (mhe_dims.dyn_par), from the plug-in's params
CAR_KEYS = ("C_AF", "C_AR", "M", "D_F", "D_R", "I_Z")   # utils/vehicle_sim.py:10-23


def dyn_params(name, params):
    """The mhe_dims.dyn_par vector of dynamics plug-in ``name`` for ``params``."""
    out = np.zeros(8)
    if name == "vehicle_dynamics_and_gnss":
        if not params or "car_params" not in params:
            raise UnsupportedPlugin("vehicle_dynamics_and_gnss needs params={'car_params': ...} (nlp/dynamics.py:151)")
        C = params["car_params"]
        out[:6] = [float(C[k]) for k in CAR_KEYS]
    return out

MEAS = {
    # name: (id, p, q, linear)              reference nlp/measurements.py
    "full_state": (1, None, 0, True),       # :4-5 (p = n)
    "pseudorange": (2, 1, 3, False),        # :56-70 (q: sat_pos)
    "vehicle_pseudorange": (3, 1, 3, False),  # :81-88
    "multi_receiver_range_3d": (4, 1, 3, False),  # :39-54 ("y" form)
    # several scalar plug-ins in one problem; rows encoded per include/mhe.h
    # (MHE_MEAS_MIXED, built by nlp.NLP from its addResidualCost calls)
    "mixed": (5, 1, 14, False),
}

# MHE_ROW_* codes of the mixed-row encoding (include/mhe.h), by reference plug-in name
ROW_CODES = {
    "pseudorange": 1, "vehicle_pseudorange": 1, "pseudorange_rate": 2,
    "multi_receiver_range_2d": 3, "multi_receiver_range_3d": 4, "multi_receiver_heading_2d": 5,
    "full_state": 6,
}
MIXED_Q = 14
MAX_EXTRA, MAX_EQ = 4, 48

# (dynamics, measurement) pairs compiled into libmhe.so (dispatch() in mhe_gn.hip)
COMPILED_PAIRS = {
    ("single_integrator", "full_state"),
    ("single_integrator_2D", "full_state"),
    ("van_der_pol", "full_state"),
    ("gnss_pos_and_bias", "pseudorange"),
    ("gnss_pos_and_bias", "full_state"),
    ("kinematic_bycicle_and_bias", "pseudorange"),
    ("double_integrator", "full_state"),
    ("vehicle_dynamics_and_gnss", "vehicle_pseudorange"),   # autonomous-car.py:190-213
    # mixed rows / extra variables / equality constraints (large-system path)
    ("van_der_pol", "mixed"),
    ("multi_receiver", "mixed"),
    ("gnss_two_receiver", "mixed"),
    ("gnss_pos_and_bias", "mixed"),
    ("kinematic_bycicle_and_bias", "mixed"),
    ("vehicle_dynamics_and_gnss", "mixed"),
    ("gnss_eight_receivers", "mixed"),
}


class UnsupportedPlugin(NotImplementedError):
    pass


def _name(fn):
    if isinstance(fn, str):
        return fn
    return getattr(fn, "__name__", None)


def dyn_model(fn):
    name = _name(fn)
    if name not in DYN:
        raise UnsupportedPlugin(
            f"dynamics plug-in {name!r} has no HIP functor; registered: {sorted(DYN)}")
    return name, DYN[name]


def meas_model(fn):
    name = _name(fn)
    if name not in MEAS:
        raise UnsupportedPlugin(
            f"measurement plug-in {name!r} has no HIP functor; registered: {sorted(MEAS)}")
    return name, MEAS[name]


def check_pair(dyn_name, meas_name):
    if (dyn_name, meas_name) not in COMPILED_PAIRS:
        raise UnsupportedPlugin(
            f"(dynamics={dyn_name!r}, measurement={meas_name!r}) is not compiled into libmhe.so; "
            f"available: {sorted(COMPILED_PAIRS)}")


# ---------------------------------------------------------------- identity checks
VERIFY_POINTS = 4
VERIFY_RTOL = 1e-12


def _twin(kind, name):
    import importlib
    mod = importlib.import_module("nlp.dynamics" if kind == "dyn" else "nlp.measurements")
    if not hasattr(mod, name):
        raise UnsupportedPlugin(f"{kind} plug-in {name!r} has no registered twin to verify against")
    return getattr(mod, name)


def _close(a, b):
    a, b = np.atleast_1d(np.asarray(a, dtype=np.float64)).ravel(), np.atleast_1d(np.asarray(b, dtype=np.float64)).ravel()
    return a.shape == b.shape and bool(np.all(np.abs(a - b) <= VERIFY_RTOL * (1.0 + np.abs(b))))


def _sample(rng, k, name):
    x = rng.normal(size=k) * 3.0
    if name == "vehicle_dynamics_and_gnss":
        x[3] = 5.0 + abs(x[3])   # forward speed away from the tyre model's pole at vx = -0.001
    return x


def verify_dyn(fn, params=None):
    """Refuse (UnsupportedPlugin) a dynamics callable whose values differ from the
    registered plug-in of the same name at seeded points (n, m from the registry).
    Strings and this package's own functions pass without evaluation."""
    name, (_, n, m) = dyn_model(fn)
    if isinstance(fn, str):
        return
    twin = _twin("dyn", name)
    if fn is twin:
        return
    rng = np.random.default_rng(20260)
    for _ in range(VERIFY_POINTS):
        x = _sample(rng, n, name)
        u = rng.normal(size=m)
        try:
            got = fn(x, u, params) if m > 0 else fn(x, params)
        except Exception as e:  # symbolic-only plug-ins cannot be compared numerically
            raise UnsupportedPlugin(f"dynamics plug-in {name!r} could not be evaluated to verify it matches the "
                                    f"device functor: {type(e).__name__}: {e}") from e
        ref = twin(x, u, params) if m > 0 else twin(x, params)
        if not _close(got, ref):
            raise UnsupportedPlugin(f"dynamics plug-in {name!r} is not the registered {name}: its values differ "
                                    "from the device functor's (same name, different math or constants)")


def verify_meas(fn, params, n):
    """As verify_dyn for a measurement callable h(x, params) on an n-state."""
    name, _ = meas_model(fn) if _name(fn) in MEAS else (_name(fn), None)
    if isinstance(fn, str):
        return
    twin = _twin("meas", name)
    if fn is twin:
        return
    rng = np.random.default_rng(20261)
    for _ in range(VERIFY_POINTS):
        x = rng.normal(size=n) * 30.0
        try:
            got = fn(x, params)
        except Exception as e:
            raise UnsupportedPlugin(f"measurement plug-in {name!r} could not be evaluated to verify it matches the "
                                    f"device functor: {type(e).__name__}: {e}") from e
        if not _close(got, twin(x, params)):
            raise UnsupportedPlugin(f"measurement plug-in {name!r} is not the registered {name}: its values differ "
                                    "from the device functor's (same name, different math or constants)")
