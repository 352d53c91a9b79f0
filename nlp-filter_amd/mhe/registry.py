"""Plug-in registry: reference plug-in functions -> HIP model ids.

User code keeps passing plug-in *functions* with the reference signatures
(``f(x, u, params)``, ``h(x, params)``, nlp/nlp.py:212-219,258).  The GPU path
has a hand-written device functor (analytic Jacobian) for each registered
plug-in; lookup is by the function's name within a ``dynamics`` /
``measurements`` module, so both this package's ``nlp.dynamics`` and the
reference's own ``nlp/dynamics.py`` functions resolve.  An unregistered
plug-in raises ``UnsupportedPlugin`` -- there is no CPU evaluation path.
"""

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
}

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
    # mixed rows / extra variables / equality constraints (large-system path)
    ("van_der_pol", "mixed"),
    ("multi_receiver", "mixed"),
    ("gnss_two_receiver", "mixed"),
    ("gnss_pos_and_bias", "mixed"),
    ("kinematic_bycicle_and_bias", "mixed"),
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
