"""autonomous-car.py's moving-horizon NLP (vehicle_dynamics_and_gnss + vehicle_pseudorange,
state bounds, prior, 11 satellite slots with R = 0 masks, warm start; L2 and
pseudo-Huber dynamics cost) through this package's facade on the GPU, window by window
against the same script on the oracle (tests/autocar.py).

The reference's stored IPOPT results for this script (nlp-l2.pkl / nlp-huber.pkl) and
its inputs are Python-2 pickles that the permitted safe loader refuses (DESIGN.md
§8), so the inputs are seeded synthetic data of the same shape and the oracle is the
checker.  Tolerance (tests/tolerance.py): 8 floor + 1e-8 (1 + max|X|), floor = the
oracle loop's own change when every pseudorange moves by eps |y| (both sides stop at
max|s| <= 1e-10 (1 + max|X|), so converged iterates agree to ~tol, not to rounding).
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

import autocar  # noqa: E402
import tolerance as tl  # noqa: E402

WINDOWS = 8


@pytest.mark.parametrize("huber", [False, True])
def test_autonomous_car_mhe_matches_oracle(huber):
    traj, gnss = autocar.synth(vary=not huber)
    XG, st, problem = autocar.facade_mhe(traj, gnss, WINDOWS, huber=huber)
    XR, rst = autocar.oracle_mhe(traj, gnss, WINDOWS, huber=huber)
    rng = np.random.default_rng(99)
    scale = [1.0 + tl.EPS * rng.choice([-1.0, 1.0], size=p.shape) for p in gnss["pr"]]
    XP, _ = autocar.oracle_mhe(traj, gnss, WINDOWS, huber=huber, pr_scale=scale)
    fl = float(np.abs(XP - XR).max())
    assert (rst == 0).all(), rst
    assert st == ["Solve_Succeeded"] * WINDOWS, st
    assert problem.engine_builds == 1, "R re-set every window must not rebuild the device constants"
    b = tl.bound(fl, XR, rel=1e-8)
    tl.check(f"autonomous-car {'huber' if huber else 'l2'} x_opt per window", np.abs(XG - XR).max(), b)
    assert b < 1e-4
    # the estimate tracks the synthetic truth (pseudorange noise 3.2 m)
    k_end = [int(round((w * autocar.DT + autocar.T) / traj["dt"])) for w in range(WINDOWS)]
    pos_err = np.abs(XG[:, -1, :2] - traj["x"][:2, k_end].T).max()
    print(f"max position error at window ends: {pos_err:.2f} m")
    assert pos_err < 10.0


def test_plugin_with_the_same_name_but_other_constants_is_refused():
    """identity by name alone would hand this function the
    built-in functor; the registry compares values and refuses it."""
    import nlp.cost_functions as cost_functions
    import nlp.measurements as measurements
    import nlp.nlp as nlp
    from mhe.registry import UnsupportedPlugin
    from nlp._ops import vertcat

    def van_der_pol(x, u, params=None):   # mu = 2 instead of the reference's 1
        return vertcat(2.0 * (1 - x[1] ** 2) * x[0] - x[1] + u[0], x[0])

    problem = nlp.fixedTimeOptimalEstimationNLP(10, 5.0, 2, 1)
    X = problem.addVariables(11, 2, name="x")
    t = np.linspace(0, 5, 11)
    problem.addDynamics(van_der_pol, X, t, np.zeros((1, 11)))
    problem.addDynamicsCost(cost_functions.weighted_l2_norm, None, {"Q": np.eye(2)})
    problem.addResidualCost(measurements.full_state, X, t, np.zeros((2, 11)), np.eye(2))
    with pytest.raises(UnsupportedPlugin, match="not the registered van_der_pol"):
        problem.solve()
