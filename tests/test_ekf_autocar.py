"""The autonomous-car EKF (autonomous-car.py:18-178) on the device.

The script defines its own EKF plug-ins, ``discrete_vehicle_dynamics`` (Euler step of
the 9-state car, Jacobian formed at the updated state) and ``vehicle_sensors_model``
(pseudoranges of x[0, 1, 8, 6, 7]).  They run as device functors
(csrc/mhe_ekf.hip EkfDiscreteVehicle / EkfVehicleSensors); the user's callables are
accepted by name only after matching the registered twins (utils/vehicle.py) at
seeded points.

Pin: tests/golden/ekf_autocar.npz -- the reference EKF with the script's own plug-in
definitions, run by tests/golden/gen_golden.py on seeded data of the script's shape
(300 steps of 10 ms, corrections every 10th step with 8-11 satellites).  The script's
stored result (data/autonomous-car/filtering/ekf.pkl) is a Python-2 pickle that the
permitted loader refuses, so it is not read.
GPU tolerance as tests/test_ekf.py: |dmu| <= 1e-9 (1 + |mu|), |dS| <= 1e-9 max|S| per step.
"""
import numpy as np
import pytest

from mhe.registry import UnsupportedPlugin
from oracle import ekf as oekf
import utils.ekf as ekf
import utils.vehicle as veh

MU_TOL, S_TOL = 1e-9, 1e-9
CAR_KEYS = ("C_AF", "C_AR", "M", "D_F", "D_R", "I_Z")


@pytest.fixture(scope="module")
def fx():
    import os
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "ekf_autocar.npz"))
    d = {k: g[k] for k in g.files}
    d["dparams"] = {"dt": float(d["dt"]), "car_params": dict(zip(CAR_KEYS, d["car"]))}
    return d


# the user's own script functions (autonomous-car.py defines them; here they delegate
# to the oracle restatement -- a different callable of the same name and math)
def discrete_vehicle_dynamics(x, u, params=None, jac=False):
    return oekf.discrete_vehicle_dynamics(x, u, params, jac)


def vehicle_sensors_model(x, params=None, jac=False):
    return oekf.vehicle_sensors_model(x, params, jac)


def _close(mu, S, mu_ref, S_ref):
    dmu = np.abs(mu - mu_ref).max(axis=-1) / (1.0 + np.abs(mu_ref).max(axis=-1))
    dS = np.abs(S - S_ref).reshape(S.shape[:-2] + (-1,)).max(-1) / np.abs(S_ref).reshape(S.shape[:-2] + (-1,)).max(-1)
    return float(dmu.max()), float(dS.max())


def _oracle_run(fx, mu0, S0, Z, nz, sat):
    f = oekf.EKF(oekf.discrete_vehicle_dynamics, oekf.vehicle_sensors_model, mu0, S0)
    mus, Ss = [], []
    for k in range(fx["U"].shape[0]):
        ns = int(nz[k])
        f.update(fx["U"][k], Z[k, :ns] if ns else None, fx["Q"],
                 np.diag(float(fx["r_pr"]) * np.ones(ns)) if ns else None, fx["dparams"], None,
                 {"sat_pos": sat[k, :ns]})
        mus.append(f.mu.copy())
        Ss.append(f.S.copy())
    return np.stack(mus), np.stack(Ss)


def test_oracle_plugins_match_reference(fx):
    for x, u, f, F, s, y, H in zip(fx["plug_x"], fx["plug_u"], fx["plug_f"], fx["plug_F"], fx["plug_sat"],
                                   fx["plug_y"], fx["plug_H"]):
        f0, J = oekf.discrete_vehicle_dynamics(x.copy(), u, fx["dparams"], jac=True)
        assert np.abs(f0 - f).max() <= 1e-14 * (1 + np.abs(f).max())
        assert np.abs(J - F).max() <= 1e-14 * (1 + np.abs(F).max())
        y0, H0 = oekf.vehicle_sensors_model(x.copy(), {"sat_pos": s}, jac=True)
        assert np.abs(y0 - y).max() <= 1e-14 * (1 + np.abs(y).max())
        assert np.abs(H0 - H).max() <= 1e-14
        # the package's twins (what user plug-ins are verified against) are the reference's math too
        f1, J1 = veh.discrete_vehicle_dynamics(x.copy(), u, fx["dparams"], jac=True)
        y1, H1 = veh.vehicle_sensors_model(x.copy(), {"sat_pos": s}, jac=True)
        assert np.abs(f1 - f).max() <= 1e-14 * (1 + np.abs(f).max()) and np.abs(J1 - F).max() <= 1e-14 * (1 + np.abs(F).max())
        assert np.abs(y1 - y).max() <= 1e-14 * (1 + np.abs(y).max()) and np.abs(H1 - H).max() <= 1e-14


def test_oracle_ekf_reproduces_reference(fx):
    mus, Ss = _oracle_run(fx, fx["mu0"], fx["S0"], fx["Z"], fx["nz"], fx["sat_pos"])
    emu, eS = _close(mus, Ss[::int(fx["S_every"])], fx["mu"], fx["S"])
    assert emu <= 1e-13 and eS <= 1e-13, (emu, eS)


def test_same_named_plugins_with_other_math_are_refused(fx):
    def discrete_vehicle_dynamics(x, u, params=None, jac=False):   # noqa: F811 -- Jacobian at the OLD state
        x0 = np.array(x, dtype=np.float64)
        xn = oekf.discrete_vehicle_dynamics(x0, u, params, False)
        _, J = oekf.discrete_vehicle_dynamics(x0 - (xn - x0), u, params, True)
        return xn, J

    def vehicle_sensors_model(x, params=None, jac=False):          # noqa: F811 -- z from x[2], not x[8]
        xs = np.array(x, dtype=np.float64)
        xs[8] = xs[2]
        return oekf.vehicle_sensors_model(xs, params, jac)

    with pytest.raises(UnsupportedPlugin):
        ekf.verify(discrete_vehicle_dynamics, veh.vehicle_sensors_model, fx["dparams"])
    with pytest.raises(UnsupportedPlugin):
        ekf.verify(veh.discrete_vehicle_dynamics, vehicle_sensors_model, fx["dparams"])
    with pytest.raises(UnsupportedPlugin):   # wrong pairing: not compiled
        ekf.models(veh.discrete_vehicle_dynamics, "multi_pseudorange")
    with pytest.raises(UnsupportedPlugin):   # car constants are required
        ekf.dyn_par(veh.discrete_vehicle_dynamics, {"dt": 0.01})
    ekf.verify(globals()["discrete_vehicle_dynamics"], globals()["vehicle_sensors_model"], fx["dparams"])


@pytest.mark.gpu
def test_autocar_ekf_class_matches_reference(fx):
    """The script's loop (autonomous-car.py:137-178) through the drop-in class, with the
    user's own plug-in callables, against the reference run step by step."""
    f = ekf.EKF(discrete_vehicle_dynamics, vehicle_sensors_model, fx["mu0"].copy(), fx["S0"].copy())
    mus, Ss = [], []
    for k in range(fx["U"].shape[0]):
        ns = int(fx["nz"][k])
        if ns:
            f.update(fx["U"][k], fx["Z"][k, :ns], fx["Q"], np.diag(float(fx["r_pr"]) * np.ones(ns)),
                     dyn_func_params=fx["dparams"], meas_func_params={"sat_pos": fx["sat_pos"][k, :ns]})
        else:
            f.update(fx["U"][k], None, fx["Q"], None, dyn_func_params=fx["dparams"],
                     meas_func_params={"sat_pos": None})
        mus.append(f.mu)
        Ss.append(f.S)
    emu, eS = _close(np.stack(mus), np.stack(Ss)[::int(fx["S_every"])], fx["mu"], fx["S"])
    print(f"autocar EKF class vs reference: mu {emu:.2e}, S {eS:.2e}")
    assert emu <= MU_TOL and eS <= S_TOL, (emu, eS)


@pytest.mark.gpu
@pytest.mark.parametrize("method", ["lane", "wave"])
def test_autocar_ekf_batch_matches_oracle(fx, method):
    """64 filters with perturbed priors and measurement noise in one launch, both device
    formulations, each instance against the oracle; instance 0 is the reference run."""
    B, T = 64, fx["U"].shape[0]
    rng = np.random.default_rng(7)
    mu0 = np.repeat(fx["mu0"][None], B, 0)
    mu0[1:, :2] += rng.normal(size=(B - 1, 2))
    mu0[1:, 6] += 5.0 * rng.normal(size=B - 1)
    S0 = np.repeat(fx["S0"][None], B, 0)
    Z = np.repeat(fx["Z"][None], B, 0)
    nzr = fx["nz"]
    for b in range(1, B):
        for k in range(T):
            Z[b, k, :nzr[k]] += 0.5 * rng.normal(size=nzr[k])
    nz = np.repeat(nzr[None], B, 0).astype(np.int32)
    sat = np.repeat(fx["sat_pos"][None], B, 0)
    pmax = Z.shape[2]
    R = np.repeat(np.diag(float(fx["r_pr"]) * np.ones(pmax))[None], T, 0)
    U = np.repeat(fx["U"][None], B, 0)
    mh, Sh, mu, S, st = ekf.run_batch(discrete_vehicle_dynamics, vehicle_sensors_model, mu0, S0, U, Z, nz,
                                      fx["Q"], R, fx["dparams"]["dt"], sat, method=method,
                                      dyn_params=fx["dparams"])
    assert int(st.abs().sum().item()) == 0
    mh, Sh = mh.cpu().numpy(), Sh.cpu().numpy()
    worst = (0.0, 0.0)
    for b in (0, 1, 17, 63):
        rmu, rS = _oracle_run(fx, mu0[b], S0[b], Z[b], nz[b], sat[b])
        emu, eS = _close(mh[b], Sh[b], rmu, rS)
        worst = (max(worst[0], emu), max(worst[1], eS))
    e0, s0 = _close(mh[0], Sh[0][::int(fx["S_every"])], fx["mu"], fx["S"])
    print(f"autocar EKF batch ({method}) vs oracle: mu {worst[0]:.2e}, S {worst[1]:.2e}; vs reference {e0:.2e}")
    assert worst[0] <= MU_TOL and worst[1] <= S_TOL, worst
    assert e0 <= MU_TOL and s0 <= S_TOL
