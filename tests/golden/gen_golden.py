"""Generate golden vectors from the reference implementation (build container only).

Run:  python tests/golden/gen_golden.py   (needs /root/reference; writes tests/golden/*.npz)

What it does
  * imports the reference's own ``nlp/collocation.py``, ``nlp/dynamics.py``,
    ``nlp/measurements.py``, ``nlp/cost_functions.py`` with a tiny numpy-backed
    stand-in for the ``casadi`` *operators* they use (vertcat, sin, cos, tan,
    sqrt, atan2, dot, norm_2, mtimes) -- CasADi itself is absent and the
    plug-ins are plain expressions over those operators;
  * ``collocation.py`` is Python-2 code: its ``range((N-a)/2 + 1)`` call gets a
    module-global ``range`` that floors float bounds (Py-2 integer division), so
    the reference's own ``__init__`` runs unmodified;
  * imports ``utils/ekf.py`` and ``utils/gnss.py`` (flat imports, as the survey
    documents) and runs the reference EKF on the gnss_stationary log;
  * runs the reference EKF with autonomous-car.py's own plug-ins (their two function
    definitions taken from the script's syntax tree; the script itself loads pickles
    and is not imported) on seeded data of the script's shape;
  * stores ONLY numbers (inputs and outputs) -- no reference source or bytecode
    is written into this repository.

The fixtures are consumed by ``tests/test_oracle_golden.py`` (oracle pinning)
and by the GPU parity tests (``tests/test_gpu_*.py``).
"""
import builtins
import importlib.util
import os
import sys
import types

import numpy as np

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


def _stub_casadi():
    m = types.ModuleType("casadi")

    def vertcat(*args):
        parts = [np.atleast_1d(np.asarray(a)).ravel() for a in args]
        return np.concatenate(parts)

    m.vertcat = vertcat
    m.sin, m.cos, m.tan, m.sqrt = np.sin, np.cos, np.tan, np.sqrt
    m.atan2 = np.arctan2
    m.dot = lambda a, b: np.sum(np.asarray(a) * np.asarray(b))
    m.norm_2 = lambda a: np.sqrt(np.sum(np.asarray(a) ** 2))

    def mtimes(a, b):
        a = np.asarray(a)
        b = np.asarray(b)
        if a.ndim == 0 or b.ndim == 0:
            return a * b
        return a @ b

    m.mtimes = mtimes
    m.__all__ = []  # collocation.py does `from casadi import *` and uses nothing
    return m


def _load(name, path, extra_globals=None):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    if extra_globals:
        mod.__dict__.update(extra_globals)
    spec.loader.exec_module(mod)
    return mod


def _py2_range(*args):
    return builtins.range(*[int(np.floor(a)) for a in args])


def load_reference():
    sys.modules.setdefault("casadi", _stub_casadi())
    if "matplotlib.pyplot" not in sys.modules:
        plt = types.ModuleType("matplotlib.pyplot")
        mpl = types.ModuleType("matplotlib")
        mpl.pyplot = plt
        sys.modules["matplotlib"] = mpl
        sys.modules["matplotlib.pyplot"] = plt
    ref = types.SimpleNamespace()
    ref.collocation = _load("ref_collocation", f"{REF}/nlp/collocation.py", {"range": _py2_range})
    ref.dynamics = _load("ref_dynamics", f"{REF}/nlp/dynamics.py")
    ref.measurements = _load("ref_measurements", f"{REF}/nlp/measurements.py")
    ref.cost_functions = _load("ref_cost_functions", f"{REF}/nlp/cost_functions.py")
    sys.path.insert(0, f"{REF}/utils")
    try:
        ref.ekf = _load("ref_ekf", f"{REF}/utils/ekf.py")
        ref.gnss = _load("ref_gnss", f"{REF}/utils/gnss.py")
        ref.gutils = _load("ref_gutils", f"{REF}/utils/utils.py")
        ref.data = _load("ref_data", f"{REF}/utils/data.py")
        sys.modules.setdefault("gnss", ref.gnss)     # leastsquares.py's flat imports
        sys.modules.setdefault("utils", ref.gutils)
        ref.ls = _load("ref_leastsquares", f"{REF}/utils/leastsquares.py")
        # utils/vehicle_sim.py: only get_parameters() is used (the car constants of
        # autonomous-car.py:102); its module-level imports are the flat utils ones
        ref.vehicle_sim = _load("ref_vehicle_sim", f"{REF}/utils/vehicle_sim.py")
    finally:
        sys.path.pop(0)
    return ref


def cstep_jac(fun, x, *rest, h=1e-30):
    """Complex-step Jacobian of a plug-in at x (works through the stub operators)."""
    x = np.asarray(x, dtype=np.float64)
    f0 = np.atleast_1d(np.real(fun(x.astype(np.complex128), *rest)))
    J = np.zeros((f0.shape[0], x.shape[0]))
    for a in range(x.shape[0]):
        xc = x.astype(np.complex128)
        xc[a] += 1j * h
        J[:, a] = np.imag(np.atleast_1d(fun(xc, *rest))) / h
    return f0, J


def cdiff_jac(fun, x, *rest, h=1e-6):
    x = np.asarray(x, dtype=np.float64)
    f0 = np.atleast_1d(fun(x, *rest)).astype(np.float64)
    J = np.zeros((f0.shape[0], x.shape[0]))
    for a in range(x.shape[0]):
        xp = x.copy(); xp[a] += h
        xm = x.copy(); xm[a] -= h
        J[:, a] = (np.atleast_1d(fun(xp, *rest)) - np.atleast_1d(fun(xm, *rest))) / (2 * h)
    return f0, J


def gen_collocation(ref):
    out = {}
    for N in (2, 3, 4, 5, 6, 7, 10, 15, 20, 50, 100, 200, 500):
        cpm = ref.collocation.ChebyshevPseudospectralMethod(N, 0, 10.0)
        out[f"tau_{N}"] = np.asarray(cpm.tau)
        D = np.ascontiguousarray(np.asarray(cpm.D, dtype=np.float64))
        if N <= 100:
            out[f"D_{N}"] = D
        else:  # large N: sha256 of the bytes + probe entries keep the fixture small
            import hashlib
            out[f"Dsha_{N}"] = np.frombuffer(hashlib.sha256(D.tobytes()).digest(), dtype=np.uint8)
            pr = np.random.default_rng(N).integers(0, N + 1, size=(256, 2))
            out[f"Dprobe_idx_{N}"] = pr
            out[f"Dprobe_val_{N}"] = D[pr[:, 0], pr[:, 1]]
            out[f"Ddiag_{N}"] = np.diag(D).copy()
        out[f"w_{N}"] = np.asarray(cpm.w)
        if N <= 20:
            ts = np.linspace(0.0, 10.0, 37)
            out[f"phi_t_{N}"] = ts
            out[f"phi_{N}"] = np.stack([cpm.evaluateLagrangePolynomials(t) for t in ts])
            X = [np.array([np.sin(k), np.cos(2 * k)]) for k in range(N + 1)]
            out[f"X_{N}"] = np.stack(X)
            out[f"xeval_{N}"] = np.stack([cpm.evaluateSolution(t, X) for t in ts])
    np.savez_compressed(os.path.join(OUT, "collocation.npz"), **out)


DYN_CASES = {
    # name: (n, m, params)
    "single_integrator": (1, 1, None),
    "single_integrator_2D": (2, 2, None),
    "single_integrator_3D": (3, 3, None),
    "double_integrator": (4, 2, None),
    "van_der_pol": (2, 1, None),
    "gnss_pos_and_bias": (5, 3, None),
    "gnss_two_receiver": (10, 6, None),
    "kinematic_bycicle_and_bias": (6, 2, None),
}


def gen_plugins(ref):
    rng = np.random.default_rng(1234)
    out = {}
    for name, (n, m, params) in DYN_CASES.items():
        f = getattr(ref.dynamics, name)
        xs = rng.normal(size=(64, n))
        us = rng.normal(size=(64, m))
        fs, Fs = [], []
        for x, u in zip(xs, us):
            f0, J = cstep_jac(lambda xx, uu: f(xx, uu, params), x, u)
            fs.append(f0)
            Fs.append(J)
        out[f"dyn_{name}_x"] = xs
        out[f"dyn_{name}_u"] = us
        out[f"dyn_{name}_f"] = np.stack(fs)
        out[f"dyn_{name}_F"] = np.stack(Fs)
    # m = 0 dynamics: f(x, params) (nlp/nlp.py:218)
    xs = rng.normal(size=(64, 8))
    fs, Fs = [], []
    for x in xs:
        f0, J = cstep_jac(lambda xx: ref.dynamics.multi_receiver(xx, None), x)
        fs.append(f0); Fs.append(J)
    out["dyn_multi_receiver_x"] = xs
    out["dyn_multi_receiver_f"] = np.stack(fs)
    out["dyn_multi_receiver_F"] = np.stack(Fs)

    # vehicle_dynamics_and_gnss (nlp/dynamics.py:148-174) with the car constants of
    # autonomous-car.py:102 (utils/vehicle_sim.get_parameters); own generator so the
    # streams of the cases above are unchanged.  vx = x[3] kept away from -0.001.
    car = ref.vehicle_sim.get_parameters()
    vr = np.random.default_rng(5678)
    xs = vr.normal(size=(64, 9))
    xs[:, 3] = 2.0 + 10.0 * np.abs(xs[:, 3])
    us = vr.normal(size=(64, 2)) * np.array([2000.0, 0.2])
    fs, Fs = [], []
    for x, u in zip(xs, us):
        f0, J = cstep_jac(lambda xx, uu: ref.dynamics.vehicle_dynamics_and_gnss(xx, uu, {"car_params": car}), x, u)
        fs.append(f0); Fs.append(J)
    out["dyn_vehicle_dynamics_and_gnss_x"] = xs
    out["dyn_vehicle_dynamics_and_gnss_u"] = us
    out["dyn_vehicle_dynamics_and_gnss_f"] = np.stack(fs)
    out["dyn_vehicle_dynamics_and_gnss_F"] = np.stack(Fs)
    out["dyn_vehicle_dynamics_and_gnss_par"] = np.array([car[k] for k in ("C_AF", "C_AR", "M", "D_F", "D_R", "I_Z")],
                                                        dtype=np.float64)

    # measurements
    def meas(name, n, mk_params, jac=cstep_jac):
        h = getattr(ref.measurements, name)
        xs = rng.normal(size=(64, n)) * 10.0
        ys, Hs, pars = [], [], []
        for x in xs:
            p = mk_params()
            y0, J = jac(lambda xx: h(xx, p), x)
            ys.append(y0); Hs.append(J); pars.append(np.concatenate([np.ravel(v) for v in p.values()]) if p else np.zeros(0))
        return xs, np.stack(ys), np.stack(Hs), np.stack(pars)

    cases = {
        "full_state": (3, lambda: None, cstep_jac),
        "pseudorange": (5, lambda: {"sat_pos": rng.normal(size=3) * 2e4}, cstep_jac),
        "vehicle_pseudorange": (9, lambda: {"sat_pos": rng.normal(size=3) * 2e4}, cstep_jac),
        "pseudorange_rate": (8, lambda: {"sat_pos": rng.normal(size=3) * 2e4, "sat_vel": rng.normal(size=3) * 3e3}, cstep_jac),
        "multi_receiver_range_3d": (10, lambda: {"y": rng.normal(size=3) * 10}, cstep_jac),
        "multi_receiver_range_2d": (4, lambda: {"y": rng.normal(size=2) * 10}, cstep_jac),
        "multi_receiver_heading_2d": (4, lambda: {"y": rng.normal(size=2) * 10}, cdiff_jac),
    }
    for name, (n, mk, jac) in cases.items():
        xs, ys, Hs, pars = meas(name, n, mk, jac)
        out[f"meas_{name}_x"] = xs
        out[f"meas_{name}_y"] = ys
        out[f"meas_{name}_H"] = Hs
        out[f"meas_{name}_par"] = pars
    # idx-variant of multi_receiver_range_3d used between receivers (gnss-multi-receiver.py)
    h = ref.measurements.multi_receiver_range_3d
    xs = rng.normal(size=(64, 10)) * 10.0
    ys, Hs = [], []
    for x in xs:
        y0, J = cstep_jac(lambda xx: h(xx, {"idxA": [0, 1, 2], "idxB": [5, 6, 7]}), x)
        ys.append(y0); Hs.append(J)
    out["meas_range3d_AB_x"] = xs
    out["meas_range3d_AB_y"] = np.stack(ys)
    out["meas_range3d_AB_H"] = np.stack(Hs)

    # cost functions (nlp/cost_functions.py)
    vs = rng.normal(size=(16, 3))
    Q = np.diag([2.0, 3.0, 0.5]) + 0.1
    out["cost_v"] = vs
    out["cost_Q"] = Q
    out["cost_weighted_l2"] = np.array([float(np.squeeze(ref.cost_functions.weighted_l2_norm(v, {"Q": Q}))) for v in vs])
    out["cost_l2"] = np.array([float(np.squeeze(ref.cost_functions.l2_norm(v))) for v in vs])
    out["cost_huber"] = np.array([float(np.squeeze(ref.cost_functions.pseudo_huber_loss(v, {"Q": Q, "delta": 0.7}))) for v in vs])
    # idxA/idxB forms of the 2-D receiver-pair models (gnss-multi-receiver.py:92-107)
    for key, fn, jac in (("heading2d_AB", ref.measurements.multi_receiver_heading_2d, cdiff_jac),
                         ("range2d_AB", ref.measurements.multi_receiver_range_2d, cstep_jac)):
        xs = rng.normal(size=(64, 10)) * 10.0
        ys, Hs = [], []
        for x in xs:
            y0, J = jac(lambda xx: fn(xx, {"idxA": [0, 1], "idxB": [5, 6]}), x)
            ys.append(y0); Hs.append(J)
        out[f"meas_{key}_x"] = xs
        out[f"meas_{key}_y"] = np.stack(ys)
        out[f"meas_{key}_H"] = np.stack(Hs)
    np.savez_compressed(os.path.join(OUT, "plugins.npz"), **out)


def gen_ekf(ref):
    """Reference EKF on the gnss_stationary log (gnss_stationary.py:71-98 recipe)."""
    data_path = f"{REF}/data/gnss_stationary/gnss_log_2020_02_05_09_14_15"
    lat0, lon0, h0 = 37.4276, -122.1670, 0
    p_ref = ref.gutils.lla2ecef(np.array([lat0, lon0, h0]))
    data = ref.data.load_gnss_logs(data_path)
    T = 50
    Q = np.diag([0.0001, 0.0001, 0.0001, 0.1, 0.001])
    r_pr = 100
    u = np.zeros((3, T + 1))
    mu0 = np.array([10.0, -5.0, 3.0, float(data["pr"][0][0]) * 0.0 + 1.0, 0.5])
    S0 = np.eye(5)
    filt = ref.ekf.EKF(ref.gnss.gnss_pos_and_bias, ref.gnss.multi_pseudorange, mu0.copy(), S0.copy())
    mus, Ss, sats, prs, nsat = [], [], [], [], []
    for k in range(T + 1):
        sat_k = np.stack([ref.gutils.ecef2enu(data["sat_pos"][k][i, :], p_ref) for i in range(data["sat_pos"][k].shape[0])])
        R = np.diag(r_pr * np.ones(data["pr"][k].shape[0]))
        filt.update(u[:, k], data["pr"][k], Q, R, dyn_func_params={"dt": 1}, meas_func_params={"sat_pos": sat_k})
        pad_s = np.zeros((12, 3)); pad_s[: sat_k.shape[0]] = sat_k
        pad_p = np.zeros(12); pad_p[: sat_k.shape[0]] = data["pr"][k]
        sats.append(pad_s); prs.append(pad_p); nsat.append(sat_k.shape[0])
        mus.append(np.array(filt.mu, dtype=np.float64).copy()); Ss.append(np.array(filt.S).copy())
    np.savez_compressed(os.path.join(OUT, "ekf_gnss_stationary.npz"), mu0=mu0, S0=S0, Q=Q, r_pr=np.array(r_pr, dtype=np.float64),
                        sat_pos=np.stack(sats), pr=np.stack(prs), nsat=np.array(nsat, dtype=np.int32),
                        mu=np.stack(mus), S=np.stack(Ss), dt=np.array(1.0))


def gen_gnss_io(ref):
    """GNSS on-disk format (utils/data.py:9-75) and geodesy (utils/utils.py:4-110).

    Inputs: a reduced copy of the gnss_stationary log -- the SVID row plus the first
    60 epochs of ``svPoss`` (T+1,12,5) and ``pseudoranges`` (T+1,12) -- written with
    scipy.io.savemat, and a 3-D ``pseudoranges`` variant (T+1,12,6: range, rate,
    velocity, time) built from it with seeded rates/velocities.  Expected outputs:
    the reference ``load_gnss_logs`` run on those files (ragged per-epoch lists
    padded to 12 slots + counts) and the reference geodesy on seeded points."""
    from scipy.io import loadmat, savemat
    src = f"{REF}/data/gnss_stationary/gnss_log_2020_02_05_09_14_15"
    sv = loadmat(src + "satposecef.mat")["svPoss"][:61].copy()
    pr = loadmat(src + "ranges.mat")["pseudoranges"][:61].copy()
    small = os.path.join(OUT, "gnss_small_")
    savemat(small + "satposecef.mat", {"svPoss": sv})
    savemat(small + "ranges.mat", {"pseudoranges": pr})
    rng = np.random.default_rng(11)
    pr3 = np.zeros(pr.shape + (6,))
    pr3[:, :, 0] = pr
    pr3[1:, :, 1] = rng.normal(size=(60, 12)) * 100.0
    pr3[1:, :, 2:5] = rng.normal(size=(60, 12, 3)) * 3e3
    pr3[1:, :, 5] = 1000.0 + np.arange(60)[:, None] + rng.uniform(0, 0.01, size=(60, 12))
    pr3[0, :, 0] = pr[0]
    small3 = os.path.join(OUT, "gnss_small3_")
    savemat(small3 + "satposecef.mat", {"svPoss": sv})
    savemat(small3 + "ranges.mat", {"pseudoranges": pr3})
    out = {}
    for tag, prefix in (("d2", small), ("d3", small3)):
        d = ref.data.load_gnss_logs(prefix)
        T = len(d["pr"])
        cnt = np.array([len(x) for x in d["pr"]], dtype=np.int32)
        sp = np.zeros((T, 12, 3))
        pv = np.zeros((T, 12))
        for k in range(T):
            sp[k, :cnt[k]] = d["sat_pos"][k]
            pv[k, :cnt[k]] = d["pr"][k]
        out[f"{tag}_t"] = np.asarray(list(d["t"]), dtype=np.float64)
        out[f"{tag}_sats"] = np.asarray(d["sats"], dtype=np.float64)
        out[f"{tag}_count"], out[f"{tag}_sat_pos"], out[f"{tag}_pr"] = cnt, sp, pv
        if "sat_vel" in d:
            sv3 = np.zeros((T, 12, 3))
            rr = np.zeros((T, 12))
            for k in range(T):
                sv3[k, :cnt[k]] = d["sat_vel"][k]
                rr[k, :cnt[k]] = d["pr_rate"][k]
            out[f"{tag}_sat_vel"], out[f"{tag}_pr_rate"] = sv3, rr
    # geodesy on seeded points around the reference site (and far away)
    lla = np.stack([rng.uniform(-80, 80, 32), rng.uniform(-180, 180, 32), rng.uniform(-100, 9000, 32)], axis=1)
    lla[0] = [37.4276, -122.1670, 0.0]
    ecef = np.stack([ref.gutils.lla2ecef(p) for p in lla])
    out["geo_lla_in"], out["geo_ecef"] = lla, ecef
    out["geo_lla_back"] = np.stack([ref.gutils.ecef2lla(p) for p in ecef])
    pts = ecef[0] + rng.normal(size=(32, 3)) * 2e4
    out["geo_pts"] = pts
    out["geo_enu"] = np.stack([ref.gutils.ecef2enu(p, ecef[0]) for p in pts])
    out["geo_enu_rot"] = np.stack([ref.gutils.ecef2enu(p, ecef[0], rotation_only=True) for p in pts])
    out["geo_enu2ecef"] = np.stack([ref.gutils.enu2ecef(e, ecef[0]) for e in out["geo_enu"]])
    tt = np.round(rng.uniform(0, 100, 200), 1)
    out["ti_t"] = tt
    out["ti_idx"] = ref.gutils.get_time_indices(tt, 20.0, 35.5).astype(np.int64)
    np.savez_compressed(os.path.join(OUT, "gnss_io.npz"), **out)


def synth_constellation(rng, T, S, p0, vel, n_min=5):
    """Seeded synthetic GNSS epochs (no reference data): satellites on a 26 560 km
    shell above the receiver's horizon, receiver moving at ``vel`` (m/s) from
    ``p0`` (ECEF), clock bias 3e4 m drifting 0.5 m/s; pseudoranges and rates with
    1 m / 0.05 m/s noise.  Returns ragged per-epoch lists like load_gnss_logs."""
    up = p0 / np.linalg.norm(p0)
    sp, pr, sv, rr = [], [], [], []
    for k in range(T):
        pos = p0 + vel * k
        b = 3e4 + 0.5 * k
        c = int(rng.integers(n_min, S + 1))
        dirs = rng.normal(size=(c, 3))
        dirs /= np.linalg.norm(dirs, axis=1, keepdims=True)
        dirs = np.where((dirs @ up)[:, None] < 0.2, -dirs, dirs)  # keep the upper hemisphere
        dirs += 0.3 * up
        dirs /= np.linalg.norm(dirs, axis=1, keepdims=True)
        s = pos + 2.0e7 * dirs
        s *= 26.56e6 / np.linalg.norm(s, axis=1, keepdims=True)
        v = rng.normal(size=(c, 3)) * 2e3
        los = (s - pos) / np.linalg.norm(s - pos, axis=1, keepdims=True)
        sp.append(s)
        sv.append(v)
        pr.append(np.linalg.norm(s - pos, axis=1) + b + rng.normal(size=c))
        rr.append(np.einsum("ij,ij->i", v - vel, los) + 0.5 + 0.05 * rng.normal(size=c))
    return {"t": np.arange(T, dtype=np.float64), "sat_pos": sp, "pr": pr, "sat_vel": sv, "pr_rate": rr}


def _pack_log(d, S=12):
    """Ragged per-epoch lists -> fixed-slot arrays."""
    T = len(d["pr"])
    cnt = np.array([len(p) for p in d["pr"]], dtype=np.int32)
    out = {"count": cnt, "t": np.asarray(d["t"], dtype=np.float64),
           "sat_pos": np.zeros((T, S, 3)), "pr": np.zeros((T, S)),
           "sat_vel": np.zeros((T, S, 3)), "pr_rate": np.zeros((T, S))}
    for k in range(T):
        c = cnt[k]
        out["sat_pos"][k, :c] = d["sat_pos"][k]
        out["pr"][k, :c] = d["pr"][k]
        out["sat_vel"][k, :c] = d["sat_vel"][k]
        out["pr_rate"][k, :c] = d["pr_rate"][k]
    return out


def gen_least_squares(ref):
    """Reference runLeastSquares (utils/leastsquares.py:97-141) on two seeded
    synthetic receivers run back to back in one process, as
    gnss-multi-receiver.py:33-34 does -- the second log's first epoch warm-starts
    from the first log's last fix through the shared default argument
    (utils/leastsquares.py:19).  Inputs are synthetic; outputs are the
    reference's."""
    rng = np.random.default_rng(4242)
    p_ref = ref.gutils.lla2ecef(np.array([37.4276, -122.1670, 0.0]))
    out = {"p_ref": p_ref}
    for tag, off, vel in (("A", [120.0, -40.0, 15.0], np.array([1.2, -0.7, 0.1])),
                          ("B", [-300.0, 90.0, -20.0], np.array([-0.4, 0.9, 0.0]))):
        d = synth_constellation(rng, 40, 12, p_ref + np.array(off), vel)
        for k, v in _pack_log(d).items():
            out[f"{tag}_{k}"] = v
        sol = ref.ls.runLeastSquares(d["t"], d["sat_pos"], d["pr"], d["sat_vel"], d["pr_rate"], p_ref)
        for key in ("x_ECEF", "y_ECEF", "z_ECEF", "bias", "xd_ECEF", "yd_ECEF", "zd_ECEF", "bias_rate",
                    "x_ENU", "y_ENU", "z_ENU", "xd_ENU", "yd_ENU", "zd_ENU", "lat", "lon", "h"):
            out[f"{tag}_ls_{key}"] = np.asarray(sol[key], dtype=np.float64)
    np.savez_compressed(os.path.join(OUT, "least_squares.npz"), **out)


def gen_c3_geometry(ref):
    """the satellite geometry of data/gnss_stationary's log -- the
    first 201 epochs of 12 slots, loaded by the reference's own load_gnss_logs and
    rotated to ENU at the scripts' reference point by its ecef2enu
    (gnss_stationary.py:19-31 recipe).  Slots an epoch lacks are flagged (count)."""
    data = ref.data.load_gnss_logs(f"{REF}/data/gnss_stationary/gnss_log_2020_02_05_09_14_15")
    p_ref = ref.gutils.lla2ecef(np.array([37.4276, -122.1670, 0.0]))
    E, S = 201, 12
    sat = np.zeros((E, S, 3))
    cnt = np.zeros(E, dtype=np.int32)
    for k in range(E):
        sp = data["sat_pos"][k]
        cnt[k] = sp.shape[0]
        for j in range(cnt[k]):
            sat[k, j] = ref.gutils.ecef2enu(sp[j, :], p_ref)
    np.savez_compressed(os.path.join(OUT, "gnss_stationary_c3.npz"), sat_enu=sat, count=cnt,
                        t=np.asarray(list(data["t"]), dtype=np.float64)[:E])


def load_autocar_plugins(ref):
    """autonomous-car.py defines its EKF plug-ins (:18-77) at module level next to code
    that loads its pickled inputs, so the script is not imported: the two function
    definitions are taken from its syntax tree and executed in a namespace holding
    the modules they use (numpy, the reference's utils/vehicle_sim.py and utils/gnss.py)."""
    import ast
    path = f"{REF}/autonomous-car.py"
    tree = ast.parse(open(path).read(), filename=path)
    keep = [n for n in tree.body if isinstance(n, ast.FunctionDef)
            and n.name in ("discrete_vehicle_dynamics", "vehicle_sensors_model")]
    ns = {"np": np, "vehicle_sim": ref.vehicle_sim, "gnss": ref.gnss}
    exec(compile(ast.Module(body=keep, type_ignores=[]), path, "exec"), ns)
    return ns["discrete_vehicle_dynamics"], ns["vehicle_sensors_model"]


def gen_autocar_ekf(ref):
    """The reference EKF with autonomous-car.py's own plug-ins (:18-77), driven as the
    script's loop (:120-178: dt = 0.01, a correction at every 10th step, R = r_pr I,
    Q_EKF = 1e-3 Q_NLP, P = I) on seeded data of the script's shape (its sim pickles are
    not readable here): a linear-tyre bicycle trajectory from the reference's own
    vehicle_dynamics, 8-11 satellites per epoch in ENU, clock b0 + alpha t."""
    fdyn, fmeas = load_autocar_plugins(ref)
    car = ref.vehicle_sim.get_parameters()
    rng = np.random.default_rng(4242)
    dt, steps, every = 0.01, 300, 10
    t = dt * np.arange(steps)
    U = np.stack([1500.0 + 800.0 * np.sin(0.35 * t), 0.04 * np.sin(0.5 * t + 0.3)], axis=1)
    x = np.array([0.0, 0.0, 0.3, 8.0, 0.0, 0.0])
    xs = []
    for k in range(steps):
        xs.append(x.copy())
        x = x + dt * ref.vehicle_sim.vehicle_dynamics(x, U[k], {"tire_model_func": ref.vehicle_sim.linear_tire_model})
    xs = np.array(xs)
    NS, r_pr, alpha, b0 = 11, 10.0, 200.0, 0.0
    dirs = rng.normal(size=(NS, 3))
    dirs[:, 2] = np.abs(dirs[:, 2]) + 0.3
    sats = 2.0e7 * dirs / np.linalg.norm(dirs, axis=1, keepdims=True)
    Z = np.zeros((steps, NS)); SP = np.zeros((steps, NS, 3)); nz = np.zeros(steps, np.int32)
    for k in range(0, steps, every):
        ns = int(rng.integers(8, NS + 1))
        p = np.array([xs[k, 0], xs[k, 1], 0.0])
        SP[k, :ns] = sats[:ns]
        Z[k, :ns] = np.linalg.norm(p - sats[:ns], axis=1) + b0 + alpha * t[k] + np.sqrt(r_pr) * rng.normal(size=ns)
        nz[k] = ns
    Q_NLP = np.diag([0.01, 0.01, 0.01, 100, 500, 500, .001, .001, .001])
    Q = .001 * Q_NLP
    mu0 = np.hstack((xs[0], np.array([b0, alpha, 0.0])))
    S0 = np.diag(np.ones(9))
    filt = ref.ekf.EKF(fdyn, fmeas, mu0.copy(), S0.copy())
    mus, Ss = [], []
    for k in range(steps):
        ns = int(nz[k])
        z = Z[k, :ns] if ns else None
        R = np.diag(r_pr * np.ones(ns)) if ns else None
        filt.update(U[k], z, Q, R, dyn_func_params={"dt": dt, "car_params": car},
                    meas_func_params={"sat_pos": SP[k, :ns] if ns else None})
        mus.append(np.array(filt.mu, dtype=np.float64).copy()); Ss.append(np.array(filt.S, dtype=np.float64).copy())
    # plug-in values / Jacobians at seeded points (the reference's own jac=True outputs)
    px = rng.normal(size=(32, 9)) * 3.0
    px[:, 3] = 4.0 + np.abs(px[:, 3]) * 5.0
    pu = rng.normal(size=(32, 2)) * np.array([1500.0, 0.1])
    pf, pF, py, pH, ps = [], [], [], [], []
    for xx, uu in zip(px, pu):
        f0, J = fdyn(xx.copy(), uu, params={"dt": dt, "car_params": car}, jac=True)
        pf.append(f0); pF.append(J)
        s = rng.normal(size=(5, 3)) * 2.0e4
        y0, H = fmeas(xx.copy(), params={"sat_pos": s}, jac=True)
        py.append(y0); pH.append(H); ps.append(s)
    np.savez_compressed(os.path.join(OUT, "ekf_autocar.npz"), mu0=mu0, S0=S0, Q=Q, r_pr=np.array(r_pr), dt=np.array(dt),
                        car=np.array([car[k] for k in ("C_AF", "C_AR", "M", "D_F", "D_R", "I_Z")]),
                        U=U, Z=Z, sat_pos=SP, nz=nz, mu=np.stack(mus), S=np.stack(Ss)[::5], S_every=np.array(5),
                        plug_x=px, plug_u=pu, plug_f=np.stack(pf), plug_F=np.stack(pF), plug_sat=np.stack(ps),
                        plug_y=np.stack(py), plug_H=np.stack(pH))


def read_ulog(path, topics):
    """Minimal ULog reader (the documented PX4 binary log format; nothing in the file is
    executed): the 16-byte header, then messages [uint16 size][uint8 type][body].
    'F' bodies are "name:type field;type field;...", 'A' bodies subscribe a topic
    (uint8 multi_id, uint16 msg_id, name), 'D' bodies are uint16 msg_id + the fields
    packed in format order.  Returns {topic: {field: array}} for multi_id 0 of `topics`,
    with the columns ulog2csv would write (padding dropped, arrays flattened as
    field[i], timestamp first)."""
    import struct
    raw = open(path, "rb").read()
    assert raw[:7] == b"ULog\x01\x125", "not a ULog file"
    sizes = {"int8_t": 1, "uint8_t": 1, "bool": 1, "char": 1, "int16_t": 2, "uint16_t": 2, "int32_t": 4,
             "uint32_t": 4, "float": 4, "int64_t": 8, "uint64_t": 8, "double": 8}
    codes = {"int8_t": "b", "uint8_t": "B", "bool": "?", "char": "c", "int16_t": "h", "uint16_t": "H",
             "int32_t": "i", "uint32_t": "I", "float": "f", "int64_t": "q", "uint64_t": "Q", "double": "d"}
    formats, subs, rows = {}, {}, {}
    off = 16
    while off + 3 <= len(raw):
        size, typ = struct.unpack_from("<HB", raw, off)
        body = raw[off + 3: off + 3 + size]
        off += 3 + size
        if len(body) < size:
            break
        if typ == ord("F"):
            name, spec = body.decode("ascii").split(":", 1)
            fields = []
            for item in spec.strip(";").split(";"):
                ftype, fname = item.split(" ")
                count = 1
                if "[" in ftype:
                    ftype, cnt = ftype[:-1].split("[")
                    count = int(cnt)
                fields.append((ftype, fname, count))
            formats[name] = fields
        elif typ == ord("A"):
            multi, msg_id = struct.unpack_from("<BH", body, 0)
            name = body[3:].decode("ascii")
            if name in topics and multi == 0:
                subs[msg_id] = name
                rows[name] = []
        elif typ == ord("D"):
            (msg_id,) = struct.unpack_from("<H", body, 0)
            if msg_id in subs:
                rows[subs[msg_id]].append(body[2:])
    out = {}
    for name in topics:
        fields = formats[name]
        fmt = "<" + "".join(codes[t] * c if c > 1 else codes[t] for t, _, c in fields)
        cols = []
        for t, fn, c in fields:
            cols += [f"{fn}[{i}]" for i in range(c)] if c > 1 else [fn]
        keep = [i for i, cn in enumerate(cols) if not cn.startswith("_padding")]
        full = struct.calcsize(fmt)   # PX4 does not log a message's trailing padding: pad it back
        vals = np.array([struct.unpack_from(fmt, r + bytes(full - len(r)), 0) for r in rows[name]], dtype=np.float64)
        names = [cols[i] for i in keep]
        order = [names.index("timestamp")] + [i for i, cn in enumerate(names) if cn != "timestamp"]
        out[name] = {"columns": [names[i] for i in order], "data": vals[:, keep][:, order]}
    return out


def gen_rc_car_c4(ref):
    """C4 inputs from the reference's rc-car logs (rc-car.py:21-38):
    * controls: data/rc-car/px4/log_164_*.ulg read with read_ulog and processed exactly
      as px4/convert.py (ulog2csv columns manual_control_setpoint[3], [4] = throttle,
      steer; sensor_combined timestamps; microseconds -> s, zeroed at the earlier first
      sample; the control interp1d'd onto the sensor times) and rc-car.py:25-37
      (throttle < 0.1 -> 0; start at the first |steer| < 0.01; times from 0).  The .pkl
      next to it (convert.py's output) is a pickle and is not read.
    * satellites: data/rc-car/gnss/gnss_log_2020_02_27_10_02_20 through the reference's
      load_gnss_logs, rotated to ENU at the scripts' reference point by its ecef2enu,
      times from 0 (rc-car.py:35); up to 12 slots per epoch (count)."""
    from scipy.interpolate import interp1d
    u = read_ulog(f"{REF}/data/rc-car/px4/log_164_2020-2-27-10-03-56.ulg", ("manual_control_setpoint", "sensor_combined"))
    mc, sc = u["manual_control_setpoint"]["data"], u["sensor_combined"]["data"]
    t1, throttle, steer = mc[:, 0] * 1e-6, mc[:, 3], mc[:, 4]
    t2 = sc[:, 0] * 1e-6
    t0 = np.min([t1[0], t2[0]])
    t1 = t1 - t0
    t2 = t2 - t0
    control = interp1d(t1, np.vstack((throttle, steer)), fill_value="extrapolate")(t2)
    for i in range(control.shape[1]):          # rc-car.py:25-28
        if control[0, i] < 0.1:
            control[0, i] = 0.0
    for k, t in enumerate(t2):                # rc-car.py:30-35
        if np.abs(control[1, k]) < 0.01:
            t2, control = t2[k:], control[:, k:]
            break
    t2 = t2 - t2[0]
    g = ref.data.load_gnss_logs(f"{REF}/data/rc-car/gnss/gnss_log_2020_02_27_10_02_20")
    tg = np.asarray(list(g["t"]), dtype=np.float64)
    tg = tg - tg[0]
    p_ref = ref.gutils.lla2ecef(np.array([37.4276, -122.1670, 0.0]))
    E, S = len(g["sat_pos"]), 12
    sat, cnt, pr = np.zeros((E, S, 3)), np.zeros(E, dtype=np.int32), np.zeros((E, S))
    for k in range(E):
        sp = g["sat_pos"][k]
        cnt[k] = sp.shape[0]
        for j in range(cnt[k]):
            sat[k, j] = ref.gutils.ecef2enu(sp[j, :], p_ref)
            pr[k, j] = g["pr"][k][j]
    np.savez_compressed(os.path.join(OUT, "rc_car_c4.npz"), t_u=t2, u=control, t_gnss=tg, sat_enu=sat, count=cnt,
                        pr=pr, ulog_columns=np.array(u["manual_control_setpoint"]["columns"][:5]))


def main(which=None):
    ref = load_reference()
    gens = {"collocation": gen_collocation, "plugins": gen_plugins, "ekf": gen_ekf, "gnss_io": gen_gnss_io,
            "least_squares": gen_least_squares, "c3_geometry": gen_c3_geometry,
            "autocar_ekf": gen_autocar_ekf, "rc_car_c4": gen_rc_car_c4}
    for name, fn in gens.items():
        if not which or name in which:
            fn(ref)
    print("golden fixtures written to", OUT)


if __name__ == "__main__":
    main(sys.argv[1:])   # e.g. `gen_golden.py plugins` regenerates plugins.npz only
