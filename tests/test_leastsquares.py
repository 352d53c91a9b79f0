"""Batched GNSS least squares (utils.leastsquares on libmhe.so, csrc/mhe_ls.hip).

Oracle: oracle/leastsquares.py (restatement of utils/leastsquares.py:6-63,97-141),
pinned to
  * tests/golden/least_squares.npz -- the reference's own runLeastSquares run on
    two seeded synthetic receivers back to back (gen_golden.py: gen_least_squares);
  * the reference's stored results for the real gnss-multi-receiver logs
    (data/gnss-multi-receiver/LS_{A,B}.csv), read in place when /root/reference
    is present (build container only; skipped elsewhere -- nothing is copied).
GPU tolerance: the kernel solves the normal equations where the reference uses
pinv(G), and stops on the same ||dx|| < 1e-7 rule, so fixes agree to
|dx| <= 1e-6 m, lat/lon to 1e-10 deg and velocities to 1e-6 m/s.
"""
import ctypes
import os

import numpy as np
import pytest

from mhe import _lib
from oracle import leastsquares as ols

REF_DATA = "/root/reference/data/gnss-multi-receiver"
X_TOL, LL_TOL, V_TOL = 1e-6, 1e-10, 1e-6


def _lists(fx, tag):
    cnt = fx[f"{tag}_count"]
    T = cnt.shape[0]
    sp = [fx[f"{tag}_sat_pos"][k, :cnt[k]] for k in range(T)]
    pr = [fx[f"{tag}_pr"][k, :cnt[k]] for k in range(T)]
    sv = [fx[f"{tag}_sat_vel"][k, :cnt[k]] for k in range(T)]
    rr = [fx[f"{tag}_pr_rate"][k, :cnt[k]] for k in range(T)]
    return sp, pr, sv, rr


@pytest.fixture(scope="module")
def lsfx(golden):
    return golden["least_squares"]


def test_oracle_reproduces_reference_runs(lsfx):
    """Two logs back to back through one shared warm-start array (gnss-multi-receiver.py:33-34)."""
    x = np.zeros(3)
    for tag in ("A", "B"):
        sp, pr, sv, rr = _lists(lsfx, tag)
        out = ols.run_least_squares(sp, pr, sv, rr, x=x)
        ref = np.stack([lsfx[f"{tag}_ls_{k}"] for k in ("x_ECEF", "y_ECEF", "z_ECEF")], 1)
        np.testing.assert_allclose(out["x"], ref, rtol=0, atol=1e-9)
        np.testing.assert_allclose(out["b"], lsfx[f"{tag}_ls_bias"], rtol=0, atol=1e-9)
        refv = np.stack([lsfx[f"{tag}_ls_{k}"] for k in ("xd_ECEF", "yd_ECEF", "zd_ECEF")], 1)
        np.testing.assert_allclose(out["v"], refv, rtol=0, atol=1e-9)
        np.testing.assert_allclose(out["bd"], lsfx[f"{tag}_ls_bias_rate"], rtol=0, atol=1e-9)


@pytest.mark.skipif(not os.path.isdir(REF_DATA), reason="reference data not present (GPU box)")
def test_oracle_reproduces_reference_stored_fixes():
    """Oracle + this package's loader/geodesy against LS_{A,B}.csv of the reference."""
    from utils import data as gd, utils as gu
    x = np.zeros(3)
    for tag, pre in (("A", "/rec1/rec1_gnss_log_50y_moving_"), ("B", "/rec2/rec2_gnss_log_50y_moving_")):
        d = gd.load_gnss_logs(REF_DATA + pre)
        out = ols.run_least_squares(d["sat_pos"], d["pr"], x=x)
        ll = np.array([gu.ecef2lla(p)[:2] for p in out["x"]])
        ref = np.loadtxt(f"{REF_DATA}/LS_{tag}.csv", delimiter=",")
        assert ll.shape == ref.shape
        assert np.abs(ll - ref).max() < 1e-12


def test_ls_abi_host_checks():
    lib = _lib.load()
    d = _lib.MheLsDims(slots=12, max_iter=100, warm=1, with_vel=0, tol=1e-7)
    nul = [None] * 12
    assert lib.mhe_ls_run(ctypes.byref(d), 0, 5, *nul, None) == 0      # empty: no launch
    d.slots = 65
    assert lib.mhe_ls_run(ctypes.byref(d), 2, 5, *nul, None) == -1     # MHE_ERR_DIMS
    d.slots = 12
    assert lib.mhe_ls_run(ctypes.byref(d), 2, 5, *nul, None) == -5     # MHE_ERR_NULL


# ---------------------------------------------------------------- GPU parity

@pytest.mark.gpu
def test_run_least_squares_matches_reference_runs(lsfx):
    import utils.leastsquares as uls
    uls._DEFAULT_X[:] = 0.0
    for tag in ("A", "B"):  # back to back: B warm-starts from A's last fix, as the reference
        sp, pr, sv, rr = _lists(lsfx, tag)
        sol = uls.runLeastSquares(lsfx[f"{tag}_t"], sp, pr, sv, rr, lsfx["p_ref"])
        for k in ("x_ECEF", "y_ECEF", "z_ECEF", "bias", "x_ENU", "y_ENU", "z_ENU"):
            assert np.abs(sol[k] - lsfx[f"{tag}_ls_{k}"]).max() <= X_TOL, k
        for k in ("lat", "lon"):
            assert np.abs(sol[k] - lsfx[f"{tag}_ls_{k}"]).max() <= LL_TOL, k
        for k in ("xd_ECEF", "yd_ECEF", "zd_ECEF", "bias_rate", "xd_ENU", "yd_ENU", "zd_ENU"):
            assert np.abs(sol[k] - lsfx[f"{tag}_ls_{k}"]).max() <= V_TOL, k
        assert (sol["iters"] > 0).all()
    np.testing.assert_allclose(uls._DEFAULT_X, [lsfx["B_ls_x_ECEF"][-1], lsfx["B_ls_y_ECEF"][-1],
                                                lsfx["B_ls_z_ECEF"][-1]], rtol=0, atol=X_TOL)


@pytest.mark.gpu
def test_iterative_least_squares_in_place_default(lsfx):
    """The shared mutable default (utils/leastsquares.py:19,34): a second call starts
    from the first call's fix, and the returned x IS the default array."""
    import utils.leastsquares as uls
    sp, pr, _, _ = _lists(lsfx, "A")
    uls._DEFAULT_X[:] = 0.0
    x1, b1 = uls.iterativeLeastSquares(sp[0], pr[0])
    assert x1 is uls._DEFAULT_X
    xo, bo, _ = ols.iterative_least_squares(sp[0], pr[0], np.zeros(3))
    assert np.abs(x1 - xo).max() <= X_TOL and abs(b1 - bo) <= X_TOL
    x2, _ = uls.iterativeLeastSquares(sp[1], pr[1])
    xo2, _, _ = ols.iterative_least_squares(sp[1], pr[1], xo.copy())
    assert np.abs(x2 - xo2).max() <= X_TOL
    own = np.array([1.0, 2.0, 3.0])
    xr, _ = uls.iterativeLeastSquares(sp[2], pr[2], own)
    assert xr is own and np.abs(own - ols.iterative_least_squares(sp[2], pr[2], np.array([1.0, 2.0, 3.0]))[0]).max() <= X_TOL


@pytest.mark.gpu
def test_velocity_alone(lsfx):
    import utils.leastsquares as uls
    sp, _, sv, rr = _lists(lsfx, "B")
    x = np.array([lsfx["B_ls_x_ECEF"][3], lsfx["B_ls_y_ECEF"][3], lsfx["B_ls_z_ECEF"][3]])
    v, bd = uls.iterativeLeastSquaresVel(sp[3], sv[3], rr[3], x)
    vo, bdo = ols.iterative_least_squares_vel(sp[3], sv[3], rr[3], x)
    assert np.abs(v - vo).max() <= 1e-9 and abs(bd - bdo) <= 1e-9


@pytest.mark.gpu
def test_batch_of_logs_both_modes(lsfx):
    """64 perturbed logs: warm chains (one wave per log) and independent epochs
    (one wave per epoch) against the oracle per log / per epoch."""
    import utils.leastsquares as uls
    rng = np.random.default_rng(11)
    C = 64
    T = lsfx["A_count"].shape[0]
    sp = np.tile(lsfx["A_sat_pos"][None], (C, 1, 1, 1))
    pr = np.tile(lsfx["A_pr"][None], (C, 1, 1)) + rng.normal(size=(C,) + lsfx["A_pr"].shape) * 3.0
    cnt = np.tile(lsfx["A_count"][None], (C, 1))
    cnt[:, 5] = np.minimum(cnt[:, 5], 5)     # ragged: fewer satellites in one epoch
    x0 = rng.normal(size=(C, 3)) * 1e3
    for warm in (True, False):
        r = uls.run_batch(sp, pr, cnt, x_init=x0, warm=warm)
        X = r["x"].cpu().numpy()
        it = r["iters"].cpu().numpy()
        assert (it > 0).all()
        for c in range(0, C, 9):
            xs = x0[c].copy()
            for k in range(T):
                start = xs if warm else x0[c].copy()
                xo, _, _ = ols.iterative_least_squares(sp[c, k, :cnt[c, k]], pr[c, k, :cnt[c, k]], start)
                assert np.abs(X[c, k] - xo).max() <= X_TOL, (warm, c, k)
        if warm:
            np.testing.assert_array_equal(r["x_last"].cpu().numpy(), X[:, -1])


@pytest.mark.gpu
def test_underdetermined_epoch_flagged(lsfx):
    import utils.leastsquares as uls
    sp = lsfx["A_sat_pos"][None, :3]
    pr = lsfx["A_pr"][None, :3]
    cnt = np.array([[3, 12, 2]], dtype=np.int32)
    cnt[0, 1] = lsfx["A_count"][1]
    r = uls.run_batch(sp, pr, cnt, warm=False)
    it = r["iters"].cpu().numpy()[0]
    assert it[0] == -1 and it[2] == -1 and it[1] > 0


@pytest.mark.gpu
def test_velocity_failure_reported_by_nan(lsfx):
    """a velocity solve that cannot be formed leaves v / bd NaN and does
    not overwrite the position fix's iteration count."""
    import utils.leastsquares as uls
    sp = lsfx["A_sat_pos"][None, :2]
    pr = lsfx["A_pr"][None, :2]
    cnt = np.array([[3, lsfx["A_count"][1]]], dtype=np.int32)
    r = uls.run_batch(sp, pr, cnt, warm=False, sat_vel=np.zeros(sp.shape), pr_rate=np.zeros(pr.shape))
    it = r["iters"].cpu().numpy()[0]
    v = r["v"].cpu().numpy()[0]
    assert it[0] == -1 and np.isnan(v[0]).all() and np.isnan(r["bd"].cpu().numpy()[0, 0])
    assert it[1] > 0 and np.isfinite(v[1]).all()
