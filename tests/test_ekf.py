"""Batched EKF (utils.ekf on libmhe.so, csrc/mhe_ekf.hip) against the reference.

Oracle: oracle/ekf.py (restatement of utils/ekf.py:20-61 + utils/gnss.py), pinned
bit-exactly to tests/golden/ekf_gnss_stationary.npz (the reference EKF run on the
gnss_stationary log).  GPU tolerance: the kernel replaces the reference's
explicit inv(P) by a Cholesky sweep, so states agree to rounding:
|dmu| <= 1e-9 (1 + |mu|) and |dS| <= 1e-9 max|S| per step over 51 steps.
"""
import ctypes

import numpy as np
import pytest

from mhe import _lib
from mhe.registry import UnsupportedPlugin
from oracle import ekf as oekf
import utils.ekf as ekf
import utils.gnss as gnss

MU_TOL, S_TOL = 1e-9, 1e-9


def _fixture(golden):
    return dict(golden["ekf_gnss_stationary"])


def _close(mu, S, mu_ref, S_ref):
    dmu = np.abs(mu - mu_ref).max(axis=-1) / (1.0 + np.abs(mu_ref).max(axis=-1))
    dS = np.abs(S - S_ref).reshape(S.shape[:-2] + (-1,)).max(-1) / np.abs(S_ref).reshape(S.shape[:-2] + (-1,)).max(-1)
    return float(dmu.max()), float(dS.max())


def test_oracle_ekf_reproduces_reference_fixture(golden):
    fx = _fixture(golden)
    mu, S = oekf.run_fixture(fx)
    np.testing.assert_array_equal(mu, fx["mu"])
    np.testing.assert_array_equal(S, fx["S"])


def test_gnss_plugins_match_oracle():
    rng = np.random.default_rng(7)
    for _ in range(16):
        x = rng.normal(size=5) * 100
        sp = rng.normal(size=(7, 3)) * 2e7
        for f, g in ((gnss.multi_pseudorange, oekf.multi_pseudorange),
                     (gnss.multi_pseudorange_and_bias, oekf.multi_pseudorange_and_bias)):
            y1, J1 = f(x, {"sat_pos": sp}, jac=True)
            y2, J2 = g(x, {"sat_pos": sp}, jac=True)
            np.testing.assert_array_equal(y1, y2)
            np.testing.assert_array_equal(J1, J2)
        u = rng.normal(size=3)
        x1, G1 = gnss.gnss_pos_and_bias(x.copy(), u, {"dt": 0.5}, jac=True)
        x2, G2 = oekf.gnss_pos_and_bias(x.copy(), u, {"dt": 0.5}, jac=True)
        np.testing.assert_array_equal(x1, x2)
        np.testing.assert_array_equal(G1, G2)


def test_unregistered_plugin_fails_loudly():
    def my_dyn(x, u, params=None, jac=False):
        return x, np.eye(5)
    with pytest.raises(UnsupportedPlugin):
        ekf.EKF(my_dyn, gnss.multi_pseudorange, np.zeros(5), np.eye(5))


def test_ekf_abi_host_checks():
    lib = _lib.load()
    d = _lib.MheEkfDims(n=5, m=3, pmax=12, q=3, dyn_model=1, meas_model=1, dt=1.0)
    # mu, S, U, u_bs, Z, z_bs, nz, nz_bs, PAR, par_bs, Q, R, r_bs, r_ss, mu_hist, S_hist, status, stream
    args = [None, None, None, 0, None, 0, None, 0, None, 0, None, None, 0, 0, None, None, None, None]
    assert lib.mhe_ekf_run(ctypes.byref(d), 0, 5, *args) == 0  # empty batch: no launch
    d.pmax = 64
    assert lib.mhe_ekf_run(ctypes.byref(d), 4, 5, *args) == -1  # MHE_ERR_DIMS


def _batch_inputs(fx, B, seed=3, drop_steps=()):
    rng = np.random.default_rng(seed)
    T = fx["pr"].shape[0]
    mu0 = np.tile(fx["mu0"], (B, 1))
    mu0[1:] += rng.normal(size=(B - 1, 5)) * np.array([3, 3, 3, 30, 0.1])
    S0 = np.tile(fx["S0"], (B, 1, 1))
    U = np.zeros((B, T, 3))
    U[1:] = rng.normal(size=(B - 1, T, 3)) * 0.1
    Z = np.tile(fx["pr"], (B, 1, 1))
    nz = np.tile(fx["nsat"], (B, 1)).astype(np.int32)
    for k in drop_steps:
        nz[:, k] = 0
    sat = np.tile(fx["sat_pos"], (B, 1, 1, 1))
    R = np.stack([np.diag(float(fx["r_pr"]) * np.ones(12)) for _ in range(T)])
    return mu0, S0, U, Z, nz, sat, R


def _oracle_batch(fx, mu0, S0, U, Z, nz, sat, meas=oekf.multi_pseudorange, extra=0):
    B, T = Z.shape[:2]
    mus = np.zeros((B, T, 5))
    Ss = np.zeros((B, T, 5, 5))
    for b in range(B):
        f = oekf.EKF(oekf.gnss_pos_and_bias, meas, mu0[b], S0[b])
        for k in range(T):
            ns = int(nz[b, k])
            if ns == 0:
                f.update(U[b, k], None, fx["Q"], None, {"dt": 1.0})
            else:
                R = np.diag(float(fx["r_pr"]) * np.ones(ns))
                f.update(U[b, k], Z[b, k, :ns], fx["Q"], R, {"dt": 1.0}, None,
                         {"sat_pos": sat[b, k, :ns - extra]})
            mus[b, k], Ss[b, k] = f.mu, f.S
    return mus, Ss


@pytest.mark.gpu
def test_ekf_class_matches_reference_fixture(golden):
    fx = _fixture(golden)
    f = ekf.EKF(gnss.gnss_pos_and_bias, gnss.multi_pseudorange, fx["mu0"].copy(), fx["S0"].copy())
    mus, Ss = [], []
    for k in range(fx["pr"].shape[0]):
        ns = int(fx["nsat"][k])
        R = np.diag(float(fx["r_pr"]) * np.ones(ns))
        f.update(np.zeros(3), fx["pr"][k, :ns], fx["Q"], R, dyn_func_params={"dt": 1.0},
                 meas_func_params={"sat_pos": fx["sat_pos"][k, :ns]})
        mus.append(f.mu)
        Ss.append(f.S)
    emu, eS = _close(np.stack(mus), np.stack(Ss), fx["mu"], fx["S"])
    assert emu <= MU_TOL and eS <= S_TOL, (emu, eS)


@pytest.mark.gpu
@pytest.mark.parametrize("method,inputs", [("lane", "batch_outer"), ("wave", "batch_outer"), ("auto", "batch_outer"),
                                           ("lane", "batch_inner"), ("wave", "batch_inner")])
def test_ekf_batch_matches_oracle_per_instance(golden, method, inputs):
    """Both device formulations: sequential scalar updates one filter per lane
    (diagonal R) and the per-wavefront augmented Cholesky sweep (any R); inputs
    batch-outermost (the reference's per-instance arrays) or batch-innermost."""
    fx = _fixture(golden)
    B = 64
    mu0, S0, U, Z, nz, sat, R = _batch_inputs(fx, B, drop_steps=(5, 6, 30))
    if inputs == "batch_inner":
        args = (np.moveaxis(U, 0, -1), np.moveaxis(Z, 0, -1), np.moveaxis(nz, 0, -1))
        sat_in = np.moveaxis(sat, 0, -1)
    else:
        args, sat_in = (U, Z, nz), sat
    mh, Sh, mu, S, st = ekf.run_batch(gnss.gnss_pos_and_bias, gnss.multi_pseudorange, mu0, S0, *args,
                                      fx["Q"], R, 1.0, sat_in, method=method, inputs=inputs)
    assert int(st.abs().sum().item()) == 0
    rmu, rS = _oracle_batch(fx, mu0, S0, U, Z, nz, sat)
    emu, eS = _close(mh.cpu().numpy(), Sh.cpu().numpy(), rmu, rS)
    assert emu <= MU_TOL and eS <= S_TOL, (emu, eS)
    np.testing.assert_array_equal(mu.cpu().numpy(), mh[:, -1].cpu().numpy())
    # instance 0 is the reference recipe (no dropped steps in the fixture: compare the prefix)
    e0, _ = _close(mh[0, :5].cpu().numpy(), Sh[0, :5].cpu().numpy(), fx["mu"][:5], fx["S"][:5])
    assert e0 <= MU_TOL


@pytest.mark.gpu
@pytest.mark.parametrize("method", ["lane", "wave"])
def test_ekf_bias_row_variant(golden, method):
    fx = _fixture(golden)
    B = 8
    mu0, S0, U, Z0, nz0, sat, _ = _batch_inputs(fx, B, seed=5)
    T = Z0.shape[1]
    Z = np.zeros((B, T, 13))
    nz = nz0 + 1
    for b in range(B):
        for k in range(T):
            ns = nz0[b, k]
            Z[b, k, :ns] = Z0[b, k, :ns]
            Z[b, k, ns] = 1.0 + 0.01 * k  # bias measurement row
    R = np.stack([np.diag(float(fx["r_pr"]) * np.ones(13)) for _ in range(T)])
    sat13 = np.zeros((B, T, 13, 3))
    sat13[:, :, :12] = sat
    mh, Sh, _, _, st = ekf.run_batch(gnss.gnss_pos_and_bias, gnss.multi_pseudorange_and_bias, mu0, S0, U, Z, nz,
                                     fx["Q"], R, 1.0, sat13, method=method)
    assert int(st.abs().sum().item()) == 0
    rmu, rS = _oracle_batch(fx, mu0, S0, U, Z, nz, sat13, meas=oekf.multi_pseudorange_and_bias, extra=1)
    emu, eS = _close(mh.cpu().numpy(), Sh.cpu().numpy(), rmu, rS)
    assert emu <= MU_TOL and eS <= S_TOL, (emu, eS)


@pytest.mark.gpu
def test_ekf_end_to_end_from_log_files():
    """On-disk log (reduced gnss_stationary .mat, utils.data) -> fixed-slot device
    layout (pack_epochs, ENU at the reference site) -> batched EKF, vs the oracle EKF
    fed the reference loader's per-epoch arrays."""
    import os
    from utils import data as gdata, utils as gutils
    G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    d = gdata.load_gnss_logs(os.path.join(G, "gnss_small_"))
    p_ref = gutils.lla2ecef(np.array([37.4276, -122.1670, 0.0]))
    pk = gdata.pack_epochs(d, p_ref, slots=12)
    T = pk["pr"].shape[0]
    B = 4
    mu0 = np.tile(np.array([10.0, -5.0, 3.0, 1.0, 0.5]), (B, 1)) + np.arange(B)[:, None]
    S0 = np.tile(np.eye(5), (B, 1, 1))
    Q = np.diag([1e-4, 1e-4, 1e-4, 0.1, 1e-3])
    R = np.tile(np.eye(12) * 100.0, (T, 1, 1))
    mh, Sh, _, _, st = ekf.run_batch(gnss.gnss_pos_and_bias, gnss.multi_pseudorange, mu0, S0, np.zeros((B, T, 3)),
                                     np.tile(pk["pr"], (B, 1, 1)), np.tile(pk["count"], (B, 1)), Q, R, 1.0,
                                     np.tile(pk["sat_pos"], (B, 1, 1, 1)))
    assert int(st.abs().sum().item()) == 0
    for b in range(B):
        f = oekf.EKF(oekf.gnss_pos_and_bias, oekf.multi_pseudorange, mu0[b], S0[b])
        for k in range(T):
            sat = gutils.ecef2enu(d["sat_pos"][k], p_ref)
            f.update(np.zeros(3), d["pr"][k], Q, np.diag(100.0 * np.ones(len(d["pr"][k]))), {"dt": 1.0}, None,
                     {"sat_pos": sat})
            emu, eS = _close(mh[b, k].cpu().numpy()[None], Sh[b, k].cpu().numpy()[None], f.mu[None], f.S[None])
            assert emu <= MU_TOL and eS <= S_TOL, (b, k, emu, eS)


@pytest.mark.gpu
def test_ekf_correlated_R_uses_general_path(golden):
    """A non-diagonal R (correlated pseudorange errors) must take the general
    per-wavefront sweep under method="auto" and match the oracle's batch update."""
    fx = _fixture(golden)
    B = 8
    mu0, S0, U, Z, nz, sat, _ = _batch_inputs(fx, B, seed=9)
    T = Z.shape[1]
    r = float(fx["r_pr"])
    Rc = r * (0.7 * np.eye(12) + 0.3 * np.ones((12, 12)))
    R = np.stack([Rc for _ in range(T)])
    mh, Sh, _, _, st = ekf.run_batch(gnss.gnss_pos_and_bias, gnss.multi_pseudorange, mu0, S0, U, Z, nz,
                                     fx["Q"], R, 1.0, sat)
    assert int(st.abs().sum().item()) == 0
    mus = np.zeros((B, T, 5))
    Ss = np.zeros((B, T, 5, 5))
    for b in range(B):
        f = oekf.EKF(oekf.gnss_pos_and_bias, oekf.multi_pseudorange, mu0[b], S0[b])
        for k in range(T):
            ns = int(nz[b, k])
            f.update(U[b, k], Z[b, k, :ns], fx["Q"], Rc[:ns, :ns], {"dt": 1.0}, None, {"sat_pos": sat[b, k, :ns]})
            mus[b, k], Ss[b, k] = f.mu, f.S
    emu, eS = _close(mh.cpu().numpy(), Sh.cpu().numpy(), mus, Ss)
    assert emu <= MU_TOL and eS <= S_TOL, (emu, eS)
