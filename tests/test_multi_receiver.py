"""The two-receiver MHE of gnss-multi-receiver.py end to end:
mixed plug-ins (range_3d / heading_2d between the receivers, pseudoranges of A
and B with per-window parameters and R = 0 slots), zA = zB at every node
(addEqConstraint), prior from the previous window, warm start.

* GPU parity: the script written against this package's facade
  (general_problems.two_rx_mhe_facade -> libmhe.so) vs the same script on the
  oracle (two_rx_mhe_oracle, dense KKT Gauss-Newton), per window, on the seeded
  synthetic two-receiver logs of tests/golden/least_squares.npz (fixes and
  velocities from the reference's runLeastSquares).  Tolerance: states at t = T
  and t = DT within 1e-6 * (1 + max|x|) (x holds clock biases ~3e4 m; the
  pseudorange rows lose log10(|y| / |y - h|) ~ 5 digits to cancellation).
* Consistency with the reference's stored IPOPT results (NLP_{A,B}.csv), read in
  place when /root/reference is present: the oracle replica on the real logs.
  PARITY UNPINNED for this case: IPOPT is absent here, our Gauss-Newton optimum is
  unique (multi-start) and KKT-stationary, yet the stored fixes differ by
  1.5-4 m (B) and 2-31 m (A, whose ~-186 m/s clock drift the model's prior on the
  drift rate cannot follow: A's pseudorange residuals reach 500 m).  The check
  below only guards the script semantics (e.g. using all 12 slots instead of
  N_sat = 10 moves every fix by ~900 m).
"""
import os

import numpy as np
import pytest

from general_problems import TWO_RX, two_rx_mhe_facade, two_rx_mhe_oracle

REF_DATA = "/root/reference/data/gnss-multi-receiver"


def _synthetic(golden):
    fx = golden["least_squares"]
    d, ls = {}, {}
    for tag in ("A", "B"):
        cnt = fx[f"{tag}_count"]
        T = cnt.shape[0]
        d[tag] = {"t": fx[f"{tag}_t"].copy(),
                  "sat_pos": [fx[f"{tag}_sat_pos"][k, :cnt[k]] for k in range(T)],
                  "pr": [fx[f"{tag}_pr"][k, :cnt[k]] for k in range(T)]}
        ls[tag] = {k: fx[f"{tag}_ls_{k}"] for k in ("x_ENU", "y_ENU", "z_ENU", "bias", "xd_ENU", "yd_ENU", "zd_ENU")}
    pa = np.stack([ls["A"][k] for k in ("x_ENU", "y_ENU", "z_ENU")], 1)
    pb = np.stack([ls["B"][k] for k in ("x_ENU", "y_ENU", "z_ENU")], 1)
    dist = float(np.mean(np.linalg.norm(pa - pb, axis=1)))  # a range measurement consistent with the logs
    return d["A"], d["B"], ls["A"], ls["B"], fx["p_ref"], {"distance": dist}


@pytest.mark.gpu
def test_two_receiver_mhe_facade_matches_oracle(golden):
    from utils import utils as gu
    dA, dB, lsA, lsB, p_ref, ov = _synthetic(golden)
    nw = 12
    XT, XD, st = two_rx_mhe_facade(dA, dB, lsA, lsB, p_ref, nw, overrides=ov)
    RT, RD, rst = two_rx_mhe_oracle(dA, dB, lsA, lsB, p_ref, nw, lambda s: gu.ecef2enu(s, p_ref), overrides=ov)
    assert all(s == "Solve_Succeeded" for s in st) and (rst == 0).all()
    scale = 1 + np.abs(RT).max()
    assert np.abs(XT - RT).max() <= 1e-6 * scale, np.abs(XT - RT).max(axis=1)
    assert np.abs(XD - RD).max() <= 1e-6 * scale
    assert np.abs(XT[:, 2] - XT[:, 7]).max() <= 1e-9 * scale   # zA = zB holds (every node, so at t = T)


@pytest.mark.skipif(not os.path.isdir(REF_DATA), reason="reference data not present (GPU box)")
def test_oracle_replica_consistent_with_stored_ipopt_results():
    from oracle import leastsquares as ols
    from utils import data as gd, utils as gu
    dA = gd.load_gnss_logs(REF_DATA + "/rec1/rec1_gnss_log_50y_moving_")
    dB = gd.load_gnss_logs(REF_DATA + "/rec2/rec2_gnss_log_50y_moving_")
    p_ref = gu.lla2ecef(np.array([37.4276, -122.1670, 0.0]))
    tA, tB = np.asarray(dA["t"], float), np.asarray(dB["t"], float)
    t0 = min(tA.min(), tB.min())
    dA["t"], dB["t"] = tA - t0, tB - t0
    x = np.zeros(3)

    def ls(d):
        o = ols.run_least_squares(d["sat_pos"], d["pr"], d["sat_vel"], d["pr_rate"], x=x)
        e = np.array([gu.ecef2enu(p, p_ref) for p in o["x"]])
        v = np.array([gu.ecef2enu(q, p_ref, rotation_only=True) for q in o["v"]])
        return {"x_ENU": e[:, 0], "y_ENU": e[:, 1], "z_ENU": e[:, 2], "bias": o["b"],
                "xd_ENU": v[:, 0], "yd_ENU": v[:, 1], "zd_ENU": v[:, 2]}

    lsA, lsB = ls(dA), ls(dB)
    nw = 8
    XT, _, st = two_rx_mhe_oracle(dA, dB, lsA, lsB, p_ref, nw, lambda s: gu.ecef2enu(s, p_ref))
    assert (st == 0).all()
    for sl, f, lim in ((slice(0, 3), "NLP_A.csv", 40.0), (slice(5, 8), "NLP_B.csv", 6.0)):
        ll = np.array([gu.ecef2lla(gu.enu2ecef(p, p_ref))[:2] for p in XT[:, sl]])
        ref = np.loadtxt(f"{REF_DATA}/{f}", delimiter=",")[:nw]
        err_m = np.abs(ll - ref).max(axis=1) * 1.11e5
        assert err_m.max() < lim, (f, err_m)
