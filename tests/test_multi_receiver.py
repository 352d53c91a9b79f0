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
* Against the reference's stored results, read in place when /root/reference is
  present (build container):
  - the least-squares fixes the script feeds the NLP (controls, first prior) match
    the stored LS_{A,B}.csv to 1e-7 m -- the data pipeline is the reference's;
  - the stored IPOPT fixes NLP_{A,B}.csv are not the optimum of the objective the
    script builds: with A's and B's horizontal positions held at the stored values
    and everything else re-minimised, the objective sits 586 above the unique optimum
    that the oracle and the GPU reach in window 0 (identical inputs and prior on both
    sides; J* = 1.1e6 -- receiver A's ~400 m pseudorange misfit dominates), and the
    objective's gradient on the held coordinates is ~190 per metre there, so no
    stationary point has those positions.  At a point converged to IPOPT's tol the excess would be second
    order in the ~1e-8 scaled dual infeasibility; 5e-4 of J is what termination away
    from stationarity leaves (CasADi's Opti accepts IPOPT's "Solved To Acceptable
    Level", whose default acceptable_dual_inf_tol is 1e10).  Named cause of the
    4 m (A) / 3.5 m (B) window-0 difference; later windows inherit different priors.
    tools/diag_multirx.py prints the per-window table (profiles/r03_multirx_gap.txt).
  - the same window-0 numbers on the REFERENCE's own objective (its nlp.py evaluated
    through tests/golden/casadi_lazy.py, tests/golden/objective.npz): J* = 1 101 297.97,
    J_c - J* = 585.78, and the reference J's gradient in the held coordinates at the
    stored fixes (xA, yA, xB, yB) = (63.7, -177.1, 28.6, -120.9) per m
    (tests/test_objective_pin.py); the replica's values below agree with them.
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


def _ref_inputs():
    from oracle import leastsquares as ols
    from utils import data as gd, utils as gu
    dA = gd.load_gnss_logs(REF_DATA + "/rec1/rec1_gnss_log_50y_moving_")
    dB = gd.load_gnss_logs(REF_DATA + "/rec2/rec2_gnss_log_50y_moving_")
    p_ref = gu.lla2ecef(np.array([37.4276, -122.1670, 0.0]))
    tA, tB = np.asarray(dA["t"], float), np.asarray(dB["t"], float)
    t0 = min(tA.min(), tB.min())
    dA["t"], dB["t"] = tA - t0, tB - t0
    x = np.zeros(3)   # the reference's shared mutable default warm start (utils/leastsquares.py:19)
    outs = {}
    for tag, d in (("A", dA), ("B", dB)):
        outs[tag] = ols.run_least_squares(d["sat_pos"], d["pr"], d["sat_vel"], d["pr_rate"], x=x)
    return dA, dB, p_ref, outs


@pytest.mark.skipif(not os.path.isdir(REF_DATA), reason="reference data not present (GPU box)")
def test_least_squares_inputs_match_stored_ls_csv():
    from utils import utils as gu
    _, _, _, outs = _ref_inputs()
    for tag in ("A", "B"):
        lla = np.array([gu.ecef2lla(p) for p in outs[tag]["x"]])[:, :2]
        ref = np.loadtxt(f"{REF_DATA}/LS_{tag}.csv", delimiter=",")
        err_m = np.abs(lla - ref).max() * 1.11e5
        print(f"LS_{tag}: max {err_m:.2e} m over {len(ref)} epochs")
        assert lla.shape == ref.shape and err_m < 1e-7


@pytest.mark.skipif(not os.path.isdir(REF_DATA), reason="reference data not present (GPU box)")
def test_stored_ipopt_fixes_are_not_stationary_for_the_script_objective():
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    import diag_multirx
    line = diag_multirx.main(1)[0]
    js, jc = (float(v) for v in (line.split("J* = ")[1].split(" ")[0], line.split("J_c = ")[1].split(" ")[0]))
    gap = jc - js
    print(line)
    assert "(status 0)" in line and "J_c" in line
    # the unique optimum (oracle) is lower than anything consistent with the stored fixes by far
    # more than rounding (~1e-9 J) or a tol-converged interior-point solve could leave
    assert gap > 1e-5 * js, gap
    # ... and so is the reference's own objective (nlp.py evaluated at the same points;
    # the replica's least-squares inputs differ from the reference's by ~1e-8 m)
    z = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "objective.npz"))
    js_ref, jc_ref = float(z["tworx_Js_ref"]), float(z["tworx_Jc_ref"])
    print(f"reference J: J* = {js_ref:.6f}, J_c - J* = {jc_ref - js_ref:.4f}")
    assert abs(js - js_ref) <= 1e-8 * js_ref and abs(gap - (jc_ref - js_ref)) <= 1e-3 * gap
