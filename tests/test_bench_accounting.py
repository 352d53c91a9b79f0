"""bench.py accounting (CPU): the roofline flop basis is SURVEY.md §8(d)'s count, the
executed count is the kernel's own, and the C2 workload is the BASELINE.json shape."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from mhe import configs  # noqa: E402


def test_survey_flop_count_matches_section_8d_table():
    # C2 d=202 -> 4.98 MFLOP per trajectory-iteration (Cholesky 2.75,
    # measurement 2.06, dynamics 0.085), 49.3 KFLOP per collocation point
    f = bench.survey_flops_per_traj_iter(101, 2, 101, 2)
    assert abs(f / 1e6 - 4.975) < 5e-3
    assert abs(f / 101 / 1e3 - 49.3) < 0.1
    d = 202
    assert abs((d ** 3 / 3 + 2 * d * d) / 1e6 - 2.83) < 0.01


def test_executed_count_below_survey_count():
    # the kernel precomputes the constant measurement contraction (linear h)
    assert bench.algorithmic_flops_per_traj_iter(101, 2, 101) < bench.survey_flops_per_traj_iter(101, 2, 101, 2)


def test_c2_workload_is_the_baseline_shape():
    w = configs.make_c2(B=4)
    assert (w.n, w.m, w.p, w.N, w.M, w.P) == (2, 1, 2, 100, 101, 101)
    assert w.dyn == "van_der_pol" and w.meas == "full_state"
    assert np.count_nonzero(np.diag(w.Rw[0])) == 2
