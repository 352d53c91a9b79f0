"""C4's inputs from the reference's rc-car logs (tests/golden/rc_car_c4.npz):
the px4 controls read from the .ulg with gen_golden.read_ulog and processed as
px4/convert.py and rc-car.py:25-37, the satellite epochs through the reference's own
load_gnss_logs.  CPU only; where /root/reference is present (build container) the
fixture is regenerated and must be bit-identical."""
import os

import numpy as np
import pytest

from mhe import configs

REF = "/root/reference/data/rc-car"


def test_fixture_shapes_and_ranges():
    z = configs.rc_car_inputs()
    assert list(z["ulog_columns"]) == ["timestamp", "x", "y", "z", "r"]   # ulog2csv columns 0..4
    t, u = z["t_u"], z["u"]
    assert t[0] == 0.0 and np.all(np.diff(t) > 0) and 100.0 < t[-1] < 110.0
    assert u.shape == (2, t.size) and np.all(np.isfinite(u))
    assert np.all((u[0] == 0.0) | (u[0] >= 0.1))                          # rc-car.py:25-28
    assert abs(u[1, 0]) < 0.01                                             # rc-car.py:30-35 start
    tg, sat, cnt = z["t_gnss"], z["sat_enu"], z["count"]
    assert tg[0] == 0.0 and np.all(np.diff(tg) > 0) and sat.shape == (tg.size, 12, 3)
    assert cnt.min() >= 4 and cnt.max() <= 12
    live = np.arange(12)[None, :] < cnt[:, None]
    r = np.linalg.norm(sat, axis=-1)
    assert np.all((r[live] > 1.9e7) & (r[live] < 2.7e7)) and np.all(r[~live] == 0.0)


def test_c4_workload_uses_the_logs():
    w = configs.make_c4(B=3)
    z = configs.rc_car_inputs()
    assert w.N == 500 and w.P * w.n == 3006 and w.T == 100.0 and w.M == 101 * 12
    live = (np.arange(12)[None, :] < z["count"][:101, None]).reshape(-1)
    assert np.array_equal(w.Rw[:, 0, 0] > 0, live) and np.all(w.Y[:, ~live, 0] == 0.0)
    assert np.array_equal(w.PAR[0].reshape(101, 12, 3), z["sat_enu"][:101])
    from scipy.interpolate import interp1d
    U = interp1d(z["t_u"], z["u"], fill_value="extrapolate")(w.cpm.tau2t(w.cpm.tau)).T
    assert np.array_equal(w.U[0], U)      # setControl's interpolation of the logged controls


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference data not present (GPU box)")
def test_fixture_regenerates_from_the_reference_logs(tmp_path):
    import sys
    here = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    sys.path.insert(0, here)
    try:
        import gen_golden as g
        out = g.OUT
        g.OUT = str(tmp_path)
        try:
            g.gen_rc_car_c4(g.load_reference())
        finally:
            g.OUT = out
    finally:
        sys.path.remove(here)
    a, b = np.load(tmp_path / "rc_car_c4.npz"), configs.rc_car_inputs()
    for k in b.files:
        assert np.array_equal(a[k], b[k]), k
