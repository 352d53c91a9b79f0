"""GNSS loaders and geodesy (utils.data / utils.utils) against the reference's outputs.

Fixture: tests/golden/gnss_io.npz + the reduced logs gnss_small*_*.mat written by
tests/golden/gen_golden.py (the reference load_gnss_logs / utils.py run on them).
Index, slot and mask work: bit-exact.  Pseudorange corrections: bit-exact (same
arithmetic).  Geodesy: <= 1e-9 relative (3x3 rotations may sum in another order)."""
import os

import numpy as np

from utils import data as gdata
from utils import utils as gutils

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _fx():
    return np.load(os.path.join(G, "gnss_io.npz"))


def test_load_gnss_logs_2d_and_3d_match_reference():
    z = _fx()
    for tag, pre in (("d2", "gnss_small_"), ("d3", "gnss_small3_")):
        d = gdata.load_gnss_logs(os.path.join(G, pre))
        pk = gdata.pack_epochs(d, slots=12)
        np.testing.assert_array_equal(pk["count"], z[f"{tag}_count"])
        np.testing.assert_array_equal(pk["sat_pos"], z[f"{tag}_sat_pos"])
        np.testing.assert_array_equal(pk["pr"], z[f"{tag}_pr"])
        np.testing.assert_array_equal(np.asarray(list(d["t"]), dtype=np.float64), z[f"{tag}_t"])
        np.testing.assert_array_equal(np.asarray(d["sats"], dtype=np.float64), z[f"{tag}_sats"])
        if tag == "d3":
            for k in range(len(d["pr"])):
                c = z["d3_count"][k]
                np.testing.assert_array_equal(d["sat_vel"][k], z["d3_sat_vel"][k, :c])
                np.testing.assert_array_equal(d["pr_rate"][k], z["d3_pr_rate"][k, :c])
        assert (pk["mask"].sum(1) == pk["count"]).all()


def test_slot_weights_zero_for_empty_slots():
    z = _fx()
    w = gdata.slot_weights(z["d2_count"], 12, 0.01)
    for k, c in enumerate(z["d2_count"]):
        assert (w[k, :c] == 0.01).all() and (w[k, c:] == 0.0).all()


def test_geodesy_matches_reference():
    z = _fx()
    ecef = gutils.lla2ecef(z["geo_lla_in"])
    assert np.abs(ecef - z["geo_ecef"]).max() <= 1e-9 * np.abs(z["geo_ecef"]).max()
    back = gutils.ecef2lla(z["geo_ecef"])
    assert np.abs(back - z["geo_lla_back"]).max() <= 1e-9 * np.abs(z["geo_lla_back"]).max()
    ref = z["geo_ecef"][0]
    enu = gutils.ecef2enu(z["geo_pts"], ref)
    assert np.abs(enu - z["geo_enu"]).max() <= 1e-9 * np.abs(z["geo_pts"] - ref).max()
    rot = gutils.ecef2enu(z["geo_pts"], ref, rotation_only=True)
    assert np.abs(rot - z["geo_enu_rot"]).max() <= 1e-9 * np.abs(z["geo_pts"]).max()
    e2e = gutils.enu2ecef(z["geo_enu"], ref)
    assert np.abs(e2e - z["geo_enu2ecef"]).max() <= 1e-9 * np.abs(ref).max()
    # single-point calls keep the reference's shapes
    assert gutils.ecef2enu(z["geo_pts"][0], ref).shape == (3,)
    assert np.all(np.isnan(gutils.ecef2lla(np.zeros(3))))


def test_get_time_indices_bit_exact():
    z = _fx()
    np.testing.assert_array_equal(gutils.get_time_indices(z["ti_t"], 20.0, 35.5), z["ti_idx"])
