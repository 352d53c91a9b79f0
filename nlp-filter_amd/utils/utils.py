"""Geodesy and time-window helpers -- kingdwd/nlp-filter utils/utils.py:4-110.

Host NumPy.  WGS-84 constants and Bowring latitude iteration as the reference;
functions accept one point (as the reference) or a stack of points (N, 3).
"""
import numpy as np

WGS84_A = 6378137.0
WGS84_F = 1.0 / 298.257223563


def ecef2lla(p_ECEF):
    """ECEF (m) -> [lat deg, lon deg, h m]; Bowring's method, 10 refinements at most
    (utils/utils.py:4-39).  The origin maps to NaNs as in the reference."""
    p = np.asarray(p_ECEF, dtype=np.float64)
    if p.ndim > 1:
        return np.stack([ecef2lla(q) for q in p])
    x, y, z = p[0], p[1], p[2]
    if x == 0.0 and y == 0.0 and z == 0.0:
        return np.nan, np.nan, np.nan
    a, f = 6378137, 1 / 298.257223563
    e2 = 2 * f - f ** 2
    s = np.sqrt(x ** 2 + y ** 2)
    beta = np.arctan(z / ((1 - f) * s))
    lat = np.arctan((z + a * np.sin(beta) ** 3 * (e2 * (1 - f) / (1 - e2))) / (s - e2 * a * np.cos(beta) ** 3))
    for _ in range(10):
        prev = lat
        beta = np.arctan((1 - f) * np.sin(lat) / (np.cos(lat)))
        lat = np.arctan((z + a * np.sin(beta) ** 3 * (e2 * (1 - f) / (1 - e2))) / (s - e2 * a * np.cos(beta) ** 3))
        if np.abs(prev - lat) < 1e-6:
            break
    rn = a / (np.sqrt(1 - e2 * np.sin(lat) ** 2))
    h = s * np.cos(lat) + (z + e2 * rn * np.sin(lat)) * np.sin(lat) - rn
    return np.array([np.rad2deg(lat), np.rad2deg(np.arctan2(y, x)), h])


def lla2ecef(p_LLA):
    """[lat deg, lon deg, h m] -> ECEF (m)  (utils/utils.py:42-56)."""
    p = np.asarray(p_LLA, dtype=np.float64)
    lat, lon, h = p[..., 0], p[..., 1], p[..., 2]
    a, finv = 6378137, 298.257223563
    e2 = 2 * (1 / finv) - (1 / finv) ** 2
    rn = a / (np.sqrt(1 - e2 * np.sin(np.deg2rad(lat)) ** 2))
    x = (rn + h) * np.cos(np.deg2rad(lat)) * np.cos(np.deg2rad(lon))
    y = (rn + h) * np.cos(np.deg2rad(lat)) * np.sin(np.deg2rad(lon))
    z = (rn * (1 - e2) + h) * np.sin(np.deg2rad(lat))
    return np.stack([x, y, z], axis=-1)


def _enu_rotation(p_ref_ECEF):
    lat_d, lon_d, _ = ecef2lla(p_ref_ECEF)
    lat, lon = np.deg2rad(lat_d), np.deg2rad(lon_d)
    return np.array([[-np.sin(lon), np.cos(lon), 0.0],
                     [-np.sin(lat) * np.cos(lon), -np.sin(lat) * np.sin(lon), np.cos(lat)],
                     [np.cos(lat) * np.cos(lon), np.cos(lat) * np.sin(lon), np.sin(lat)]])


def ecef2enu(p_ECEF, p_ref_ECEF, rotation_only=False):
    """ECEF -> ENU at p_ref (utils/utils.py:59-84); rotation_only for velocities.
    Accepts (3,) or (N, 3)."""
    R = _enu_rotation(p_ref_ECEF)
    p = np.asarray(p_ECEF, dtype=np.float64)
    v = p if rotation_only else p - np.asarray(p_ref_ECEF, dtype=np.float64)
    return v @ R.T if v.ndim > 1 else R @ v


def enu2ecef(p_ENU, p_ref_ECEF):
    """ENU at p_ref -> ECEF (utils/utils.py:87-104)."""
    R = _enu_rotation(p_ref_ECEF).T
    p = np.asarray(p_ENU, dtype=np.float64)
    ref = np.asarray(p_ref_ECEF, dtype=np.float64)
    return (p @ R.T if p.ndim > 1 else R @ p) + ref


def get_time_indices(t, t0, tf):
    """Indices i with t0 <= t[i] <= tf, ascending (utils/utils.py:107-110)."""
    t = np.asarray(t)
    return np.flatnonzero((t >= t0) & (t <= tf))
