"""GNSS logs on disk -> fixed-slot device layout -- kingdwd/nlp-filter utils/data.py:9-75
and the 12-slot measurement packing of autonomous-car.py:245-263.

``load_gnss_logs(prefix)`` returns the reference's dict (per-epoch ragged lists,
ionosphere and satellite-clock corrections applied, empty / NaN slots dropped).
``pack_epochs`` turns it into the batch-outermost arrays the kernels read:
satellite ENU positions (T, S, 3), pseudoranges (T, S), a validity mask and
per-epoch counts; unused slots carry zeros, and ``slot_weights`` gives them
weight 0 (R = 0) exactly as the reference MHE does.
"""
import numpy as np
from scipy.io import loadmat

from .utils import ecef2enu

C = 299792458  # speed of light (m/s)


def load_gnss_logs(prefix):
    """prefix + 'satposecef.mat' (svPoss: row 0 = SVIDs, then [x, y, z, ion m, clock s])
    and prefix + 'ranges.mat' (pseudoranges (T+1, S) or (T+1, S, 5|6): range, rate,
    velocity xyz[, time])."""
    sv = loadmat(prefix + "satposecef.mat")["svPoss"]
    sat_pos_all = sv[1:, :, :3]
    ion = sv[1:, :, 3]
    clk = sv[1:, :, 4]
    raw = loadmat(prefix + "ranges.mat")["pseudoranges"]
    pos_only = raw.ndim == 2
    if pos_only:
        pr_all = raw[1:, :] + ion + C * clk
        sats = raw[0, :]
        times = range(pr_all.shape[0])
    else:
        pr_all = raw[1:, :, 0] + ion + C * clk
        rate_all = raw[1:, :, 1]
        vel_all = raw[1:, :, 2:5]
        times = np.max(raw[1:, :, 5], axis=1) if raw.shape[2] == 6 else range(pr_all.shape[0])
        sats = raw[0, :, 0]
    keep = ~np.all(sat_pos_all == 0.0, axis=2) & ~np.isnan(pr_all)  # (T, S)
    data = {"t": times, "sats": sats,
            "sat_pos": [sat_pos_all[k][keep[k]].reshape(-1, 3) for k in range(pr_all.shape[0])],
            "pr": [pr_all[k][keep[k]] for k in range(pr_all.shape[0])]}
    if not pos_only:
        data["sat_vel"] = [vel_all[k][keep[k]].reshape(-1, 3) for k in range(pr_all.shape[0])]
        data["pr_rate"] = [rate_all[k][keep[k]] for k in range(pr_all.shape[0])]
    return data


def pack_epochs(data, p_ref_ECEF=None, slots=12, epochs=None):
    """Fixed-slot layout of the selected epochs (default: all).  Satellite positions
    are converted to ENU at p_ref_ECEF when given.  Returns a dict of arrays:
    sat_pos (T, slots, 3), pr (T, slots), count (T,) int32, mask (T, slots) bool."""
    ks = range(len(data["pr"])) if epochs is None else epochs
    ks = list(ks)
    T = len(ks)
    sp = np.zeros((T, slots, 3))
    pr = np.zeros((T, slots))
    cnt = np.zeros(T, dtype=np.int32)
    for r, k in enumerate(ks):
        c = min(len(data["pr"][k]), slots)
        cnt[r] = c
        pos = np.asarray(data["sat_pos"][k][:c], dtype=np.float64)
        sp[r, :c] = ecef2enu(pos, p_ref_ECEF) if (p_ref_ECEF is not None and c) else pos
        pr[r, :c] = data["pr"][k][:c]
    mask = np.arange(slots)[None, :] < cnt[:, None]
    return {"sat_pos": sp, "pr": pr, "count": cnt, "mask": mask}


def slot_weights(count, slots, w):
    """Per-slot measurement weight (R^-1 entries): w for occupied slots, 0 for the
    empty ones (autonomous-car.py:250-263).  Returns (T, slots)."""
    count = np.asarray(count)
    return np.where(np.arange(slots)[None, :] < count[:, None], float(w), 0.0)
