"""mhe_resjac: the per-collocation-point residual and Jacobian evaluation (SURVEY §8(a)
a5-a7) on the GPU vs the oracle's restated plug-ins, element by element.

Tolerance (<= 1e-14 relative): W_k = a sum_j D_kj X_j - f sums P terms
in another order, so |dW| <= 64 eps (a sum_j |D_kj| |X_j| + |f|) per entry; F, H are
closed-form (<= 16 eps of the entry's scale); e = y - h cancels in any order, so
|de| <= 8 eps (|y| + |h|).
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

from mhe import configs, solver  # noqa: E402
from oracle import gn, models  # noqa: E402

EPS = np.finfo(np.float64).eps


def _cases():
    yield "c2_n100", configs.make_c2(B=5, N=100), {}
    yield "c2_n150_big", configs.make_c2(B=3, N=150), {}
    yield "gnss_small", configs.make_gnss_small(B=3), {}
    yield "c3_real_geometry_big", configs.make_c3(B=2), {}
    yield "c4_big", configs.make_c4(B=1), {}


@pytest.mark.parametrize("name,w,kw", list(_cases()), ids=lambda v: v if isinstance(v, str) else "")
def test_resjac_matches_oracle(name, w, kw):
    s = solver.from_workload(w, **kw)
    W, F, E, Hm = (t.cpu().numpy() for t in s.resjac(w.X_init, w.U, w.Y, w.PAR))
    pb = gn.Problem(w.N, w.T, w.n, w.m, w.dyn, w.meas, w.cpm.D, (w.T / 2) * w.cpm.w,
                    w.cpm.lagrange_matrix(w.t_meas), w.Qw, w.Rw, meas_static=w.meas_static)
    U = np.broadcast_to(w.U, (w.B,) + w.U.shape[1:])
    PAR = None if w.PAR is None else np.broadcast_to(w.PAR, (w.B,) + w.PAR.shape[1:])
    f, Fr = models.dyn_eval(w.dyn, w.X_init, U)
    Wr = pb.alpha * np.einsum("kj,bja->bka", pb.D, w.X_init) - f
    scale_W = pb.alpha * np.einsum("kj,bja->bka", np.abs(pb.D), np.abs(w.X_init)) + np.abs(f)
    xi = np.einsum("ij,bja->bia", pb.Phi, w.X_init)
    h, Hr = models.meas_eval(w.meas, xi, PAR, w.meas_static)
    live = ~gn.masked_rows(pb.Rw if pb.Rw.ndim == 4 else pb.Rw[None])[0]      # R = 0 slots: h undefined there
    Er = w.Y - h
    dW = np.abs(W - Wr) / scale_W.clip(1e-300)
    dF = np.abs(F - Fr).max() / max(1.0, np.abs(Fr).max())
    dE = (np.abs(E - Er) / (np.abs(w.Y) + np.abs(h)).clip(1e-300))[:, live]
    dH = np.abs(Hm - Hr)[:, live].max() / max(1.0, np.abs(Hr).max())
    print(f"{name}: W {dW.max() / EPS:.1f} eps, F {dF / EPS:.1f} eps, e {dE.max() / EPS:.1f} eps, "
          f"H {dH / EPS:.1f} eps (relative to each entry's scale)")
    assert dW.max() <= 64 * EPS and dF <= 16 * EPS and dE.max() <= 8 * EPS and dH <= 16 * EPS
