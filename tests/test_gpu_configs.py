"""The C4 (rc-car) and C5 (multi-receiver) workload shapes of BASELINE.json on the
large-system path, against the oracle.

* C4 at full size (N=500, d=3006, 501 epochs x 12 pseudoranges): two GN iterations
  vs oracle.gn (structured normal equations, LAPACK Cholesky), tolerance
  8 floor + 1e-10 (1 + max|X|) (tests/tolerance.py: floor = the oracle's own change
  when every y, or every entry of H and g, moves by eps of its magnitude) -- ~1 cm
  here: moving H by eps moves X by ~1 mm at N = 500 (cond(H)), whatever the order.
* C5 (mixed rows: pseudorange, pseudorange rate, 2-D range to the extra variable
  XA): at N=30 two iterations vs oracle.gn_general (dense KKT, row by row --
  too slow at N=200), same tolerance; at the full N=200 shape size-independent properties: all
  trajectories converge (the GN step itself, max|delta| <= tol (1 + max|X|), is the
  stationarity check), the cost ends below its start (undamped GN need not decrease
  it monotonically), XA[2] (no row depends on it) is held bit-exactly, and the
  synthetic truth is recovered to the noise level.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

from mhe import configs, solver  # noqa: E402
from oracle import gn  # noqa: E402
from oracle import gn_general as gg  # noqa: E402

import tolerance as tl  # noqa: E402


def _np(ts):
    return [t.cpu().numpy() for t in ts]


def test_c4_full_shape_matches_oracle():
    w = configs.make_c4(B=2)
    s = solver.from_workload(w)
    assert s.large_system
    X, cost, iters, status = _np(s.solve(w.X_init, w.U, w.Y, w.PAR, max_iter=2, tol=0.0))
    pb = gn.Problem(w.N, w.T, w.n, w.m, w.dyn, w.meas, w.cpm.D, (w.T / 2) * w.cpm.w,
                    w.cpm.lagrange_matrix(w.t_meas), w.Qw, w.Rw, meas_static=w.meas_static)
    PAR = np.broadcast_to(w.PAR, (w.B,) + w.PAR.shape[1:])
    run = lambda Y, pt=None: gn.gauss_newton(pb, w.X_init, w.U, Y, PAR, max_iter=2, tol=0.0, perturb=pt)  # noqa: E731
    Xr, cr, ir, sr = run(w.Y)
    fx, fc = tl.floor(lambda Y, pt: run(Y, pt)[:2], w.Y)
    assert iters.tolist() == ir.tolist() == [2, 2] and status.tolist() == sr.tolist()
    b = tl.bound(fx, Xr)
    tl.check("C4 X", np.abs(X - Xr).max(), b, " m")   # floor ~1 mm: H's conditioning at N = 500
    tl.check("C4 cost", np.abs(cost - cr).max(), tl.FLOOR_MULT * fc + 1e-10 * np.abs(cr).max())


def _c5_solver(w):
    s = solver.from_workload(w)
    assert s.large_system and s.n_extra == 3
    return s


def test_c5_reduced_matches_kkt_oracle():
    w = configs.make_c5(B=2, N=30)
    s = _c5_solver(w)
    X, cost, iters, st, Z = _np(s.solve(w.X_init, None, w.Y, w.PAR, max_iter=2, tol=0.0, Z0=w.Z_init))
    pb = gg.GeneralProblem(w.N, w.T, w.n, w.m, w.dyn, "mixed", w.cpm.D, (w.T / 2) * w.cpm.w,
                           w.cpm.lagrange_matrix(w.t_meas), w.Qw, w.Rw, n_extra=3)
    run = lambda Y, pt=None: gg.gauss_newton_general(pb, w.X_init, w.Z_init, None, Y, w.PAR, None,  # noqa: E731
                                            max_iter=2, tol=0.0, perturb=pt)
    Xr, Zr, cr, ir, sr = run(w.Y)
    fx, fz, fc = tl.floor(lambda Y, pt: run(Y, pt)[:3], w.Y)
    assert iters.tolist() == ir.tolist() == [2, 2] and st.tolist() == sr.tolist()
    bx, bz = tl.bound(fx, Xr), tl.bound(fz, Zr)
    tl.check("C5 X", np.abs(X - Xr).max(), bx, " m")
    tl.check("C5 Z", np.abs(Z - Zr).max(), bz, " m")
    assert max(bx, bz) < 1e-4
    tl.check("C5 cost", np.abs(cost - cr).max(), tl.FLOOR_MULT * fc + 1e-10 * np.abs(cr).max())


def test_c5_full_shape_properties():
    w = configs.make_c5(B=4)
    s = _c5_solver(w)
    X, c0, iters, st, Z = _np(s.solve(w.X_init, None, w.Y, w.PAR, max_iter=0, tol=0.0, Z0=w.Z_init))
    assert np.all(np.isfinite(c0)) and iters.tolist() == [0] * w.B
    X, cost, iters, st, Z = _np(s.solve(w.X_init, None, w.Y, w.PAR, max_iter=60, tol=1e-9, Z0=w.Z_init))
    assert st.tolist() == [0] * w.B, (st, iters)
    assert np.all(cost < c0)
    assert np.array_equal(Z[:, 2], w.Z_init[:, 2])          # XA[2] enters no row: held
    assert np.abs(X[:, :, :3] - w.X_true[:, :, :3]).max() < 10.0  # sigma_pr = 10 m
    assert np.abs(Z[:, :2] - w.Z_true[:, :2]).max() < 3.0
