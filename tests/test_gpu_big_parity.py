"""Kernel-level parity of the LARGE-SYSTEM path (csrc/mhe_big.h), through the C-ABI
(mhe_assemble_ws / mhe_chol_solve_ws, ABI v5) at the C3, C4 and C5 shapes.

The iterate checks of tests/test_gpu_configs.py are conditioning-limited at C4 (moving H
by eps moves X by ~1 mm at N = 500).  These checks are not: they test the two kernels
that carry C3-C5 directly.

* k_big_resid + k_big_assemble: H and g at the configs' initial iterates vs the oracle's
  normal equations of the reference objective (nlp/nlp.py:242-273; oracle.gn /
  oracle.gn_general), both in node-major order (the binding permutes the kernels'
  component-major tiles; padding nodes last).  H entrywise, scaled by the SPD bound
  |H_ij| <= sqrt(H_ii H_jj):  |dH_ij| <= 1e-12 sqrt(H_ii H_jj)  -- a 1e-7 relative error in
  any entry of any tile fails.  g: <= 8 floor_g + 1e-12 max|g| (floor_g: the oracle's own
  change when every y moves by eps|y|, the rounding of y - h at |y| ~ 2e7 m).
* k_big_chol (blocked Cholesky + both triangular solves): the normwise backward error of
  delta = -H^-1 g on the device's own H, eta = ||H delta + g|| / (||H|| ||delta|| + ||g||)
  (residual in extended precision) <= 64 eps -- independent of cond(H).
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

from mhe import configs, solver  # noqa: E402
from oracle import gn  # noqa: E402
from oracle import gn_general as gg  # noqa: E402

import tolerance as tl  # noqa: E402
from big_oracle import backward_error as _backward_error, c5_normal_epochs as _c5_normal_epochs  # noqa: E402
from big_oracle import c5_problem as _c5_pb, g_rounding_floor  # noqa: E402

EPS = np.finfo(np.float64).eps


def _np(ts):
    return [t.cpu().numpy() for t in ts]


def _pb(w):
    return gn.Problem(w.N, w.T, w.n, w.m, w.dyn, w.meas, w.cpm.D, (w.T / 2) * w.cpm.w,
                      w.cpm.lagrange_matrix(w.t_meas), w.Qw, w.Rw, Pw=w.Pw, meas_static=w.meas_static)


def _bcast(a, B):
    return None if a is None else np.broadcast_to(a, (B,) + a.shape[1:])


def _check_H(name, H, Hr):
    d = Hr.shape[-1]
    Hd = H[:, :d, :d]
    dg = np.sqrt(np.abs(np.einsum("bii->bi", Hr)))
    scaled = np.abs(Hd - Hr) / (dg[:, :, None] * dg[:, None, :])
    print(f"{name}: max |dH| / sqrt(H_ii H_jj) {scaled.max():.3e}; max |dH| / max|H| "
          f"{np.abs(Hd - Hr).max() / np.abs(Hr).max():.3e}; asymmetry {np.abs(H - np.swapaxes(H, 1, 2)).max():.1e}")
    tl.check(f"{name} H (diagonal-scaled)", scaled.max(), 1e-12)
    assert np.array_equal(H, np.swapaxes(H, 1, 2))  # both triangles from the same tile element


def _check_padding(H, g, d):
    dp = H.shape[-1]
    if dp > d:
        assert np.array_equal(H[:, d:, d:], np.broadcast_to(np.eye(dp - d), H[:, d:, d:].shape))
        assert not H[:, :d, d:].any() and not H[:, d:, :d].any() and not g[:, d:].any()


def _check_solve(name, s, H, g):
    delta, status = _np(s.chol_solve(H, g))
    assert status.tolist() == [0] * H.shape[0]
    for b in range(H.shape[0]):
        eta = _backward_error(H[b], g[b], delta[b])
        tl.check(f"{name} solve backward error [{b}]", eta, 64 * EPS)


def _assemble_vs_oracle(name, w, B=2):
    s = solver.from_workload(w)
    assert s.large_system
    H, g, cost, status = _np(s.assemble(w.X_init, w.U, w.Y, w.PAR, status_out=True))
    assert status.tolist() == [0] * B
    pb = _pb(w)
    run = lambda Y: gn.normal_equations(pb, w.X_init, _bcast(w.U, B), Y, _bcast(w.PAR, B))  # noqa: E731
    Hr, gr, cr = run(w.Y)
    _, fg, fc = tl.floor(lambda Y, pt: run(Y), w.Y, conditioning=False)
    d = pb.d
    _check_H(name, H, Hr)
    # g entry by entry against its own rounding level (big_oracle.g_rounding_floor)
    gb = tl.FLOOR_MULT * g_rounding_floor(pb, w.X_init, w.Y, _bcast(w.PAR, B), _bcast(w.U, B)) + 1e-12 * np.abs(gr).max()
    print(f"{name} g: max |dg| {np.abs(g[:, :d] - gr).max():.3e}, random-eps floor {fg:.3e}, "
          f"first-order floor {np.max(gb):.3e}")
    tl.check(f"{name} g (entrywise / bound)", (np.abs(g[:, :d] - gr) / gb).max(), 1.0)
    tl.check(f"{name} cost", np.abs(cost - cr).max(), tl.FLOOR_MULT * fc + 1e-12 * np.abs(cr).max())
    _check_padding(H, g, d)
    return s, H, g


def test_c3_assemble_and_solve():
    """C3 (gnss_stationary, N = 200, d = 1005, the log's real satellite epochs)."""
    s, H, g = _assemble_vs_oracle("C3", configs.make_c3(B=2))
    _check_solve("C3", s, H, g)


def test_c4_assemble_and_solve():
    """C4 (rc-car, N = 500, d = 3006, the reference's own px4 / GNSS logs)."""
    s, H, g = _assemble_vs_oracle("C4", configs.make_c4(B=2))
    _check_solve("C4", s, H, g)


def test_forced_large_assemble_equals_register_path():
    """C2 through both device paths: the same normal equations (node-major, padding
    aside) and the same solve, to 1e-12 / 64 eps."""
    w = configs.make_c2(B=3, N=100)
    sr, sb = solver.from_workload(w), solver.from_workload(w, force_large=True)
    assert not sr.large_system and sb.large_system
    Hr, gr, cr = _np(sr.assemble(w.X_init, w.U, w.Y))
    Hb, gb, cb = _np(sb.assemble(w.X_init, w.U, w.Y))
    d = w.P * w.n
    _check_H("C2 large vs register", Hb, Hr[:, :d, :d])
    assert np.abs(gb[:, :d] - gr[:, :d]).max() <= 1e-12 * np.abs(gr).max()
    assert np.abs(cb - cr).max() <= 1e-12 * np.abs(cr).max()
    _check_padding(Hb, gb, d)
    _check_solve("C2 large path", sb, Hb, gb)


def test_large_chol_solve_random_spd_and_non_spd():
    """k_big_chol on random SPD matrices (vs LAPACK) and on non-SPD / non-finite input."""
    w = configs.make_c3(B=1, N=60)
    s = solver.from_workload(w)
    assert s.large_system
    rng = np.random.default_rng(11)
    B, dp = 3, s.dp
    A = rng.normal(size=(B, dp, dp))
    H = A @ np.swapaxes(A, 1, 2) + dp * np.eye(dp)[None]
    g = rng.normal(size=(B, dp))
    delta, status = _np(s.chol_solve(H, g))
    ref = -np.linalg.solve(H, g[..., None])[..., 0]
    assert status.tolist() == [0] * B
    tl.check("random SPD solve", np.abs(delta - ref).max(), 1e-10 * np.abs(ref).max())
    for b in range(B):
        assert _backward_error(H[b], g[b], delta[b]) <= 64 * EPS
    H = np.stack([np.eye(dp)] * 3)
    H[1, dp // 2, dp // 2] = -1.0
    H[2, 3, 3] = np.nan
    delta, status = _np(s.chol_solve(H, np.ones((3, dp))))
    assert status.tolist() == [0, 2, 2]
    assert np.allclose(delta[0], -1.0) and np.isnan(delta[1:]).all()


def test_large_chol_solve_wide_split_spd_and_non_spd():
    """The wide-system factorization (C4 shape, NT = 188 tile columns: per block column a
    diagonal-stage launch and a k_big_rows launch, then the solve launch): a random SPD
    system against LAPACK, and a non-SPD pivot in a middle block column / a NaN in a late
    one -- the diagonal stage that meets it stops the trajectory, the later launches skip
    it, the others are unaffected."""
    w = configs.make_c4(B=1)
    s = solver.from_workload(w)
    assert s.large_system and s.dp // 16 >= 128
    rng = np.random.default_rng(12)
    dp = s.dp
    A = rng.normal(size=(dp, dp)) / np.sqrt(dp)
    H1 = A @ A.T + np.eye(dp)
    g1 = rng.normal(size=dp)
    H = np.stack([H1, np.eye(dp), np.eye(dp)])
    H[1, dp // 2, dp // 2] = -1.0
    H[2, dp - 20, dp - 20] = np.nan
    g = np.stack([g1, np.ones(dp), np.ones(dp)])
    delta, status = _np(s.chol_solve(H, g))
    assert status.tolist() == [0, 2, 2]
    ref = -np.linalg.solve(H1, g1)
    tl.check("wide random SPD solve", np.abs(delta[0] - ref).max(), 1e-10 * np.abs(ref).max())
    assert _backward_error(H1, g1, delta[0]) <= 64 * EPS
    assert np.isnan(delta[1:]).all()


def test_wide_split_non_spd_neighbours_leave_healthy_deltas_bitwise():
    """The split factorization's solve launch (k_big_chol SPLIT = 2) takes no flag from LDS
    (a flag left by an earlier workgroup could stop some waves of a healthy
    trajectory).  A batch alternating non-SPD and healthy SPD systems at the C4 shape: the
    healthy deltas are bitwise those of the one-launch right-looking kernel on the healthy
    systems alone, and the non-SPD ones are stopped."""
    from mhe import _lib
    w = configs.make_c4(B=1)
    s = solver.from_workload(w)
    assert s.large_system and s.dp // 16 >= 128
    rng = np.random.default_rng(13)
    dp, nh = s.dp, 4
    Hh, gh = [], []
    for _ in range(nh):
        A = rng.normal(size=(dp, dp)) / np.sqrt(dp)
        Hh.append(A @ A.T + np.eye(dp))
        gh.append(rng.normal(size=dp))
    H, g = [], []
    for i in range(nh):
        bad = np.eye(dp)
        bad[(i * 397) % dp, (i * 397) % dp] = -1.0  # a non-SPD pivot in a different block column each
        H += [bad, Hh[i]]
        g += [np.ones(dp), gh[i]]
    delta, status = _np(s.chol_solve(np.stack(H), np.stack(g)))
    assert status.tolist() == [2, 0] * nh
    try:
        assert s.lib.mhe_set_option(_lib.OPT_BIG_RIGHT_LOOKING, 1) >= 0
        ref, rst = _np(s.chol_solve(np.stack(Hh), np.stack(gh)))
    finally:
        s.lib.mhe_set_option(_lib.OPT_BIG_RIGHT_LOOKING, 0)
    assert rst.tolist() == [0] * nh
    assert np.array_equal(delta[1::2], ref)
    assert np.isnan(delta[0::2]).all()


def test_constants_of_other_dims_refused_by_parity_entry_points():
    w = configs.make_c3(B=2, N=60)
    s = solver.from_workload(w)
    other = solver.from_workload(configs.make_c3(B=2, N=61))
    s.cbuf, saved = other.cbuf, s.cbuf
    try:
        H, g, cost, status = _np(s.assemble(w.X_init, w.U, w.Y, w.PAR, status_out=True))
    finally:
        s.cbuf = saved
    assert status.tolist() == [solver.STATUS_BAD_CONSTANTS] * 2
    assert np.isnan(H).all() and np.isnan(g).all() and np.isnan(cost).all()


# ---------------------------------------------------------------- C5 (n = 40)
def _c5_assemble(w, s):
    H, g, cost, status = _np(s.assemble(w.X_init, w.U, w.Y, w.PAR, status_out=True))
    assert status.tolist() == [0] * w.B
    return H, g, cost


def test_c5_reduced_assemble_vs_dense_oracle():
    """C5's structure (8 receivers, n = 40) at N = 10 (d = 440): H, g vs the row-by-row
    dense oracle -- which also pins the epoch-regrouped oracle used at full size."""
    w = configs.make_c5(B=2, N=10)
    s = solver.from_workload(w)
    assert s.large_system and s.n == 40
    H, g, cost = _c5_assemble(w, s)
    pb = _c5_pb(w)
    run = lambda Y: gg.normal_equations_full(pb, w.X_init, None, w.U, Y, w.PAR)  # noqa: E731
    Hr, gr, cr = run(w.Y)
    He, ge_, ce = _c5_normal_epochs(pb, w.X_init, w.U, w.Y, w.PAR)
    assert np.abs(He - Hr).max() <= 1e-12 * np.abs(Hr).max() and np.abs(ge_ - gr).max() <= 1e-12 * np.abs(gr).max()
    _, fg, fc = tl.floor(lambda Y, pt: run(Y), w.Y, conditioning=False)
    d = pb.d
    _check_H("C5 N=10", H, Hr)
    tl.check("C5 N=10 g", np.abs(g[:, :d] - gr).max(), tl.FLOOR_MULT * fg + 1e-12 * np.abs(gr).max())
    tl.check("C5 N=10 cost", np.abs(cost - cr).max(), tl.FLOOR_MULT * fc + 1e-12 * np.abs(cr).max())
    _check_padding(H, g, d)
    _check_solve("C5 N=10", s, H, g)


def test_c5_full_shape_assemble_and_solve():
    """C5 at the shape SURVEY §8(d) names (N = 200, n = 40, d = 8040), one trajectory:
    H, g vs the epoch-regrouped oracle and the solve's backward error."""
    w = configs.make_c5(B=1)
    s = solver.from_workload(w)
    assert s.dp == 40 * 208
    H, g, cost = _c5_assemble(w, s)
    pb = _c5_pb(w)
    run = lambda Y: _c5_normal_epochs(pb, w.X_init, w.U, Y, w.PAR)  # noqa: E731
    Hr, gr, cr = run(w.Y)
    fg, fc = tl.floor(lambda Y, pt: run(Y)[1:], w.Y, conditioning=False)
    d = pb.d
    _check_H("C5 d=8040", H, Hr)
    del Hr
    tl.check("C5 d=8040 g", np.abs(g[:, :d] - gr).max(), tl.FLOOR_MULT * fg + 1e-12 * np.abs(gr).max())
    tl.check("C5 d=8040 cost", np.abs(cost - cr).max(), tl.FLOOR_MULT * fc + 1e-12 * np.abs(cr).max())
    _check_padding(H, g, d)
    _check_solve("C5 d=8040", s, H, g)
