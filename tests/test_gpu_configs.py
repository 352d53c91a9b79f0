"""The C4 (rc-car) and C5 (multi-receiver) workload shapes of BASELINE.json on the
large-system path, against the oracle.

* C4 at full size (N=500, d=3006, 501 epochs x 12 pseudoranges): two GN iterations
  vs oracle.gn (structured normal equations, LAPACK Cholesky), tolerance
  8 floor + 1e-10 (1 + max|X|) (tests/tolerance.py: floor = the oracle's own change
  when every y, or every entry of H and g, moves by eps of its magnitude) -- ~1 cm
  here: moving H by eps moves X by ~1 mm at N = 500 (cond(H)), whatever the order.
* C5 as SURVEY.md §8(d) defines it (8 receivers, n = 40, d = 8040 at N = 200; mixed
  pseudorange rows per receiver + range_3d between adjacent receivers): at N = 10
  (d = 440) two iterations vs oracle.gn_general (dense, row by row), same tolerance;
  at the full shape, properties (below) and batch chunking bit-identical to one launch.
* C5s (the reference's own multi-receiver.py structure, n = 8 + the extra variable XA;
  mixed rows: pseudorange, pseudorange rate, 2-D range to XA): at N=30 two iterations
  vs oracle.gn_general, same tolerance; at the full N=200 shape size-independent properties: all
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
    U = np.broadcast_to(w.U, (w.B,) + w.U.shape[1:])   # the rc-car controls, shared by the batch
    run = lambda Y, pt=None: gn.gauss_newton(pb, w.X_init, U, Y, PAR, max_iter=2, tol=0.0, perturb=pt)  # noqa: E731
    Xr, cr, ir, sr = run(w.Y)
    fx, fc = tl.floor(lambda Y, pt: run(Y, pt)[:2], w.Y)
    assert iters.tolist() == ir.tolist() == [2, 2] and status.tolist() == sr.tolist()
    b = tl.bound(fx, Xr)
    tl.check("C4 X", np.abs(X - Xr).max(), b, " m")   # floor ~1 mm: H's conditioning at N = 500
    tl.check("C4 cost", np.abs(cost - cr).max(), tl.FLOOR_MULT * fc + 1e-10 * np.abs(cr).max())


def test_c3_full_shape_real_geometry_matches_oracle():
    """C3 as SURVEY §8(d) specifies it: the satellite epochs of data/gnss_stationary's log
    (tests/golden/gnss_stationary_c3.npz; 57 empty slots masked with R = 0)."""
    w = configs.make_c3(B=2)
    s = solver.from_workload(w)
    assert s.large_system and (w.Rw == 0).any()
    X, cost, iters, status = _np(s.solve(w.X_init, w.U, w.Y, w.PAR, max_iter=3, tol=0.0))
    pb = gn.Problem(w.N, w.T, w.n, w.m, w.dyn, w.meas, w.cpm.D, (w.T / 2) * w.cpm.w,
                    w.cpm.lagrange_matrix(w.t_meas), w.Qw, w.Rw, meas_static=w.meas_static)
    U = np.broadcast_to(w.U, (w.B,) + w.U.shape[1:])
    PAR = np.broadcast_to(w.PAR, (w.B,) + w.PAR.shape[1:])
    run = lambda Y, pt=None: gn.gauss_newton(pb, w.X_init, U, Y, PAR, max_iter=3, tol=0.0, perturb=pt)  # noqa: E731
    Xr, cr, ir, sr = run(w.Y)
    fx, fc = tl.floor(lambda Y, pt: run(Y, pt)[:2], w.Y)
    assert iters.tolist() == ir.tolist() == [3, 3] and status.tolist() == sr.tolist()
    b = tl.bound(fx, Xr)
    tl.check("C3 X", np.abs(X - Xr).max(), b, " m")
    assert b < 1e-4
    tl.check("C3 cost", np.abs(cost - cr).max(), tl.FLOOR_MULT * fc + 1e-10 * np.abs(cr).max())


def _c5_solver(w):
    s = solver.from_workload(w)
    assert s.large_system and s.n_extra == 3
    return s


def test_c5s_reduced_matches_kkt_oracle():
    w = configs.make_c5_small(B=2, N=30)
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


def test_c5s_full_shape_properties():
    w = configs.make_c5_small(B=4)
    s = _c5_solver(w)
    X, c0, iters, st, Z = _np(s.solve(w.X_init, None, w.Y, w.PAR, max_iter=0, tol=0.0, Z0=w.Z_init))
    assert np.all(np.isfinite(c0)) and iters.tolist() == [0] * w.B
    X, cost, iters, st, Z = _np(s.solve(w.X_init, None, w.Y, w.PAR, max_iter=60, tol=1e-9, Z0=w.Z_init))
    assert st.tolist() == [0] * w.B, (st, iters)
    assert np.all(cost < c0)
    assert np.array_equal(Z[:, 2], w.Z_init[:, 2])          # XA[2] enters no row: held
    assert np.abs(X[:, :, :3] - w.X_true[:, :, :3]).max() < 10.0  # sigma_pr = 10 m
    assert np.abs(Z[:, :2] - w.Z_true[:, :2]).max() < 3.0


def _c5_pb(w):
    return gg.GeneralProblem(w.N, w.T, w.n, w.m, w.dyn, "mixed", w.cpm.D, (w.T / 2) * w.cpm.w,
                             w.cpm.lagrange_matrix(w.t_meas), w.Qw, w.Rw)


def test_c5_eight_receivers_reduced_matches_oracle():
    """SURVEY §8(d) C5 structure (n = 40) at N = 10 (d = 440) vs the dense oracle."""
    w = configs.make_c5(B=2, N=10)
    s = solver.from_workload(w)
    assert s.large_system and s.n == 40 and s.m == 24
    X, cost, iters, st = _np(s.solve(w.X_init, w.U, w.Y, w.PAR, max_iter=2, tol=0.0))
    pb = _c5_pb(w)
    run = lambda Y, pt=None: gg.gauss_newton_general(pb, w.X_init, None, w.U, Y, w.PAR, None,  # noqa: E731
                                                     max_iter=2, tol=0.0, perturb=pt)
    Xr, _, cr, ir, sr = run(w.Y)
    fx, fc = tl.floor(lambda Y, pt: (lambda r: (r[0], r[2]))(run(Y, pt)), w.Y)
    assert iters.tolist() == ir.tolist() == [2, 2] and st.tolist() == sr.tolist()
    b = tl.bound(fx, Xr)
    tl.check("C5 (n=40, N=10) X", np.abs(X - Xr).max(), b, " m")
    assert b < 1e-4
    tl.check("C5 cost", np.abs(cost - cr).max(), tl.FLOOR_MULT * fc + 1e-10 * np.abs(cr).max())


def test_c5_eight_receivers_full_shape():
    """d = 8040 (N = 200, n = 40): every trajectory converges, the cost drops, the
    receivers are recovered to the noise level (sigma_pr = 1 m, 96 pseudoranges an
    epoch), and streaming the batch through a 1-trajectory workspace (chunking: C5's
    2048 trajectories per GPU x 0.28 GB do not fit 288 GB at once) is bit-identical."""
    w = configs.make_c5(B=3)
    s = solver.from_workload(w)
    assert s.dp == 40 * 208 and s.large_system
    X, c0, iters, st = _np(s.solve(w.X_init, w.U, w.Y, w.PAR, max_iter=0, tol=0.0))
    X, cost, iters, st = _np(s.solve(w.X_init, w.U, w.Y, w.PAR, max_iter=30, tol=1e-9))
    print("C5 d=8040: iterations", iters.tolist(), "status", st.tolist())
    assert st.tolist() == [0] * w.B and np.all(cost < c0)
    pos = [c for r in range(8) for c in (5 * r, 5 * r + 1, 5 * r + 2)]
    err = np.abs(X[:, :, pos] - w.X_true[:, :, pos]).max()
    print(f"C5 d=8040: max position error {err:.2f} m")
    assert err < 3.0
    a = _np(s.solve(w.X_init, w.U, w.Y, w.PAR, max_iter=2, tol=0.0))
    per = s.lib.mhe_workspace_bytes(s.dims, 1)
    s.ws_budget = per          # one trajectory per launch
    try:
        b = _np(s.solve(w.X_init, w.U, w.Y, w.PAR, max_iter=2, tol=0.0))
    finally:
        s.ws_budget = None
    for x, y in zip(a, b):
        assert np.array_equal(x, y)


def test_chunks_are_whole_cu_fulls():
    """BatchSolver._chunk: a batch whose workspace does not fit is streamed in equal
    chunks of whole CU-fulls when the budget allows more than one (C5: 2048 trajectories
    at 0.52 GB each -> 8 x 256 on a 256-CU MI355X, not 5 x 410 with an idle tail round)."""
    w = configs.make_c3(B=2, N=60)
    s = solver.from_workload(w)
    assert s.large_system
    per = s.lib.mhe_workspace_bytes(s.dims, 1)
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    try:
        s.ws_budget = per * (cus + cus // 2 + 10)
        assert s._chunk(8 * cus) == cus
        s.ws_budget = per * (cus // 2)
        assert s._chunk(8 * cus) == cus // 2
        s.ws_budget = None
        assert s._chunk(3) == 3
    finally:
        s.ws_budget = None


def _subset_vs_oracle(w, X, cost, iters, status, idx, its, what):
    """Strided trajectories of a configured-size batch vs the oracle on those inputs
    (catches batch-index and workspace-offset bugs that a B = 2 run cannot)."""
    pb = gn.Problem(w.N, w.T, w.n, w.m, w.dyn, w.meas, w.cpm.D, (w.T / 2) * w.cpm.w,
                    w.cpm.lagrange_matrix(w.t_meas), w.Qw, w.Rw, meas_static=w.meas_static)
    U = np.broadcast_to(w.U, (w.B,) + w.U.shape[1:])[idx] if w.U.shape[0] == 1 else w.U[idx]
    PAR = np.broadcast_to(w.PAR, (idx.size,) + w.PAR.shape[1:])
    run = lambda Y, pt=None: gn.gauss_newton(pb, w.X_init[idx], U, Y, PAR, max_iter=its, tol=0.0,  # noqa: E731
                                             perturb=pt)
    Xr, cr, ir, sr = run(w.Y[idx])
    fx, fc = tl.floor(lambda Y, pt: run(Y, pt)[:2], w.Y[idx])
    assert iters[idx].tolist() == ir.tolist() == [its] * idx.size and status[idx].tolist() == sr.tolist()
    assert iters.tolist() == [its] * w.B and status.tolist() == [status[0]] * w.B
    b = tl.bound(fx, Xr)
    tl.check(f"{what} X (trajectories {idx.tolist()})", np.abs(X[idx] - Xr).max(), b, " m")
    tl.check(f"{what} cost", np.abs(cost[idx] - cr).max(), tl.FLOOR_MULT * fc + 1e-10 * np.abs(cr).max())
    return b


def test_c3_configured_batch_strided_subset_matches_oracle():
    """C3 at its configured batch (B = 4096, real geometry), 2 GN iterations on the
    device; 8 trajectories spread over the batch (first, last, strided) vs the oracle."""
    w = configs.make_c3(B=4096)
    s = solver.from_workload(w)
    X, cost, iters, status = _np(s.solve(w.X_init, w.U, w.Y, w.PAR, max_iter=2, tol=0.0))
    idx = np.unique(np.r_[np.arange(0, w.B, w.B // 7), w.B - 1])[:8]
    assert _subset_vs_oracle(w, X, cost, iters, status, idx, 2, "C3 B=4096") < 1e-4


def test_c4_configured_batch_strided_subset_matches_oracle():
    """C4 at its configured per-GPU batch (B = 1024, d = 3006), 2 GN iterations (the
    batch chunked through one workspace if the free HBM asks for it); 3 strided
    trajectories vs the oracle under C4's conditioning-limited bound (~1 cm)."""
    w = configs.make_c4(B=1024)
    s = solver.from_workload(w)
    print("C4 B=1024 chunk", s._chunk(w.B))
    X, cost, iters, status = _np(s.solve(w.X_init, w.U, w.Y, w.PAR, max_iter=2, tol=0.0))
    idx = np.array([0, 511, 1023])
    _subset_vs_oracle(w, X, cost, iters, status, idx, 2, "C4 B=1024")


def test_c5_configured_shard_chunked():
    """C5 at its configured per-GPU shard (B = 2048, d = 8040: 0.52 GB of workspace per
    trajectory, so the batch is streamed through one workspace in chunks of whole
    CU-fulls, BatchSolver._chunk), 1 and 2 GN iterations.
      * every trajectory runs the same iterations with the same status;
      * trajectories at the ends, the middle and both sides of every chunk boundary equal
        the same trajectories solved alone in one small launch, bitwise (a batch- or
        chunk-offset bug shows here first);
      * the first step of trajectories 0 and 2047 solves the ORACLE's normal equations at
        X_init (tests/big_oracle.c5_normal_epochs, pinned to the dense oracle at N = 10):
        normwise backward error of delta = X1 - X0 <= 1e-12 (the assembly tolerance of
        tests/test_gpu_big_parity.py) + 8 eps max|X1| / max|delta| (X1 - X0 rounding) --
        independent of cond(H).  Reference problem: gnss-multi-receiver.py:141-243."""
    from big_oracle import backward_error, c5_normal_epochs, c5_problem
    w = configs.make_c5(B=2048)
    s = solver.from_workload(w)
    chunk = s._chunk(w.B)
    print(f"C5 B=2048: chunk {chunk}")
    X1, c1, i1, st1 = _np(s.solve(w.X_init, w.U, w.Y, w.PAR, max_iter=1, tol=0.0))
    X2, c2, i2, st2 = _np(s.solve(w.X_init, w.U, w.Y, w.PAR, max_iter=2, tol=0.0))
    assert i1.tolist() == [1] * w.B and i2.tolist() == [2] * w.B
    assert st1.tolist() == [solver.STATUS_MAX_ITER] * w.B and st2.tolist() == [solver.STATUS_MAX_ITER] * w.B
    assert np.all(np.isfinite(X2)) and np.all(np.isfinite(c2))
    edges = [e for k in range(chunk, w.B, chunk) for e in (k - 1, k)]
    idx = np.unique(np.r_[0, w.B // 2 - 1, w.B - 1, edges]).astype(np.int64)
    sub = s.solve(w.X_init[idx], w.U[idx], w.Y[idx], w.PAR, max_iter=2, tol=0.0)
    Xs, cs, _, _ = _np(sub)
    assert np.array_equal(Xs, X2[idx]) and np.array_equal(cs, c2[idx]), idx
    pb = c5_problem(w)
    for b in (0, w.B - 1):
        H, g, _ = c5_normal_epochs(pb, w.X_init[b:b + 1], w.U[b:b + 1], w.Y[b:b + 1], w.PAR)
        delta = (X1[b] - w.X_init[b]).ravel()
        eta = backward_error(H[0], g[0], delta)
        bnd = 1e-12 + 8 * np.finfo(np.float64).eps * np.abs(X1[b]).max() / np.abs(delta).max()
        tl.check(f"C5 B=2048 trajectory {b}: first step vs oracle H, g (backward error)", eta, bnd)
