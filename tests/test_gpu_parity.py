"""HIP path (through the C-ABI) vs the CPU oracle on identical seeded inputs.

Tolerances (fp64 throughout; tests/tolerance.py derives them and every test prints
the observed error beside its bound):
  assembly  H, cost        <= 1e-12 relative to max|.|   (same formulas, different summation order)
            g              <= 8 floor_g + 1e-12 max|g|  (floor: the change of the oracle's g when
                              every y moves by eps |y| -- the rounding of y - h(x) any evaluation
                              order has; ~5e-9 m per pseudorange row at |y| ~ 2.2e7 m)
  dense SPD solve          <= 1e-10 relative              (cond(H) ~ 1e5 for C2)
  Gauss-Newton iterate     <= 8 floor_X + 1e-10 (1 + max|X|) after the same number of iterations
                              (SURVEY.md §8(c)); converged optimum (tol 1e-9 stopping rule on both
                              sides, iteration counts within 1) <= 8 floor_X + 1e-8 (1 + max|X|)
  index / status / iteration counts: exact
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

from mhe import configs, solver  # noqa: E402
from oracle import gn  # noqa: E402

import tolerance as tl  # noqa: E402


def _problem(w):
    return gn.Problem(w.N, w.T, w.n, w.m, w.dyn, w.meas, w.cpm.D, (w.T / 2) * w.cpm.w,
                      w.cpm.lagrange_matrix(w.t_meas), w.Qw, w.Rw, Pw=w.Pw, meas_static=w.meas_static)


def _U(w):
    return np.broadcast_to(w.U, (w.B,) + w.U.shape[1:])


def _PAR(w):
    return None if w.PAR is None else np.broadcast_to(w.PAR, (w.B,) + w.PAR.shape[1:])


WORKLOADS = {
    "c1": lambda: configs.make_c1(),
    "c2_n20": lambda: configs.make_c2(B=6, N=20),
    "c2_n100": lambda: configs.make_c2(B=6, N=100),
    "gnss_small": lambda: configs.make_gnss_small(B=4),
}


@pytest.fixture(scope="module", params=sorted(WORKLOADS))
def case(request):
    w = WORKLOADS[request.param]()
    return w, solver.from_workload(w), _problem(w)


def test_assemble_matches_oracle(case):
    w, s, pb = case
    H, g, cost = s.assemble(w.X_init, w.U, w.Y, w.PAR)
    H, g, cost = H.cpu().numpy(), g.cpu().numpy(), cost.cpu().numpy()
    run = lambda Y: gn.normal_equations(pb, w.X_init, _U(w), Y, _PAR(w))  # noqa: E731
    Hr, gr, cr = run(w.Y)
    _, fg, fc = tl.floor(lambda Y, pt: run(Y), w.Y, conditioning=False)
    d = pb.d
    tl.check("H", np.abs(H[:, :d, :d] - Hr).max(), 1e-12 * np.abs(Hr).max())
    tl.check("g", np.abs(g[:, :d] - gr).max(), tl.FLOOR_MULT * fg + 1e-12 * np.abs(gr).max())
    tl.check("cost", np.abs(cost - cr).max(), tl.FLOOR_MULT * fc + 1e-12 * np.abs(cr).max())
    # padding: identity block, zero coupling, zero gradient
    if s.dp > d:
        assert np.array_equal(H[:, d:, d:], np.broadcast_to(np.eye(s.dp - d), H[:, d:, d:].shape))
        assert not H[:, :d, d:].any() and not H[:, d:, :d].any() and not g[:, d:].any()


def test_chol_solve_matches_numpy(case):
    w, s, pb = case
    rng = np.random.default_rng(7)
    B, dp = 5, s.dp
    A = rng.normal(size=(B, dp, dp))
    H = A @ np.swapaxes(A, 1, 2) + dp * np.eye(dp)[None]
    g = rng.normal(size=(B, dp))
    delta, status = s.chol_solve(H, g)
    ref = -np.linalg.solve(H, g[..., None])[..., 0]
    assert np.all(status.cpu().numpy() == 0)
    assert np.abs(delta.cpu().numpy() - ref).max() <= 1e-10 * np.abs(ref).max()


def test_chol_solve_detects_non_spd(case):
    w, s, pb = case
    dp = s.dp
    H = np.stack([np.eye(dp), np.eye(dp), np.eye(dp)])
    H[1, dp // 2, dp // 2] = -1.0     # negative pivot
    H[2, 3, 3] = np.nan               # non-finite pivot
    delta, status = s.chol_solve(H, np.ones((3, dp)))
    assert status.cpu().numpy().tolist() == [0, 2, 2]
    assert np.allclose(delta.cpu().numpy()[0], -1.0)


def test_gn_iterates_match_oracle(case):
    w, s, pb = case
    it = 4
    X, cost, iters, status = s.solve(w.X_init, w.U, w.Y, w.PAR, max_iter=it, tol=0.0)
    run = lambda Y, pt=None: gn.gauss_newton(pb, w.X_init, _U(w), Y, _PAR(w), max_iter=it, tol=0.0, perturb=pt)  # noqa: E731
    Xr, cr, ir, sr = run(w.Y)
    fx, fc = tl.floor(lambda Y, pt: run(Y, pt)[:2], w.Y)
    assert iters.cpu().numpy().tolist() == ir.tolist() == [it] * w.B
    assert status.cpu().numpy().tolist() == sr.tolist() == [1] * w.B
    tl.check("X", np.abs(X.cpu().numpy() - Xr).max(), tl.bound(fx, Xr))
    tl.check("cost", np.abs(cost.cpu().numpy() - cr).max(), tl.FLOOR_MULT * fc + 1e-10 * np.abs(cr).max())


def test_gn_converges_to_oracle_optimum(case):
    w, s, pb = case
    X, cost, iters, status = s.solve(w.X_init, w.U, w.Y, w.PAR, max_iter=50, tol=1e-9)
    run = lambda Y, pt=None: gn.gauss_newton(pb, w.X_init, _U(w), Y, _PAR(w), max_iter=50, tol=1e-9, perturb=pt)  # noqa: E731
    Xr, cr, ir, sr = run(w.Y)
    fx, fc = tl.floor(lambda Y, pt: run(Y, pt)[:2], w.Y)
    assert status.cpu().numpy().tolist() == sr.tolist() == [0] * w.B
    assert np.all(np.abs(iters.cpu().numpy() - ir) <= 1)
    tl.check("X", np.abs(X.cpu().numpy() - Xr).max(), tl.bound(fx, Xr, rel=1e-8))
    tl.check("cost", np.abs(cost.cpu().numpy() - cr).max(), tl.FLOOR_MULT * fc + 1e-10 * np.abs(cr).max())


def test_max_iter_zero_returns_initial_iterate():
    w = configs.make_c2(B=3, N=20)
    s = solver.from_workload(w)
    X, cost, iters, status = s.solve(w.X_init, w.U, w.Y, max_iter=0)
    assert np.array_equal(X.cpu().numpy(), w.X_init)
    assert iters.cpu().numpy().tolist() == [0, 0, 0]
    _, _, _, cr = gn.residuals(_problem(w), w.X_init, _U(w), w.Y)
    assert np.allclose(cost.cpu().numpy(), cr, rtol=1e-12)


def test_empty_batch_is_noop():
    w = configs.make_c2(B=1, N=20)
    s = solver.from_workload(w)
    X, cost, iters, status = s.solve(np.zeros((0, w.P, w.n)), w.U, np.zeros((0, w.M, w.p)), max_iter=3)
    assert X.shape == (0, w.P, w.n)


def test_nonfinite_input_is_reported_not_fatal():
    w = configs.make_c2(B=3, N=20)
    s = solver.from_workload(w)
    X0 = w.X_init.copy()
    X0[1, 5, 0] = np.nan
    X, cost, iters, status = s.solve(X0, w.U, w.Y, max_iter=40, tol=1e-9)
    st = status.cpu().numpy().tolist()
    assert st[0] == 0 and st[2] == 0 and st[1] in (2, 3)


def test_c2_full_batch_properties():
    """BASELINE configs[1] at full size (B=1024, N=100): every trajectory converges,
    the cost drops, and a subset matches the oracle."""
    w = configs.make_c2(B=1024)
    s = solver.from_workload(w)
    X, cost, iters, status = s.solve(w.X_init, w.U, w.Y, max_iter=30, tol=1e-9)
    st = status.cpu().numpy()
    assert (st == 0).all()
    pb = _problem(w)
    _, _, _, c0 = gn.residuals(pb, w.X_init, _U(w), w.Y)
    assert (cost.cpu().numpy() < c0).all()
    sub = np.arange(0, 1024, 128)
    Xr, cr, ir, sr = gn.gauss_newton(pb, w.X_init[sub], _U(w)[sub], w.Y[sub], max_iter=30, tol=1e-9)
    assert np.abs(X.cpu().numpy()[sub] - Xr).max() <= 1e-8 * (1 + np.abs(Xr).max())


def test_bitwise_deterministic_full_occupancy():
    """Two workgroups per CU (B=1024) stress intra-workgroup LDS hand-offs: the same
    inputs must give bitwise-identical results run to run (a race shows up here first)."""
    w = configs.make_c2(B=1024)
    s = solver.from_workload(w)
    r1 = [t.cpu().numpy() for t in s.solve(w.X_init, w.U, w.Y, max_iter=3, tol=0.0)]
    r2 = [t.cpu().numpy() for t in s.solve(w.X_init, w.U, w.Y, max_iter=3, tol=0.0)]
    for a, b in zip(r1, r2):
        assert np.array_equal(a, b)
    H, g, _ = s.assemble(w.X_init, w.U, w.Y)
    d1, s1 = s.chol_solve(H, g)
    d2, s2 = s.chol_solve(H, g)
    assert torch.equal(d1, d2) and (s1.cpu().numpy() == 0).all()


def test_small_batch_instance_matches_full_occupancy_instance():
    """launch_gn runs the small-batch instance of k_gn (launch bounds of 2 waves per SIMD)
    when the batch gives each CU at most one trajectory, and the two-workgroups-per-CU
    instance otherwise.  They differ only in register allocation, so the same trajectories
    solved in a small batch and inside a large one agree bit for bit."""
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    w = configs.make_c2(B=2 * cus + 8)
    s = solver.from_workload(w)
    big = [t.cpu().numpy() for t in s.solve(w.X_init, w.U, w.Y, max_iter=4, tol=0.0)]
    sub = slice(0, min(cus, 96))
    assert sub.stop <= cus  # the small batch runs the small-batch instance (batch <= CUs)
    small = [t.cpu().numpy() for t in s.solve(w.X_init[sub], w.U, w.Y[sub], max_iter=4, tol=0.0)]
    for a, b in zip(small, big):
        assert np.array_equal(a, b[sub])


FULL_OCC = {
    "c1": lambda B: configs.make_c1(B=B),                 # single_integrator pair (nlp/dynamics.py:4-7)
    "c2_n20": lambda B: configs.make_c2(B=B, N=20),       # van der Pol pair
    "gnss_small": lambda B: configs.make_gnss_small(B=B),  # pseudorange pair (nlp/measurements.py:56-70)
}


@pytest.mark.parametrize("name", sorted(FULL_OCC))
def test_full_occupancy_instance_iterates_match_oracle(name):
    """B = CUs + 8 runs the two-workgroups-per-CU instance k_gn<..., MAX_SLOTS, MODE_SOLVE>
    (not the small-batch one the B <= 6 cases above select): 4 GN iterations at tol 0 of
    every trajectory against the oracle, for each shipped model pair family."""
    import ctypes
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    w = FULL_OCC[name](cus + 8)
    s = solver.from_workload(w)
    buf = ctypes.create_string_buffer(256)
    st = torch.cuda.current_stream()
    assert s.lib.mhe_solve_kernel_name(s.dims, w.B, ctypes.c_void_p(st.cuda_stream), buf, 256) == 0
    print(buf.value.decode())
    assert b"two workgroups per CU" in buf.value and b"SB=true" not in buf.value
    pb = _problem(w)
    it = 4
    X, cost, iters, status = s.solve(w.X_init, w.U, w.Y, w.PAR, max_iter=it, tol=0.0)
    run = lambda Y, pt=None: gn.gauss_newton(pb, w.X_init, _U(w), Y, _PAR(w), max_iter=it, tol=0.0, perturb=pt)  # noqa: E731
    Xr, cr, ir, sr = run(w.Y)
    fx, fc = tl.floor(lambda Y, pt: run(Y, pt)[:2], w.Y)
    assert iters.cpu().numpy().tolist() == ir.tolist() == [it] * w.B
    assert status.cpu().numpy().tolist() == sr.tolist() == [1] * w.B
    tl.check(f"{name} B={w.B} X", np.abs(X.cpu().numpy() - Xr).max(), tl.bound(fx, Xr))
    tl.check(f"{name} B={w.B} cost", np.abs(cost.cpu().numpy() - cr).max(), tl.FLOOR_MULT * fc + 1e-10 * np.abs(cr).max())
    head = lambda a: None if a is None else (a[:6] if a.shape[0] > 1 else a)  # noqa: E731
    sb = s.solve(w.X_init[:6], head(w.U), w.Y[:6], head(w.PAR), max_iter=it, tol=0.0)[0].cpu().numpy()
    assert np.array_equal(sb, X.cpu().numpy()[:6])  # and bitwise what the small-batch instance gives
