"""General problems on the GPU: mixed scalar rows, extra decision
variables and equality constraints through mhe_gn_solve_ext (large-system path,
bordered KKT step in k_big_border) vs the dense-KKT oracle (oracle/gn_general.py).

Tolerances (fp64, tests/tolerance.py): pseudoranges (~2e7 m) carry eps |y| of
rounding in y - h in any evaluation order; its effect (floor) is measured by
re-running the oracle with every y moved by eps |y|, so
  one GN step                       <= 8 floor + 1e-10 (1 + max|X|)
  converged iterate (tol 1e-10)     <= 8 floor + 1e-8 (1 + max|X|)
  constraints after every step      |v[a] - v[b]| <= 1e-9 * (1 + max|X|)
  held (unobservable) extra variable: bit-identical to its start value
  status exact, iteration counts within 1.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

from mhe import solver  # noqa: E402
from oracle import collocation as oc  # noqa: E402
from oracle import gn  # noqa: E402
from oracle import gn_general as gg  # noqa: E402

from general_problems import multi_receiver_problem, row, two_receiver_problem  # noqa: E402
import tolerance as tl  # noqa: E402


def _solver(pb):
    return solver.BatchSolver(pb.N, pb.T, pb.dyn, "mixed", pb.D, pb.c, pb.Phi, pb.Qw, pb.Rw, Pw=pb.Pw,
                              n_extra=pb.n_extra, eq=pb.eq if pb.eq.size else None)


def test_two_receiver_one_step_matches_kkt_oracle():
    pb, X0, U, Y, PAR, x0, _ = two_receiver_problem(B=4)
    s = _solver(pb)
    assert s.large_system
    X, cost, iters, st = s.solve(X0, U, Y, PAR, x0, max_iter=1, tol=0.0)
    run = lambda Yv, pt=None: gg.gauss_newton_general(pb, X0, None, U, Yv, PAR, x0, max_iter=1, tol=0.0, perturb=pt)  # noqa: E731
    Xr, _, cr, ir, sr = run(Y)
    fx, = tl.floor(lambda Yv, pt: run(Yv, pt)[:1], Y)
    X = X.cpu().numpy()
    assert iters.cpu().numpy().tolist() == ir.tolist() == [1] * 4
    tl.check("X", np.abs(X - Xr).max(), tl.bound(fx, Xr), " m")
    assert np.abs(X[:, :, 2] - X[:, :, 7]).max() <= 1e-9 * (1 + np.abs(X).max())


def test_two_receiver_converges_to_kkt_oracle():
    pb, X0, U, Y, PAR, x0, _ = two_receiver_problem(B=6, seed=4)
    s = _solver(pb)
    X, cost, iters, st = s.solve(X0, U, Y, PAR, x0, max_iter=40, tol=1e-10)
    run = lambda Yv, pt=None: gg.gauss_newton_general(pb, X0, None, U, Yv, PAR, x0, max_iter=40, tol=1e-10, perturb=pt)  # noqa: E731
    Xr, _, cr, ir, sr = run(Y)
    fx, fc = tl.floor(lambda Yv, pt: (lambda r: (r[0], r[2]))(run(Yv, pt)), Y)
    assert st.cpu().numpy().tolist() == sr.tolist() == [0] * 6
    assert np.all(np.abs(iters.cpu().numpy() - ir) <= 1)
    X = X.cpu().numpy()
    tl.check("X", np.abs(X - Xr).max(), tl.bound(fx, Xr, rel=1e-8), " m")
    tl.check("cost", np.abs(cost.cpu().numpy() - cr).max(), tl.FLOOR_MULT * fc + 1e-10 * np.abs(cr).max())
    assert np.abs(X[:, :, 2] - X[:, :, 7]).max() <= 1e-9 * (1 + np.abs(X).max())


def test_extra_variables_match_oracle_and_hold_unobservable():
    pb, X0, Z0, U, Y, PAR, xt, zt = multi_receiver_problem(B=4)
    s = _solver(pb)
    X, cost, iters, st, Z = s.solve(X0, None, Y, PAR, max_iter=40, tol=1e-10, Z0=Z0)
    run = lambda Yv, pt=None: gg.gauss_newton_general(pb, X0, Z0, None, Yv, PAR, None, max_iter=40, tol=1e-10, perturb=pt)  # noqa: E731
    Xr, Zr, cr, ir, sr = run(Y)
    fx, fz = tl.floor(lambda Yv, pt: run(Yv, pt)[:2], Y)
    assert st.cpu().numpy().tolist() == sr.tolist() == [0] * 4
    X, Z = X.cpu().numpy(), Z.cpu().numpy()
    tl.check("X", np.abs(X - Xr).max(), tl.bound(fx, Xr, rel=1e-8), " m")
    tl.check("Z", np.abs(Z - Zr).max(), tl.bound(fz, Zr, rel=1e-8), " m")
    assert np.array_equal(Z[:, 2], Z0[:, 2])  # XA[2] enters no row: held exactly


def test_mixed_component_rows_equal_fused_full_state_path():
    """van der Pol with full_state measurements written as mixed COMPONENT rows
    (large-system path) must reach the fused kernel's optimum (register path)."""
    from mhe import configs
    w = configs.make_c2(B=4, N=20)
    s_ref = solver.from_workload(w)
    assert not s_ref.large_system
    Xf, cf, _, sf = s_ref.solve(w.X_init, w.U, w.Y, max_iter=30, tol=1e-11)
    Phi = w.cpm.lagrange_matrix(w.t_meas)
    rows, Phi2, Rw, Y2 = [], [], [], []
    for i in range(Phi.shape[0]):
        for a in range(w.n):
            rows.append(row(gg.ROW_COMP, [a]))
            Phi2.append(Phi[i])
            Rw.append(w.Rw[i][a, a])
    Y2 = w.Y.reshape(w.B, -1, 1)
    s_mix = solver.BatchSolver(w.N, w.T, w.dyn, "mixed", w.cpm.D, (w.T / 2.0) * w.cpm.w, np.array(Phi2), w.Qw,
                               np.array(Rw), Pw=w.Pw)
    assert s_mix.large_system
    Xm, cm, _, sm = s_mix.solve(w.X_init, w.U, Y2, np.array(rows)[None], max_iter=30, tol=1e-11)
    assert sf.cpu().numpy().tolist() == sm.cpu().numpy().tolist() == [0] * 4
    Xf, Xm = Xf.cpu().numpy(), Xm.cpu().numpy()
    assert np.abs(Xf - Xm).max() <= 1e-9 * (1 + np.abs(Xf).max())
    assert np.allclose(cf.cpu().numpy(), cm.cpu().numpy(), rtol=1e-10)


def test_constraints_with_a_single_model_problem():
    """Equality constraints are independent of the mixed encoding: van der Pol with
    full_state rows and X_j[0] = X_j[1] at every other node, vs the oracle."""
    from mhe import configs
    w = configs.make_c2(B=3, N=12)
    n, P = w.n, w.P
    eq = np.array([[j * n + 0, j * n + 1] for j in range(0, P, 2)])
    s = solver.BatchSolver(w.N, w.T, w.dyn, w.meas, w.cpm.D, (w.T / 2.0) * w.cpm.w, w.cpm.lagrange_matrix(w.t_meas),
                           w.Qw, w.Rw, Pw=w.Pw, eq=eq)
    assert s.large_system
    X, cost, iters, st = s.solve(w.X_init, w.U, w.Y, max_iter=30, tol=1e-11)
    # oracle: the same objective as COMPONENT rows
    Phi = w.cpm.lagrange_matrix(w.t_meas)
    rows = np.array([row(gg.ROW_COMP, [a]) for i in range(Phi.shape[0]) for a in range(n)])
    Phi2 = np.repeat(Phi, n, axis=0)
    Rw = np.array([w.Rw[i][a, a] for i in range(Phi.shape[0]) for a in range(n)])
    pb = gg.GeneralProblem(w.N, w.T, n, w.m, w.dyn, "mixed", w.cpm.D, (w.T / 2.0) * w.cpm.w, Phi2, w.Qw, Rw,
                           Pw=w.Pw, eq=eq)
    U = np.broadcast_to(w.U, (w.B,) + w.U.shape[1:])
    Xr, _, cr, ir, sr = gg.gauss_newton_general(pb, w.X_init, None, U, w.Y.reshape(w.B, -1, 1),
                                                np.tile(rows[None], (w.B, 1, 1)), None, max_iter=30, tol=1e-11)
    assert st.cpu().numpy().tolist() == sr.tolist() == [0] * 3
    X = X.cpu().numpy()
    assert np.abs(X - Xr).max() <= 1e-9 * (1 + np.abs(Xr).max())
    assert np.abs(X[:, ::2, 0] - X[:, ::2, 1]).max() <= 1e-10 * (1 + np.abs(X).max())


def test_general_path_bitwise_deterministic():
    pb, X0, U, Y, PAR, x0, _ = two_receiver_problem(B=64, seed=7)
    s = _solver(pb)
    a = s.solve(X0, U, Y, PAR, x0, max_iter=8, tol=1e-10)[0].cpu().numpy()
    b = s.solve(X0, U, Y, PAR, x0, max_iter=8, tol=1e-10)[0].cpu().numpy()
    assert np.array_equal(a, b)
