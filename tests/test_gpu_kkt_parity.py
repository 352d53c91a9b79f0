"""Kernel-level parity of the BORDERED (KKT) system of the large-system path, through the
C-ABI (mhe_assemble_kkt_ws / mhe_chol_solve_ws with n_extra / n_eq > 0, ABI v6).

Reference: extra decision variables (nlp/nlp.py:40-47 addVariables; the XA variable of
multi-receiver.py:73,99) and addEqConstraint rows (nlp/nlp.py:49-53 with
constraints.equality_constaint; gnss-multi-receiver.py:76-78 holds zA = zB at every node).
Each bordered GN step solves

    [ H    H_xz  C^T ] [dx]     [ g_x     ]
    [ H_zx H_zz  0   ] [dz] = - [ g_z     ]
    [ C    0     0   ] [l ]     [ C v - r ]

* the exported matrix against oracle.gn_general's dense KKT system (normal_equations_full
  + constraint_rows, the row-by-row independent assembly): entrywise, scaled by
  sqrt(|A_ii A_jj|) on the unknowns' rows, <= 1e-12; the constraint rows / columns (exact
  +-1 / 0 coefficients) and any entry whose scale is 0 (an extra variable no row depends
  on: multi_receiver's XA[2]) exactly;
* g_x, g_z against 8 x the oracle's own random-eps floor + 1e-12 max|g|; C v - r to 1e-14;
* the device's bordered solve of that system (k_big_chol, then k_big_border's Schur step):
  its normwise backward error on the KKT matrix (residual in extended precision) <= 64 eps.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

from mhe import configs, solver  # noqa: E402
from oracle import gn_general as gg  # noqa: E402

import tolerance as tl  # noqa: E402
from big_oracle import backward_error  # noqa: E402
from general_problems import multi_receiver_problem, two_receiver_problem  # noqa: E402

EPS = np.finfo(np.float64).eps


def _solver(pb):
    return solver.BatchSolver(pb.N, pb.T, pb.dyn, "mixed", pb.D, pb.c, pb.Phi, pb.Qw, pb.Rw, Pw=pb.Pw,
                              n_extra=pb.n_extra, eq=pb.eq if pb.eq.size else None)


def _oracle_kkt(pb, X, Z, U, Y, PAR, x0):
    """The dense KKT matrix and g of every trajectory in the device's index order:
    node-major x (padding nodes of the dp block left as the device's: identity), then z,
    then the constraint rows."""
    H, g, cost = gg.normal_equations_full(pb, X, Z, U, Y, PAR, x0)
    B, P, n = X.shape
    d, nz = P * n, pb.n_extra
    C = gg.constraint_rows(pb, d, nz)
    v = np.concatenate([X.reshape(B, -1), np.zeros((B, 0)) if Z is None else Z], axis=1)
    cval = v @ C.T - pb.eq_rhs
    return H, g, cost, C, cval


def _embed(s, H, g, C, cval):
    """oracle (d + nz [+ nc]) -> device (dk) order."""
    B = H.shape[0]
    dp, dk = s.dp, s.kkt_dim
    d, nz, nc = s.P * s.n, s.n_extra, s.n_eq
    idx = np.concatenate([np.arange(d), dp + np.arange(nz)])
    A = np.zeros((B, dk, dk))
    A[:, d:dp, d:dp] = np.eye(dp - d)
    A[np.ix_(np.arange(B), idx, idx)] = H
    A[:, dp + nz:, idx] = C[None]
    A[:, idx[:, None], (dp + nz + np.arange(nc))[None, :]] = np.swapaxes(C, 0, 1)[None]
    G = np.zeros((B, dk))
    G[:, idx] = g
    G[:, dp + nz:] = cval
    return A, G


def _check(name, s, pb, X, Z, U, Y, PAR, x0):
    B = X.shape[0]
    Hd, gd, cd, st = [t.cpu().numpy() for t in s.assemble(X, U, Y, PAR, x0, status_out=True, Z=Z)]
    assert st.tolist() == [0] * B
    Hr, gr, cr, C, cval = _oracle_kkt(pb, X, Z, U, Y, PAR, x0)
    A, G = _embed(s, Hr, gr, C, cval)
    dp, nz, nc = s.dp, s.n_extra, s.n_eq
    nu = dp + nz  # unknowns' rows (scaled comparison); the constraint rows are exact
    dg = np.sqrt(np.abs(np.einsum("bii->bi", A[:, :nu, :nu])))
    sc = dg[:, :, None] * dg[:, None, :]
    diff = np.abs(Hd[:, :nu, :nu] - A[:, :nu, :nu])
    assert np.all(diff[sc == 0.0] == 0.0), f"{name}: entries of an unobserved variable differ"
    scaled = np.where(sc > 0, diff / np.where(sc > 0, sc, 1.0), 0.0)
    tl.check(f"{name} KKT H block (diagonal-scaled)", scaled.max(), 1e-12)
    assert np.array_equal(Hd[:, nu:, :], A[:, nu:, :]), f"{name}: constraint rows differ"
    assert np.array_equal(Hd[:, :, nu:], A[:, :, nu:]), f"{name}: constraint columns differ"
    assert np.array_equal(Hd, np.swapaxes(Hd, 1, 2))
    print(f"{name}: dk = {s.kkt_dim} (dp {dp}, n_extra {nz}, n_eq {nc}); H_xz max {np.abs(A[:, :dp, dp:nu]).max() if nz else 0:.3e}")

    def run(Yv, pt=None):
        return _oracle_kkt(pb, X, Z, U, Yv, PAR, x0)[1:3]
    fg, fc = tl.floor(run, Y, conditioning=False)
    d = s.P * s.n
    idx = np.concatenate([np.arange(d), dp + np.arange(nz)])
    tl.check(f"{name} g_x, g_z", np.abs(gd[:, idx] - gr).max(), tl.FLOOR_MULT * fg + 1e-12 * np.abs(gr).max())
    assert not gd[:, d:dp].any()
    if nc:
        tl.check(f"{name} C v - r", np.abs(gd[:, nu:] - cval).max(), 1e-14 * (1 + np.abs(X).max()))
    tl.check(f"{name} cost", np.abs(cd - cr).max(), tl.FLOOR_MULT * fc + 1e-12 * np.abs(cr).max())
    # the device's bordered solve of its own KKT system
    delta, st2 = [t.cpu().numpy() for t in s.chol_solve(Hd, gd)]
    assert st2.tolist() == [0] * B
    for b in range(B):
        keep = ~((np.abs(Hd[b]).sum(1) == 0.0))  # a held variable: zero row and column, delta 0
        Ab = Hd[b][np.ix_(keep, keep)]
        eta = backward_error(Ab, gd[b][keep], delta[b][keep])
        tl.check(f"{name} KKT solve backward error [{b}]", eta, 64 * EPS)
        assert np.all(delta[b][~keep] == 0.0)
    return Hd, gd, delta


def test_two_receiver_equality_rows_kkt():
    """gnss-multi-receiver.py's structure (mixed pseudorange / range / heading rows, a prior
    and zA = zB at every node, gnss-multi-receiver.py:76-78): n_eq = P rows."""
    pb, X0, U, Y, PAR, x0, _ = two_receiver_problem(N=20, B=3, seed=5)
    s = _solver(pb)
    assert s.large_system and s.n_eq == pb.N + 1 and s.n_extra == 0
    _check("two-receiver eq", s, pb, X0, None, U, Y, PAR, x0)


def test_multi_receiver_extra_variables_kkt():
    """multi-receiver.py's XA extra variable (3 components, XA[2] in no row: held)."""
    pb, X0, Z0, U, Y, PAR, _, _ = multi_receiver_problem(B=3)
    s = _solver(pb)
    assert s.large_system and s.n_extra == pb.n_extra > 0
    _check("multi-receiver z", s, pb, X0, Z0, U, Y, PAR, None)


def test_c5s_extra_variables_kkt():
    """C5s (the multi-receiver.py structure, 12 pseudoranges + 12 rates + the 2-D range to
    XA per epoch) at a reduced horizon N = 40 (d = 328): the dense oracle assembles row by
    row."""
    w = configs.make_c5_small(B=2, N=40)
    Phi = w.cpm.lagrange_matrix(w.t_meas)
    pb = gg.GeneralProblem(w.N, w.T, w.n, w.m, w.dyn, "mixed", w.cpm.D, (w.T / 2.0) * w.cpm.w, Phi, w.Qw, w.Rw,
                           Pw=None, n_extra=w.n_extra)
    s = solver.from_workload(w)
    PAR = np.broadcast_to(w.PAR, (w.B,) + w.PAR.shape[1:])
    _check("C5s N=40", s, pb, w.X_init, w.Z_init, None, w.Y, PAR, None)


def test_kkt_solve_matches_one_bordered_gn_step():
    """The exported system IS the one a GN step solves: X + dx from chol_solve of the
    assembled KKT equals one device GN iteration (mhe_solve, max_iter 1, tol 0) to the
    rounding of the two evaluation orders (the GN step re-forms the same values)."""
    pb, X0, U, Y, PAR, x0, _ = two_receiver_problem(N=12, B=2, seed=9)
    s = _solver(pb)
    Hd, gd, _, _ = [t.cpu().numpy() for t in s.assemble(X0, U, Y, PAR, x0, status_out=True)]
    delta = s.chol_solve(Hd, gd)[0].cpu().numpy()
    d = s.P * s.n
    X1 = X0 + delta[:, :d].reshape(X0.shape)
    Xg = s.solve(X0, U, Y, PAR, x0, max_iter=1, tol=0.0)[0].cpu().numpy()
    lam = s.lam.cpu().numpy()
    err = np.abs(X1 - Xg).max()
    tl.check("assembled KKT step vs GN step", err, 1e-9 * (1 + np.abs(Xg).max()))
    tl.check("multipliers", np.abs(delta[:, s.dp:] - lam).max(), 1e-6 * (1 + np.abs(lam).max()))
