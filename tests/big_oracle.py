"""Oracle helpers for the large-system tests -- TEST INFRASTRUCTURE (imports oracle/).

* c5_normal_epochs: oracle.gn_general.normal_equations_full regrouped by epoch, for the
  C5 shape (d = 8040) where the row-by-row dense form is out of reach; pinned to the
  dense form at N = 10 (tests/test_gpu_big_parity.py).
* backward_error: normwise backward error of a computed solution of H delta = -g, the
  residual formed in extended precision (independent of cond(H)).
"""
import numpy as np

from oracle import gn
from oracle import gn_general as gg


def c5_problem(w):
    return gg.GeneralProblem(w.N, w.T, w.n, w.m, w.dyn, "mixed", w.cpm.D, (w.T / 2) * w.cpm.w,
                             w.cpm.lagrange_matrix(w.t_meas), w.Qw, w.Rw)


def c5_normal_epochs(pb, X, U, Y, PAR):
    """oracle.gn_general.normal_equations_full regrouped: the rows of one epoch share
    their Phi row, so sum_i R_i (Phi_i Phi_i^T) (x) (G_i G_i^T) is contracted per epoch
    (oracle.gn._meas_block) -- the same sums, reachable at d = 8040 where the row-by-row
    dense form is not (checked against it at N = 10 below)."""
    X = np.asarray(X, dtype=np.float64)
    B, P, n = X.shape
    Hd, gd, cost = gg._dynamics_part(pb, X, U, None)
    cost = cost.copy()
    XI = np.einsum("ij,bjc->bic", pb.Phi, X)
    G = np.zeros((B, pb.M, n, n))
    ge = np.zeros((B, pb.M, n))
    for b in range(B):
        Rw = pb.Rw[b] if pb.Rw.ndim == 2 else pb.Rw
        for i in range(pb.M):
            R = float(np.ravel(Rw[i])[0])
            if R == 0.0:
                continue
            h, Gr = gg.mixed_row(PAR[min(b, PAR.shape[0] - 1), i], XI[b, i])
            e = float(np.ravel(Y[b, i])[0]) - h
            Gx = Gr[:n]
            G[b, i] = R * np.outer(Gx, Gx)
            ge[b, i] = Gx * (R * e)
            cost[b] += R * e * e
    H = Hd.reshape(B, P, n, P, n) + gn._meas_block(pb.Phi, G)
    g = gd.reshape(B, P, n) - np.einsum("ij,bia->bja", pb.Phi, ge)
    return H.reshape(B, P * n, P * n), g.reshape(B, P * n), cost


def backward_error(H, g, delta):
    """Normwise backward error of H delta = -g, the residual formed in extended precision."""
    Hl, dl, gl = H.astype(np.longdouble), delta.astype(np.longdouble), g.astype(np.longdouble)
    r = np.einsum("ij,j->i", Hl, dl) + gl
    nH = np.abs(Hl).sum(1).max()
    return float(np.abs(r).max() / (nH * np.abs(dl).max() + np.abs(gl).max()))


def g_rounding_floor(pb, X, Y, PAR=None, U=None):
    """Per-entry first-order rounding level of g = J^T W r at X (B, P n), whatever the
    evaluation order (the bound oracle.gn.cost_noise uses for the cost, entry by entry; a
    random eps perturbation of y, tests/tolerance.floor, can cancel to well below it):
      measurements  e = y - h(x) carries eps (|y| + |h|) (pseudoranges: |y| ~ 2e7 m), so
                    Phi^T H^T R e carries |Phi|^T |H|^T |R| eps (|y| + |h|);
      dynamics      W = a D X - f carries eps (a |D| |X| + |f|), so V = c Qw W carries
                    c |Qw| of that (+ eps |V|), and a D^T V - F^T V carries
                    (a |D|^T + |F|^T) of V's plus eps (a |D|^T |V| + |F|^T |V|)."""
    from oracle import models
    eps = np.finfo(np.float64).eps
    X = np.asarray(X, dtype=np.float64)
    B, P, n = X.shape
    # dynamics (L2 cost)
    f, F = models.dyn_eval(pb.dyn, X, U, pb.dyn_par)
    W = pb.alpha * np.einsum("kj,bja->bka", pb.D, X) - f
    Wr = eps * (pb.alpha * np.einsum("kj,bja->bka", np.abs(pb.D), np.abs(X)) + np.abs(f))
    V = np.einsum("k,ac,bkc->bka", pb.c, pb.Qw, W)
    Vr = np.einsum("k,ac,bkc->bka", pb.c, np.abs(pb.Qw), Wr) + eps * np.abs(V)
    aV = np.abs(V) * eps + Vr
    gd = pb.alpha * np.einsum("kj,bka->bja", np.abs(pb.D), aV) + np.einsum("bjca,bjc->bja", np.abs(F), aV)
    # measurements
    xi = np.einsum("ij,bja->bia", pb.Phi, X)
    h, Hm = models.meas_eval(pb.meas, xi, PAR, pb.meas_static)
    Rw = pb.Rw if pb.Rw.ndim == 4 else pb.Rw[None]
    mask = gn.masked_rows(Rw)[..., None]
    with np.errstate(invalid="ignore"):
        mag = np.where(mask, 0.0, np.abs(Y) + np.abs(h)) * eps
    Hm = np.where(mask[..., None], 0.0, Hm)
    ge = np.einsum("bipa,bipq,biq->bia", np.abs(Hm), np.abs(np.broadcast_to(Rw, Hm.shape[:2] + (Hm.shape[2],) * 2)), mag)
    gm = np.einsum("ij,bia->bja", np.abs(pb.Phi), ge)
    return (gd + gm).reshape(B, P * n)
