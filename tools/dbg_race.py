import os, sys, numpy as np, torch
sys.path.insert(0,'nlp-filter_amd'); sys.path.insert(0,'.')
from mhe import configs, solver
from oracle import gn
w = configs.make_c2(B=1024)
s = solver.from_workload(w)
pb = gn.Problem(w.N, w.T, w.n, w.m, w.dyn, w.meas, w.cpm.D, (w.T/2)*w.cpm.w, w.cpm.lagrange_matrix(w.t_meas), w.Qw, w.Rw)
U = np.broadcast_to(w.U, (w.B,)+w.U.shape[1:])
# assemble determinism
H1, g1, c1 = s.assemble(w.X_init, w.U, w.Y); H2, g2, c2 = s.assemble(w.X_init, w.U, w.Y)
print("assemble det:", torch.equal(H1, H2), torch.equal(g1, g2))
# linsolve determinism + correctness on the real H
d1, st1 = s.chol_solve(H1, g1); d2, st2 = s.chol_solve(H1, g1)
print("chol det:", torch.equal(d1, d2), "status", np.bincount(st1.cpu().numpy(), minlength=4))
Hn = H1.cpu().numpy(); gnn = g1.cpu().numpy()
ref = -np.linalg.solve(Hn, gnn[..., None])[..., 0]
err = np.abs(d1.cpu().numpy() - ref).max(axis=1) / np.abs(ref).max(axis=1)
print("chol err max", err.max(), "n bad", (err > 1e-8).sum(), np.nonzero(err > 1e-8)[0][:10])
# one GN iteration
outs = [s.solve(w.X_init, w.U, w.Y, max_iter=1, tol=0.0) for _ in range(3)]
X = [o[0].cpu().numpy() for o in outs]
print("gn1 det:", np.array_equal(X[0], X[1]), np.array_equal(X[0], X[2]))
Xr, _, _, _ = gn.gauss_newton(pb, w.X_init, U, w.Y, max_iter=1, tol=0.0)
e = np.abs(X[0] - Xr).reshape(1024, -1).max(1)
print("gn1 err max", e.max(), "n bad", (e > 1e-8).sum(), np.nonzero(e > 1e-8)[0][:10])
