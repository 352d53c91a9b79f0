"""Dump one large-path solve (C3 / C4 / C5 shapes, 2 GN iterations) to an .npz, for a bitwise
comparison of two builds (MHE_LIB): python tools/dump_big_solve.py <C3|C4|C5> <B> <out.npz>"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "nlp-filter_amd"))
import numpy as np  # noqa: E402
from mhe import configs, solver  # noqa: E402

cfg, B, out = sys.argv[1], int(sys.argv[2]), sys.argv[3]
w = {"C3": configs.make_c3, "C4": configs.make_c4, "C5": configs.make_c5}[cfg](B=B)
s = solver.from_workload(w)
X, cost, iters, status = [t.cpu().numpy() for t in s.solve(w.X_init, w.U, w.Y, w.PAR, max_iter=2, tol=0.0)]
np.savez(out, X=X, cost=cost, iters=iters, status=status)
print(cfg, B, "status", np.unique(status), "cost[0]", cost[0])
