"""C5 (d = 8040) convergence trace (tools only): max|X_k - X_{k-1}| and the cost per
GN iteration, from solves with max_iter = k, tol = 0."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "nlp-filter_amd"))
import numpy as np  # noqa: E402
from mhe import configs, solver  # noqa: E402

w = configs.make_c5(B=2)
s = solver.from_workload(w)
prev = None
for k in range(0, 21):
    X, cost, it, st = [t.cpu().numpy() for t in s.solve(w.X_init, w.U, w.Y, w.PAR, max_iter=k, tol=0.0)]
    d = None if prev is None else np.abs(X - prev).max(axis=(1, 2))
    print(k, "cost", cost.tolist(), "max|dX|", None if d is None else d.tolist(), "max|X|",
          np.abs(X).max(axis=(1, 2)).tolist(), "status", st.tolist(), flush=True)
    prev = X
