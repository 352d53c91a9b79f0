import os, sys, numpy as np, torch
sys.path.insert(0,'nlp-filter_amd'); sys.path.insert(0,'.')
from mhe import _lib, configs, solver
pad = int(os.environ.get("SMEM_PAD", "0"))  # tool argument, passed to the library explicitly
w = configs.make_c2(B=1024)
s = solver.from_workload(w)
s.lib.mhe_set_option(_lib.OPT_DEBUG_SMEM_PAD, pad)
for rep in range(3):
    X, cost, iters, status = s.solve(w.X_init, w.U, w.Y, max_iter=30, tol=1e-9)
    st = status.cpu().numpy(); it = iters.cpu().numpy()
    print(pad, "rep", rep, "status hist", np.bincount(st, minlength=4), "iters<6", (it<6).sum())
