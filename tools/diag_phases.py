"""Phase breakdown of the fused GN kernel from the MHE_DIAG build (s_memtime stamps).

python tools/diag_phases.py  (needs tools/libmhe_diag.so; GPU)
Phases (cycles per GN iteration, averaged over workgroups): 7 loop head,
0 node+meas, 1 gradient, 2 tile build, 3 Cholesky+forward, 4 backward,
5 exit (+update).  Diagnostic only: the stamps serialise the phases.
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["MHE_LIB"] = os.environ.get("MHE_DIAG_LIB", os.path.join(ROOT, "tools", "libmhe_diag.so"))
sys.path.insert(0, os.path.join(ROOT, "nlp-filter_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from mhe import _lib, configs, solver  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 4
lib = _lib.load()
lib.mhe_diag_set_buffer.argtypes = [ctypes.c_void_p]
dbg = torch.zeros(B * 16 + 128, dtype=torch.int64, device="cuda")
lib.mhe_diag_set_buffer(ctypes.c_void_p(dbg.data_ptr()))
w = configs.make_c2(B=B)
s = solver.from_workload(w)
for _ in range(2):
    X, c, it, st = s.solve(w.X_init, w.U, w.Y, max_iter=iters, tol=0.0)
torch.cuda.synchronize()
ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
ev0.record()
X, c, it, st = s.solve(w.X_init, w.U, w.Y, max_iter=iters, tol=0.0)
ev1.record()
torch.cuda.synchronize()
allv = dbg.cpu().numpy().astype(np.float64)
d = allv[:B * 16].reshape(B, 16) / iters
busy = allv[B * 16:].reshape(8, 16) / (iters * 3)  # block 0, summed over the launches
names = {7: "loop head", 6: "node/meas rows", 14: "node mat-vec loop", 0: "node+meas barrier", 1: "gradient", 15: "tile build", 2: "tile barrier", 3: "chol tail", 4: "backward", 5: "exit",
         8: "  T (trsm) | SB: CP pre-panel", 9: "  barrier1 | SB: slowest worker busy", 12: "  U: rhs/panel", 13: "  U: slots | SB: wave 4 busy", 10: "  U: diag | SB: slowest worker over CP", 11: "  barrier2"}
tot = d.sum(1).mean()
print(f"B={B} iters={iters} kernel {ev0.elapsed_time(ev1):.3f} ms; cycles/iter/WG (s_memtime) total {tot:.0f}")
for i, nm in names.items():
    print(f"  {nm:10s} {d[:, i].mean():10.0f}  ({100 * d[:, i].mean() / tot:5.1f} %)  max {d[:, i].max():.0f}")
if busy.any():
    print("small-batch factorization, block 0: busy cycles per interval (rows: waves 0..7, cols: k)")
    for w in range(8):
        print(f"  wave {w}: " + " ".join(f"{v:6.0f}" for v in busy[w][:13]) + f"   sum {busy[w].sum():7.0f}")
