"""PCIe-inclusive rate of the C2 workload (tools only; NOT the bench metric).

    python tools/bench_pcie.py [B] [iters] [reps]

Host NumPy inputs in (X0, U, Y), host NumPy outputs back (X, cost, iters, status):
the facade path a reference user calls (BatchSolver.solve on host arrays), timed
with perf_counter around H2D + the fused launch + D2H.  Reported beside the
device-resident rate of the same launch (inputs already in HBM).
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "nlp-filter_amd"))
import torch  # noqa: E402
from mhe import configs, solver  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 10
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
w = configs.make_c2(B=B)
s = solver.from_workload(w)


def host_solve():
    X, c, it, st = s.solve(w.X_init, w.U, w.Y, max_iter=iters, tol=0.0)
    return X.cpu().numpy(), c.cpu().numpy(), it.cpu().numpy(), st.cpu().numpy()


for _ in range(3):
    host_solve()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(reps):
    host_solve()
torch.cuda.synchronize()
t_host = (time.perf_counter() - t0) / reps

staged = s.prepare(w.X_init, w.U, w.Y)
outs = (torch.empty_like(staged[0]), torch.empty(B, dtype=torch.float64, device="cuda"),
        torch.empty(B, dtype=torch.int32, device="cuda"), torch.empty(B, dtype=torch.int32, device="cuda"))
stream = torch.cuda.current_stream()
for _ in range(3):
    s.solve_staged(staged, outs, iters, 0.0, stream)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(reps):
    s.solve_staged(staged, outs, iters, 0.0, stream)
torch.cuda.synchronize()
t_dev = (time.perf_counter() - t0) / reps

in_bytes = sum(a.nbytes for a in (w.X_init, w.U, w.Y))
out_bytes = w.X_init.nbytes + B * (8 + 4 + 4)
print(json.dumps({"workload": "C2", "B": B, "iters": iters,
                  "pcie_inclusive_pt_updates_per_s": B * w.P * iters / t_host, "ms_host_to_host": t_host * 1e3,
                  "device_resident_pt_updates_per_s": B * w.P * iters / t_dev, "ms_device_resident": t_dev * 1e3,
                  "host_bytes_in": in_bytes, "host_bytes_out": out_bytes}))
