"""Large-system path timing (C3 shape): GN collocation-point updates/s at batch B (tools only).
    python tools/bench_big.py [B] [iters]"""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "nlp-filter_amd"))
import torch  # noqa: E402
from mhe import configs, solver  # noqa: E402
B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
it = int(sys.argv[2]) if len(sys.argv) > 2 else 3
w = configs.make_c3(B=B)
s = solver.from_workload(w)
st = s.prepare(w.X_init, w.U, w.Y, w.PAR)
outs = (torch.empty_like(st[0]), torch.empty(B, dtype=torch.float64, device="cuda"),
        torch.empty(B, dtype=torch.int32, device="cuda"), torch.empty(B, dtype=torch.int32, device="cuda"))
s.solve_staged(st, outs, 1, 0.0)
torch.cuda.synchronize()
t0 = time.perf_counter()
s.solve_staged(st, outs, it, 0.0)
torch.cuda.synchronize()
dt = time.perf_counter() - t0
print(f"C3 large-system path B={B} iters={it}: {dt * 1e3:.1f} ms, {B * w.P * it / dt:.3e} pt-updates/s, "
      f"workspace {s.lib.mhe_workspace_bytes(s.dims, B) / 2**30:.2f} GiB, status {outs[3].cpu().unique().tolist()}")
