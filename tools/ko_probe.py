"""Knock-out timing of the factorization (tools only): mhe_chol_solve on B random SPD
systems with a libmhe_ko<mask>.so build; results are wrong by design.  GPU.
    python tools/ko_probe.py <mask>"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
m = int(sys.argv[1]) if len(sys.argv) > 1 else 0
os.environ["MHE_LIB"] = os.path.join(ROOT, "tools", f"libmhe_ko{m}.so")
sys.path.insert(0, os.path.join(ROOT, "nlp-filter_amd"))
import numpy as np, torch  # noqa: E402
from mhe import configs, solver  # noqa: E402
w = configs.make_c2(B=8)
B, dp = 1024, 208
rng = np.random.default_rng(0)
Q = rng.standard_normal((dp, dp)) / np.sqrt(dp)
H = Q @ Q.T + np.eye(dp) * 2
Ht = torch.tensor(np.broadcast_to(H, (B, dp, dp)).copy(), device="cuda")
g = torch.tensor(rng.standard_normal((B, dp)), device="cuda")
s = solver.from_workload(w)
for _ in range(3):
    s.chol_solve(Ht, g)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(20):
    s.chol_solve(Ht, g)
e1.record()
torch.cuda.synchronize()
print(f"mask {m:3d}: {e0.elapsed_time(e1) / 20 * 1000:8.1f} us per chol_solve launch (B={B})")
