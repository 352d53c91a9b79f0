"""Batched GNSS least-squares throughput (utils.leastsquares on mhe_ls_run).

    python tools/bench_ls.py [C]

Workload: the reference's receiver-A log (40 epochs x 12 satellite slots, committed
fixture tests/golden/least_squares.npz) replicated over C logs with perturbed
pseudoranges (sigma 3 m) and starting points (synthetic), with the velocity solve.
Metric: position fixes/s = C * T / kernel time (HIP events around one run_batch
launch, inputs resident), for the reference's warm-started chains (one wave walks a
log's epochs in order) and for independent epochs (one wave per epoch).
CPU baseline: oracle/leastsquares.py (the reference's iterativeLeastSquares +
iterativeLeastSquaresVel) on one core over a bounded sample.
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "nlp-filter_amd"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import utils.leastsquares as uls  # noqa: E402
from oracle import leastsquares as ols  # noqa: E402

C = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
fx = dict(np.load(os.path.join(ROOT, "tests", "golden", "least_squares.npz")))
rng = np.random.default_rng(5)
T = fx["A_count"].shape[0]
sp = np.tile(fx["A_sat_pos"][None], (C, 1, 1, 1))
pr = np.tile(fx["A_pr"][None], (C, 1, 1)) + rng.normal(size=(C,) + fx["A_pr"].shape) * 3.0
sv = np.tile(fx["A_sat_vel"][None], (C, 1, 1, 1))
rr = np.tile(fx["A_pr_rate"][None], (C, 1, 1))
cnt = np.tile(fx["A_count"][None], (C, 1)).astype(np.int32)
x0 = rng.normal(size=(C, 3)) * 1e3
dev = torch.device("cuda", 0)
spt, prt, svt, rrt, cntt, x0t = (torch.as_tensor(a, device=dev) for a in (sp, pr, sv, rr, cnt, x0))

res = {"metric": "GNSS least-squares fixes/s", "unit": "fixes/s",
       "workload": f"receiver-A log (T={T} epochs x 12 slots) x C={C} logs, position + velocity"}
for warm in (True, False):
    run = lambda: uls.run_batch(spt, prt, cntt, x_init=x0t, sat_vel=svt, pr_rate=rrt, warm=warm)  # noqa: E731
    out = run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        run()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 5
    it = out["iters"].float().mean().item()
    res["warm" if warm else "independent"] = {"value": C * T / (ms * 1e-3), "ms_per_launch": ms,
                                               "mean_gn_iterations": it}
res["value"] = res["warm"]["value"]
# algorithmic bytes per fix: satellite positions + velocities (12 x 6), pseudoranges +
# rates (12 x 2), count in; x, b, v, bd, iterations out
by = 8.0 * (12 * 6 + 12 * 2) + 4 + 8.0 * 8 + 4
res["roofline"] = {"bound": "hbm", "achieved": by * res["value"] / 1e9, "peak": 8000.0, "unit": "GB/s",
                   "frac": by * res["value"] / 1e9 / 8000.0, "bytes_per_fix": by,
                   "note": "latency-bound: one lane per log walks its epochs in order (warm start); strided per-lane rows"}

nb, t0 = 0, time.perf_counter()
while time.perf_counter() - t0 < 3.0:
    c = nb % C
    x = x0[c].copy()
    for k in range(T):
        n = int(cnt[c, k])
        xo, b, _ = ols.iterative_least_squares(sp[c, k, :n], pr[c, k, :n], x)
        ols.iterative_least_squares_vel(sp[c, k, :n], sv[c, k, :n], rr[c, k, :n], xo)
    nb += 1
dt = time.perf_counter() - t0
res["cpu_baseline"] = {"value": nb * T / dt, "unit": "fixes/s", "cores": 1, "kind": "port",
                       "sample": f"{nb} logs x {T} epochs, warm chains, oracle/leastsquares.py on one core, "
                                 f"{dt:.1f} s"}
print(json.dumps(res))
