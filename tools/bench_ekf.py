"""Batched EKF throughput (utils.ekf.EKF on mhe_ekf_run).

    python tools/bench_ekf.py [B] [reps]

Workload: the gnss_stationary EKF recipe of the reference (gnss_stationary.py:
gnss_pos_and_bias + multi_pseudorange, 12 satellite slots, 51 epochs from the
committed fixture tests/golden/ekf_gnss_stationary.npz), replicated over B
independent filters with perturbed initial states and controls (synthetic).
Metric: filter-step updates/s = B * T / kernel time (HIP events around one
run_batch launch with inputs resident, history kept).

Roofline per filter-step (n = 5, p = 12): algorithmic bytes = Z (12) + sat_pos
(36) + U (3) doubles read, mu/S history (5 + 25) doubles written, nz (4 B):
652 B -- the bound is HBM.  Flops for context, as executed by the diagonal-R
kernel (k_ekf_lane: predict G S G^T 4 n^3, per row h/H ~20 + e 2n + v = S H^T
2n^2 + s 2n + mu 2n + S 2n^2 + n): ~2.4 KFLOP.
CPU baseline: the oracle EKF (oracle/ekf.py, the reference's update with
np.linalg.inv) on one host core over a bounded sample.
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

import utils.ekf as ekf  # noqa: E402
import utils.gnss as gnss  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
REPS = int(sys.argv[2]) if len(sys.argv) > 2 else 10
fx = dict(np.load(os.path.join(ROOT, "tests", "golden", "ekf_gnss_stationary.npz")))
T, pmax, n = fx["pr"].shape[0], 12, 5
rng = np.random.default_rng(7)
mu0 = np.tile(fx["mu0"], (B, 1))
mu0[1:] += rng.normal(size=(B - 1, 5)) * np.array([3, 3, 3, 30, 0.1])
S0 = np.tile(fx["S0"], (B, 1, 1))
U = rng.normal(size=(B, T, 3)) * 0.1
Z = np.tile(fx["pr"], (B, 1, 1))
nz = np.tile(fx["nsat"], (B, 1)).astype(np.int32)
sat = np.tile(fx["sat_pos"], (B, 1, 1, 1))
R = np.stack([np.diag(float(fx["r_pr"]) * np.ones(pmax)) for _ in range(T)])

dev = torch.device("cuda", 0)
LAYOUT = os.environ.get("EKF_INPUTS", "batch_inner")
if LAYOUT == "batch_inner":  # synthetic inputs generated batch-innermost: coalesced device reads
    U, Z, nz, sat_in = (np.ascontiguousarray(np.moveaxis(x, 0, -1)) for x in (U, Z, nz, sat))
else:
    sat_in = sat
args = [torch.as_tensor(a, device=dev) for a in (mu0, S0, U, Z, nz, sat_in)]
Rt = torch.as_tensor(R, device=dev)
Qt = torch.as_tensor(fx["Q"], device=dev)


def run(method="lane"):
    return ekf.run_batch(gnss.gnss_pos_and_bias, gnss.multi_pseudorange, args[0], args[1], args[2], args[3],
                         args[4], Qt, Rt, 1.0, args[5], method=method, inputs=LAYOUT)


out = run("auto")   # diagonal R: auto selects the per-lane kernel
torch.cuda.synchronize()
assert int(out[4].abs().sum().item()) == 0
ref = run("wave")    # general per-wavefront sweep, same inputs: agreement and its speed
torch.cuda.synchronize()
dmu = float(((out[0] - ref[0]).abs().amax(-1) / (1 + ref[0].abs().amax(-1))).max().item())
ew0, ew1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
ew0.record()
run("wave")
ew1.record()
torch.cuda.synchronize()
wave_ms = ew0.elapsed_time(ew1)
del out, ref  # the history buffers are reused by the timed calls (no allocation inside the timing)
run()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(REPS):
    run()
e1.record()
torch.cuda.synchronize()
wall = e0.elapsed_time(e1) / REPS / 1e3   # per launch (includes the tensor staging in run_batch)

ps = fx["nsat"].astype(np.float64)
# flops per filter-step as executed by k_ekf_lane: predict 4 n^3; per row h/H ~20, e 2n, v = S H^T 2n^2,
# s 2n, mu 2n, S 2n^2 + n
fl = np.mean(4 * n ** 3 + ps * (20 + 2 * n + 2 * n * n + 2 * n + 2 * n + 2 * n * n + n))
by = 8.0 * (pmax + 3 * pmax + 3 + n + n * n) + 4
steps = B * T

# CPU: the oracle EKF, one core, bounded sample (per-instance arrays)
from oracle import ekf as oekf  # noqa: E402
if LAYOUT == "batch_inner":
    U, Z, nz = (np.moveaxis(x, -1, 0) for x in (U, Z, nz))
nb, t0 = 0, time.perf_counter()
while time.perf_counter() - t0 < (0.0 if os.environ.get("NO_CPU") else 5.0):
    b = nb % B
    f = oekf.EKF(oekf.gnss_pos_and_bias, oekf.multi_pseudorange, mu0[b], S0[b])
    for k in range(T):
        ns = int(nz[b, k])
        f.update(U[b, k], Z[b, k, :ns], fx["Q"], np.diag(float(fx["r_pr"]) * np.ones(ns)), {"dt": 1.0}, None,
                 {"sat_pos": sat[b, k, :ns]})
    nb += 1
cpu_dt = time.perf_counter() - t0

res = {"metric": "EKF filter-step updates/s", "value": steps / wall, "unit": "filter-steps/s",
       "workload": f"gnss_stationary EKF recipe (n=5, 12 satellite slots, T={T}) x B={B} filters, "
                   f"inputs {LAYOUT}",
       "B": B, "T": T, "ms_per_launch": wall * 1e3,
       "kernel": "mhe_ekf::k_ekf_lane (diagonal R, one filter per lane)",
       "roofline": {"bound": "hbm", "achieved": by * steps / wall / 1e9, "peak": 8000.0, "unit": "GB/s",
                    "frac": by * steps / wall / 1e9 / 8000.0, "bytes_per_step": by,
                    "flops_per_step": fl, "achieved_tflops": fl * steps / wall / 1e12},
       "general_R_kernel": {"kernel": "mhe_ekf::k_ekf (one wavefront per filter, augmented Cholesky sweep)",
                            "ms_per_launch": wave_ms, "value": steps / (wave_ms * 1e-3),
                            "max_rel_dmu_vs_lane": dmu},
       "cpu_baseline": {"value": nb * T / cpu_dt, "unit": "filter-steps/s", "cores": 1, "kind": "port",
                        "sample": f"{nb} filters x {T} steps with oracle/ekf.py (the reference's update, "
                                  f"np.linalg.inv), one core, {cpu_dt:.1f} s"}}
print(json.dumps(res))
