"""Batched autonomous-car EKF throughput (autonomous-car.py:120-178 on mhe_ekf_run).

    python tools/bench_ekf_autocar.py [B] [reps]

Workload: the script's own plug-ins (discrete_vehicle_dynamics, n = 9, m = 2;
vehicle_sensors_model, 8-11 pseudoranges at every 10th step) on the 300-step input
of tests/golden/ekf_autocar.npz, replicated over B filters with perturbed priors
(synthetic), inputs batch-innermost, history kept.  Metric: filter-step updates/s =
B * T / kernel time (HIP events around one run_batch launch, inputs resident).

Algorithmic bytes per filter-step (average over the 300 steps): U (2) doubles and nz
(4 B) read every step, Z + satellite positions (4 doubles per row) on the correction
steps, the mu/S history (9 + 81 doubles) written: ~777 B -- HBM-bound.
CPU baseline: the oracle EKF (oracle/ekf.py: the reference's update with
np.linalg.inv and the script's plug-ins restated) on one host core over a bounded sample.
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
import utils.vehicle as veh  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
REPS = int(sys.argv[2]) if len(sys.argv) > 2 else 5
fx = dict(np.load(os.path.join(ROOT, "tests", "golden", "ekf_autocar.npz")))
car = dict(zip(("C_AF", "C_AR", "M", "D_F", "D_R", "I_Z"), fx["car"]))
dparams = {"dt": float(fx["dt"]), "car_params": car}
T, pmax, n = fx["U"].shape[0], fx["Z"].shape[1], 9
rng = np.random.default_rng(11)
mu0 = np.tile(fx["mu0"], (B, 1))
mu0[1:, :2] += rng.normal(size=(B - 1, 2))
S0 = np.tile(fx["S0"], (B, 1, 1))
# batch-innermost inputs: U (T,m,B), Z (T,pmax,B), nz (T,B), sat (T,pmax,3,B)
U = np.ascontiguousarray(np.repeat(fx["U"][..., None], B, -1))
Z = np.ascontiguousarray(np.repeat(fx["Z"][..., None], B, -1))
nz = np.ascontiguousarray(np.repeat(fx["nz"][:, None], B, -1).astype(np.int32))
sat = np.ascontiguousarray(np.repeat(fx["sat_pos"][..., None], B, -1))
R = np.stack([np.diag(float(fx["r_pr"]) * np.ones(pmax)) for _ in range(T)])
dev = torch.device("cuda", 0)
args = [torch.as_tensor(a, device=dev) for a in (mu0, S0, U, Z, nz, sat)]
Rt, Qt = torch.as_tensor(R, device=dev), torch.as_tensor(fx["Q"], device=dev)


def run(method="lane"):
    return ekf.run_batch(veh.discrete_vehicle_dynamics, veh.vehicle_sensors_model, args[0], args[1], args[2],
                         args[3], args[4], Qt, Rt, dparams["dt"], args[5], method=method, inputs="batch_inner",
                         dyn_params=dparams)


out = run()
torch.cuda.synchronize()
assert int(out[4].abs().sum().item()) == 0
del out  # the history buffers are reused by the timed calls (no allocation inside the timing)
run()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(REPS):
    run()
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / REPS
rows = float(fx["nz"].sum()) / T
bytes_step = 8 * 2 + 4 + rows * 4 * 8 + 8 * (9 + 81)
rate = B * T / (ms * 1e-3)

# CPU baseline: the oracle EKF, one core, bounded sample
from oracle import ekf as oe  # noqa: E402
nb, t0 = 0, time.perf_counter()
while time.perf_counter() - t0 < (0.0 if os.environ.get("NO_CPU") else 10.0) and nb < 64:
    f = oe.EKF(oe.discrete_vehicle_dynamics, oe.vehicle_sensors_model, mu0[nb], S0[nb])
    for k in range(T):
        ns = int(fx["nz"][k])
        f.update(fx["U"][k], fx["Z"][k, :ns] if ns else None, fx["Q"],
                 np.diag(float(fx["r_pr"]) * np.ones(ns)) if ns else None, dparams, None, {"sat_pos": fx["sat_pos"][k, :ns]})
    nb += 1
cpu_rate = nb * T / (time.perf_counter() - t0)
print(json.dumps({"workload": "autonomous-car EKF (discrete_vehicle_dynamics + vehicle_sensors_model, n=9)",
                  "B": B, "T": T, "kernel_ms": ms, "filter_steps_per_s": rate,
                  "bytes_per_filter_step": bytes_step, "achieved_GBs": rate * bytes_step / 1e9,
                  "hbm_frac": rate * bytes_step / 8e12,
                  "cpu_baseline": {"filter_steps_per_s": cpu_rate, "cores": 1, "kind": "port",
                                   "sample": f"{nb} filters x {T} steps, oracle EKF"}}))
