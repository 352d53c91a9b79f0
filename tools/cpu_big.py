"""CPU baseline for the large-system configs (tools only; SURVEY.md §8(d): "for C3-C5,
time a B' = 64 subset on CPU and report per-trajectory rates").

    python tools/cpu_big.py [C3|C4|C5 ...] [--subset B'] [--threads T]

Times the oracle's vectorised GN iteration (oracle.gn.gn_step_batched: normal
equations by einsum, np.linalg.cholesky on the (B', d, d) stack, two triangular
solves; C5's extra variables and constraints through oracle.gn_general's dense KKT
step) on a B'-trajectory subset of the same seeded workload, after one warm-up
iteration, and reports seconds per trajectory-iteration and the implied
point-updates/s.  A subset rate, not extrapolated: the label says so.  The oracle is
the checker here, timed as the CPU port of the same algorithm (cpu_baseline kind
"port").
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "nlp-filter_amd"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

from mhe import configs  # noqa: E402
from oracle import gn  # noqa: E402

DEFAULT_SUBSET = {"C3": 64, "C4": 8, "C5": 16}


def problem(w):
    return gn.Problem(w.N, w.T, w.n, w.m, w.dyn, w.meas, w.cpm.D, (w.T / 2) * w.cpm.w,
                      w.cpm.lagrange_matrix(w.t_meas), w.Qw, w.Rw, Pw=w.Pw, meas_static=w.meas_static)


def one_config(cfg, Bs, reps, N=None):
    w = configs.CONFIGS[cfg](B=Bs, **({} if N is None else {"N": N}))
    U = None if w.U is None else np.broadcast_to(w.U, (w.B,) + w.U.shape[1:])
    PAR = None if w.PAR is None else np.broadcast_to(w.PAR, (w.B,) + w.PAR.shape[1:])
    if w.meas == "mixed":  # C5: mixed rows (+ extra variables z) -> oracle.gn_general's dense KKT step
        from oracle import gn_general as gg
        Z0 = getattr(w, "Z_init", None)
        gp = gg.GeneralProblem(w.N, w.T, w.n, w.m, w.dyn, "mixed", w.cpm.D, (w.T / 2) * w.cpm.w,
                               w.cpm.lagrange_matrix(w.t_meas), w.Qw, w.Rw,
                               **({} if Z0 is None else {"n_extra": Z0.shape[-1]}))
        step = lambda X: gg.gauss_newton_general(gp, X, Z0, U, w.Y, w.PAR, None,  # noqa: E731
                                                 max_iter=1, tol=0.0)
    else:
        pb = problem(w)
        step = lambda X: gn.gn_step_batched(pb, X, U, w.Y, PAR)  # noqa: E731
    step(w.X_init)  # warm-up (BLAS thread pool, page-in)
    t0 = time.perf_counter()
    for _ in range(reps):
        step(w.X_init)
    dt = (time.perf_counter() - t0) / reps
    return {"config": cfg, "workload": w.name, "subset_B": Bs, "d": w.P * w.n, "P": w.P,
            "s_per_traj_iter": dt / Bs, "pt_updates_per_s": Bs * w.P / dt,
            "note": f"CPU subset of {Bs} trajectories, {reps} timed GN iteration(s) after 1 warm-up"
                    + ("" if N is None else f"; REDUCED horizon N = {N} (not the config's shape)")}


def main():
    args = sys.argv[1:]
    cfgs = [a for a in args if a in DEFAULT_SUBSET] or ["C3", "C4"]
    n_red = int(args[args.index("--N") + 1]) if "--N" in args else None  # reduced horizon (C5: labelled)
    sub = int(args[args.index("--subset") + 1]) if "--subset" in args else None
    threads = len(os.sched_getaffinity(0))
    for cfg in cfgs:
        r = one_config(cfg, sub or DEFAULT_SUBSET[cfg], 1, n_red)
        r["threads"] = int(os.environ.get("OMP_NUM_THREADS", threads))
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
