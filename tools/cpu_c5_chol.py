"""CPU lower bound for one C5 trajectory-iteration (d = 8040): np.linalg.cholesky of one
d x d SPD matrix on the host threads, median of 3 after a warm-up.  The factorization
alone -- the mixed-row assembly is not included, so this bounds the CPU time from below.
    python tools/cpu_c5_chol.py
"""
import json, os, time
import numpy as np
d = 8040
rng = np.random.default_rng(0)
A = rng.normal(size=(d, d))
H = A @ A.T + d * np.eye(d)
t0 = time.perf_counter(); np.linalg.cholesky(H); t1 = time.perf_counter()
reps = []
for _ in range(3):
    t0 = time.perf_counter(); L = np.linalg.cholesky(H); reps.append(time.perf_counter() - t0)
med = float(np.median(reps))
print(json.dumps({"config": "C5", "d": d, "what": "np.linalg.cholesky of one d x d SPD matrix (the factorization alone: a LOWER bound on one C5 trajectory-iteration on CPU; the mixed-row assembly is not included)", "seconds_median_of_3": med, "gflops": d**3 / 3 / med / 1e9, "threads": len(os.sched_getaffinity(0)), "host": "build container"}))
