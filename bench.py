"""Benchmark: Gauss-Newton collocation-point updates/sec (BASELINE.json metric).

Workload (BASELINE.json configs[1] and north star): van der Pol
(nlp/dynamics.py:61-66), full_state measurements, N=100 (P=101 CGL nodes), T=10,
M=101, ONE seeded batch of 1024 independent trajectories split over the G GPUs
(strong scaling, the north star's "batch-1024 at 1, 2, 4 and 8 MI355X"): rank r
generates only its contiguous shard [r*1024/G, (r+1)*1024/G) of that batch
(configs.make_c2(shard=...), bitwise the slice of the full batch), rank 0 builds
the model constants and the other ranks RECEIVE them by one RCCL broadcast
(setup, untimed); the only other collectives are the max-over-ranks of the elapsed
time and the sum of the iteration counts.  ``--weak`` gives every rank its own
seeded batch of ``--batch`` trajectories instead (weak scaling).

One step = one mhe_solve launch over the resident shard doing exactly GN_ITERS
full Gauss-Newton iterations per trajectory (tol = 0): residual + Jacobian,
J^T W J / J^T W r assembly, register-tiled Cholesky, two triangular solves,
update.  value = (all ranks) sum of B_r * P * GN_ITERS * K / max-rank wall.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--no-cpu] [--global-batch G] [--weak [--batch B]]
N > 1: under torch.distributed.run (RANK/LOCAL_RANK/WORLD_SIZE set) each process is one
rank; run plainly, bench.py starts the N ranks itself (mhe.launch, before any GPU call)
and exits with their code.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "nlp-filter_amd"))
sys.path.insert(0, ROOT)

GN_ITERS = 10
FP64_PEAK_TFLOPS = 78.6   # MI355X FP64 vector / matrix (spec); MI355X_MICROARCH.md lists no fp64 row
HBM_PEAK_GBS = 8000.0


def algorithmic_flops_per_traj_iter(P, n, M):
    """FLOPs one GN iteration of one trajectory needs (d = P n):
    Cholesky d^3/3, two triangular solves 2 d^2, X-dependent J^T W J terms
    (6 flops per lower-triangle element), residual/gradient mat-vecs
    (D X, D^T V, Phi X, Phi^T G e: 2 P^2 n + 2 P^2 n + 2 M P n + 2 M P n)."""
    d = P * n
    return d ** 3 / 3.0 + 2.0 * d * d + 6.0 * d * (d + 1) / 2.0 + 4.0 * P * P * n + 4.0 * M * P * n


def gn_kernel_name(s, B, stream):
    """The k_gn instance the library's launch_gn selects for this solver and per-GPU
    batch on this stream's device (mhe_solve_kernel_name: the same conditions as the
    launch -- batch vs CUs, Huber, bounds, LDS fit)."""
    import ctypes
    buf = ctypes.create_string_buffer(256)
    rc = s.lib.mhe_solve_kernel_name(s.dims, B, ctypes.c_void_p(stream.cuda_stream), buf, 256)
    return buf.value.decode() if rc == 0 else f"unknown (rc {rc})"


def survey_flops_per_traj_iter(P, n, E, nnz_g):
    """SURVEY.md §8(d) algorithmic FLOPs per trajectory per GN iteration (the
    roofline's `achieved` basis): Cholesky d^3/3 + two triangular solves 2 d^2
    + epoch-grouped measurement contraction sum_e P^2 nnz(G_e) + dynamics terms
    2 P^2 n^2 + 4 P n^3.  C2 (P=101, n=2, E=101, nnz(G_e)=2 for full_state with
    diagonal R): 4.975 MFLOP = 49.3 KFLOP per collocation point, as §8(d)'s table.
    The kernel executes fewer (the contraction is constant for a linear h and
    precomputed once): see algorithmic_flops_per_traj_iter."""
    d = P * n
    return d ** 3 / 3.0 + 2.0 * d * d + E * P * P * nnz_g + 2.0 * P * P * n * n + 4.0 * P * n ** 3


def algorithmic_bytes_per_traj(P, n, m, M, p):
    """HBM bytes per trajectory per launch: X in, U, Y in, X out, cost/iters/status.
    (Constants -- D, Phi, the constant J^T W J tiles -- are shared by every
    workgroup and L2/MALL resident; they are not per-trajectory traffic.)"""
    return 8.0 * (P * n + M * p + P * n) + 8 + 4 + 4


def cpu_baseline(w, iters, sample_B, target_s=10.0):
    """The oracle's CPU port of the same GN iteration on the host cores
    (thread pool over trajectories, BLAS single-threaded inside each worker).
    Repeats the sample until ~target_s of wall time has been spent."""
    from concurrent.futures import ThreadPoolExecutor
    from threadpoolctl import threadpool_limits
    from oracle import gn

    cores = len(os.sched_getaffinity(0))
    cores = min(cores, int(os.environ.get("OMP_NUM_THREADS", cores)))
    pb = gn.Problem(w.N, w.T, w.n, w.m, w.dyn, w.meas, w.cpm.D, (w.T / 2) * w.cpm.w,
                    w.cpm.lagrange_matrix(w.t_meas), w.Qw, w.Rw)
    port = gn.CpuPort(pb)
    B = min(sample_B, w.B)
    U = np.broadcast_to(w.U, (B,) + w.U.shape[1:])
    chunks = np.array_split(np.arange(B), cores)

    def work(ix):
        X = w.X_init[ix].copy()
        for _ in range(iters):
            X = port.iteration(X, U[ix], w.Y[ix])
        return X

    # the median of >= 5 repetitions after a warm-up, each repetition one
    # pass of `iters` GN iterations over the sample, repeated until ~target_s of wall
    reps = []
    with threadpool_limits(1), ThreadPoolExecutor(max_workers=cores) as ex:
        work(chunks[0][:2])  # warm-up
        t0 = time.perf_counter()
        while len(reps) < 5 or time.perf_counter() - t0 < target_s:
            t1 = time.perf_counter()
            list(ex.map(work, chunks))
            reps.append(time.perf_counter() - t1)
    dt = time.perf_counter() - t0
    med = float(np.median(reps))
    # the 1-core figure: a 64-trajectory slice, ~target_s / 3
    one = np.arange(min(64, B))
    reps1 = []
    with threadpool_limits(1):
        work(one[:2])
        t0 = time.perf_counter()
        while len(reps1) < 5 or time.perf_counter() - t0 < target_s / 3:
            t1 = time.perf_counter()
            work(one)
            reps1.append(time.perf_counter() - t1)
    med1 = float(np.median(reps1))
    return {"value": B * w.P * iters / med, "unit": "GN collocation-point updates/s", "cores": cores,
            "kind": "port",
            "value_1core": len(one) * w.P * iters / med1,
            "statistic": "median over repetitions",
            "sample": f"median of {len(reps)} repetitions ({dt:.1f} s wall) of ({B} of the {w.B} C2 trajectories x "
                      f"{iters} GN iterations) with oracle.gn.CpuPort (same algorithm: constant J^T W J part "
                      f"precomputed, LAPACK dpotrf + 2 trsv per trajectory), {cores} worker threads; value_1core: "
                      f"median of {len(reps1)} repetitions of {len(one)} trajectories x {iters} iterations on one "
                      f"thread"}


def rank_workload(world, rank, global_batch=1024, weak=False, batch=1024, N=100):
    """The C2 trajectories rank `rank` of `world` solves.  Strong (default): its
    contiguous shard of ONE seeded batch of `global_batch` (seed 1), generated alone;
    weak: its own seeded batch of `batch` (seed 1 + 1000 rank).  tests/test_dist_gloo.py
    checks that the shards of the strong split are the full batch, bitwise."""
    from mhe import configs, dist
    if weak:
        return configs.make_c2(B=batch, seed=dist.shard_seed(1, rank), N=N)
    return configs.make_c2(B=global_batch, seed=1, N=N, shard=dist.shard_range(global_batch, world, rank))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--global-batch", type=int, default=1024,
                    help="strong scaling (default): this many trajectories in total, split over the "
                         "ranks (dist.shard_range) -- the north star's fixed batch-1024 at 1/2/4/8 GPUs")
    ap.add_argument("--weak", action="store_true",
                    help="weak scaling instead: --batch trajectories per GPU, a seeded batch per rank")
    ap.add_argument("--batch", type=int, default=1024, help="trajectories per GPU with --weak")
    ap.add_argument("--iters", type=int, default=GN_ITERS)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--cpu-sample", type=int, default=1024)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    args = ap.parse_args()

    # `python bench.py --gpus N` on its own: start the N ranks here, before anything
    # touches the GPU (mhe.launch imports no torch), and exit with their code.  Under
    # torch.distributed.run (WORLD_SIZE set) this returns at once.
    from mhe import launch
    launch.relaunch_if_needed(args.gpus)

    import torch

    from mhe import configs, dist, solver

    world, rank, local = dist.world()
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    dist.init("nccl", dev)

    w = rank_workload(world, rank, args.global_batch, args.weak, args.batch)
    # model constants: built once on rank 0; the other ranks only allocate the buffer and
    # receive rank 0's bytes over RCCL/xGMI (one-time, untimed).  The kernels check the
    # buffer's layout stamp against their own dims before using it.
    s = solver.from_workload(w, device=dev, constants="build" if rank == 0 else "receive")
    dist.broadcast_(s.cbuf, src=0)
    if rank != 0:
        s.constants_ready()
    # the line proves its rank count by collectives: every rank adds 1, and 1 more when its
    # received constants carry rank 0's digest (the layout stamp and every byte after it)
    ranks_seen, constants_ok_ranks = dist.verify_broadcast(s.cbuf, dev)
    if ranks_seen != world or constants_ok_ranks != world:
        raise SystemExit(f"rank {rank}: {ranks_seen} ranks seen, {constants_ok_ranks} with rank 0's constants "
                         f"(WORLD_SIZE={world})")
    staged = s.prepare(w.X_init, w.U, w.Y)
    B = w.B
    outs = (torch.empty_like(staged[0]), torch.empty(B, dtype=torch.float64, device=dev),
            torch.empty(B, dtype=torch.int32, device=dev), torch.empty(B, dtype=torch.int32, device=dev))
    stream = torch.cuda.current_stream(dev)

    for _ in range(args.warmup):
        s.solve_staged(staged, outs, args.iters, 0.0, stream)
    torch.cuda.synchronize(dev)
    dist.barrier()
    torch.cuda.synchronize(dev)
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        s.solve_staged(staged, outs, args.iters, 0.0, stream)
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    dist.barrier()
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    kern_ms = ev0.elapsed_time(ev1) / args.steps  # launches are back to back on `stream`

    wall = dist.max_over_ranks(wall, dev)
    iters_done = dist.sum_over_ranks(outs[2].sum().item(), dev)
    total_updates = iters_done * w.P * args.steps  # sum over ranks of B * P * iters per step
    value = total_updates / wall

    if rank == 0:
        fl = survey_flops_per_traj_iter(w.P, w.n, w.M, int(np.count_nonzero(np.diag(w.Rw[0])))) * B * args.iters
        achieved = fl / (kern_ms * 1e-3) / 1e12
        fl_exec = algorithmic_flops_per_traj_iter(w.P, w.n, w.M) * B * args.iters
        rec = {
            "metric": "Gauss-Newton collocation-point updates/sec",
            "value": value,
            "unit": "GN collocation-point updates/s",
            "n_gpus": world,
            "ranks_seen": ranks_seen,              # all-reduce sum of 1 over the process group
            "constants_ok_ranks": constants_ok_ranks,  # ranks whose broadcast constants match rank 0's
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": wall / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak" if args.weak else "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (seeded van der Pol truth via RK4 + Gaussian noise, R/Q from estimation_example.py)",
            "config": {"workload": "C2 van_der_pol: n=2, m=1, full_state p=2, N=100 (P=101, d=202), T=10, M=101",
                       "global_batch": B * world if args.weak else args.global_batch,
                       "batch_per_gpu": B,  # rank 0's (strong: its shard_range of the global batch)
                       "gn_iters_per_step": args.iters,
                       "parallelism": f"dp{world} (independent trajectories; RCCL broadcast of constants only)"},
            "roofline": {"bound": "mfma", "achieved": achieved, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                         "frac": achieved / FP64_PEAK_TFLOPS, "traffic": None,
                         "kernel": gn_kernel_name(s, B, stream),
                         "kernel_ms": kern_ms,
                         "flops_per_launch": fl,
                         "flops_basis": "SURVEY.md 8(d): d^3/3 + 2d^2 + sum_e P^2 nnz(G_e) + 2P^2n^2 + 4Pn^3 "
                                        "per trajectory-iteration x B x iters",
                         "executed_flops_per_launch": fl_exec,
                         "executed_tflops": fl_exec / (kern_ms * 1e-3) / 1e12,
                         "executed_frac": fl_exec / (kern_ms * 1e-3) / 1e12 / FP64_PEAK_TFLOPS,
                         "hbm_algorithmic_GBs": algorithmic_bytes_per_traj(w.P, w.n, w.m, w.M, w.p) * B / (kern_ms * 1e-3) / 1e9},
        }
        pmc = os.path.join(ROOT, "profiles", "pmc_summary.json")
        if os.path.exists(pmc):
            # PMC counters come from separate rocprofv3 passes (tools/profile_round.sh);
            # they are attached only when they measured THIS build of libmhe.so
            from mhe._lib import lib_digest
            with open(pmc) as f:
                ps = json.load(f)
            same = (ps.get("kernel_sig") == "k_gn<DynVanDerPol" and ps.get("batch") == B
                    and ps.get("iters") == args.iters)
            if same and ps.get("lib_sha") == lib_digest():
                rec["roofline"]["traffic"] = ps["hbm_bytes_per_launch"]
                rec["roofline"]["traffic_note"] = ps["note"] + f"; profiled build {ps['lib_sha']} ({ps['tag']})"
                rec["roofline"]["mfma_util_pmc"] = ps.get("mfma_util")
                if ps.get("trace_ms_timed_launches"):
                    # the same quantity as kernel_ms from the rocprof trace of that build: the
                    # average over the profiled bench's timed launches (its warm-up excluded)
                    rec["roofline"]["kernel_ms_rocprof_timed"] = ps["trace_ms_timed_launches"]
                    rec["roofline"]["kernel_ms_rocprof_all"] = ps["trace_ms_all_launches"]
                    # frac on the rocprof basis (the tracer's own timing of those launches,
                    # profiles/<tag>_kernel_stats.csv), next to frac on the HIP-event basis
                    rec["roofline"]["frac_rocprof_timed"] = (fl / (ps["trace_ms_timed_launches"] * 1e-3) / 1e12
                                                             / FP64_PEAK_TFLOPS)
            elif same:
                rec["roofline"]["traffic_note"] = (f"profiles/pmc_summary.json measured build {ps.get('lib_sha')}, "
                                                   f"not this libmhe.so ({lib_digest()}): traffic omitted")
        if world == 1 and not args.no_cpu:
            rec["cpu_baseline"] = cpu_baseline(w, args.iters, args.cpu_sample, args.cpu_seconds)
        print(json.dumps(rec))
    if world > 1:
        import torch.distributed as tdist
        tdist.destroy_process_group()


if __name__ == "__main__":
    main()
