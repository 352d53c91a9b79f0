"""Self-launch of a one-process-per-GPU job (no torch import: nothing here may touch
the GPU, so the parent can start its ranks before any HIP call).

``python bench.py --gpus N`` without a ``torch.distributed.run`` around it comes here:
the parent starts N copies of the same command as ranks 0..N-1 of one job (RANK,
LOCAL_RANK, WORLD_SIZE, LOCAL_WORLD_SIZE, MASTER_ADDR = 127.0.0.1, a free MASTER_PORT),
waits for all of them, and exits with the first failing rank's code; if one rank fails
the others are terminated (a rank blocked in a collective would otherwise wait for the
dead one forever).  Rank 0 prints the result; the parent prints nothing of its own.
"""
import os
import socket
import subprocess
import sys
import time


def free_port(host="127.0.0.1"):
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind((host, 0))
        return s.getsockname()[1]


def rank_env(rank, world, port, base=None):
    env = dict(os.environ if base is None else base)
    env.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world),
               MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on this pool (RCCL)
    return env


def launch(argv, nprocs, stdout=None, stderr=None, poll_s=0.05, grace_s=10.0):
    """Run ``argv`` as ranks 0..nprocs-1 of one job on this node; returns 0 when every
    rank exits 0, else the first nonzero exit code observed (a rank killed by a
    signal counts as 128 + signal)."""
    if nprocs < 1:
        raise ValueError("nprocs must be >= 1")
    port = free_port()
    procs = [subprocess.Popen(argv, env=rank_env(r, nprocs, port), stdout=stdout, stderr=stderr)
             for r in range(nprocs)]
    rc = 0
    try:
        while True:
            codes = [p.poll() for p in procs]
            bad = [c for c in codes if c is not None and c != 0]
            if bad:
                rc = bad[0] if bad[0] > 0 else 128 - bad[0]
                break
            if all(c == 0 for c in codes):
                return 0
            time.sleep(poll_s)
    except BaseException:
        rc = rc or 1
        raise
    finally:
        if rc:
            for p in procs:
                if p.poll() is None:
                    p.terminate()
            t0 = time.time()
            for p in procs:
                try:
                    p.wait(timeout=max(0.1, grace_s - (time.time() - t0)))
                except subprocess.TimeoutExpired:
                    p.kill()
                    p.wait()
    return rc


def relaunch_if_needed(nprocs, argv=None):
    """In the parent of a self-launched job (WORLD_SIZE unset, nprocs > 1): start the
    ranks and exit with their code.  Returns (does nothing) inside a rank or for one
    process."""
    if nprocs <= 1 or "WORLD_SIZE" in os.environ:
        return
    argv = [sys.executable] + ([os.path.abspath(sys.argv[0])] + sys.argv[1:] if argv is None else argv)
    sys.stdout.flush()
    sys.exit(launch(argv, nprocs))
