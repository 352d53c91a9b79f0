"""World-size-2 data-parallel path on CPU (gloo): per-rank shards, one-time
constant broadcast, sum / max reductions -- the same plumbing bench.py uses
over RCCL.  The per-rank work is the oracle's CPU port of the GN iteration."""
import os
import socket

import numpy as np
import torch
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, ws, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(ws), RANK=str(rank),
                      LOCAL_RANK=str(rank))
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "nlp-filter_amd"), root]
    from mhe import configs, dist
    from oracle import gn
    dist.init("gloo")
    w = configs.make_c2(B=4, N=20, seed=dist.shard_seed(1, rank))
    # constants: rank 0's copy is broadcast; every rank must hold identical bytes
    Dt = torch.tensor(w.cpm.D if rank == 0 else np.zeros_like(w.cpm.D))
    dist.broadcast_(Dt, 0)
    same = bool(np.array_equal(Dt.numpy(), w.cpm.D))
    pb = gn.Problem(w.N, w.T, w.n, w.m, w.dyn, w.meas, Dt.numpy(), (w.T / 2) * w.cpm.w,
                    w.cpm.lagrange_matrix(w.t_meas), w.Qw, w.Rw)
    port = gn.CpuPort(pb)
    X = port.iteration(w.X_init, np.broadcast_to(w.U, (w.B,) + w.U.shape[1:]), w.Y)
    updates = w.B * w.P * 1
    total = dist.sum_over_ranks(updates, "cpu")
    tmax = dist.max_over_ranks(float(rank + 1), "cpu")
    out[rank] = (same, total, tmax, float(np.abs(X).sum()), float(w.Y.sum()))
    torch.distributed.destroy_process_group()


def test_two_rank_gloo_sharding():
    ws = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(ws, _free_port(), out), nprocs=ws, join=True)
    r0, r1 = out[0], out[1]
    assert r0[0] and r1[0]                       # broadcast constants identical
    assert r0[1] == r1[1] == 2 * 4 * 21          # weak scaling: sum of per-rank updates
    assert r0[2] == r1[2] == 2.0                 # max over ranks
    assert r0[4] != r1[4]                        # distinct seeded shards


def _strong_worker(rank, ws, port, out, total, iters):
    """bench.py's strong path on CPU: rank_workload's shard of one seeded batch, the
    constants received from rank 0 (a rank > 0 starts from zeros), `iters` GN iterations
    of the oracle's CPU port, the shards' X gathered to compare with one rank."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(ws), RANK=str(rank),
                      LOCAL_RANK=str(rank))
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "nlp-filter_amd"), root]
    import bench
    from mhe import dist
    from oracle import gn
    dist.init("gloo")
    w = bench.rank_workload(ws, rank, global_batch=total, N=20)
    consts = np.concatenate([w.cpm.D.ravel(), w.cpm.w, w.Qw.ravel()])
    buf = torch.tensor(consts if rank == 0 else np.zeros_like(consts))
    dist.broadcast_(buf, 0)
    P = w.P
    D = buf[:P * P].numpy().reshape(P, P)
    wq = buf[P * P:P * P + P].numpy()
    Qw = buf[P * P + P:].numpy().reshape(w.n, w.n)
    pb = gn.Problem(w.N, w.T, w.n, w.m, w.dyn, w.meas, D, (w.T / 2) * wq, w.cpm.lagrange_matrix(w.t_meas), Qw, w.Rw)
    port = gn.CpuPort(pb)
    X = w.X_init
    for _ in range(iters):
        X = port.iteration(X, np.broadcast_to(w.U, (w.B,) + w.U.shape[1:]), w.Y)
    parts = [None] * ws
    torch.distributed.all_gather_object(parts, (w.shard, X, w.Y))
    total_updates = dist.sum_over_ranks(w.B * iters, "cpu")
    out[rank] = (parts, total_updates)
    torch.distributed.destroy_process_group()


def test_two_rank_strong_split_equals_one_rank():
    """Strong scaling (bench.py's default): the two ranks' shards of the seeded batch are
    the single-rank batch bitwise (inputs and iterates after 3 GN iterations), and the
    summed iteration count is B * iters."""
    import bench
    from mhe import configs
    from oracle import gn
    total, iters, ws = 9, 3, 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_strong_worker, args=(ws, _free_port(), out, total, iters), nprocs=ws, join=True)
    parts, upd = out[0]
    assert out[1][1] == upd == total * iters
    assert [p[0] for p in parts] == [(0, 5), (5, 9)]
    one = bench.rank_workload(1, 0, global_batch=total, N=20)
    assert one.shard == (0, total)
    full = configs.make_c2(B=total, seed=1, N=20)
    assert np.array_equal(full.Y, one.Y) and np.array_equal(full.X_init, one.X_init)
    pb = gn.Problem(one.N, one.T, one.n, one.m, one.dyn, one.meas, one.cpm.D, (one.T / 2) * one.cpm.w,
                    one.cpm.lagrange_matrix(one.t_meas), one.Qw, one.Rw)
    port = gn.CpuPort(pb)
    X = one.X_init
    for _ in range(iters):
        X = port.iteration(X, np.broadcast_to(one.U, (total,) + one.U.shape[1:]), one.Y)
    assert np.array_equal(np.concatenate([p[2] for p in parts]), one.Y)
    assert np.array_equal(np.concatenate([p[1] for p in parts]), X)


def test_shard_range_partitions():
    from mhe import dist
    for total in (0, 1, 7, 1024, 1025):
        for ws in (1, 2, 3, 8):
            parts = [dist.shard_range(total, ws, r) for r in range(ws)]
            assert parts[0][0] == 0 and parts[-1][1] == total
            assert all(a[1] == b[0] for a, b in zip(parts, parts[1:]))
            assert max(h - l for l, h in parts) - min(h - l for l, h in parts) <= 1
