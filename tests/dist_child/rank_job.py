"""One rank of a CPU (gloo) job started by mhe.launch -- tests/test_launch.py.

The same plumbing bench.py's ranks use, on the CPU: rank / world from the environment
the launcher set, gloo init at MASTER_ADDR:MASTER_PORT, rank 0's constants broadcast,
the strong split of one seeded batch, the max-over-ranks time and the sum of the
per-rank work; rank 0 prints one JSON line.  ``--fail-rank r`` makes rank r exit 3
after init (the others then block in the next collective until the launcher ends them).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "nlp-filter_amd"), ROOT]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from mhe import configs, dist  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--fail-rank", type=int, default=-1)
args = ap.parse_args()
world, rank, local = dist.world()
dist.init("gloo")
if rank == args.fail_rank:
    sys.exit(3)
w = configs.make_c2(B=8, N=20, seed=1, shard=dist.shard_range(8, world, rank))
D = torch.tensor(w.cpm.D if rank == 0 else np.zeros_like(w.cpm.D))
dist.broadcast_(D, 0)
t0 = time.perf_counter()
work = w.B * w.P
wall = dist.max_over_ranks(time.perf_counter() - t0, "cpu")
total = dist.sum_over_ranks(work, "cpu")
same = dist.sum_over_ranks(float(np.array_equal(D.numpy(), w.cpm.D)), "cpu")
ranks_seen, ok_ranks = dist.verify_broadcast(D, "cpu")  # bench.py's self-proving rank count
if rank == 0:
    print(json.dumps({"world": world, "total": total, "same": same, "wall": wall,
                      "ranks_seen": ranks_seen, "constants_ok_ranks": ok_ranks,
                      "env": [os.environ["MASTER_ADDR"], os.environ["LOCAL_RANK"]]}))
torch.distributed.destroy_process_group()
