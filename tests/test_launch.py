"""mhe.launch: ``python bench.py --gpus N`` starts its own N ranks (no torch.distributed.run
around it), before any GPU call.  Driven here through the same spawn code with a gloo
world of 2 on the CPU (tests/dist_child/rank_job.py: bench.py's rank plumbing)."""
import json
import os
import subprocess
import sys

import pytest

from mhe import launch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = os.path.join(ROOT, "tests", "dist_child", "rank_job.py")


def _env_clean(monkeypatch):
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        monkeypatch.delenv(k, raising=False)


def test_launch_two_gloo_ranks(monkeypatch, tmp_path):
    _env_clean(monkeypatch)
    out = tmp_path / "out.txt"
    with open(out, "w") as f:
        rc = launch.launch([sys.executable, CHILD], 2, stdout=f)
    assert rc == 0
    lines = [ln for ln in out.read_text().splitlines() if ln.startswith("{")]  # (gloo prints its own lines)
    assert len(lines) == 1                       # rank 0 alone prints
    r = json.loads(lines[0])
    assert r["world"] == 2 and r["total"] == 8 * 21 and r["same"] == 2.0
    assert r["ranks_seen"] == 2 and r["constants_ok_ranks"] == 2  # counted by collectives
    assert r["env"] == ["127.0.0.1", "0"]


def test_launch_failing_rank_ends_the_job(monkeypatch, tmp_path):
    """Rank 1 exits 3 after init; rank 0 would wait in its broadcast forever: the
    launcher returns 3 and terminates it."""
    _env_clean(monkeypatch)
    with open(tmp_path / "o.txt", "w") as f:
        rc = launch.launch([sys.executable, CHILD, "--fail-rank", "1"], 2, stdout=f, stderr=subprocess.STDOUT,
                           grace_s=5.0)
    assert rc == 3


def test_relaunch_is_a_no_op_inside_a_rank(monkeypatch):
    monkeypatch.setenv("WORLD_SIZE", "2")
    launch.relaunch_if_needed(2)                 # returns: already a rank
    monkeypatch.delenv("WORLD_SIZE")
    launch.relaunch_if_needed(1)                 # returns: one process


def test_bench_self_launch_reaches_the_ranks(monkeypatch, tmp_path):
    """bench.py --gpus 2 with no launcher around it: the parent starts two ranks (here
    without a GPU each rank stops at its first device call -- the point is that the
    parent no longer refuses with 'WORLD_SIZE=1' and that a rank's failure is the
    job's exit code)."""
    _env_clean(monkeypatch)
    pytest.importorskip("torch")
    import torch
    if torch.cuda.is_available():
        pytest.skip("CPU-only check (on a GPU box the bench runs for real)")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1",
                        "--warmup", "0", "--no-cpu"], capture_output=True, text=True, timeout=300)
    assert p.returncode != 0
    assert "WORLD_SIZE=1" not in p.stderr + p.stdout
