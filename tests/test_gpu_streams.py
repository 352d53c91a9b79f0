"""Stream-ordered launches (include/mhe.h: every call only enqueues on its stream;
mhe.streams): solves on two side streams with no synchronisation in between give the
current-stream result bit for bit, on both device paths; the per-stream workspace
cache of the large-system path stays bounded."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

from mhe import configs, solver  # noqa: E402


@pytest.mark.parametrize("force_large", [False, True])
def test_side_streams_match_current_stream(force_large):
    w = configs.make_c2(B=6, N=40)
    s = solver.from_workload(w, force_large=force_large)
    ref = [t.cpu().numpy() for t in s.solve(w.X_init, w.U, w.Y, max_iter=5, tol=0.0)]
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    halves = (slice(0, 3), slice(3, 6))
    outs = []
    for st, sl in zip((s1, s2, s1), halves + (slice(0, 6),)):
        outs.append(s.solve(w.X_init[sl], w.U, w.Y[sl], max_iter=5, tol=0.0, stream=st))  # no sync in between
    torch.cuda.synchronize()
    for o, sl in zip(outs, halves + (slice(0, 6),)):
        for a, r in zip(o, ref):
            assert np.array_equal(a.cpu().numpy(), r[sl])
    assert len(s._ws) <= solver.BatchSolver.WS_CACHE
    for _ in range(4):  # more streams than the cache holds
        s.solve(w.X_init, w.U, w.Y, max_iter=1, tol=0.0, stream=torch.cuda.Stream())
    torch.cuda.synchronize()
    assert len(s._ws) <= solver.BatchSolver.WS_CACHE


def test_two_streams_chunked_under_a_small_budget():
    """the chunk budget on the large-system path with two streams in flight --
    a budget of two trajectories' workspace streams each solve in chunks through its own
    stream's workspace; both match the unchunked current-stream solve bit for bit."""
    w = configs.make_c2(B=6, N=40)
    s = solver.from_workload(w, force_large=True)
    ref = [t.cpu().numpy() for t in s.solve(w.X_init, w.U, w.Y, max_iter=4, tol=0.0)]
    per = s.lib.mhe_workspace_bytes(s.dims, 1)
    s.ws_budget = 2 * per
    try:
        assert s._chunk(6, None) == 2
        s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
        outs = [s.solve(w.X_init, w.U, w.Y, max_iter=4, tol=0.0, stream=st) for st in (s1, s2)]
        torch.cuda.synchronize()
    finally:
        s.ws_budget = None
    for o in outs:
        for a, r in zip(o, ref):
            assert np.array_equal(a.cpu().numpy(), r)
    assert len(s._ws) <= solver.BatchSolver.WS_CACHE
