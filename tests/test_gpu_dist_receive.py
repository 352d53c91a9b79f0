"""The multi-GPU constants hand-off on one device (bench.py's ranks > 0).

A rank > 0 constructs its solver with constants="receive" (only the buffer is
allocated), gets rank 0's bytes by one RCCL broadcast (mhe.dist.broadcast_) and calls
constants_ready().  RCCL needs one device per rank, so on a one-GPU box the broadcast is
stood in for by a device copy of the same bytes; everything around it is the code every
rank > 0 runs:
  * before constants_ready() the solver refuses to launch;
  * after it, the receiving solver's solve equals the building solver's BITWISE (both
    device paths);
  * bytes built for other dims are refused per trajectory by the kernels' layout stamp
    (status 4 = MHE_STATUS_BAD_CONSTANTS, no iterations, X untouched, cost NaN).
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

from mhe import _lib, configs, solver  # noqa: E402


def _np(ts):
    return [t.cpu().numpy() for t in ts]


CASES = {
    "register_c2": lambda: (configs.make_c2(B=16, N=100), configs.make_c2(B=16, N=99)),
    "large_c3": lambda: (configs.make_c3(B=4, N=60), configs.make_c3(B=4, N=61)),
}


@pytest.mark.parametrize("case", sorted(CASES))
def test_received_constants_solve_bitwise_and_stamp_refusal(case):
    w, w_other = CASES[case]()
    src = solver.from_workload(w)                          # rank 0: builds
    dst = solver.from_workload(w, constants="receive")     # rank > 0: allocates only
    assert dst.cbuf.numel() == src.cbuf.numel()
    with pytest.raises(_lib.MheCallError):
        dst.solve(w.X_init, w.U, w.Y, w.PAR, max_iter=1)
    dst.cbuf.copy_(src.cbuf)                               # stands in for dist.broadcast_(cbuf, 0)
    dst.constants_ready()
    a = _np(src.solve(w.X_init, w.U, w.Y, w.PAR, max_iter=4, tol=0.0))
    b = _np(dst.solve(w.X_init, w.U, w.Y, w.PAR, max_iter=4, tol=0.0))
    for x, y in zip(a, b):
        assert np.array_equal(x, y)
    assert a[2].tolist() == [4] * w.B

    # bytes built for other dims (another N): the stamp at offset 0 differs
    other = solver.from_workload(w_other)
    bad = solver.from_workload(w, constants="receive")
    k = min(bad.cbuf.numel(), other.cbuf.numel())
    bad.cbuf.zero_()
    bad.cbuf[:k].copy_(other.cbuf[:k])
    bad.constants_ready()
    X, cost, iters, status = _np(bad.solve(w.X_init, w.U, w.Y, w.PAR, max_iter=3, tol=0.0))
    assert status.tolist() == [solver.STATUS_BAD_CONSTANTS] * w.B and iters.tolist() == [0] * w.B
    assert np.array_equal(X, w.X_init) and np.isnan(cost).all()
