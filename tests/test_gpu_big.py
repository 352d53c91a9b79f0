"""Large-system GN path (csrc/mhe_big.h: workspace, HBM-resident tiles) vs the
register-resident kernel and the CPU oracle.

Tolerances as tests/test_gpu_parity.py (tests/tolerance.py): iterates <= 8 floor +
1e-10 (1 + max|X|) after the same number of iterations (floor: the oracle's own
change when every y moves by eps |y| -- pseudorange rounding), converged optimum
<= 8 floor + 1e-8 (1 + max|X|); iteration counts and statuses exact.  The two
device paths on identical inputs: 1e-10 (1 + max|X|).  force_large=True (mhe_dims.force_large) routes C2 through the large-system
path, so the two device paths are compared on identical inputs.
"""

import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

from mhe import _lib, configs, solver  # noqa: E402
from oracle import gn  # noqa: E402

import tolerance as tl  # noqa: E402


def _problem(w):
    return gn.Problem(w.N, w.T, w.n, w.m, w.dyn, w.meas, w.cpm.D, (w.T / 2) * w.cpm.w,
                      w.cpm.lagrange_matrix(w.t_meas), w.Qw, w.Rw, Pw=w.Pw, meas_static=w.meas_static)


def _U(w):
    return np.broadcast_to(w.U, (w.B,) + w.U.shape[1:])


def _PAR(w):
    return None if w.PAR is None else np.broadcast_to(w.PAR, (w.B,) + w.PAR.shape[1:])


def _np(ts):
    return [t.cpu().numpy() for t in ts]


def _forced_big(w):
    s = solver.from_workload(w, force_large=True)
    assert s.large_system
    return s


def _solve_forced(s, w, **kw):
    out = _np(s.solve(w.X_init, w.U, w.Y, w.PAR, **kw))
    torch.cuda.synchronize()
    return out


def test_constants_of_other_dims_are_refused_on_device():
    """the path and layout are fixed when the constants are built; a
    solve with dims that disagree (here: the other path) computes nothing and says so."""
    w = configs.make_c2(B=2, N=20)
    reg = solver.from_workload(w)
    big = solver.from_workload(w, force_large=True)
    assert not reg.large_system and big.large_system
    for s, other in ((reg, big), (big, reg)):
        s.cbuf, saved = other.cbuf, s.cbuf   # constants laid out for the other path
        try:
            X, cost, iters, status = _np(s.solve(w.X_init, w.U, w.Y, max_iter=3))
        finally:
            s.cbuf = saved
        assert status.tolist() == [solver.STATUS_BAD_CONSTANTS] * 2 and iters.tolist() == [0, 0]
        assert np.array_equal(X, w.X_init) and np.isnan(cost).all()


def test_forced_big_path_matches_register_path_c2():
    w = configs.make_c2(B=8, N=100)
    sr = solver.from_workload(w)
    assert not sr.large_system
    Xr, cr, ir, str_ = _np(sr.solve(w.X_init, w.U, w.Y, max_iter=4, tol=0.0))
    sb = _forced_big(w)
    Xb, cb, ib, stb = _solve_forced(sb, w, max_iter=4, tol=0.0)
    assert ib.tolist() == ir.tolist() == [4] * w.B and stb.tolist() == str_.tolist()
    tl.check("X big vs register", np.abs(Xb - Xr).max(), 1e-10 * (1 + np.abs(Xr).max()))
    tl.check("cost big vs register", np.abs(cb - cr).max(), 1e-10 * np.abs(cr).max())
    # converged: same optimum, same statuses
    Xr, cr, ir, str_ = _np(sr.solve(w.X_init, w.U, w.Y, max_iter=50, tol=1e-9))
    Xb, cb, ib, stb = _solve_forced(sb, w, max_iter=50, tol=1e-9)
    assert stb.tolist() == str_.tolist() == [0] * w.B
    assert np.all(np.abs(ib - ir) <= 1)
    tl.check("X big vs register (converged)", np.abs(Xb - Xr).max(), 1e-8 * (1 + np.abs(Xr).max()))


def test_big_vdp_n150_matches_oracle():
    w = configs.make_c2(B=3, N=150)  # d = 302 > 208: large-system path by size
    s = solver.from_workload(w)
    assert s.large_system
    X, cost, iters, status = _np(s.solve(w.X_init, w.U, w.Y, max_iter=3, tol=0.0))
    pb = _problem(w)
    Xr, cr, ir, sr = gn.gauss_newton(pb, w.X_init, _U(w), w.Y, max_iter=3, tol=0.0)
    assert iters.tolist() == ir.tolist() and status.tolist() == sr.tolist()
    tl.check("X", np.abs(X - Xr).max(), 1e-10 * (1 + np.abs(Xr).max()))
    tl.check("cost", np.abs(cost - cr).max(), 1e-10 * np.abs(cr).max())


@pytest.mark.parametrize("N", [60, 200])
def test_big_gnss_matches_oracle(N):
    """N=200 is the C3 shape (d = 1005, 201 epochs x 12 pseudoranges)."""
    w = configs.make_gnss_small(B=2, N=N, T=float(N), n_sat=12, epochs=N + 1)
    s = solver.from_workload(w)
    assert s.large_system
    pb = _problem(w)
    X, cost, iters, status = _np(s.solve(w.X_init, w.U, w.Y, w.PAR, max_iter=3, tol=0.0))
    _check_oracle(w, pb, X, cost, iters, status, 3)


def _check_oracle(w, pb, X, cost, iters, status, it, resolve=1e-4):
    run = lambda Y, pt=None: gn.gauss_newton(pb, w.X_init, _U(w), Y, _PAR(w), max_iter=it, tol=0.0, perturb=pt)  # noqa: E731
    Xr, cr, ir, sr = run(w.Y)
    fx, fc = tl.floor(lambda Y, pt: run(Y, pt)[:2], w.Y)
    assert iters.tolist() == ir.tolist() and status.tolist() == sr.tolist()
    b = tl.bound(fx, Xr)
    tl.check("X", np.abs(X - Xr).max(), b, " m")
    if resolve is not None:
        assert b < resolve, f"the bound must resolve {resolve:g} m errors"
    tl.check("cost", np.abs(cost - cr).max(), tl.FLOOR_MULT * fc + 1e-10 * np.abs(cr).max())


def test_big_max_iter_zero_and_empty_batch():
    w = configs.make_c2(B=2, N=150)
    s = solver.from_workload(w)
    X, cost, iters, status = _np(s.solve(w.X_init, w.U, w.Y, max_iter=0))
    assert np.array_equal(X, w.X_init) and iters.tolist() == [0, 0] and status.tolist() == [1, 1]
    _, _, _, cr = gn.residuals(_problem(w), w.X_init, _U(w), w.Y)
    assert np.allclose(cost, cr, rtol=1e-12)
    X, cost, iters, status = s.solve(np.zeros((0, w.P, w.n)), w.U, np.zeros((0, w.M, w.p)), max_iter=3)
    assert X.shape == (0, w.P, w.n)


def test_big_wide_slab_c4_shape_matches_oracle():
    """The C4 shape (bicycle + pseudorange, N = 500, d = 3006, NT = 188 tile
    columns) takes k_big_chol<8> (wide trailing slab, NT >= BIG_WIDE_NT)."""
    w = configs.make_c4(B=1)
    s = solver.from_workload(w)
    assert s.large_system and w.P * w.n // 16 + 1 >= 128
    pb = _problem(w)
    X, cost, iters, status = _np(s.solve(w.X_init, w.U, w.Y, w.PAR, max_iter=2, tol=0.0))
    # C4's conditioning floor is ~1 mm (tests/tolerance.py): the bound cannot resolve 0.1 mm
    _check_oracle(w, pb, X, cost, iters, status, 2, resolve=None)


@pytest.mark.parametrize("cfg", ["c3", "c4", "c5"])
def test_left_and_right_looking_factorizations_agree(cfg):
    """k_big_chol's left-looking block-column update (default) and the right-looking
    trailing update (mhe_set_option(MHE_OPT_BIG_RIGHT_LOOKING, 1), kept for A/B runs)
    accumulate every tile's updates in
    the same k order (the right-looking form only stores and reloads the partial sums
    between super-blocks, which is exact): iterates after 2 GN steps are bitwise
    identical (C3 reduced N = 60 with the 4-wide instance, C4 full shape with the 8-wide
    one, C5's eight receivers at N = 20, whose component-pair sparsity the split form's
    envelope skips -- the skipped terms are products with exact zeros)."""
    if cfg == "c5":
        w = configs.make_c5(B=2, N=20)
    else:
        w = configs.make_c3(B=2, N=60) if cfg == "c3" else configs.make_c4(B=1)
    s = solver.from_workload(w)
    assert s.large_system
    out = {}
    try:
        for ll in ("1", "0"):
            assert s.lib.mhe_set_option(_lib.OPT_BIG_RIGHT_LOOKING, 0 if ll == "1" else 1) >= 0
            out[ll] = _np(s.solve(w.X_init, w.U, w.Y, w.PAR, max_iter=2, tol=0.0))
            torch.cuda.synchronize()
    finally:
        s.lib.mhe_set_option(_lib.OPT_BIG_RIGHT_LOOKING, 0)
    Xa, Xb = out["1"][0], out["0"][0]
    assert (out["1"][3] == out["0"][3]).all() and (out["1"][2] == out["0"][2]).all()
    print(f"{cfg}: left- vs right-looking max|dX| = {np.abs(Xa - Xb).max():.3e}")
    assert np.array_equal(Xa, Xb) and np.array_equal(out["1"][1], out["0"][1])


def test_split_factorization_is_batch_invariant():
    """C4 (NT = 188 >= 128 tile columns) runs the split factorization: per block column a
    diagonal stage and k_big_rows, one workgroup per 8 rows of one trajectory; a batch that
    is a multiple of 8 is remapped so a trajectory's row groups share an XCD.  A batch of 8
    (remapped) agrees bitwise with the right-looking one-launch kernel on the same batch and
    with trajectory 5 solved alone (batch 1: no remap, other workgroup ids)."""
    w = configs.make_c4(B=8)
    s = solver.from_workload(w)
    assert s.large_system
    split = _np(s.solve(w.X_init, w.U, w.Y, w.PAR, max_iter=2, tol=0.0))
    torch.cuda.synchronize()
    try:
        assert s.lib.mhe_set_option(_lib.OPT_BIG_RIGHT_LOOKING, 1) >= 0
        mono = _np(s.solve(w.X_init, w.U, w.Y, w.PAR, max_iter=2, tol=0.0))
        torch.cuda.synchronize()
    finally:
        s.lib.mhe_set_option(_lib.OPT_BIG_RIGHT_LOOKING, 0)
    one = _np(s.solve(w.X_init[5:6], w.U, w.Y[5:6], w.PAR, max_iter=2, tol=0.0))
    assert (split[3] == split[3][0]).all()
    for a, b in zip(split, mono):
        assert np.array_equal(a, b)
    for a, b in zip(one, split):
        assert np.array_equal(a, b[5:6])


def test_envelope_of_the_eight_receiver_system():
    """The split factorization's envelope (mhe_big_envelope, ABI v7) is the structure of
    C5's normal matrix, component by component (N = 20: 2 tiles per component): receiver
    r's x, y, z rows start at receiver r - 1's x (the range rows to the previous receiver;
    receiver 0 at column 0), its clock bias b at its own x (pseudoranges), its drift alpha
    at its own b (dynamics b' = alpha) -- formed on the device from the component pairs
    k_big_resid finds coupled, so nothing coupled is skipped and nothing uncoupled kept."""
    import ctypes
    w = configs.make_c5(B=2, N=20)
    s = solver.from_workload(w)
    assert s.large_system
    s.solve(w.X_init, w.U, w.Y, w.PAR, max_iter=1, tol=0.0)
    torch.cuda.synchronize()
    NT = s.lib.mhe_padded_dim(s.dims) // 16
    NTc = NT // w.n
    fc = (ctypes.c_int32 * NT)()
    ws = list(s._ws.values())[-1]
    nb = s.lib.mhe_workspace_bytes(s.dims, s._chunk(2))
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    assert s.lib.mhe_big_envelope(s.dims, ctypes.c_void_p(ws.data_ptr()), nb, 1, fc, NT, stream) == NT
    assert s.lib.mhe_big_envelope(s.dims, ctypes.c_void_p(ws.data_ptr()), nb, 2, fc, NT, stream) == -1  # past the batch
    expect = []
    for a in range(w.n):
        r, c = divmod(a, 5)
        first = (5 * (r - 1) if r > 0 else 0) if c < 3 else (5 * r if c == 3 else 5 * r + 3)
        expect += [first * NTc] * NTc
    assert list(fc) == expect
