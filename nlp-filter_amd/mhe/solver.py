"""Batched Gauss-Newton solver on libmhe.so (device-resident, torch as container).

``BatchSolver`` owns the device constants of one problem structure (N, T,
models, measurement times, weights) and solves many independent trajectories
that share it:  X (B, P, n), U (B|1, P, m), Y (B, M, p), PAR (B|1, M, q),
x0 (B, n).  Everything is fp64 and stays in HBM between calls; the HIP work is
enqueued on the current torch stream (or the one passed in: inputs are staged and
outputs allocated on that stream after it waits for the current one, and every
tensor the launch touches is kept alive for it -- mhe.streams).  The large-system
workspace is cached per stream, so concurrent solves on different streams never
share one.
"""
import collections
import ctypes

import numpy as np
import torch

from . import _lib, registry
from .streams import keep_alive, launch_stream

STATUS_CONVERGED, STATUS_MAX_ITER, STATUS_NOT_SPD, STATUS_NONFINITE, STATUS_BAD_CONSTANTS = 0, 1, 2, 3, 4


def _dev(x, device, shape=None):
    if x is None:
        return None
    if isinstance(x, torch.Tensor):
        t = x.to(device=device, dtype=torch.float64)
    else:
        t = torch.as_tensor(np.asarray(x, dtype=np.float64), device=device)
    t = t.contiguous()
    if shape is not None and tuple(t.shape) != tuple(shape):
        raise ValueError(f"expected shape {shape}, got {tuple(t.shape)}")
    return t


def _ptr(t):
    return None if t is None else ctypes_ptr(t)


def _at(t, lo, per, itemsize=8):
    """Pointer to trajectory ``lo`` of a batch-outermost tensor with ``per`` elements per
    trajectory (per = 0: an input shared by the batch)."""
    if t is None:
        return None
    return ctypes.c_void_p(t.data_ptr() + itemsize * lo * per)


def ctypes_ptr(t):
    import ctypes
    return ctypes.c_void_p(t.data_ptr())


def _handle(s):
    import ctypes
    return ctypes.c_void_p(s.cuda_stream)


class BatchSolver:
    """Device constants + launch wrappers for one problem structure.

    Parameters (host numpy or torch):
      N, T            collocation order and window length
      dyn, meas       plug-in functions (or names) -- see mhe.registry
      D (P,P), cw (P) differentiation matrix, (T/2) * quadrature weights
      Phi (M,P)       Lagrange basis at the measurement times
      Qw (n,n)        dynamics-cost information (weighted_l2_norm params["Q"])
      Rw (M,p,p)      measurement information (R passed to addResidualCost)
      Pw (n,n)|None   prior information (addInitialCost), None = no prior
      meas_idx        static index parameters of the measurement model
      dyn_cost        "l2" (weighted_l2_norm) or "huber" (pseudo_huber_loss, IRLS; huber_delta)
      bounds          [(state component, lb, ub), ...] enforced by projected Newton (addVarBounds)
      n_extra         extra decision variables z (meas="mixed" rows may reference them)
      eq              (K, 2) equality constraints v[a] - v[b] = r on the node-major state
                      vector (b = -1: v[a] = r), met by every GN step (bordered KKT solve);
                      after each solve ``self.lam`` (B, K) holds their multipliers
                      (L = J + lam^T (C v - r))
      eq_rhs          (K,) the constants r (None: 0, the addEqConstraint rows)
      force_large     take the large-system path even when the register-resident kernel
                      fits (parity tests of the two paths; fixed at construction)
      dyn_par         static dynamics parameters (mhe_dims.dyn_par; registry.dyn_params turns a
                      plug-in's params dict into it, e.g. car_params for vehicle_dynamics_and_gnss)
      constants       "build" (default): build the device constants here; "receive": only
                      allocate ``cbuf`` -- a data-parallel rank > 0 receives rank 0's bytes
                      (mhe.dist.broadcast_) and then calls constants_ready()
    With meas="mixed", PAR rows follow include/mhe.h (q = 14) and Rw is (M,) weights.
    """

    WS_CACHE = 2  # large-system workspaces kept alive (one per recently used stream)
    ws_budget = None  # bytes of workspace one launch may use (None: 85 % of the free HBM)

    def __init__(self, N, T, dyn, meas, D, cw, Phi, Qw, Rw, Pw=None, meas_idx=None, device="cuda",
                 dyn_cost="l2", huber_delta=None, bounds=None, n_extra=0, eq=None, force_large=False,
                 dyn_par=None, eq_rhs=None, constants="build"):
        self.lib = _lib.load()
        if not torch.cuda.is_available():
            raise _lib.MheLibraryError("no HIP device visible: the estimator has no CPU path")
        self.device = torch.device(device)
        dname, (did, n, m) = registry.dyn_model(dyn)
        mname, (mid, p, q, linear) = registry.meas_model(meas)
        registry.check_pair(dname, mname)
        p = n if p is None else p
        self.N, self.T, self.n, self.m, self.p, self.q = int(N), float(T), n, m, p, q
        self.P = self.N + 1
        Phi = np.asarray(Phi, dtype=np.float64).reshape(-1, self.P)
        self.M = Phi.shape[0]
        self.dyn_name, self.meas_name, self.linear_meas = dname, mname, linear
        dims = _lib.MheDims()
        dims.N, dims.n, dims.m, dims.p, dims.M, dims.q = self.N, n, m, p, self.M, q
        dims.dyn_model, dims.meas_model = did, mid
        dims.has_prior = 0 if Pw is None else 1
        idx = list(meas_idx) if meas_idx is not None else [0, 1, 2, 3]
        for i in range(8):
            dims.meas_idx[i] = idx[i] if i < len(idx) else 0
        dims.T = self.T
        if dyn_cost not in ("l2", "huber"):
            raise ValueError(f"dyn_cost must be 'l2' or 'huber', got {dyn_cost!r}")
        dims.dyn_cost = 1 if dyn_cost == "huber" else 0
        dims.huber_delta = float(huber_delta) if huber_delta is not None else 0.0
        bounds = list(bounds or [])
        if len(bounds) > 8:
            raise ValueError("at most 8 bounded state components")
        dims.n_bounds = len(bounds)
        for i, (c, lo, hi) in enumerate(bounds):
            dims.bound_idx[i] = int(c)
            dims.bound_lb[i] = -np.inf if lo is None else float(lo)
            dims.bound_ub[i] = np.inf if hi is None else float(hi)
        self.dyn_cost, self.huber_delta, self.bounds = dyn_cost, huber_delta, bounds
        self.n_extra = int(n_extra)
        if self.n_extra and mname != "mixed":
            raise ValueError("extra variables enter mixed measurement rows only (meas='mixed')")
        dims.n_extra = self.n_extra
        self._eq = np.zeros(0, dtype=np.int32) if eq is None else np.ascontiguousarray(
            np.asarray(eq, dtype=np.int32).reshape(-1, 2).ravel())
        dims.n_eq = self._eq.size // 2
        self._eq_rhs = np.zeros(dims.n_eq) if eq_rhs is None else np.ascontiguousarray(
            np.asarray(eq_rhs, dtype=np.float64).ravel())
        if self._eq_rhs.size != dims.n_eq:
            raise ValueError("eq_rhs needs one constant per equality row")
        if dims.n_eq:
            import ctypes
            dims.eq_idx = self._eq.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))  # self._eq keeps it alive
            dims.eq_rhs = self._eq_rhs.ctypes.data_as(ctypes.POINTER(ctypes.c_double))
        self.n_eq = dims.n_eq
        self.lam = None
        dims.force_large = 1 if force_large else 0
        if dyn_par is None and dname == "vehicle_dynamics_and_gnss":
            raise ValueError("vehicle_dynamics_and_gnss needs dyn_par (registry.dyn_params(name, params))")
        dp = np.zeros(8) if dyn_par is None else np.asarray(dyn_par, dtype=np.float64).ravel()
        for i in range(8):
            dims.dyn_par[i] = float(dp[i]) if i < dp.size else 0.0
        self.dyn_par = dp
        self.dims = dims
        self.dp = self.lib.mhe_padded_dim(dims)
        if self.dp < 0:
            raise _lib.MheCallError("mhe_padded_dim: unsupported dims (system too large for this build?)")
        nbytes = self.lib.mhe_const_bytes(dims)
        if nbytes == 0:
            raise _lib.MheCallError("mhe_const_bytes: invalid dims")
        dev = self.device
        self.cbuf = torch.empty(nbytes, dtype=torch.uint8, device=dev)
        self._ws = collections.OrderedDict()  # large-system workspace per stream handle (LRU, <= WS_CACHE)
        self._built = torch.cuda.Event()  # launches on any stream wait for the constants
        if constants == "receive":
            # another process builds the buffer (rank 0 of a data-parallel job); the caller
            # fills self.cbuf (mhe.dist.broadcast_) and then calls constants_ready()
            self._ready = False
            return
        if constants != "build":
            raise ValueError(f"constants must be 'build' or 'receive', got {constants!r}")
        self._ready = True
        src = dict(D=np.asarray(D, np.float64), cw=np.asarray(cw, np.float64), Phi=Phi,
                   Qw=np.asarray(Qw, np.float64), Rw=np.asarray(Rw, np.float64).reshape(self.M, p, p),
                   Pw=None if Pw is None else np.asarray(Pw, np.float64))
        src = {k: _dev(v, dev) for k, v in src.items() if v is not None}
        cur = torch.cuda.current_stream(dev)
        rc = self.lib.mhe_build_constants(
            self.dims, _ptr(src["D"]), _ptr(src["cw"]), _ptr(src["Phi"]),
            _ptr(src["Qw"]), _ptr(src["Rw"]), _ptr(src.get("Pw")), _ptr(self.cbuf), _handle(cur))
        _lib.check(rc, "mhe_build_constants")
        # the staging tensors may be freed now: the build reads them on `cur`, where the
        # caching allocator orders their reuse
        self._built.record(cur)

    def constants_ready(self, stream=None):
        """A solver built with constants="receive": self.cbuf now holds the bytes another
        process built for the same dims (enqueued on ``stream``, default the current one);
        later launches on any stream wait for that point.  A buffer built for other dims
        is refused per trajectory by the kernels' layout stamp (MHE_STATUS_BAD_CONSTANTS)."""
        s = torch.cuda.current_stream(self.device) if stream is None else stream
        self._built.record(s)
        self._ready = True

    def _check_ready(self):
        if not self._ready:
            raise _lib.MheCallError("constants not received yet: fill cbuf and call constants_ready()")

    # ------------------------------------------------------------------ inputs
    def _inputs(self, X, U, Y, PAR, x0):
        dev = self.device
        X = _dev(X, dev)
        if X.dim() != 3 or X.shape[1:] != (self.P, self.n):
            raise ValueError(f"X must be (B, {self.P}, {self.n}), got {tuple(X.shape)}")
        B = X.shape[0]
        U_t, ustr = None, 0
        if self.m > 0:
            if U is None:
                raise ValueError("controls U are required for this dynamics model")
            U_t = _dev(U, dev)
            if U_t.dim() == 2:
                U_t = U_t[None]
            if U_t.shape[1:] != (self.P, self.m) or U_t.shape[0] not in (1, B):
                raise ValueError(f"U must be (B|1, {self.P}, {self.m}), got {tuple(U_t.shape)}")
            ustr = 0 if U_t.shape[0] == 1 else self.P * self.m
        Y_t = _dev(Y, dev, (B, self.M, self.p))
        PAR_t, pstr = None, 0
        if self.q > 0:
            PAR_t = _dev(PAR, dev)
            if PAR_t.dim() == 2:
                PAR_t = PAR_t[None]
            if PAR_t.shape[1:] != (self.M, self.q) or PAR_t.shape[0] not in (1, B):
                raise ValueError(f"PAR must be (B|1, {self.M}, {self.q}), got {tuple(PAR_t.shape)}")
            pstr = 0 if PAR_t.shape[0] == 1 else self.M * self.q
        x0_t = None
        if self.dims.has_prior:
            x0_t = _dev(x0, dev, (B, self.n))
        return X, B, U_t, ustr, Y_t, PAR_t, pstr, x0_t

    @property
    def large_system(self):
        """True when the problem exceeds the register-resident kernel (C3-C5):
        mhe_gn_solve_ws then needs a device workspace (allocated here, cached)."""
        return self.lib.mhe_workspace_bytes(self.dims, 1) > 0

    def _chunk(self, B, s=None):
        """Trajectories per launch on the large-system path: all B unless their
        workspace exceeds the budget (ws_budget bytes, default 85 % of the free HBM
        plus the workspace this solver holds for stream ``s``, which the launch
        replaces) -- then the batch is streamed in equal chunks through one workspace
        (C5: 2048 trajectories x 0.28 GB).  Workspaces cached for OTHER streams stay
        allocated (a launch there may still be using them), so they are not counted
        as free."""
        per = self.lib.mhe_workspace_bytes(self.dims, 1)
        if per == 0 or B == 0:
            return B
        budget = self.ws_budget
        if budget is None:
            free, _ = torch.cuda.mem_get_info(self.device)
            own = self._ws.get(s.cuda_stream) if s is not None else None
            budget = int(0.85 * (free + (own.numel() if own is not None else 0)))
        k = max(1, min(B, budget // per))
        if k >= B:
            return B
        # k_big_chol runs one workgroup per trajectory: a chunk that is a whole number of
        # CU-fulls leaves no CUs idle in a tail round (C5: 410 -> 256, 0.39 -> 0.46 of peak)
        cus = torch.cuda.get_device_properties(self.device).multi_processor_count
        if k > cus:
            k -= k % cus
        nch = -(-B // k)
        return -(-B // nch)  # equal chunks

    def _workspace(self, B, s):
        """Workspace for B trajectories on stream s (allocated on s: one per stream, so
        concurrent solves on different streams never share or free each other's)."""
        nb = self.lib.mhe_workspace_bytes(self.dims, B)
        if nb == 0:
            return None, 0
        key = s.cuda_stream
        ws = self._ws.pop(key, None)
        if ws is None or ws.numel() < nb:
            ws = None  # release the old one before allocating the larger one
            ws = torch.empty(nb, dtype=torch.uint8, device=self.device)
        self._ws[key] = ws  # most recently used last
        while len(self._ws) > self.WS_CACHE:
            # dropping the reference is safe: a launch on another stream recorded its
            # workspace on that stream (keep_alive), so the allocator reuses it only
            # after that stream's work is done
            self._ws.popitem(last=False)
        return ws, nb

    def _rw(self, Rw, B):
        """Per-solve measurement weights (mhe_solve_args.Rw): (B|1, M, p, p), or (B|1, M)
        for mixed rows; None = the weights the constants were built with."""
        if Rw is None:
            return None, 0
        if self.linear_meas:
            raise ValueError("per-solve Rw needs a nonlinear measurement model (a linear h folds R into the constants)")
        shape = (self.M,) if self.meas_name == "mixed" else (self.M, self.p, self.p)
        t = _dev(Rw, self.device)
        if t.shape == shape:
            t = t[None]
        if t.shape[1:] != shape or t.shape[0] not in (1, B):
            raise ValueError(f"Rw must be (B|1,) + {shape}, got {tuple(t.shape)}")
        return t, (0 if t.shape[0] == 1 else int(np.prod(shape)))

    def _gn(self, s, cur, B, X, Xo, U_t, ustr, Y_t, PAR_t, pstr, x0_t, cost, iters, status, max_iter, tol,
            Z=None, Zo=None, Rw=None, lam=None):
        Rw_t, rstr = self._rw(Rw, B)
        if B == 0:
            return
        chunk = self._chunk(B, s)
        ws, nb = self._workspace(chunk, s)
        P, n, M = self.P, self.n, self.M
        for lo in range(0, B, chunk):
            c = min(chunk, B - lo)
            a = _lib.MheSolveArgs()

            def at(t, per, stride=None):
                if t is None:
                    return None
                st = per if stride is None else stride
                return ctypes.c_void_p(t.data_ptr() + 8 * lo * st) if st else ctypes.c_void_p(t.data_ptr())

            a.batch = c
            a.X0, a.X_out = at(X, P * n), at(Xo, P * n)
            a.Z0, a.Z_out = at(Z, self.n_extra), at(Zo, self.n_extra)
            a.U, a.u_bstride = at(U_t, 0, ustr), ustr
            a.Y = at(Y_t, M * self.p)
            a.PAR, a.par_bstride = at(PAR_t, 0, pstr), pstr
            a.Rw, a.rw_bstride = at(Rw_t, 0, rstr), rstr
            a.x0 = at(x0_t, n)
            a.cost_out = at(cost, 1)
            a.iters_out = ctypes.c_void_p(iters.data_ptr() + 4 * lo)
            a.status_out = ctypes.c_void_p(status.data_ptr() + 4 * lo)
            a.max_iter, a.tol = int(max_iter), float(tol)
            a.workspace, a.workspace_bytes = (None if ws is None else ctypes.c_void_p(ws.data_ptr())), nb
            a.lambda_out = at(lam, self.n_eq)
            rc = self.lib.mhe_solve(self.dims, _ptr(self.cbuf), ctypes.byref(a), _handle(s))
            _lib.check(rc, "mhe_solve")
        keep_alive(s, cur, X, Xo, Z, Zo, U_t, Y_t, PAR_t, Rw_t, x0_t, cost, iters, status, ws, lam)

    # ------------------------------------------------------------------ calls
    def solve(self, X0, U, Y, PAR=None, x0=None, max_iter=20, tol=1e-10, stream=None, out=None, Z0=None, Rw=None,
              lam_out=None):
        """Gauss-Newton to convergence. Returns (X, cost, iters, status) device tensors,
        and the extra variables Z (B, n_extra) as a fifth element when n_extra > 0.
        ``Rw`` (B|1, M, p, p) -- (B|1, M) for mixed rows -- replaces the measurement
        weights of the constants for this solve (nonlinear models; the MHE windows'
        R = 0 slot masks).  With ``stream`` the work (staging included) is ordered on
        that stream; consume the outputs there or make the consuming stream wait for it.
        ``lam_out`` (B, n_eq) float64 device tensor: receives this solve's constraint
        multipliers (the per-call way; ``self.lam`` is the last solve's on any stream,
        kept for single-stream callers)."""
        self._check_ready()
        with launch_stream(stream, self.device, (self._built,)) as (s, cur):
            X, B, U_t, ustr, Y_t, PAR_t, pstr, x0_t = self._inputs(X0, U, Y, PAR, x0)
            if out is None:
                Xo = torch.empty_like(X)
                cost = torch.empty(B, dtype=torch.float64, device=self.device)
                iters = torch.empty(B, dtype=torch.int32, device=self.device)
                status = torch.empty(B, dtype=torch.int32, device=self.device)
            else:
                Xo, cost, iters, status = out
            Z = Zo = None
            if self.n_extra:
                Z = _dev(np.zeros((B, self.n_extra)) if Z0 is None else Z0, self.device, (B, self.n_extra))
                Zo = torch.empty_like(Z)
            lam = None
            if self.n_eq:
                if lam_out is not None:
                    if tuple(lam_out.shape) != (B, self.n_eq) or lam_out.dtype != torch.float64:
                        raise ValueError(f"lam_out must be float64 ({B}, {self.n_eq})")
                    lam = lam_out
                    lam.zero_()
                else:
                    lam = torch.zeros((B, self.n_eq), dtype=torch.float64, device=self.device)
            self._gn(s, cur, B, X, Xo, U_t, ustr, Y_t, PAR_t, pstr, x0_t, cost, iters, status, max_iter, tol, Z, Zo,
                     Rw, lam)
            self.lam = lam
        if self.n_extra:
            return Xo, cost, iters, status, Zo
        return Xo, cost, iters, status

    def prepare(self, X0, U, Y, PAR=None, x0=None):
        """Pre-stage device inputs once (bench: inputs resident before timing)."""
        return self._inputs(X0, U, Y, PAR, x0)

    def solve_staged(self, staged, outs, max_iter, tol, stream=None):
        X, B, U_t, ustr, Y_t, PAR_t, pstr, x0_t = staged
        Xo, cost, iters, status = outs
        self._check_ready()
        with launch_stream(stream, self.device, (self._built,)) as (s, cur):
            self._gn(s, cur, B, X, Xo, U_t, ustr, Y_t, PAR_t, pstr, x0_t, cost, iters, status, max_iter, tol)

    def resjac(self, X, U, Y, PAR=None, stream=None):
        """Per-node defects W (B,P,n) and dynamics Jacobians F (B,P,n,n), per-row
        residuals E (B,M,p) and measurement Jacobians Hm (B,M,p,n) at X (mhe_resjac)."""
        self._check_ready()
        with launch_stream(stream, self.device, (self._built,)) as (s, cur):
            X, B, U_t, ustr, Y_t, PAR_t, pstr, _ = self._inputs(X, U, Y, PAR, np.zeros((X.shape[0], self.n))
                                                                if self.dims.has_prior else None)
            f64 = dict(dtype=torch.float64, device=self.device)
            W = torch.empty((B, self.P, self.n), **f64)
            F = torch.empty((B, self.P, self.n, self.n), **f64)
            E = torch.empty((B, self.M, self.p), **f64)
            Hm = torch.empty((B, self.M, self.p, self.n), **f64)
            rc = self.lib.mhe_resjac(self.dims, _ptr(self.cbuf), B, _ptr(X), _ptr(U_t), ustr, _ptr(Y_t), _ptr(PAR_t),
                                     pstr, _ptr(W), _ptr(F), _ptr(E), _ptr(Hm), _handle(s))
            _lib.check(rc, "mhe_resjac")
            keep_alive(s, cur, X, U_t, Y_t, PAR_t, W, F, E, Hm)
        return W, F, E, Hm

    @property
    def kkt_dim(self):
        """Rows of the system assemble() / chol_solve() exchange: dp, plus n_extra + n_eq
        border rows for a bordered (KKT) problem (mhe_kkt_dim)."""
        return self.lib.mhe_kkt_dim(self.dims)

    def assemble(self, X, U, Y, PAR=None, x0=None, stream=None, status_out=False, Z=None):
        """GN normal equations at X: H (B,dp,dp), g (B,dp), cost (B) -- dense, node-major
        (row j*n + c; padding nodes last) on both paths.  The large-system path runs the
        solve's own k_big_resid + k_big_assemble over a workspace (mhe_assemble_kkt_ws) and
        copies H out of their component-major tiles.  A bordered problem (n_extra / n_eq
        > 0) returns the KKT system of kkt_dim rows instead (H_xz, H_zz, the constraint
        rows; g = [g_x; g_z; C v - r]) at (X, Z).  ``status_out``: also return the
        per-trajectory status (0, or 4 = constants built for other dims)."""
        self._check_ready()
        with launch_stream(stream, self.device, (self._built,)) as (s, cur):
            X, B, U_t, ustr, Y_t, PAR_t, pstr, x0_t = self._inputs(X, U, Y, PAR, x0)
            Z_t = None
            if self.n_extra:
                Z_t = _dev(np.zeros((B, self.n_extra)) if Z is None else Z, self.device, (B, self.n_extra))
            dk = self.kkt_dim
            H = torch.empty((B, dk, dk), dtype=torch.float64, device=self.device)
            g = torch.empty((B, dk), dtype=torch.float64, device=self.device)
            cost = torch.empty(B, dtype=torch.float64, device=self.device)
            status = torch.empty(B, dtype=torch.int32, device=self.device)
            # the large-system workspace is streamed in chunks like solve()'s (C5: 0.28 GB per
            # trajectory), the outputs written in place at each chunk's offset
            chunk = max(1, self._chunk(B, s))
            ws, nb = self._workspace(chunk, s)
            P, n, M = self.P, self.n, self.M
            for lo in range(0, B, chunk):
                c = min(chunk, B - lo)
                rc = self.lib.mhe_assemble_kkt_ws(
                    self.dims, _ptr(self.cbuf), c, _at(X, lo, P * n), _at(Z_t, lo, self.n_extra), _at(U_t, lo, ustr),
                    ustr, _at(Y_t, lo, M * self.p), _at(PAR_t, lo, pstr), pstr, _at(x0_t, lo, n), _at(H, lo, dk * dk),
                    _at(g, lo, dk), _at(cost, lo, 1), _at(status, lo, 1, 4), _ptr(ws), nb, _handle(s))
                _lib.check(rc, "mhe_assemble_kkt_ws")
            keep_alive(s, cur, X, Z_t, U_t, Y_t, PAR_t, x0_t, H, g, cost, status, ws)
        if status_out:
            return H, g, cost, status
        return H, g, cost

    def chol_solve(self, H, g, stream=None):
        """delta = -H^{-1} g with the solver's own factorization (H: (B,dp,dp) SPD,
        node-major as ``assemble`` returns it; lower triangle read): the register-tiled
        kernel, or on the large-system path k_big_chol over a workspace (mhe_chol_solve_ws).
        A bordered problem takes the KKT system of kkt_dim rows (``assemble``'s) and
        returns delta = [dx; dz; lambda], solved as every bordered GN step (k_big_border)."""
        self._check_ready()
        with launch_stream(stream, self.device, (self._built,)) as (s, cur):
            H = _dev(H, self.device)
            g = _dev(g, self.device)
            B = H.shape[0]
            dk = self.kkt_dim
            if H.shape[1:] != (dk, dk) or g.shape != (B, dk):
                raise ValueError(f"H must be (B,{dk},{dk}) and g (B,{dk})")
            delta = torch.empty((B, dk), dtype=torch.float64, device=self.device)
            status = torch.empty(B, dtype=torch.int32, device=self.device)
            chunk = max(1, self._chunk(B, s))
            ws, nb = self._workspace(chunk, s)
            for lo in range(0, B, chunk):
                c = min(chunk, B - lo)
                rc = self.lib.mhe_chol_solve_ws(self.dims, _ptr(self.cbuf), c, _at(H, lo, dk * dk), _at(g, lo, dk),
                                                _at(delta, lo, dk), _at(status, lo, 1, 4), _ptr(ws), nb, _handle(s))
                _lib.check(rc, "mhe_chol_solve_ws")
            keep_alive(s, cur, H, g, delta, status, ws)
        return delta, status


def from_workload(w, device="cuda", **kw):
    """BatchSolver for a mhe.configs.Workload (kw: dyn_cost, huber_delta, bounds)."""
    Phi = w.cpm.lagrange_matrix(w.t_meas)
    kw.setdefault("n_extra", getattr(w, "n_extra", 0))
    if getattr(w, "dyn_par", None) is not None:
        kw.setdefault("dyn_par", w.dyn_par)
    return BatchSolver(w.N, w.T, w.dyn, w.meas, w.cpm.D, (w.T / 2.0) * w.cpm.w, Phi, w.Qw, w.Rw,
                       Pw=w.Pw, meas_idx=w.meas_static.get("idx"), device=device, **kw)
