"""ctypes binding of libmhe.so (the C-ABI declared in include/mhe.h).

The library is built in-tree (``python __graft_entry__.py`` / ``make -C
nlp-filter_amd/csrc``) to ``nlp-filter_amd/mhe/libmhe.so``.  There is no CPU
fallback: if the library is missing or fails to load, every solver entry point
raises ``MheLibraryError``.
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MHE_LIB", os.path.join(HERE, "libmhe.so"))

MHE_OK = 0
ERRORS = {-1: "MHE_ERR_DIMS", -2: "MHE_ERR_MODEL", -3: "MHE_ERR_HIP", -4: "MHE_ERR_UNSUPPORTED", -5: "MHE_ERR_NULL"}
STATUS = {0: "converged", 1: "max_iter", 2: "not_spd", 3: "nonfinite", 4: "bad_constants"}
OPT_BIG_RIGHT_LOOKING, OPT_DEBUG_SMEM_PAD = 1, 2  # mhe_set_option (A/B runs and tests only)

# symbol -> (restype, argtypes); must match include/mhe.h exactly
c_i32, c_i64, c_dbl, c_vp, c_sz = ctypes.c_int32, ctypes.c_int64, ctypes.c_double, ctypes.c_void_p, ctypes.c_size_t


class _Sized(ctypes.Structure):
    """ctypes mirror of an include/mhe.h dims struct: struct_size (first field) is set
    to this declaration's size, which the library checks against its own sizeof."""

    def __init__(self, *a, **kw):
        super().__init__(*a, **kw)
        self.struct_size = ctypes.sizeof(self)


class MheDims(_Sized):
    _fields_ = [
        ("struct_size", c_i32), ("N", c_i32), ("n", c_i32), ("m", c_i32), ("p", c_i32), ("M", c_i32), ("q", c_i32),
        ("dyn_model", c_i32), ("meas_model", c_i32), ("has_prior", c_i32),
        ("meas_idx", c_i32 * 8), ("T", c_dbl),
        ("dyn_cost", c_i32), ("n_bounds", c_i32), ("huber_delta", c_dbl),
        ("bound_idx", c_i32 * 8), ("bound_lb", c_dbl * 8), ("bound_ub", c_dbl * 8),
        ("n_extra", c_i32), ("n_eq", c_i32), ("eq_idx", ctypes.POINTER(c_i32)),
        ("force_large", c_i32), ("dyn_par", c_dbl * 8), ("eq_rhs", ctypes.POINTER(c_dbl)),
    ]


class MheEkfDims(_Sized):
    _fields_ = [("struct_size", c_i32), ("n", c_i32), ("m", c_i32), ("pmax", c_i32), ("q", c_i32),
                ("dyn_model", c_i32), ("meas_model", c_i32), ("dt", c_dbl), ("r_diag", c_i32),
                ("hist_batch_inner", c_i32), ("in_batch_inner", c_i32), ("dyn_par", c_dbl * 8)]


class MheLsDims(_Sized):
    _fields_ = [("struct_size", c_i32), ("slots", c_i32), ("max_iter", c_i32), ("warm", c_i32), ("with_vel", c_i32), ("tol", c_dbl)]


class MheSolveArgs(_Sized):
    _fields_ = [("struct_size", c_i32), ("batch", c_i32), ("X0", c_vp), ("X_out", c_vp), ("Z0", c_vp), ("Z_out", c_vp),
                ("U", c_vp), ("u_bstride", c_i64), ("Y", c_vp), ("PAR", c_vp), ("par_bstride", c_i64),
                ("Rw", c_vp), ("rw_bstride", c_i64), ("x0", c_vp), ("cost_out", c_vp), ("iters_out", c_vp),
                ("status_out", c_vp), ("max_iter", c_i32), ("tol", c_dbl), ("workspace", c_vp),
                ("workspace_bytes", c_sz), ("lambda_out", c_vp)]


_P = ctypes.POINTER(MheDims)
_PE = ctypes.POINTER(MheEkfDims)
_PL = ctypes.POINTER(MheLsDims)
SIGNATURES = {
    "mhe_version": (ctypes.c_char_p, []),
    "mhe_set_option": (c_i32, [c_i32, c_i32]),
    "mhe_padded_dim": (c_i32, [_P]),
    "mhe_const_bytes": (c_sz, [_P]),
    "mhe_build_constants": (ctypes.c_int, [_P, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "mhe_gn_solve": (ctypes.c_int, [_P, c_vp, c_i32, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_i64, c_vp,
                                    c_vp, c_vp, c_vp, c_i32, c_dbl, c_vp]),
    "mhe_workspace_bytes": (c_sz, [_P, c_i32]),
    "mhe_gn_solve_ws": (ctypes.c_int, [_P, c_vp, c_i32, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_i64, c_vp,
                                       c_vp, c_vp, c_vp, c_i32, c_dbl, c_vp, c_sz, c_vp]),
    "mhe_gn_solve_ext": (ctypes.c_int, [_P, c_vp, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_i64,
                                        c_vp, c_vp, c_vp, c_vp, c_i32, c_dbl, c_vp, c_sz, c_vp]),
    "mhe_solve": (ctypes.c_int, [_P, c_vp, ctypes.POINTER(MheSolveArgs), c_vp]),
    "mhe_resjac": (ctypes.c_int, [_P, c_vp, c_i32, c_vp, c_vp, c_i64, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp,
                                  c_vp]),
    "mhe_assemble": (ctypes.c_int, [_P, c_vp, c_i32, c_vp, c_vp, c_i64, c_vp, c_vp, c_i64, c_vp,
                                    c_vp, c_vp, c_vp, c_vp]),
    "mhe_chol_solve": (ctypes.c_int, [_P, c_vp, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "mhe_assemble_ws": (ctypes.c_int, [_P, c_vp, c_i32, c_vp, c_vp, c_i64, c_vp, c_vp, c_i64, c_vp,
                                       c_vp, c_vp, c_vp, c_vp, c_vp, c_sz, c_vp]),
    "mhe_chol_solve_ws": (ctypes.c_int, [_P, c_vp, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_sz, c_vp]),
    "mhe_kkt_dim": (c_i32, [_P]),
    "mhe_solve_kernel_name": (c_i32, [_P, c_i32, c_vp, ctypes.c_char_p, c_i32]),
    "mhe_big_envelope": (c_i32, [_P, c_vp, c_sz, c_i32, c_vp, c_i32, c_vp]),
    "mhe_assemble_kkt_ws": (ctypes.c_int, [_P, c_vp, c_i32, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_i64, c_vp,
                                           c_vp, c_vp, c_vp, c_vp, c_vp, c_sz, c_vp]),
    "mhe_ekf_run": (ctypes.c_int, [_PE, c_i32, c_i32, c_vp, c_vp, c_vp, c_i64, c_vp, c_i64, c_vp, c_i64,
                                   c_vp, c_i64, c_vp, c_vp, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp]),
    "mhe_ls_run": (ctypes.c_int, [_PL, c_i32, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                                  c_vp, c_vp, c_vp, c_vp]),
}


class MheLibraryError(RuntimeError):
    pass


class MheCallError(RuntimeError):
    pass


_lib = None


def load(path=None):
    """Load libmhe.so once (raises MheLibraryError if absent)."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise MheLibraryError(
            f"libmhe.so not found at {p}: build it with `python __graft_entry__.py` "
            "(hipcc --offload-arch=gfx950). There is no CPU fallback.")
    try:
        import torch  # noqa: F401  (bind to the HIP runtime torch already loaded)
    except Exception:
        pass
    lib = ctypes.CDLL(p)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if path is None:
        _lib = lib
    return lib


def lib_digest(path=None):
    """sha256 (16 hex digits) of the libmhe.so file -- stamps profiles with the
    exact build they measured (tools/parse_pmc.py, bench.py)."""
    import hashlib
    with open(path or LIB_PATH, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()[:16]


def check(rc, what):
    if rc != MHE_OK:
        raise MheCallError(f"{what} failed: {ERRORS.get(rc, rc)}")
