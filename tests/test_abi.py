"""The C-ABI library loads and exports every symbol include/mhe.h declares (no GPU calls)."""
import ctypes
import os
import re

from mhe import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    src = open(os.path.join(ROOT, "include", "mhe.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(mhe_[a-z_]+)\s*\(", src)))


def test_header_symbols_exported():
    lib = ctypes.CDLL(_lib.LIB_PATH)
    declared = _declared()
    assert "mhe_gn_solve" in declared and "mhe_build_constants" in declared
    for name in declared:
        assert hasattr(lib, name), f"{name} declared in mhe.h but not exported"
    assert set(declared) == set(_lib.SIGNATURES), "ctypes signature table out of sync with mhe.h"


def test_host_side_entry_points_without_gpu():
    lib = _lib.load()
    assert lib.mhe_version().startswith(b"libmhe")
    d = _lib.MheDims()
    d.N, d.n, d.m, d.p, d.M, d.q, d.dyn_model, d.meas_model, d.T = 100, 2, 1, 2, 101, 0, 5, 1, 10.0
    assert lib.mhe_padded_dim(d) == 208
    assert lib.mhe_const_bytes(d) > 0
    d.n = 3  # inconsistent with van der Pol
    assert lib.mhe_const_bytes(d) == 0
    assert lib.mhe_padded_dim(d) == -1
    d.n, d.dyn_model = 2, 99
    assert lib.mhe_const_bytes(d) == 0
    assert lib.mhe_workspace_bytes(d, 1024) == 0  # register-resident path needs no workspace
    d.dyn_model, d.N = 5, 500  # beyond the register-resident limit: large-system path
    assert lib.mhe_padded_dim(d) == 2 * 512  # component-major, P padded to 16 per component
    assert lib.mhe_workspace_bytes(d, 2) > 2 * 8 * (64 * 65 // 2) * 256


def test_set_option_is_explicit_and_bounded():
    """The A/B options are set only through mhe_set_option (no environment variable is
    read): it returns the previous value and refuses unknown options / bad values."""
    lib = _lib.load()
    assert lib.mhe_set_option(_lib.OPT_BIG_RIGHT_LOOKING, 1) == 0
    assert lib.mhe_set_option(_lib.OPT_BIG_RIGHT_LOOKING, 0) == 1
    assert lib.mhe_set_option(_lib.OPT_DEBUG_SMEM_PAD, 0) == 0
    assert lib.mhe_set_option(_lib.OPT_DEBUG_SMEM_PAD, -5) == -1
    assert lib.mhe_set_option(77, 1) == -1
    src = open(os.path.join(ROOT, "nlp-filter_amd", "csrc", "mhe_core.h")).read()
    src += open(os.path.join(ROOT, "nlp-filter_amd", "csrc", "mhe_gn.hip")).read()
    assert "getenv" not in src


def test_general_problem_dims_validation():
    """Extra variables / equality constraints / mixed rows: host-side checks."""
    lib = _lib.load()
    d = _lib.MheDims()
    d.N, d.n, d.m, d.p, d.M, d.q, d.dyn_model, d.meas_model, d.T = 10, 10, 6, 1, 30, 14, 8, 5, 5.0  # mixed
    assert lib.mhe_padded_dim(d) == 10 * 16           # always the large-system path
    assert lib.mhe_workspace_bytes(d, 4) > 0
    pairs = (ctypes.c_int32 * 22)(*[v for j in range(11) for v in (j * 10 + 2, j * 10 + 7)])
    d.n_eq, d.eq_idx = 11, ctypes.cast(pairs, ctypes.POINTER(ctypes.c_int32))
    assert lib.mhe_const_bytes(d) > 0
    d.n_extra = 3
    assert lib.mhe_padded_dim(d) == 160
    d.n_extra = 5                                      # > MHE_MAX_EXTRA
    assert lib.mhe_padded_dim(d) == -1
    d.n_extra = 0
    pairs[1] = 110                                     # index past P*n
    assert lib.mhe_padded_dim(d) == -1
    pairs[1] = 7
    d.eq_idx = ctypes.POINTER(ctypes.c_int32)()        # NULL table
    assert lib.mhe_padded_dim(d) == -1
    d.eq_idx = ctypes.cast(pairs, ctypes.POINTER(ctypes.c_int32))
    d.n_bounds, d.bound_idx[0], d.bound_lb[0], d.bound_ub[0] = 1, 0, -1.0, 1.0
    assert lib.mhe_padded_dim(d) == -1                 # bounds + constraints: unsupported
    d.n_bounds, d.n_eq = 0, 0
    d.meas_model, d.q, d.n_extra = 2, 3, 2             # extra variables need mixed rows
    d.dyn_model, d.n, d.m = 6, 5, 3
    assert lib.mhe_padded_dim(d) == -1


def test_struct_size_guards_stale_bindings():
    """ABI r02 (VERDICT weak #7): a binding that declares a truncated struct (the old
    INTEGRATION.md stub stopped after T) is refused with MHE_ERR_DIMS before any later
    field is read; so is one that omits struct_size (N lands in its place)."""
    lib = _lib.load()

    class Truncated(ctypes.Structure):   # struct_size .. T, nothing after
        _fields_ = [f for f in _lib.MheDims._fields_ if f[0] != "dyn_cost"][:12]

    assert Truncated._fields_[-1][0] == "T"
    t = Truncated()
    t.struct_size = ctypes.sizeof(t)
    t.N, t.n, t.m, t.p, t.M, t.q, t.dyn_model, t.meas_model, t.T = 100, 2, 1, 2, 101, 0, 5, 1, 10.0
    fn = lib.mhe_padded_dim
    pd = ctypes.CFUNCTYPE(ctypes.c_int32, ctypes.POINTER(Truncated))(ctypes.cast(fn, ctypes.c_void_p).value)
    assert pd(ctypes.byref(t)) == -1
    cb = ctypes.CFUNCTYPE(ctypes.c_size_t, ctypes.POINTER(Truncated))(ctypes.cast(lib.mhe_const_bytes, ctypes.c_void_p).value)
    assert cb(ctypes.byref(t)) == 0
    # a solve entry point returns MHE_ERR_DIMS (no device pointer is touched)
    sv = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.POINTER(Truncated), ctypes.c_void_p, ctypes.c_int32,
                          *([ctypes.c_void_p] * 3), ctypes.c_int64, *([ctypes.c_void_p] * 2), ctypes.c_int64,
                          *([ctypes.c_void_p] * 4), ctypes.c_int32, ctypes.c_double, ctypes.c_void_p)(
        ctypes.cast(lib.mhe_gn_solve, ctypes.c_void_p).value)
    assert sv(ctypes.byref(t), None, 1, None, None, None, 0, None, None, 0, None, None, None, None, 5, 1e-10, None) == -1

    class NoSize(ctypes.Structure):      # the round-2 layout: N first
        _fields_ = _lib.MheDims._fields_[1:]

    o = NoSize()
    o.N, o.n, o.m, o.p, o.M, o.q, o.dyn_model, o.meas_model, o.T = 100, 2, 1, 2, 101, 0, 5, 1, 10.0
    pd2 = ctypes.CFUNCTYPE(ctypes.c_int32, ctypes.POINTER(NoSize))(ctypes.cast(fn, ctypes.c_void_p).value)
    assert pd2(ctypes.byref(o)) == -1
    # the full, current struct works
    d = _lib.MheDims()
    d.N, d.n, d.m, d.p, d.M, d.q, d.dyn_model, d.meas_model, d.T = 100, 2, 1, 2, 101, 0, 5, 1, 10.0
    assert d.struct_size == ctypes.sizeof(_lib.MheDims) and lib.mhe_padded_dim(d) == 208
    # EKF and least-squares structs: same guard
    e = _lib.MheEkfDims()
    e.struct_size -= 4
    assert lib.mhe_ekf_run(e, 1, 1, None, None, None, 0, None, 0, None, 0, None, 0, None, None, 0, 0,
                           None, None, None, None) == -1
    ls = _lib.MheLsDims()
    ls.struct_size = 0
    assert lib.mhe_ls_run(ls, 1, 1, *([None] * 13)) == -1


def test_integration_stub_declares_the_full_struct():
    """INTEGRATION.md's ctypes stub must declare mhe_dims exactly as the library does."""
    import re as _re
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    m = _re.search(r"class mhe_dims\(ctypes.Structure\):.*?_fields_ = \[(.*?)\]\n", text, _re.S)
    assert m, "INTEGRATION.md has no mhe_dims stub"
    names = _re.findall(r'\("([a-z_A-Z]+)"', m.group(1))
    assert names == [f[0] for f in _lib.MheDims._fields_]


def test_kkt_dim_and_kernel_name_queries_without_gpu():
    """Host-only ABI v6/v7 queries: mhe_kkt_dim = padded dim + n_extra + n_eq, and
    mhe_solve_kernel_name names the instance the launch would pick (batch vs CUs; no
    device here, so the CU count falls back to 256) or the large-system sequence;
    mhe_big_envelope's argument checks (no copy without a workspace)."""
    import numpy as np
    lib = _lib.load()
    d = _lib.MheDims()
    d.N, d.n, d.m, d.p, d.M, d.q, d.dyn_model, d.meas_model, d.T = 100, 2, 1, 2, 101, 0, 5, 1, 10.0
    assert lib.mhe_kkt_dim(d) == lib.mhe_padded_dim(d) == 208
    buf = ctypes.create_string_buffer(256)
    assert lib.mhe_solve_kernel_name(d, 1024, None, buf, 256) == 0 and b"two workgroups per CU" in buf.value
    assert lib.mhe_solve_kernel_name(d, 128, None, buf, 256) == 0 and b"SB=true" in buf.value
    assert lib.mhe_solve_kernel_name(d, 128, None, None, 0) == -5  # MHE_ERR_NULL
    fc = (ctypes.c_int32 * 64)()
    assert lib.mhe_big_envelope(d, None, 0, 0, fc, 64, None) == -4  # ABI v7: register path, no envelope
    d.N = 500
    assert lib.mhe_solve_kernel_name(d, 8, None, buf, 256) == 0 and buf.value.startswith(b"large-system path")
    assert lib.mhe_big_envelope(d, None, 0, 0, fc, 64, None) == -5  # no workspace (MHE_ERR_NULL)
    # a bordered problem: equality rows (host pointer) -> dp + n_eq rows
    eq = np.array([[0, 1], [2, 3], [4, -1]], dtype=np.int32)
    d.n_eq = 3
    d.eq_idx = eq.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))
    assert lib.mhe_kkt_dim(d) == lib.mhe_padded_dim(d) + 3
    d.struct_size = 8  # a truncated struct is refused
    assert lib.mhe_kkt_dim(d) == -1
