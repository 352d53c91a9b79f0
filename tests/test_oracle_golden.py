"""Pin the CPU oracle (and the product's host constants) to the reference's own outputs.

Golden vectors come from tests/golden/gen_golden.py, which runs the reference
code (nlp/collocation.py, nlp/dynamics.py, nlp/measurements.py,
nlp/cost_functions.py) in the build container.
"""
import hashlib

import numpy as np
import pytest

from oracle import collocation as oc
from oracle import models as om
from nlp.collocation import ChebyshevPseudospectralMethod

NS = (2, 3, 4, 5, 6, 7, 10, 15, 20, 50, 100, 200, 500)


def _D_ok(D, g, N):
    if N <= 100:
        return np.array_equal(D, g[f"D_{N}"])
    return hashlib.sha256(np.ascontiguousarray(D).tobytes()).digest() == bytes(g[f"Dsha_{N}"])


@pytest.mark.parametrize("N", NS)
def test_oracle_constants_bit_exact(golden, N):
    g = golden["collocation"]
    assert np.array_equal(oc.nodes(N), g[f"tau_{N}"])
    assert _D_ok(oc.diff_matrix(N), g, N)
    assert np.array_equal(oc.quad_weights(N), g[f"w_{N}"])  # bug-compatible weights


@pytest.mark.parametrize("N", NS)
def test_product_constants_bit_exact(golden, N):
    g = golden["collocation"]
    c = ChebyshevPseudospectralMethod(N, 0, 10.0)
    assert np.array_equal(c.tau, g[f"tau_{N}"])
    assert _D_ok(c.D, g, N)
    assert np.array_equal(c.w, g[f"w_{N}"])
    if N > 100:
        idx = g[f"Dprobe_idx_{N}"]
        assert np.array_equal(c.D[idx[:, 0], idx[:, 1]], g[f"Dprobe_val_{N}"])


def test_weight_quirks(golden):
    # collocation.py:82-83 inside the inner loop -> w[2] never set for N = 3
    assert oc.quad_weights(3)[2] == 0.0
    assert abs(oc.quad_weights(10).sum() - 2.0060606060606) < 1e-12


@pytest.mark.parametrize("N", (2, 3, 4, 5, 6, 7, 10, 15, 20))
def test_lagrange_basis(golden, N):
    g = golden["collocation"]
    t = g[f"phi_t_{N}"]
    # poly1d mode reproduces the reference bit-for-bit
    assert np.array_equal(oc.interp_matrix(N, 10.0, t, mode="poly1d"), g[f"phi_{N}"])
    c = ChebyshevPseudospectralMethod(N, 0, 10.0, phi_mode="poly1d")
    assert np.array_equal(c.lagrange_matrix(t), g[f"phi_{N}"])
    # barycentric (the product default) = same basis without poly1d cancellation;
    # the reference's poly1d error grows with N: 5e-8 at N=20
    tol = {20: 1e-7, 15: 1e-9}.get(N, 1e-12)
    assert np.abs(oc.interp_matrix(N, 10.0, t) - g[f"phi_{N}"]).max() < tol
    cb = ChebyshevPseudospectralMethod(N, 0, 10.0)
    assert np.abs(cb.lagrange_matrix(t) - g[f"phi_{N}"]).max() < tol
    # evaluateSolution (collocation.py:113-121)
    X = g[f"X_{N}"]
    xe = np.stack([c.evaluateSolution(tt, X) for tt in t])
    assert np.allclose(xe, g[f"xeval_{N}"], rtol=0, atol=1e-13)


DYN = ["single_integrator", "single_integrator_2D", "single_integrator_3D", "double_integrator",
       "van_der_pol", "gnss_pos_and_bias", "gnss_two_receiver", "kinematic_bycicle_and_bias"]


@pytest.mark.parametrize("name", DYN)
def test_oracle_dynamics_vs_reference(golden, name):
    g = golden["plugins"]
    f, F = om.dyn_eval(name, g[f"dyn_{name}_x"], g[f"dyn_{name}_u"])
    assert np.allclose(f, g[f"dyn_{name}_f"], rtol=1e-14, atol=1e-14)
    assert np.allclose(F, g[f"dyn_{name}_F"], rtol=1e-13, atol=1e-13)


def test_oracle_vehicle_dynamics_and_gnss_vs_reference(golden):
    """nlp/dynamics.py:148-174 with the reference car constants (params["car_params"]),
    values and complex-step Jacobians of the reference plug-in."""
    g = golden["plugins"]
    name = "vehicle_dynamics_and_gnss"
    f, F = om.dyn_eval(name, g[f"dyn_{name}_x"], g[f"dyn_{name}_u"], g[f"dyn_{name}_par"])
    assert np.allclose(f, g[f"dyn_{name}_f"], rtol=1e-13, atol=1e-12)
    assert np.allclose(F, g[f"dyn_{name}_F"], rtol=1e-12, atol=1e-12)


def test_oracle_multi_receiver_m0(golden):
    g = golden["plugins"]
    f, F = om.dyn_eval("multi_receiver", g["dyn_multi_receiver_x"], None)
    assert np.allclose(f, g["dyn_multi_receiver_f"], atol=1e-14)
    assert np.allclose(F, g["dyn_multi_receiver_F"], atol=1e-14)


@pytest.mark.parametrize("name", ["full_state", "pseudorange", "vehicle_pseudorange", "multi_receiver_range_3d"])
def test_oracle_measurements_vs_reference(golden, name):
    g = golden["plugins"]
    x, par = g[f"meas_{name}_x"], g[f"meas_{name}_par"]
    h, H = om.meas_eval(name, x, par if par.size else None)
    assert np.allclose(h, g[f"meas_{name}_y"], rtol=1e-13, atol=1e-10)
    assert np.allclose(H, g[f"meas_{name}_H"], rtol=1e-12, atol=1e-12)


def test_oracle_range3d_between_receivers(golden):
    g = golden["plugins"]
    h, H = om.meas_eval("multi_receiver_range_3d", g["meas_range3d_AB_x"], None,
                        {"idxA": [0, 1, 2], "idxB": [5, 6, 7]})
    assert np.allclose(h, g["meas_range3d_AB_y"], rtol=1e-13)
    assert np.allclose(H, g["meas_range3d_AB_H"], atol=1e-12)


def test_cost_functions(golden):
    g = golden["plugins"]
    v, Q = g["cost_v"], g["cost_Q"]
    assert np.allclose(np.einsum("bi,ij,bj->b", v, Q, v), g["cost_weighted_l2"], rtol=1e-14)
    assert np.allclose(np.einsum("bi,bi->b", v, v), g["cost_l2"], rtol=1e-14)
