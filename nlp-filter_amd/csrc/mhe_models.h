// Device functors for the reference plug-ins (nlp/dynamics.py, nlp/measurements.py).
//
// Each dynamics functor: static n, m; eval(x, u, dp, f, F) writes f (n) and the
// Jacobian F = df/dx (n*n, row-major); dp = mhe_dims.dyn_par (the plug-in's params,
// e.g. params["car_params"]).  Each measurement functor: static p,
// q, LINEAR; eval(x, par, idx, h, H) writes h (p) and H = dh/dx (p*n).
// Jacobians are analytic; their parity against the reference's own plug-ins
// (complex-step through the reference code) is pinned by tests/golden/plugins.npz.
#pragma once
#include <hip/hip_runtime.h>

#include "mhe.h"

namespace mhe {

// nlp/dynamics.py:4-8  xdot = u[0]
struct DynSingleIntegrator {
  static constexpr int n = 1, m = 1;
  __device__ static void eval(const double* x, const double* u, const double*, double* f, double* F) {
    f[0] = u[0];
    F[0] = 0.0;
  }
};

// nlp/dynamics.py:10-27  xdot = u
template <int N_>
struct DynSingleIntegratorND {
  static constexpr int n = N_, m = N_;
  __device__ static void eval(const double* x, const double* u, const double*, double* f, double* F) {
#pragma unroll
    for (int a = 0; a < n; ++a) {
      f[a] = u[a];
#pragma unroll
      for (int b = 0; b < n; ++b) F[a * n + b] = 0.0;
    }
  }
};

// nlp/dynamics.py:29-38
struct DynDoubleIntegrator {
  static constexpr int n = 4, m = 2;
  __device__ static void eval(const double* x, const double* u, const double*, double* f, double* F) {
    f[0] = x[2]; f[1] = x[3]; f[2] = u[0]; f[3] = u[1];
#pragma unroll
    for (int i = 0; i < 16; ++i) F[i] = 0.0;
    F[0 * 4 + 2] = 1.0;
    F[1 * 4 + 3] = 1.0;
  }
};

// nlp/dynamics.py:61-66  [(1 - x1^2) x0 - x1 + u, x0]
struct DynVanDerPol {
  static constexpr int n = 2, m = 1;
  __device__ static void eval(const double* x, const double* u, const double*, double* f, double* F) {
    const double x0 = x[0], x1 = x[1];
    const double s = 1.0 - x1 * x1;
    f[0] = s * x0 - x1 + u[0];
    f[1] = x0;
    F[0] = s;
    F[1] = -2.0 * x1 * x0 - 1.0;
    F[2] = 1.0;
    F[3] = 0.0;
  }
};

// nlp/dynamics.py:68-79  [u0, u1, u2, x4, 0]
struct DynGnssPosAndBias {
  static constexpr int n = 5, m = 3;
  __device__ static void eval(const double* x, const double* u, const double*, double* f, double* F) {
    f[0] = u[0]; f[1] = u[1]; f[2] = u[2]; f[3] = x[4]; f[4] = 0.0;
#pragma unroll
    for (int i = 0; i < 25; ++i) F[i] = 0.0;
    F[3 * 5 + 4] = 1.0;
  }
};

// nlp/dynamics.py:81-96 (m = 0: f(x, params), nlp/nlp.py:216-219)
struct DynMultiReceiver {
  static constexpr int n = 8, m = 0;
  __device__ static void eval(const double* x, const double*, const double*, double* f, double* F) {
#pragma unroll
    for (int i = 0; i < 64; ++i) F[i] = 0.0;
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      f[a] = x[a + 4];
      f[a + 4] = 0.0;
      F[a * 8 + a + 4] = 1.0;
    }
  }
};

// nlp/dynamics.py:98-115
struct DynGnssTwoReceiver {
  static constexpr int n = 10, m = 6;
  __device__ static void eval(const double* x, const double* u, const double*, double* f, double* F) {
    f[0] = u[0]; f[1] = u[1]; f[2] = u[2]; f[3] = x[4]; f[4] = 0.0;
    f[5] = u[3]; f[6] = u[4]; f[7] = u[5]; f[8] = x[9]; f[9] = 0.0;
#pragma unroll
    for (int i = 0; i < 100; ++i) F[i] = 0.0;
    F[3 * 10 + 4] = 1.0;
    F[8 * 10 + 9] = 1.0;
  }
};

// nlp/dynamics.py:117-136 (kinematic_bycicle_and_bias; the reference code uses
// x[2] as the heading inside cos/sin, reproduced verbatim)
struct DynKinematicBicycle {
  static constexpr int n = 6, m = 2;
  __device__ static void eval(const double* x, const double* u, const double*, double* f, double* F) {
    const double L = 0.28;
    const double v = 8.72649116358 * u[0] - 0.856053299155;
    const double delta = 0.48869219055841229 * u[1];  // np.deg2rad(28)
    double sn, cs;
    sincos(x[2], &sn, &cs);
    f[0] = v * cs; f[1] = v * sn; f[2] = 0.0; f[3] = x[4]; f[4] = 0.0;
    f[5] = (v / L) * tan(delta);
#pragma unroll
    for (int i = 0; i < 36; ++i) F[i] = 0.0;
    F[0 * 6 + 2] = -v * sn;
    F[1 * 6 + 2] = v * cs;
    F[3 * 6 + 4] = 1.0;
  }
};

// R receivers, each the per-receiver block of gnss_two_receiver (nlp/dynamics.py:98-115):
// x = [x, y, z, b, alpha] per receiver (n = 5R), u = receiver velocities (m = 3R);
// xdot_r = u_r, bdot_r = alpha_r, alphadot_r = 0.  SURVEY.md §8(d) C5 (R = 8, n = 40).
// The Jacobian has R nonzeros (d b_r / d alpha_r = 1): SPARSE functors also give it as
// (row, col, value) triples so the large-system path never forms an n x n array.
template <int R_>
struct DynGnssReceivers {
  static constexpr int n = 5 * R_, m = 3 * R_;
  static constexpr bool SPARSE = true;
  static constexpr int NNZ = R_;
  __device__ static int frow(int k) { return 5 * k + 3; }
  __device__ static int fcol(int k) { return 5 * k + 4; }
  __device__ static void eval_sparse(const double* x, const double* u, const double*, double* f, double* Fv) {
#pragma unroll
    for (int r = 0; r < R_; ++r) {
      f[5 * r + 0] = u[3 * r + 0];
      f[5 * r + 1] = u[3 * r + 1];
      f[5 * r + 2] = u[3 * r + 2];
      f[5 * r + 3] = x[5 * r + 4];
      f[5 * r + 4] = 0.0;
      Fv[r] = 1.0;
    }
  }
  __device__ static void eval(const double* x, const double* u, const double* dp, double* f, double* F) {
    double Fv[NNZ];
    eval_sparse(x, u, dp, f, Fv);
    for (int i = 0; i < n * n; ++i) F[i] = 0.0;
    for (int k = 0; k < NNZ; ++k) F[frow(k) * n + fcol(k)] = Fv[k];
  }
};

// SPARSE detection: functors without the member are dense
template <class DYN, class = void>
struct dyn_sparse {
  static constexpr bool value = false;
};
template <class DYN>
struct dyn_sparse<DYN, decltype(void(DYN::SPARSE))> {
  static constexpr bool value = DYN::SPARSE;
};

// nlp/dynamics.py:148-174  vehicle_dynamics_and_gnss: x = [px, py, psi, vx, vy, r, b, bd, pz],
// u = [F_xr, delta]; the dynamic bicycle of vehicle_dynamics (:148-164, linear tyres with
// vx + 0.001 in the slip angles) plus bdot = bd.  dp = params["car_params"] as
// [C_AF, C_AR, M, D_F, D_R, I_Z] (utils/vehicle_sim.py:10-23).
struct DynVehicleGnss {
  static constexpr int n = 9, m = 2;
  __device__ static void eval(const double* x, const double* u, const double* dp, double* f, double* F) {
    const double C_AF = dp[0], C_AR = dp[1], Mv = dp[2], D_F = dp[3], D_R = dp[4], I_Z = dp[5];
    const double iv = 1.0 / (x[3] + 0.001);  // epsilon = .001 (nlp/dynamics.py:153)
    const double ar = (x[4] - D_R * x[5]) * iv, af = (x[4] + D_F * x[5]) * iv;
    const double F_yr = -C_AR * ar;
    const double F_yf = -C_AF * (af - u[1]);
    double sp, cp, su, cu;
    sincos(x[2], &sp, &cp);
    sincos(u[1], &su, &cu);
    f[0] = x[3] * cp - x[4] * sp;
    f[1] = x[3] * sp + x[4] * cp;
    f[2] = x[5];
    f[3] = (-F_yf * su + u[0]) / Mv + x[5] * x[4];
    f[4] = (F_yf * cu + F_yr) / Mv - x[5] * x[3];
    f[5] = (D_F * F_yf * cu - D_R * F_yr) / I_Z;
    f[6] = x[7];
    f[7] = 0.0;
    f[8] = 0.0;
#pragma unroll
    for (int i = 0; i < 81; ++i) F[i] = 0.0;
    // tyre forces w.r.t. vx, vy, r
    const double fr3 = C_AR * ar * iv, fr4 = -C_AR * iv, fr5 = C_AR * D_R * iv;
    const double ff3 = C_AF * af * iv, ff4 = -C_AF * iv, ff5 = -C_AF * D_F * iv;
    F[0 * 9 + 2] = -x[3] * sp - x[4] * cp;
    F[0 * 9 + 3] = cp;
    F[0 * 9 + 4] = -sp;
    F[1 * 9 + 2] = x[3] * cp - x[4] * sp;
    F[1 * 9 + 3] = sp;
    F[1 * 9 + 4] = cp;
    F[2 * 9 + 5] = 1.0;
    F[3 * 9 + 3] = -su * ff3 / Mv;
    F[3 * 9 + 4] = -su * ff4 / Mv + x[5];
    F[3 * 9 + 5] = -su * ff5 / Mv + x[4];
    F[4 * 9 + 3] = (cu * ff3 + fr3) / Mv - x[5];
    F[4 * 9 + 4] = (cu * ff4 + fr4) / Mv;
    F[4 * 9 + 5] = (cu * ff5 + fr5) / Mv - x[3];
    F[5 * 9 + 3] = (D_F * cu * ff3 - D_R * fr3) / I_Z;
    F[5 * 9 + 4] = (D_F * cu * ff4 - D_R * fr4) / I_Z;
    F[5 * 9 + 5] = (D_F * cu * ff5 - D_R * fr5) / I_Z;
    F[6 * 9 + 7] = 1.0;
  }
};

// ---------------------------------------------------------------- measurements

// nlp/measurements.py:4-5  h = x (linear: its Gauss-Newton Hessian term is constant)
template <int N_>
struct MeasFullState {
  static constexpr int p = N_, q = 0;
  static constexpr bool LINEAR = true, MIXED = false;
  __device__ static void eval(const double* x, const double*, const int*, double* h, double* H) {
#pragma unroll
    for (int a = 0; a < p; ++a) {
      h[a] = x[a];
#pragma unroll
      for (int b = 0; b < p; ++b) H[a * p + b] = (a == b) ? 1.0 : 0.0;
    }
  }
};

// nlp/measurements.py:56-70  ||x[idx0:3] - sat|| + x[idx3]
template <int N_>
struct MeasPseudorange {
  static constexpr int p = 1, q = 3;
  static constexpr bool LINEAR = false, MIXED = false;
  __device__ static void eval(const double* x, const double* par, const int* idx, double* h, double* H) {
    const double d0 = x[idx[0]] - par[0], d1 = x[idx[1]] - par[1], d2 = x[idx[2]] - par[2];
    const double rho = sqrt(d0 * d0 + d1 * d1 + d2 * d2);
    h[0] = rho + x[idx[3]];
#pragma unroll
    for (int a = 0; a < N_; ++a) H[a] = 0.0;
    const double ir = 1.0 / rho;
    H[idx[0]] += d0 * ir;
    H[idx[1]] += d1 * ir;
    H[idx[2]] += d2 * ir;
    H[idx[3]] += 1.0;
  }
};

// nlp/measurements.py:81-88  vehicle_pseudorange: |[x0, x1, x8] - sat| + x6 (fixed indices)
struct MeasVehiclePseudorange {
  static constexpr int p = 1, q = 3;
  static constexpr bool LINEAR = false, MIXED = false;
  __device__ static void eval(const double* x, const double* par, const int*, double* h, double* H) {
    const double d0 = x[0] - par[0], d1 = x[1] - par[1], d2 = x[8] - par[2];
    const double rho = sqrt(d0 * d0 + d1 * d1 + d2 * d2);
    h[0] = rho + x[6];
#pragma unroll
    for (int a = 0; a < 9; ++a) H[a] = 0.0;
    const double ir = 1.0 / rho;
    H[0] = d0 * ir;
    H[1] = d1 * ir;
    H[8] = d2 * ir;
    H[6] = 1.0;
  }
};

// nlp/measurements.py:39-54  ("y" form) sqrt(sum (x[idx] - y)^2 + 1e-6)
template <int N_>
struct MeasRange3D {
  static constexpr int p = 1, q = 3;
  static constexpr bool LINEAR = false, MIXED = false;
  __device__ static void eval(const double* x, const double* par, const int* idx, double* h, double* H) {
    const double d0 = x[idx[0]] - par[0], d1 = x[idx[1]] - par[1], d2 = x[idx[2]] - par[2];
    const double r = sqrt(d0 * d0 + d1 * d1 + d2 * d2 + 0.000001);
    h[0] = r;
#pragma unroll
    for (int a = 0; a < N_; ++a) H[a] = 0.0;
    const double ir = 1.0 / r;
    H[idx[0]] += d0 * ir;
    H[idx[1]] += d1 * ir;
    H[idx[2]] += d2 * ir;
  }
};

// A measurement row whose weight matrix is all zero contributes nothing (the reference
// masks empty satellite slots with R = 0, autonomous-car.py:260-263, gnss-multi-receiver.py:196-204).
template <int p>
__device__ __forceinline__ bool masked_row(const double* R) {
  bool z = true;
#pragma unroll
  for (int c = 0; c < p * p; ++c) z = z && R[c] == 0.0;
  return z;
}

// MHE_MEAS_MIXED: one scalar row of any of the reference plug-ins (include/mhe.h
// documents the PAR row [code, i0..i6, v0..v5]).  x has N_ + MHE_MAX_EXTRA entries
// ([x(t_i) ; z]), G (same length) receives dh/d[x ; z].  An index outside
// [0, N_ + nz) contributes nothing (rows are device data: never read out of range).
template <int N_>
struct MeasMixed {
  static constexpr int p = 1, q = MHE_MIXED_Q, NA = N_ + MHE_MAX_EXTRA;
  static constexpr bool LINEAR = false, MIXED = true;
  __device__ static void eval(const double* x, const double* par, int nz, double& h, double* G) {
#pragma unroll
    for (int c = 0; c < NA; ++c) G[c] = 0.0;
    int id[7];
    row_ids(par, nz, id);
    eval_core([&](int k) { return id[k] >= 0 ? x[id[k]] : 0.0; },
              [&](int k, double g) {
                if (id[k] >= 0) G[id[k]] += g;
              },
              par, h);
  }
  // the row's state / extra-variable index per slot (-1: none or out of range)
  __device__ static void row_ids(const double* par, int nz, int* id) {
#pragma unroll
    for (int k = 0; k < 7; ++k) {
      const int v = (int)par[1 + k];
      id[k] = (v >= 0 && v < N_ + nz) ? v : -1;
    }
  }
  // Per-slot form (k_big_resid): the row's values read through xget(index) and its
  // gradient left per slot, gs[k] = dh/dx[id[k]] (each slot receives one term), so no
  // array is indexed by a row's data -- the dense x / G arrays of eval() sit in scratch
  // memory at n = 40.
  template <class XG>
  __device__ static void eval_slots(XG xget, const double* par, int nz, double& h, int* id, double* gs) {
    row_ids(par, nz, id);
#pragma unroll
    for (int k = 0; k < 7; ++k) gs[k] = 0.0;
    eval_core([&](int k) { return id[k] >= 0 ? xget(id[k]) : 0.0; }, [&](int k, double g) { gs[k] += g; }, par, h);
  }
  template <class XF, class AF>
  __device__ static void eval_core(XF X, AF add, const double* par, double& h) {
    const double* v = par + 8;
    switch ((int)par[0]) {
      case MHE_ROW_PSEUDORANGE: {  // nlp/measurements.py:56-70
        const double d0 = X(0) - v[0], d1 = X(1) - v[1], d2 = X(2) - v[2];
        const double rho = sqrt(d0 * d0 + d1 * d1 + d2 * d2);
        h = rho + X(3);
        add(0, d0 / rho); add(1, d1 / rho); add(2, d2 / rho); add(3, 1.0);
        break;
      }
      case MHE_ROW_PSEUDORANGE_RATE: {  // nlp/measurements.py:72-79
        const double r0 = v[0] - X(0), r1 = v[1] - X(1), r2 = v[2] - X(2);
        const double nr = sqrt(r0 * r0 + r1 * r1 + r2 * r2);
        const double l0 = r0 / nr, l1 = r1 / nr, l2 = r2 / nr;
        const double w0 = v[3] - X(3), w1 = v[4] - X(4), w2 = v[5] - X(5);
        const double wl = w0 * l0 + w1 * l1 + w2 * l2;
        h = wl + X(6);
        // d/dx_pos = -(w - (w.l) l) / |r|,  d/dx_vel = -l
        add(0, -(w0 - wl * l0) / nr); add(1, -(w1 - wl * l1) / nr); add(2, -(w2 - wl * l2) / nr);
        add(3, -l0); add(4, -l1); add(5, -l2); add(6, 1.0);
        break;
      }
      case MHE_ROW_RANGE_2D:
      case MHE_ROW_RANGE_3D: {  // nlp/measurements.py:7-20, 39-54
        const int K = (int)par[0] == MHE_ROW_RANGE_2D ? 2 : 3;
        double d[3] = {0.0, 0.0, 0.0}, s = 0.000001;
        for (int k = 0; k < K; ++k) {
          d[k] = X(k) - X(k + K) - v[k];
          s += d[k] * d[k];
        }
        const double r = sqrt(s);
        h = r;
        for (int k = 0; k < K; ++k) {
          add(k, d[k] / r);
          add(k + K, -d[k] / r);
        }
        break;
      }
      case MHE_ROW_HEADING_2D: {  // nlp/measurements.py:22-37: atan2(r_x, r_y)
        const double rx = X(0) - X(1) + v[0], ry = X(2) - X(3) + v[1];
        const double q2 = rx * rx + ry * ry;
        h = atan2(rx, ry);
        add(0, ry / q2); add(1, -ry / q2); add(2, -rx / q2); add(3, rx / q2);
        break;
      }
      case MHE_ROW_COMPONENT:  // nlp/measurements.py:4-5, one component
        h = X(0);
        add(0, 1.0);
        break;
      default:
        h = 0.0;
        break;
    }
  }
};

}  // namespace mhe
