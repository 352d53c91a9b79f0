// libmhe: batched extended Kalman filter for MI355X (gfx950).
//
// Replaces utils/ekf.py:20-61 (EKF.update -> predict / correct, kingdwd/nlp-filter)
// for many independent filter instances at once: ONE WAVEFRONT PER FILTER runs
// all `steps` updates of its instance; four instances per workgroup.  Per step
//   predict:  mu- = f(mu, u),  S- = G S G^T + Q                (utils/ekf.py:40-45)
//   correct:  P = H S- H^T + R,  K = S- H^T P^-1,
//             mu = mu- + K (z - h(mu-)),  S = S- - K H S-        (utils/ekf.py:47-61)
// The reference forms P^-1 explicitly (utils/ekf.py:55).  Here one augmented
// right-looking Cholesky sweep over [P | H S- | e] (row per lane, pivots and
// L_jc broadcast by v_readlane) gives Y = L^-1 H S- and w = L^-1 e, so that
//   K e = Y^T w   and   K H S- = Y^T Y
// -- no inverse and no back substitution; S stays symmetric by construction.
// Results agree with the reference to floating-point rounding (tests state the
// tolerance).  Plug-ins are the utils/gnss.py models as device functors.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "mhe.h"

namespace mhe_ekf {

constexpr int NWF = 4;     // filters (waves) per workgroup
constexpr int MAXP = 32;   // measurement rows per step (nz <= MAXP)

// ---------------------------------------------------------------- plug-ins
// gnss_pos_and_bias, utils/gnss.py:79-90: x+ = x + dt [u0, u1, u2, x4, 0],
// G = I + dt e_3 e_4^T (the reference updates x in place; G does not depend on x).
// gnz(r, c): structural non-zeros of G (compile-time; the predict skips the rest).
struct EkfGnssPosAndBias {
  static constexpr int n = 5, m = 3;
  static constexpr bool gnz(int r, int c) { return r == c || (r == 3 && c == 4); }
  __device__ static void step(const double* x, const double* u, double dt, const double* /*dp*/, double* xp,
                              double* G) {
    xp[0] = x[0] + dt * u[0];
    xp[1] = x[1] + dt * u[1];
    xp[2] = x[2] + dt * u[2];
    xp[3] = x[3] + dt * x[4];
    xp[4] = x[4] + dt * 0.0;
    for (int i = 0; i < n * n; ++i) G[i] = 0.0;
    for (int i = 0; i < n; ++i) G[i * n + i] = 1.0;
    G[3 * n + 4] = dt;
  }
};

// discrete_vehicle_dynamics of autonomous-car.py:18-52 (a script-defined EKF plug-in):
// x = [px, py, psi, vx, vy, r, b, bd, pz], u = [F_xr, delta]; explicit Euler on the
// dynamic bicycle of utils/vehicle_sim.py:72-85 with the linear tyres of :58-66
// (slip angles (vy -+ D r)/vx, no epsilon), plus b+ = b + dt bd.
// dp = car_params as [C_AF, C_AR, M, D_F, D_R, I_Z].  Bug-compatible with the
// reference: x is updated IN PLACE before the Jacobian is formed (autonomous-car.py:23),
// so every entry of G below is evaluated at the PREDICTED state x+, and G holds exactly
// the entries the reference writes.
struct EkfDiscreteVehicle {
  static constexpr int n = 9, m = 2;
  static constexpr bool gnz(int r, int c) {
    return r == c || ((r == 0 || r == 1) && c >= 2 && c <= 4) || (r == 2 && c == 5) ||
           (r >= 3 && r <= 5 && c >= 3 && c <= 5) || (r == 6 && c == 7);
  }
  __device__ static void step(const double* x, const double* u, double dt, const double* dp, double* xp,
                              double* G) {
    const double C_AF = dp[0], C_AR = dp[1], Mv = dp[2], D_F = dp[3], D_R = dp[4], I_Z = dp[5];
    {  // xd at x (utils/vehicle_sim.py:72-85 with linear_tire_model)
      const double a_r = (x[4] - D_R * x[5]) / x[3];
      const double a_f = (x[4] + D_F * x[5]) / x[3] - u[1];
      const double F_yr = -C_AR * a_r, F_yf = -C_AF * a_f;
      double sp, cp, su, cu;
      sincos(x[2], &sp, &cp);
      sincos(u[1], &su, &cu);
      xp[0] = x[0] + dt * (x[3] * cp - x[4] * sp);
      xp[1] = x[1] + dt * (x[3] * sp + x[4] * cp);
      xp[2] = x[2] + dt * x[5];
      xp[3] = x[3] + dt * ((-F_yf * su + u[0]) / Mv + x[5] * x[4]);
      xp[4] = x[4] + dt * ((F_yf * cu + F_yr) / Mv - x[5] * x[3]);
      xp[5] = x[5] + dt * ((D_F * F_yf * cu - D_R * F_yr) / I_Z);
      xp[6] = x[6] + dt * x[7];
      xp[7] = x[7] + dt * 0.0;
      xp[8] = x[8] + dt * 0.0;
    }
    // Jacobian at x+ (autonomous-car.py:27-51)
    const double* y = xp;
    const double ivx = 1.0 / (y[3] * y[3]);
    const double dfyf_dvx = C_AF * (y[4] + D_F * y[5]) * ivx;
    const double dfyf_dvy = -C_AF / y[3];
    const double dfyf_dr = -C_AF * D_F / y[3];
    const double dfyr_dvx = C_AR * (y[4] - D_R * y[5]) * ivx;
    const double dfyr_dvy = -C_AR / y[3];
    const double dfyr_dr = C_AR * D_R / y[3];
    double sp, cp, su, cu;
    sincos(y[2], &sp, &cp);
    sincos(u[1], &su, &cu);
    for (int i = 0; i < n * n; ++i) G[i] = 0.0;
    for (int i = 0; i < n; ++i) G[i * n + i] = 1.0;
    G[0 * n + 2] += dt * (-y[3] * sp - y[4] * cp);
    G[0 * n + 3] += dt * cp;
    G[0 * n + 4] += -dt * sp;
    G[1 * n + 2] += dt * (y[3] * cp - y[4] * sp);
    G[1 * n + 3] += dt * sp;
    G[1 * n + 4] += dt * cp;
    G[2 * n + 5] += dt;
    G[3 * n + 3] += -(dt / Mv) * (su * dfyf_dvx);
    G[3 * n + 4] += dt * (y[5] - (su * dfyf_dvy) / Mv);
    G[3 * n + 5] += dt * (y[4] - (su * dfyf_dr) / Mv);
    G[4 * n + 3] += dt * ((cu * dfyf_dvx + dfyr_dvx) / Mv - y[5]);
    G[4 * n + 4] += (dt / Mv) * (cu * dfyf_dvy + dfyr_dvy);
    G[4 * n + 5] += dt * ((cu * dfyf_dr + dfyr_dr) / Mv - y[3]);
    G[5 * n + 3] += (dt / I_Z) * (D_F * cu * dfyf_dvx - D_R * dfyr_dvx);
    G[5 * n + 4] += (dt / I_Z) * (D_F * cu * dfyf_dvy - D_R * dfyr_dvy);
    G[5 * n + 5] += (dt / I_Z) * (D_F * cu * dfyf_dr - D_R * dfyr_dr);
    G[6 * n + 7] += dt;
  }
};

// Row i of multi_pseudorange (utils/gnss.py:27-45 via pseudorange :4-24):
//   h = |x[:3] - s_i| + x[3],  H = [-(s_i - x[:3]) / |s_i - x[:3]|, 1, 0]
// with_bias (multi_pseudorange_and_bias, :48-61): the extra last row is h = x[3]
// and -- bug-compatible -- an all-zero Jacobian row.
template <bool with_bias>
struct EkfMultiPseudorange {
  static constexpr int q = 3;
  static constexpr int lane_minw = with_bias ? 2 : 4;  // k_ekf_lane waves per SIMD (no spills)
  template <int n>
  __device__ static void row(const double* x, const double* par, int i, int nz, double& h, double* H) {
    if (with_bias && i == nz - 1) {
      h = x[3];
      for (int c = 0; c < n; ++c) H[c] = 0.0;
      return;
    }
    const double l0 = par[0] - x[0], l1 = par[1] - x[1], l2 = par[2] - x[2];
    const double r = sqrt(l0 * l0 + l1 * l1 + l2 * l2);
    h = sqrt((x[0] - par[0]) * (x[0] - par[0]) + (x[1] - par[1]) * (x[1] - par[1]) +
             (x[2] - par[2]) * (x[2] - par[2])) + x[3];
    for (int c = 0; c < n; ++c) H[c] = 0.0;
    H[0] = -l0 / r;
    H[1] = -l1 / r;
    H[2] = -l2 / r;
    H[3] = 1.0;
  }
};

// vehicle_sensors_model of autonomous-car.py:54-77: multi_pseudorange on
// x_meas = [px, py, pz, b, bd] = x[0, 1, 8, 6, 7]; row i: h = |p - s_i| + b and the
// 5-column Jacobian scattered back to the 9-state (columns 0, 1, 8, 6, 7).
struct EkfVehicleSensors {
  static constexpr int q = 3;
  static constexpr int lane_minw = 2;
  template <int n>
  __device__ static void row(const double* x, const double* par, int /*i*/, int /*nz*/, double& h, double* H) {
    const double l0 = par[0] - x[0], l1 = par[1] - x[1], l2 = par[2] - x[8];
    const double r = sqrt(l0 * l0 + l1 * l1 + l2 * l2);
    h = sqrt((x[0] - par[0]) * (x[0] - par[0]) + (x[1] - par[1]) * (x[1] - par[1]) +
             (x[8] - par[2]) * (x[8] - par[2])) + x[6];
    for (int c = 0; c < n; ++c) H[c] = 0.0;
    H[0] = -l0 / r;
    H[1] = -l1 / r;
    H[8] = -l2 / r;
    H[6] = 1.0;
  }
};

struct EkfArgs {
  int batch, steps, nmeas_rows_max;
  double dt;
  double dp[8];  // static dynamics parameters (mhe_ekf_dims.dyn_par)
  double* mu;
  double* S;
  const double* U;
  long long u_bstride;
  const double* Z;
  long long z_bstride;
  const int* nz;
  long long nz_bstride;
  const double* PAR;
  long long par_bstride;
  const double* Q;
  const double* R;
  long long r_bstride, r_sstride;
  double* mu_hist;
  double* S_hist;
  int hist_bi;  // 1: histories batch-innermost, mu_hist (steps, n, B), S_hist (steps, n, n, B)
  long long es;  // element stride of U / Z / nz / PAR: 1 (batch outermost) or batch (batch innermost,
                 // the b-strides are then 1): entry e of step k of instance b at b*bstride + (k*W + e)*es
  int* status;
};

// element (b, k, e) of a per-step history with `w` entries per step
__device__ __forceinline__ size_t hist_at(const EkfArgs& a, int b, int k, int e, int w) {
  return a.hist_bi ? ((size_t)k * w + e) * a.batch + b : ((size_t)b * a.steps + k) * w + e;
}

__device__ __forceinline__ double readlane_d(double v, int lane) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)b, lane);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), lane);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// per-wave LDS scratch (doubles)
template <int n>
struct WaveSmem {
  static constexpr int MU = 0, S = MU + n, G = S + n * n, SP = G + n * n, MP = SP + n * n, H = MP + n,
                       T1 = H + MAXP * n, E = T1 + MAXP * n, Y = E + MAXP, W = Y + MAXP * n, total = W + MAXP;
};

template <class DYN, class MEAS>
__global__ __launch_bounds__(NWF * 64) void k_ekf(EkfArgs a) {
  constexpr int n = DYN::n, m = DYN::m, q = MEAS::q;
  using WS = WaveSmem<n>;
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int b = blockIdx.x * NWF + wave;
  if (b >= a.batch) return;  // whole wave exits; no workgroup barrier is used below
  double* sw = smem + wave * WS::total;
  double* mu = sw + WS::MU;
  double* S = sw + WS::S;
  double* G = sw + WS::G;
  double* SP = sw + WS::SP;
  double* MP = sw + WS::MP;
  double* H = sw + WS::H;
  double* T1 = sw + WS::T1;
  double* E = sw + WS::E;
  double* Y = sw + WS::Y;
  double* W = sw + WS::W;
  for (int t = lane; t < n; t += 64) mu[t] = a.mu[(size_t)b * n + t];
  for (int t = lane; t < n * n; t += 64) S[t] = a.S[(size_t)b * n * n + t];
  int status = 0;
  __builtin_amdgcn_wave_barrier();
  for (int k = 0; k < a.steps; ++k) {
    // ---- predict (utils/ekf.py:40-45)
    if (lane == 0) {
      double x[n], u[m > 0 ? m : 1], xp[n], Gl[n * n];
      for (int c = 0; c < n; ++c) x[c] = mu[c];
      for (int c = 0; c < m; ++c) u[c] = a.U[(long long)b * a.u_bstride + ((long long)k * m + c) * a.es];
      DYN::step(x, u, a.dt, a.dp, xp, Gl);
      for (int c = 0; c < n; ++c) MP[c] = xp[c];
      for (int c = 0; c < n * n; ++c) G[c] = Gl[c];
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    for (int t = lane; t < n * n; t += 64) {  // S- = G S G^T + Q
      const int r = t / n, c = t % n;
      double acc = 0.0;
      for (int kk = 0; kk < n; ++kk) {
        double gs = 0.0;
        for (int l = 0; l < n; ++l) gs += S[kk * n + l] * G[c * n + l];  // (S G^T)[kk][c]
        acc += G[r * n + kk] * gs;
      }
      SP[t] = acc + a.Q[t];
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    const int nz = a.nz[(long long)b * a.nz_bstride + (long long)k * a.es];
    if (nz > 0 && nz <= MAXP) {
      // ---- measurement rows at mu- (utils/ekf.py:51)
      const long long rk = (long long)k * a.nmeas_rows_max + lane;  // row index within the instance
      if (lane < nz) {
        double x[n], h, Hr[n], par[q > 0 ? q : 1];
        for (int c = 0; c < n; ++c) x[c] = MP[c];
        for (int c = 0; c < q; ++c) par[c] = a.PAR[(long long)b * a.par_bstride + (rk * q + c) * a.es];
        MEAS::template row<n>(x, par, lane, nz, h, Hr);
        for (int c = 0; c < n; ++c) H[lane * n + c] = Hr[c];
        E[lane] = a.Z[(long long)b * a.z_bstride + rk * a.es] - h;
      }
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      for (int t = lane; t < nz * n; t += 64) {  // T1 = H S-
        const int i = t / n, c = t % n;
        double acc = 0.0;
        for (int l = 0; l < n; ++l) acc += H[i * n + l] * SP[l * n + c];
        T1[t] = acc;
      }
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      // ---- augmented sweep: lane i holds row i of [P | T1 | e], P = T1 H^T + R
      const double* Rk = a.R + (long long)b * a.r_bstride + (long long)k * a.r_sstride;
      const int i = lane;
      const bool row = i < nz;
      double p[MAXP], t1[n], e = 0.0;
#pragma unroll
      for (int j = 0; j < MAXP; ++j) {
        double acc = 0.0;
        if (row && j < nz) {
          for (int l = 0; l < n; ++l) acc += T1[i * n + l] * H[j * n + l];
          acc += Rk[i * a.nmeas_rows_max + j];
        }
        p[j] = acc;
      }
#pragma unroll
      for (int c = 0; c < n; ++c) t1[c] = row ? T1[i * n + c] : 0.0;
      if (row) e = E[i];
      double idg = 0.0;
      bool bad = false;
#pragma unroll
      for (int c = 0; c < MAXP; ++c) {
        if (c < nz) {
          const double piv = readlane_d(p[c], c);
          bad |= !(piv > 0.0 && piv < INFINITY);
          const double rs = 1.0 / sqrt(piv);
          const double qv = p[c] * rs;                 // L_ic (i > c)
          const double mm = (i > c && row) ? qv * rs : 0.0;  // A'_ic / A'_cc
          idg = (i == c) ? rs : idg;
#pragma unroll
          for (int j = c + 1; j < MAXP; ++j)
            if (j < nz) p[j] -= qv * readlane_d(qv, j);
#pragma unroll
          for (int cc = 0; cc < n; ++cc) t1[cc] -= mm * readlane_d(t1[cc], c);
          e -= mm * readlane_d(e, c);
        }
      }
      if (bad) status = 1;
      if (row) {
#pragma unroll
        for (int c = 0; c < n; ++c) Y[i * n + c] = t1[c] * idg;  // Y = L^-1 H S-
        W[i] = e * idg;                                         // w = L^-1 e
      }
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      // mu = mu- + Y^T w ; S = S- - Y^T Y   (utils/ekf.py:34-35, 58-59)
      for (int t = lane; t < n * n; t += 64) {
        const int r = t / n, c = t % n;
        double acc = 0.0;
        for (int ii = 0; ii < nz; ++ii) acc += Y[ii * n + r] * Y[ii * n + c];
        S[t] = SP[t] - acc;
      }
      for (int t = lane; t < n; t += 64) {
        double acc = 0.0;
        for (int ii = 0; ii < nz; ++ii) acc += Y[ii * n + t] * W[ii];
        mu[t] = MP[t] + acc;
      }
    } else {
      if (nz > MAXP) status = 2;
      for (int t = lane; t < n * n; t += 64) S[t] = SP[t];
      for (int t = lane; t < n; t += 64) mu[t] = MP[t];
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    if (a.mu_hist)
      for (int t = lane; t < n; t += 64) a.mu_hist[hist_at(a, b, k, t, n)] = mu[t];
    if (a.S_hist)
      for (int t = lane; t < n * n; t += 64) a.S_hist[hist_at(a, b, k, t, n * n)] = S[t];
  }
  for (int t = lane; t < n; t += 64) a.mu[(size_t)b * n + t] = mu[t];
  for (int t = lane; t < n * n; t += 64) a.S[(size_t)b * n * n + t] = S[t];
  if (a.status && lane == 0) a.status[b] = status;
}

// ---------------------------------------------------------------- one filter per lane
// When every step's R is diagonal (dims->r_diag, checked by the caller) the
// correction is done as nz sequential SCALAR updates, all linearised at the
// prediction mu- (row i: h_i, H_i at mu-; innovation e_i = z_i - h_i(mu-) -
// H_i (mu - mu-) against the running mean).  For a linear(ised) measurement
// model with diagonal R this is algebraically the reference's batch update
// (utils/ekf.py:51-59: K = S- H^T P^-1, mu = mu- + K e, S = S- - K H S-):
//   v = S H_i^T,  s = H_i v + R_ii,  mu += v e_i / s,  S -= v v^T / s.
// The whole filter lives in one lane's registers (mu, mu-, S: 35 doubles), so a
// wave runs 64 filters with no broadcasts, barriers or LDS: O(p n^2) work per
// step instead of the sweep's O(p^3), and no lane idles on the row loop.
// S storage in one lane: full n x n for small n; for larger n (the 9-state vehicle)
// the upper triangle only (45 instead of 81 doubles, so S and S- fit the registers).
// The symmetric form reads S[r][c] = S[c][r] = stored (min, max) entry.
template <int n>
struct LaneS {
  static constexpr bool sym = true;
  static constexpr int size = sym ? n * (n + 1) / 2 : n * n;
  static constexpr int at(int r, int c) {
    return sym ? (r <= c ? r * n - r * (r - 1) / 2 + (c - r) : c * n - c * (c - 1) / 2 + (r - c)) : r * n + c;
  }
};

template <class DYN, class MEAS>
__global__ __launch_bounds__(256, MEAS::lane_minw) void k_ekf_lane(EkfArgs a) {
  constexpr int n = DYN::n, m = DYN::m, q = MEAS::q;
  using LS = LaneS<n>;
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= a.batch) return;  // no barriers below
  double mu[n], S[LS::size];
#pragma unroll
  for (int c = 0; c < n; ++c) mu[c] = a.mu[(size_t)b * n + c];
#pragma unroll
  for (int r = 0; r < n; ++r)
#pragma unroll
    for (int c = 0; c < n; ++c)
      if (!LS::sym || c >= r) S[LS::at(r, c)] = a.S[(size_t)b * n * n + r * n + c];
  int status = 0;
  for (int k = 0; k < a.steps; ++k) {
    // ---- predict: mu- = f(mu, u), S- = G S G^T + Q   (utils/ekf.py:40-45); only the
    // structural non-zeros of G (DYN::gnz, compile time) enter the products
    double u[m > 0 ? m : 1], mp[n], G[n * n];
#pragma unroll
    for (int c = 0; c < m; ++c) u[c] = a.U[(long long)b * a.u_bstride + ((long long)k * m + c) * a.es];
    DYN::step(mu, u, a.dt, a.dp, mp, G);
    double SN[LS::size];
#pragma unroll
    for (int c = 0; c < n; ++c) {
      double v[n];  // (S G^T)[:, c]
#pragma unroll
      for (int l = 0; l < n; ++l) {
        double acc = 0.0;
#pragma unroll
        for (int kk = 0; kk < n; ++kk)
          if (DYN::gnz(c, kk)) acc += S[LS::at(l, kk)] * G[c * n + kk];
        v[l] = acc;
      }
#pragma unroll
      for (int r = 0; r < n; ++r) {
        if (LS::sym && r > c) continue;
        double acc = 0.0;
#pragma unroll
        for (int l = 0; l < n; ++l)
          if (DYN::gnz(r, l)) acc += G[r * n + l] * v[l];
        SN[LS::at(r, c)] = acc + a.Q[r * n + c];
      }
    }
#pragma unroll
    for (int i = 0; i < LS::size; ++i) S[i] = SN[i];
#pragma unroll
    for (int c = 0; c < n; ++c) mu[c] = mp[c];
    // ---- correct: sequential scalar updates at the linearisation point mu-
    const int nz = a.nz[(long long)b * a.nz_bstride + (long long)k * a.es];
    if (nz > MAXP) status = 2;
    const int rows = nz <= MAXP ? nz : 0;
    // with batch-innermost inputs (es = batch) consecutive lanes read consecutive words
    const double* zk = a.Z + (long long)b * a.z_bstride + (long long)k * a.nmeas_rows_max * a.es;
    const double* pk = a.PAR + (long long)b * a.par_bstride + (long long)k * a.nmeas_rows_max * q * a.es;
    const double* Rk = a.R + (long long)b * a.r_bstride + (long long)k * a.r_sstride;
    // rows in chunks of RCH: all of a chunk's inputs (z, satellite position, R_ii) are
    // loaded before its first update, so a step costs ceil(nz / RCH) memory round
    // trips instead of nz (clamped rows read valid memory and are skipped)
    constexpr int RCH = 8;
    for (int i0 = 0; i0 < rows; i0 += RCH) {
      double zr[RCH], pr[RCH][q > 0 ? q : 1], rr[RCH];
#pragma unroll
      for (int u = 0; u < RCH; ++u) {
        const int ic = min(i0 + u, rows - 1);
        zr[u] = zk[ic * a.es];
#pragma unroll
        for (int c = 0; c < q; ++c) pr[u][c] = pk[(ic * q + c) * a.es];
        rr[u] = Rk[ic * a.nmeas_rows_max + ic];
      }
#pragma unroll
      for (int u = 0; u < RCH; ++u) {
        if (i0 + u >= rows) break;
        double h, H[n];
        MEAS::template row<n>(mp, pr[u], i0 + u, nz, h, H);
        double e = zr[u] - h;
#pragma unroll
        for (int c = 0; c < n; ++c) e -= H[c] * (mu[c] - mp[c]);
        double v[n];
#pragma unroll
        for (int r = 0; r < n; ++r) {
          double acc = 0.0;
#pragma unroll
          for (int c = 0; c < n; ++c) acc += S[LS::at(r, c)] * H[c];
          v[r] = acc;
        }
        double sv = rr[u];
#pragma unroll
        for (int c = 0; c < n; ++c) sv += H[c] * v[c];
        if (!(sv > 0.0 && sv < INFINITY)) status = 1;
        const double inv = 1.0 / sv;
        const double ge = e * inv;
#pragma unroll
        for (int r = 0; r < n; ++r) mu[r] += v[r] * ge;
#pragma unroll
        for (int r = 0; r < n; ++r) {
          const double vr = v[r] * inv;
#pragma unroll
          for (int c = 0; c < n; ++c)
            if (!LS::sym || c >= r) S[LS::at(r, c)] -= vr * v[c];
        }
      }
    }
    // histories: with the batch-innermost layout (hist_bi) consecutive lanes write
    // consecutive words -- one coalesced 512-B store per entry instead of 64 partial lines
    if (a.mu_hist) {
#pragma unroll
      for (int c = 0; c < n; ++c) a.mu_hist[hist_at(a, b, k, c, n)] = mu[c];
    }
    if (a.S_hist) {
#pragma unroll
      for (int r = 0; r < n; ++r)
#pragma unroll
        for (int c = 0; c < n; ++c) a.S_hist[hist_at(a, b, k, r * n + c, n * n)] = S[LS::at(r, c)];
    }
  }
#pragma unroll
  for (int c = 0; c < n; ++c) a.mu[(size_t)b * n + c] = mu[c];
#pragma unroll
  for (int r = 0; r < n; ++r)
#pragma unroll
    for (int c = 0; c < n; ++c) a.S[(size_t)b * n * n + r * n + c] = S[LS::at(r, c)];
  if (a.status) a.status[b] = status;
}

template <class DYN, class MEAS>
int launch(EkfArgs& a, hipStream_t st, bool r_diag) {
  if (r_diag) {
    hipLaunchKernelGGL((k_ekf_lane<DYN, MEAS>), dim3((a.batch + 255) / 256), dim3(256), 0, st, a);
  } else {
    const int smem = NWF * WaveSmem<DYN::n>::total * (int)sizeof(double);
    hipLaunchKernelGGL((k_ekf<DYN, MEAS>), dim3((a.batch + NWF - 1) / NWF), dim3(NWF * 64), smem, st, a);
  }
  return hipGetLastError() == hipSuccess ? MHE_OK : MHE_ERR_HIP;
}

}  // namespace mhe_ekf

extern "C" int mhe_ekf_run(const mhe_ekf_dims* dims, int32_t batch, int32_t steps, double* mu, double* S,
                           const double* U, int64_t u_bstride, const double* Z, int64_t z_bstride, const int32_t* nz,
                           int64_t nz_bstride, const double* PAR, int64_t par_bstride, const double* Q,
                           const double* R, int64_t r_bstride, int64_t r_sstride, double* mu_hist, double* S_hist,
                           int32_t* status, void* stream) {
  using namespace mhe_ekf;
  if (!dims) return MHE_ERR_NULL;
  if (dims->struct_size != (int32_t)sizeof(mhe_ekf_dims)) return MHE_ERR_DIMS;  // stale / truncated binding
  if (batch < 0 || steps < 0 || dims->pmax < 1 || dims->pmax > MAXP) return MHE_ERR_DIMS;
  if (batch == 0 || steps == 0) return MHE_OK;
  if (!mu || !S || !Q || !nz || !Z || !R || (dims->m > 0 && !U)) return MHE_ERR_NULL;
  EkfArgs a = {};
  a.batch = batch; a.steps = steps; a.nmeas_rows_max = dims->pmax; a.dt = dims->dt;
  a.mu = mu; a.S = S; a.U = U; a.u_bstride = u_bstride; a.Z = Z; a.z_bstride = z_bstride; a.nz = nz;
  a.nz_bstride = nz_bstride; a.PAR = PAR; a.par_bstride = par_bstride; a.Q = Q; a.R = R; a.r_bstride = r_bstride;
  a.r_sstride = r_sstride; a.mu_hist = mu_hist; a.S_hist = S_hist; a.status = status;
  a.hist_bi = dims->hist_batch_inner != 0;
  a.es = 1;
  if (dims->in_batch_inner) {  // U (steps, m, B), Z (steps, pmax, B), nz (steps, B), PAR (steps, pmax, q, B)
    a.es = batch;
    a.u_bstride = a.z_bstride = a.nz_bstride = a.par_bstride = 1;
  }
  hipStream_t st = (hipStream_t)stream;
  for (int i = 0; i < 8; ++i) a.dp[i] = dims->dyn_par[i];
  if (dims->q != 3) return MHE_ERR_DIMS;
  if (!PAR) return MHE_ERR_NULL;
  const bool rd = dims->r_diag != 0;
  if (dims->dyn_model == MHE_EKF_DYN_GNSS_POS_AND_BIAS) {
    if (dims->n != 5 || dims->m != 3) return MHE_ERR_MODEL;
    switch (dims->meas_model) {
      case MHE_EKF_MEAS_MULTI_PSEUDORANGE:
        return launch<EkfGnssPosAndBias, EkfMultiPseudorange<false>>(a, st, rd);
      case MHE_EKF_MEAS_MULTI_PSEUDORANGE_AND_BIAS:
        return launch<EkfGnssPosAndBias, EkfMultiPseudorange<true>>(a, st, rd);
    }
  } else if (dims->dyn_model == MHE_EKF_DYN_DISCRETE_VEHICLE) {
    if (dims->n != 9 || dims->m != 2) return MHE_ERR_MODEL;
    if (!(dims->dyn_par[2] != 0.0 && dims->dyn_par[5] != 0.0)) return MHE_ERR_DIMS;  // M, I_Z unset
    if (dims->meas_model == MHE_EKF_MEAS_VEHICLE_SENSORS)
      return launch<EkfDiscreteVehicle, EkfVehicleSensors>(a, st, rd);
  }
  return MHE_ERR_MODEL;
}
