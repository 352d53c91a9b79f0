// libmhe: batched GNSS least-squares fixes for MI355X (gfx950).
//
// Replaces the per-epoch initialiser of kingdwd/nlp-filter:
//   iterativeLeastSquares     utils/leastsquares.py:19-42  position + clock bias,
//                             GN steps dx = pinv(G) drho, stop at ||dx|| < tol
//   iterativeLeastSquaresVel  utils/leastsquares.py:45-63  velocity + bias rate
//                             (one linear solve at the converged position)
//   runLeastSquares           utils/leastsquares.py:97-141 the per-epoch loop
// for many logs ("chains") at once.  ONE LANE PER TASK: a lane forms the geometry
// rows [-(s - x)/|s - x|, 1] and residuals of its epoch's satellites one after the
// other, accumulates the 4x4 normal equations G^T G dx = G^T drho in registers and
// solves them by a register Cholesky.
// For full-column-rank G this is the pinv(G) drho of the reference; results
// agree to rounding (tests state the tolerance).
//
// warm = 1 reproduces the reference's warm start: the default argument x of
// iterativeLeastSquares is one shared array that every call updates in place,
// so epoch k starts from epoch k-1's fix (b restarts at 0 every call) -- one
// lane walks its chain's epochs in order.  warm = 0 solves every epoch
// independently from x_init (one lane per epoch: all epochs in parallel).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "mhe.h"

namespace mhe_ls {

struct LsArgs {
  int chains, epochs, slots, max_iter, warm, with_vel;
  double tol;
  const double *sat_pos, *pr, *sat_vel, *pr_rate, *x_init;
  const int32_t* nsat;
  double *x_out, *b_out, *v_out, *bd_out, *x_last;
  int32_t* iters;
};

// Solve the 4x4 SPD system A s = v (A packed upper: 00 01 02 03 11 12 13 22 23 33).
// Returns false on a non-positive pivot (fewer than 4 independent rows).
__device__ bool solve4(const double* A, const double* v, double* s) {
  double L[4][4] = {};
  const int id[4][4] = {{0, 1, 2, 3}, {1, 4, 5, 6}, {2, 5, 7, 8}, {3, 6, 8, 9}};
  for (int j = 0; j < 4; ++j) {
    double d = A[id[j][j]];
    for (int k = 0; k < j; ++k) d -= L[j][k] * L[j][k];
    if (!(d > 0.0)) return false;
    L[j][j] = sqrt(d);
    for (int i = j + 1; i < 4; ++i) {
      double t = A[id[i][j]];
      for (int k = 0; k < j; ++k) t -= L[i][k] * L[j][k];
      L[i][j] = t / L[j][j];
    }
  }
  double y[4];
  for (int i = 0; i < 4; ++i) {
    double t = v[i];
    for (int k = 0; k < i; ++k) t -= L[i][k] * y[k];
    y[i] = t / L[i][i];
  }
  for (int i = 3; i >= 0; --i) {
    double t = y[i];
    for (int k = i + 1; k < 4; ++k) t -= L[k][i] * s[k];
    s[i] = t / L[i][i];
  }
  return true;
}

// One task per LANE: a lane walks its log's epochs (warm) or solves one epoch,
// accumulating the 4x4 normal equations of its satellite rows sequentially in
// registers -- no cross-lane reductions, 64 tasks per wavefront.
__device__ __forceinline__ void row_geom(double sp0, double sp1, double sp2, double x0, double x1, double x2,
                                         double g[4], double& nrm) {
  const double l0 = sp0 - x0, l1 = sp1 - x1, l2 = sp2 - x2;
  nrm = sqrt(l0 * l0 + l1 * l1 + l2 * l2);
  g[0] = -l0 / nrm; g[1] = -l1 / nrm; g[2] = -l2 / nrm; g[3] = 1.0;
}

__device__ __forceinline__ void accum(double A[10], double v[4], const double g[4], double r) {
  int t = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
#pragma unroll
    for (int j = i; j < 4; ++j) A[t++] += g[i] * g[j];
    v[i] += g[i] * r;
  }
}

__global__ __launch_bounds__(256) void k_ls(LsArgs a) {
  const int task = blockIdx.x * blockDim.x + threadIdx.x;
  const int ntask = a.warm ? a.chains : a.chains * a.epochs;
  if (task >= ntask) return;
  const int c = a.warm ? task : task / a.epochs;
  const int k0 = a.warm ? 0 : task % a.epochs;
  const int k1 = a.warm ? a.epochs : k0 + 1;
  double x0 = a.x_init[3 * c], x1 = a.x_init[3 * c + 1], x2 = a.x_init[3 * c + 2];
  for (int k = k0; k < k1; ++k) {
    const size_t e = (size_t)c * a.epochs + k;
    const int ns = min((int)a.nsat[e], a.slots);  // slots beyond the layout are never read
    const double* S = a.sat_pos + e * a.slots * 3;
    const double* PR = a.pr + e * a.slots;
    double b = 0.0;
    int it = 0;
    // fewer than 4 rows cannot fix 4 unknowns: flagged (a rank-deficient G^T G would
    // otherwise leave the last pivot at rounding level, of either sign)
    bool ok = ns >= 4;
    for (int i = 0; i < a.max_iter && ok; ++i) {
      double A[10] = {}, v[4] = {};
      for (int q = 0; q < ns; ++q) {
        double g[4], nrm;
        row_geom(S[3 * q], S[3 * q + 1], S[3 * q + 2], x0, x1, x2, g, nrm);
        accum(A, v, g, PR[q] - nrm - b);
      }
      double dx[4];
      if (!solve4(A, v, dx)) {
        ok = false;
        break;
      }
      x0 += dx[0]; x1 += dx[1]; x2 += dx[2];
      b += dx[3];
      ++it;
      if (sqrt(dx[0] * dx[0] + dx[1] * dx[1] + dx[2] * dx[2] + dx[3] * dx[3]) < a.tol) break;
    }
    a.x_out[e * 3] = x0; a.x_out[e * 3 + 1] = x1; a.x_out[e * 3 + 2] = x2;
    a.b_out[e] = b;
    a.iters[e] = ok ? it : -1;
    if (a.with_vel) {  // utils/leastsquares.py:45-63 at the fix just computed
      const double* V = a.sat_vel + e * a.slots * 3;
      const double* RR = a.pr_rate + e * a.slots;
      double A[10] = {}, v[4] = {};
      for (int q = 0; q < ns; ++q) {
        double g[4], nrm;
        row_geom(S[3 * q], S[3 * q + 1], S[3 * q + 2], x0, x1, x2, g, nrm);
        accum(A, v, g, RR[q] - (V[3 * q] * -g[0] + V[3 * q + 1] * -g[1] + V[3 * q + 2] * -g[2]));
      }
      // a singular velocity system leaves v / bd NaN; iters keeps the position fix's
      // count (velocity failure is told apart from position failure by the NaN)
      double sv[4] = {NAN, NAN, NAN, NAN};
      if (ns >= 4) (void)solve4(A, v, sv);  // sv untouched (NaN) when singular
      a.v_out[e * 3] = sv[0]; a.v_out[e * 3 + 1] = sv[1]; a.v_out[e * 3 + 2] = sv[2];
      a.bd_out[e] = sv[3];
    }
  }
  if (a.warm && a.x_last) {
    a.x_last[3 * c] = x0; a.x_last[3 * c + 1] = x1; a.x_last[3 * c + 2] = x2;
  }
}

}  // namespace mhe_ls

extern "C" int mhe_ls_run(const mhe_ls_dims* dims, int32_t chains, int32_t epochs, const double* sat_pos,
                          const double* pr, const int32_t* nsat, const double* sat_vel, const double* pr_rate,
                          const double* x_init, double* x_out, double* b_out, double* v_out, double* bd_out,
                          int32_t* iters_out, double* x_last, void* stream) {
  using namespace mhe_ls;
  if (!dims) return MHE_ERR_NULL;
  if (dims->struct_size != (int32_t)sizeof(mhe_ls_dims)) return MHE_ERR_DIMS;  // stale / truncated binding
  if (chains < 0 || epochs < 0 || dims->slots < 1 || dims->slots > 64 || dims->max_iter < 0 ||
      !(dims->tol >= 0.0))
    return MHE_ERR_DIMS;
  if (chains == 0 || epochs == 0) return MHE_OK;
  if (!sat_pos || !pr || !nsat || !x_init || !x_out || !b_out || !iters_out) return MHE_ERR_NULL;
  if (dims->with_vel && (!sat_vel || !pr_rate || !v_out || !bd_out)) return MHE_ERR_NULL;
  LsArgs a = {};
  a.chains = chains; a.epochs = epochs; a.slots = dims->slots; a.max_iter = dims->max_iter;
  a.warm = dims->warm ? 1 : 0; a.with_vel = dims->with_vel ? 1 : 0; a.tol = dims->tol;
  a.sat_pos = sat_pos; a.pr = pr; a.nsat = nsat; a.sat_vel = sat_vel; a.pr_rate = pr_rate; a.x_init = x_init;
  a.x_out = x_out; a.b_out = b_out; a.v_out = v_out; a.bd_out = bd_out; a.iters = iters_out; a.x_last = x_last;
  const long long ntask = a.warm ? (long long)chains : (long long)chains * epochs;
  const int blocks = (int)((ntask + 255) / 256);
  hipLaunchKernelGGL(k_ls, dim3(blocks), dim3(256), 0, (hipStream_t)stream, a);
  return hipGetLastError() == hipSuccess ? MHE_OK : MHE_ERR_HIP;
}
