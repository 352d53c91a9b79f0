// libmhe: batched collocation Gauss-Newton for MI355X (gfx950, CDNA4) -- the C-ABI
// (include/mhe.h), argument checks, constants building and dispatch to the
// per-pair launch templates (mhe_core.h, pair_*.hip).
//
// What replaces what (reference kingdwd/nlp-filter):
//   fixedTimeOptimalEstimationNLP objective   nlp/nlp.py:202-286
//   NLP.solve() -> CasADi/IPOPT               nlp/nlp.py:61-83
// is re-built here as ONE fused kernel per batch: one workgroup (8 waves) per
// trajectory runs the whole Gauss-Newton loop
//     residual + Jacobian  ->  J^T W J, J^T W r  ->  Cholesky  ->  2 triangular
//     solves  ->  X += delta  ->  convergence test
// with the d x d normal matrix (d = (N+1) n, padded to 16*NT) held in the MFMA
// accumulator registers of the 8 waves as 16x16 fp64 tiles (off-diagonal tiles,
// 2 KB per tile, 8 VGPRs per lane; diagonal tiles in LDS).  The right-looking blocked Cholesky
// factors one 16-column panel per step in registers (row-per-lane sweep with
// scalar broadcasts), streams the panel through LDS and applies the trailing
// update with v_mfma_f64_16x16x4f64.  The forward solve rides along with the
// panel sweep (augmented column); the backward solve reads L straight from the
// tile registers.  Trajectories are independent: no inter-workgroup traffic.
//
// See DESIGN.md for the data layout, the roofline and the measurements.
#include <cstdio>
#include <string.h>

#include "mhe_core.h"

namespace mhe {

// ------------------------------------------------------------ register-path constants
__global__ void k_copy_consts(int P, int M, int n, int p, int NT, const double* D, const double* cw,
                              const double* Phi, const double* Qw, const double* Rw, const double* Pw,
                              char* cbuf) {
  const ConstLayout CL = const_layout(P, M, n, p, NT);
  double* oD = (double*)(cbuf + CL.D);
  double* oDt = (double*)(cbuf + CL.Dt);
  double* oPhi = (double*)(cbuf + CL.Phi);
  double* oPhiT = (double*)(cbuf + CL.PhiT);
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;
  const int stride = gridDim.x * blockDim.x;
  for (int e = gid; e < P * P; e += stride) {
    const int k = e / P, j = e % P;
    oD[e] = D[e];
    oDt[j * P + k] = D[e];
  }
  for (int e = gid; e < M * P; e += stride) {
    const int i = e / P, j = e % P;
    oPhi[e] = Phi[e];
    oPhiT[j * M + i] = Phi[e];
  }
  for (int e = gid; e < P; e += stride) ((double*)(cbuf + CL.cw))[e] = cw[e];
  for (int e = gid; e < n * n; e += stride) {
    ((double*)(cbuf + CL.Qw))[e] = Qw[e];
    ((double*)(cbuf + CL.Pw))[e] = Pw ? Pw[e] : 0.0;
  }
  for (int e = gid; e < M * p * p; e += stride) ((double*)(cbuf + CL.Rw))[e] = Rw[e];
}

// ------------------------------------------------------------ large-system path (mhe_big.h)
// Every trajectory starts RUNNING -- or, when the constants buffer's stamp does not
// match these dims, BAD_CONSTANTS: then no kernel of the solve touches the constants
// (X_out keeps X0, cost NaN).
__global__ void k_big_init(BigArgs a, int batch) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b < batch) {
    const bool ok = *(const unsigned long long*)a.cbuf == a.tag;
    a.state[b] = ok ? BIG_RUNNING : MHE_STATUS_BAD_CONSTANTS;
    a.iters[b] = 0;
    if (!ok) a.cost[b] = NAN;
  }
}

__global__ void k_big_finish(int batch, int* state) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b < batch && state[b] == BIG_RUNNING) state[b] = MHE_STATUS_MAX_ITER;
}

// ------------------------------------------------------------ constants
__global__ void k_big_consts(int P, int M, int n, int p, const double* D, const double* cw, const double* Qw,
                             const double* Rw, const double* Pw, char* cbuf) {
  const BigConst CL = big_const_layout(P, M, n, p);
  const int gid = blockIdx.x * blockDim.x + threadIdx.x, stride = gridDim.x * blockDim.x;
  double* oD = (double*)(cbuf + CL.D);
  double* oDt = (double*)(cbuf + CL.Dt);
  double* oDCD = (double*)(cbuf + CL.DCD);
  for (int e = gid; e < P * P; e += stride) {
    const int k = e / P, j = e % P;
    oD[e] = D[e];
    oDt[j * P + k] = D[e];
    // (D^T C D)[k][j] with C = diag(cw): element (row k, col j), formed in the same order
    // for (k, j) and (j, k) -- exactly symmetric, so k_big_assemble may read either
    const int lo = k < j ? k : j, hi = k < j ? j : k;
    double s = 0.0;
    for (int t = 0; t < P; ++t) s += D[t * P + lo] * cw[t] * D[t * P + hi];
    oDCD[e] = s;
  }
  for (int e = gid; e < P; e += stride) ((double*)(cbuf + CL.cw))[e] = cw[e];
  for (int e = gid; e < n * n; e += stride) {
    ((double*)(cbuf + CL.Qw))[e] = Qw[e];
    ((double*)(cbuf + CL.Pw))[e] = Pw ? Pw[e] : 0.0;
  }
  for (int e = gid; e < M * p * p; e += stride) ((double*)(cbuf + CL.Rw))[e] = Rw[e];
}

// equality-constraint index pairs, passed by value (kernel arguments) so that
// building constants stays a pure stream-ordered enqueue
struct EqPairs {
  int v[2 * MHE_MAX_EQ];
  double r[MHE_MAX_EQ];
};
__global__ void k_big_eq_consts(int P, int M, int n, int p, int nc, EqPairs e, char* cbuf) {
  const BigConst CL = big_const_layout(P, M, n, p, nc);
  int* o = (int*)(cbuf + CL.eq);
  double* orr = (double*)(cbuf + CL.eqr);
  for (int i = threadIdx.x; i < 2 * nc; i += blockDim.x) o[i] = e.v[i];
  for (int i = threadIdx.x; i < nc; i += blockDim.x) orr[i] = e.r[i];
}

// epoch detection: row i starts an epoch unless its Phi row equals row i-1 bitwise
__global__ void k_big_epoch_flags(int P, int M, int n, int p, const double* Phi, char* cbuf) {
  const BigConst CL = big_const_layout(P, M, n, p);
  int* flag = (int*)(cbuf + CL.flag);
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < M; i += gridDim.x * blockDim.x) {
    int f = (i == 0);
    if (!f)
      for (int j = 0; j < P; ++j)
        if (__double_as_longlong(Phi[(size_t)i * P + j]) != __double_as_longlong(Phi[(size_t)(i - 1) * P + j])) {
          f = 1;
          break;
        }
    flag[i] = f;
  }
}

__global__ void k_big_epoch_scan(int P, int M, int n, int p, char* cbuf) {
  const BigConst CL = big_const_layout(P, M, n, p);
  const int* flag = (const int*)(cbuf + CL.flag);
  int* erow = (int*)(cbuf + CL.erow);
  int E = 0;
  for (int i = 0; i < M; ++i)
    if (flag[i]) erow[E++] = i;
  erow[E] = M;
  *(int*)(cbuf + CL.ne) = E;
}

__global__ void k_big_epoch_rows(int P, int M, int n, int p, const double* Phi, char* cbuf) {
  const BigConst CL = big_const_layout(P, M, n, p);
  const int* erow = (const int*)(cbuf + CL.erow);
  const int E = *(const int*)(cbuf + CL.ne);
  double* PhiE = (double*)(cbuf + CL.PhiE);
  double* PhiET = (double*)(cbuf + CL.PhiET);
  const int Mr = M > 0 ? M : 1;
  for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < E * P; t += gridDim.x * blockDim.x) {
    const int e = t / P, j = t % P;
    const double v = Phi[(size_t)erow[e] * P + j];
    PhiE[(size_t)e * P + j] = v;
    PhiET[(size_t)j * Mr + e] = v;
  }
}

__global__ void k_write_tag(unsigned long long* p, unsigned long long tag) { *p = tag; }

int g_opt_big_right_looking = 0;
int g_opt_smem_pad = 0;

}  // namespace mhe

// ================================================================ dispatch
using namespace mhe;

#ifdef MHE_DIAG
static unsigned long long* g_dbg = nullptr;
#endif

namespace {

// The (dynamics, measurement) pairs compiled into this library (mhe/registry.py
// COMPILED_PAIRS mirrors this list).
const PairOps* find_pair(const mhe_dims* dm) {
  const PairOps* ops = pairs_vdp(dm->dyn_model, dm->meas_model);
#ifndef MHE_FAST_BUILD  // -DMHE_FAST_BUILD: van der Pol only (kernel development)
  if (!ops) ops = pairs_integrators(dm->dyn_model, dm->meas_model);
  if (!ops) ops = pairs_gnss(dm->dyn_model, dm->meas_model);
  if (!ops) ops = pairs_vehicles(dm->dyn_model, dm->meas_model);
  if (!ops) ops = pairs_receivers(dm->dyn_model, dm->meas_model);
#endif
  return ops;
}

// Every entry point validates the caller's struct first: struct_size must be
// sizeof(mhe_dims) of this build, so a binding that declares an older or truncated
// struct gets MHE_ERR_DIMS before any field past struct_size is read.
int check_dims(const mhe_dims* dm, int* NT_out) {
  if (!dm) return MHE_ERR_NULL;
  if (dm->struct_size != (int32_t)sizeof(mhe_dims)) return MHE_ERR_DIMS;
  int n, m, p, q;
  bool lin;
  if (!dyn_info(dm->dyn_model, n, m)) return MHE_ERR_MODEL;
  if (!meas_info(dm->meas_model, n, p, q, lin)) return MHE_ERR_MODEL;
  if (dm->n != n || dm->m != m || dm->p != p || dm->q != q) return MHE_ERR_DIMS;
  if (dm->N < 1 || dm->M < 0 || !(dm->T > 0.0)) return MHE_ERR_DIMS;
  if (dm->dyn_cost != MHE_COST_L2 && dm->dyn_cost != MHE_COST_HUBER) return MHE_ERR_MODEL;
  if (dm->dyn_cost == MHE_COST_HUBER && !(dm->huber_delta > 0.0)) return MHE_ERR_DIMS;
  if (dm->n_bounds < 0 || dm->n_bounds > 8) return MHE_ERR_DIMS;
  for (int i = 0; i < dm->n_bounds; ++i)
    if (dm->bound_idx[i] < 0 || dm->bound_idx[i] >= n || !(dm->bound_lb[i] <= dm->bound_ub[i])) return MHE_ERR_DIMS;
  if (dm->meas_model == MHE_MEAS_VEHICLE_PSEUDORANGE && dm->dyn_model != MHE_DYN_VEHICLE_GNSS) return MHE_ERR_DIMS;
  for (int i = 0; i < 4; ++i)
    if ((dm->meas_model == MHE_MEAS_PSEUDORANGE && (dm->meas_idx[i] < 0 || dm->meas_idx[i] >= n)) ||
        (dm->meas_model == MHE_MEAS_RANGE_3D && i < 3 && (dm->meas_idx[i] < 0 || dm->meas_idx[i] >= n)))
      return MHE_ERR_DIMS;
  const int P = dm->N + 1;
  if (dm->n_extra < 0 || dm->n_extra > MHE_MAX_EXTRA || dm->n_eq < 0 || dm->n_extra + dm->n_eq > MHE_MAX_EQ)
    return MHE_ERR_DIMS;
  if (dm->n_extra > 0 && dm->meas_model != MHE_MEAS_MIXED) return MHE_ERR_DIMS;  // z enters mixed rows only
  if (dm->n_eq > 0) {
    if (!dm->eq_idx) return MHE_ERR_NULL;
    for (int i = 0; i < dm->n_eq; ++i) {
      const int ia = dm->eq_idx[2 * i], ib = dm->eq_idx[2 * i + 1];
      if (ia < 0 || ia >= P * n || ib < -1 || ib >= P * n || ia == ib) return MHE_ERR_DIMS;
    }
  }
  if (dm->n_bounds > 0 && (dm->n_eq > 0 || dm->n_extra > 0)) return MHE_ERR_UNSUPPORTED;
  int NT = (P * n + 15) / 16;
  if (is_big(dm)) NT = n * big_pp(P) / 16;  // large-system path (mhe_big.h), component-major tiles
  if (NT_out) *NT_out = NT;
  return MHE_OK;
}

// bytes of the constants buffer: the 256-B header (layout stamp at offset 0) and the
// constants proper
size_t const_total_bytes(const mhe_dims* dm, int NT) {
  if (is_big(dm)) return big_const_layout(dm->N + 1, dm->M, dm->n, dm->p, dm->n_eq).total;
  return const_layout(dm->N + 1, dm->M, dm->n, dm->p, NT).total;
}

// FNV-1a over the dims that define the constants' layout and contents, including the
// equality rows (eq_idx pairs and the bits of eq_rhs), which mhe_build_constants copies
// into the buffer: a solve whose dims carry other rows than the buffer was built with
// is refused (MHE_STATUS_BAD_CONSTANTS) instead of silently using the old rows.
unsigned long long const_tag(const mhe_dims* dm, int NT) {
  unsigned long long h = 1469598103934665603ull;
  auto mix = [&h](long long x) {
    h ^= (unsigned long long)x;
    h *= 1099511628211ull;
  };
  const long long v[] = {0x4D4845, is_big(dm) ? 1 : 0, dm->N, dm->n, dm->m, dm->p, dm->M, dm->q, dm->dyn_model,
                         dm->meas_model, dm->has_prior, dm->dyn_cost, NT, dm->n_eq, dm->n_extra};
  for (long long x : v) mix(x);
  if (dm->n_eq > 0 && dm->eq_idx)  // check_dims has validated n_eq <= MHE_MAX_EQ and eq_idx
    for (int i = 0; i < 2 * dm->n_eq; ++i) mix(dm->eq_idx[i]);
  for (int i = 0; i < dm->n_eq; ++i) {  // NULL eq_rhs = all 0 (as the build); -0 and +0 alike
    const double r = (dm->eq_rhs ? dm->eq_rhs[i] : 0.0) + 0.0;
    long long bits;
    memcpy(&bits, &r, sizeof bits);
    mix(bits);
  }
  return h | 1ull;
}

// Constants of the large-system path: model-independent (D, D^T, D^T C D, weights,
// the epoch-compressed basis and the equality-constraint pairs).
int build_big_consts(const mhe_dims* dm, const double* D, const double* cw, const double* Phi, const double* Qw,
                     const double* Rw, const double* Pw, char* cbuf, hipStream_t st) {
  const int P = dm->N + 1;
  hipLaunchKernelGGL(k_big_consts, dim3(256), dim3(256), 0, st, P, dm->M, dm->n, dm->p, D, cw, Qw, Rw, Pw, cbuf);
  if (dm->M > 0) {
    hipLaunchKernelGGL(k_big_epoch_flags, dim3((dm->M + 255) / 256), dim3(256), 0, st, P, dm->M, dm->n, dm->p, Phi,
                       cbuf);
    hipLaunchKernelGGL(k_big_epoch_scan, dim3(1), dim3(1), 0, st, P, dm->M, dm->n, dm->p, cbuf);
    hipLaunchKernelGGL(k_big_epoch_rows, dim3(256), dim3(256), 0, st, P, dm->M, dm->n, dm->p, Phi, cbuf);
  }
  if (dm->n_eq > 0) {
    EqPairs e = {};
    for (int i = 0; i < 2 * dm->n_eq; ++i) e.v[i] = dm->eq_idx[i];
    for (int i = 0; i < dm->n_eq; ++i) e.r[i] = dm->eq_rhs ? dm->eq_rhs[i] : 0.0;
    hipLaunchKernelGGL(k_big_eq_consts, dim3(1), dim3(128), 0, st, P, dm->M, dm->n, dm->p, dm->n_eq, e, cbuf);
  }
  return hipGetLastError() == hipSuccess ? MHE_OK : MHE_ERR_HIP;
}

GnArgs make_args(const mhe_dims* dm, const void* cbuf, int NT) {
  GnArgs a = {};
#ifdef MHE_DIAG
  a.dbg = g_dbg;
#endif
  a.cbuf = (const char*)cbuf;
  a.P = dm->N + 1;
  a.M = dm->M;
  a.d = a.P * dm->n;
  a.NT = NT;
  a.ntiles = NT * (NT + 1) / 2;
  a.q = dm->q;
  a.has_prior = dm->has_prior;
  for (int i = 0; i < 8; ++i) a.idx[i] = dm->meas_idx[i];
  a.alpha = 2.0 / dm->T;
  a.huber_delta = dm->huber_delta;
  a.n_bounds = dm->n_bounds;
  a.tag = const_tag(dm, NT);
  for (int i = 0; i < 8; ++i) {
    a.bidx[i] = dm->bound_idx[i];
    a.blb[i] = dm->bound_lb[i];
    a.bub[i] = dm->bound_ub[i];
    a.dpar[i] = dm->dyn_par[i];
  }
  return a;
}

// The large-system path's launch arguments that follow from the dims and the
// constants / workspace alone (the per-solve pointers are set by the caller).
BigArgs make_big_args(const mhe_dims* dims, const void* cbuf, int NT, void* workspace) {
  BigArgs A = {};
  A.cbuf = (const char*)cbuf;
  A.P = dims->N + 1; A.M = dims->M; A.n = dims->n; A.Pp = big_pp(A.P); A.NTc = A.Pp / 16; A.NT = NT;
  A.q = dims->q; A.has_prior = dims->has_prior;
  for (int i = 0; i < 8; ++i) A.idx[i] = dims->meas_idx[i];
  A.alpha = 2.0 / dims->T;
  A.ws = (double*)workspace; A.ws_stride = big_ws_doubles(dims, NT);
  A.n_bounds = dims->n_bounds;
  for (int i = 0; i < 8; ++i) {
    A.bidx[i] = dims->bound_idx[i];
    A.blb[i] = dims->bound_lb[i];
    A.bub[i] = dims->bound_ub[i];
    A.dpar[i] = dims->dyn_par[i];
  }
  A.nz = dims->n_extra;
  A.nc = dims->n_eq;
  A.huber = dims->dyn_cost == MHE_COST_HUBER;
  A.huber_delta = dims->huber_delta;
  A.tag = const_tag(dims, NT);
  return A;
}

}  // namespace

// ------------------------------------------------------------ large-system parity I/O
// mhe_assemble_ws / mhe_chol_solve_ws on the large-system path: the kernels keep H as
// the lower 16x16 tiles (row-major inside a tile) of the COMPONENT-MAJOR system
// (unknown (node j, component c) at row c*Pp + j); the caller sees the dense NODE-MAJOR
// system of mhe_assemble (row j*n + c, j < Pp: the first P*n rows are the oracle's
// order, padding nodes last).  cm(r) maps a node-major row to its component-major one.
namespace mhe {

__device__ __forceinline__ int big_cm(int r, int n, int Pp) { return (r % n) * Pp + r / n; }

// state word per trajectory: running, or BAD_CONSTANTS when the buffer's stamp does
// not match these dims (then nothing of the stage runs and the outputs are NaN)
__global__ void k_big_parity_init(BigArgs a, int batch) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b < batch) {
    const bool ok = *(const unsigned long long*)a.cbuf == a.tag;
    a.state[b] = ok ? BIG_RUNNING : MHE_STATUS_BAD_CONSTANTS;
    if (!ok && a.cost) a.cost[b] = NAN;
    if (MHE_BIG_ENV) {  // the envelope flags k_big_import_hg sets from the caller's system
      const BigWs WL = big_ws_layout(a.P, a.M, a.n, a.NT, a.nz, a.nc);
      int* EM = big_env_mask(a.ws + (size_t)b * a.ws_stride, WL);
      for (int e = 0; e < a.n * a.n; ++e) EM[e] = 0;
    }
  }
}

__global__ void k_big_parity_finish(int batch, int* state) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b < batch && state[b] == BIG_RUNNING) state[b] = MHE_STATUS_CONVERGED;
}

// dense node-major H (full, both triangles) and g = -BV from the tiles into the leading
// dp x dp block of a ld x ld matrix per trajectory (ld = dp, or dp + K for the KKT
// system: k_big_export_border fills the rest); grid (x, batch)
__global__ void k_big_export_hg(BigArgs a, int batch, int ld, double* Hout, double* gout) {
  const int b = blockIdx.y;
  const int dp = a.n * a.Pp;
  const BigWs WL = big_ws_layout(a.P, a.M, a.n, a.NT, a.nz, a.nc);
  const double* ws = a.ws + (size_t)b * a.ws_stride;
  const bool ok = a.state[b] == BIG_RUNNING;
  const size_t nel = (size_t)dp * dp;
  for (size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < nel; e += (size_t)gridDim.x * blockDim.x) {
    const int r = (int)(e / dp), c = (int)(e % dp);
    const int R = big_cm(r, a.n, a.Pp), C = big_cm(c, a.n, a.Pp);
    const int hi = R >= C ? R : C, lo = R >= C ? C : R;
    const double v = ws[WL.H + (size_t)big_tile_index(hi >> 4, lo >> 4, a.NT) * 256 + (hi & 15) * 16 + (lo & 15)];
    Hout[(size_t)b * ld * ld + (size_t)r * ld + c] = ok ? v : NAN;
    if (c == 0) gout[(size_t)b * ld + r] = ok ? -ws[WL.BV + R] : NAN;
  }
}

// The border of the KKT system at X (mhe_assemble_kkt_ws), in the rows / columns dp ..
// dp + K - 1 after the dense H block:  [H  B; B^T  S] and g = [g_x; g_z; c(v) - r], the
// values k_big_border forms for the solve (big_border_col / _s / _rhs); grid (K, batch)
__global__ void k_big_export_border(BigArgs a, int batch, int p, double* Hout, double* gout) {
  const int b = blockIdx.y, col = blockIdx.x;
  const int n = a.n, dp = n * a.Pp, K = a.nz + a.nc, ld = dp + K;
  const BigConst CL = big_const_layout(a.P, a.M, n, p, a.nc);
  const BigWs WL = big_ws_layout(a.P, a.M, n, a.NT, a.nz, a.nc);
  const double* ws = a.ws + (size_t)b * a.ws_stride;
  const double* PhiE = (const double*)(a.cbuf + CL.PhiE);
  const int* eq = (const int*)(a.cbuf + CL.eq);
  const double* eqr = (const double*)(a.cbuf + CL.eqr);
  const int E = a.M > 0 ? *(const int*)(a.cbuf + CL.ne) : 0;
  const double* X = a.X + (size_t)b * a.P * n;
  const bool ok = a.state[b] == BIG_RUNNING;
  double* Hb = Hout + (size_t)b * ld * ld;
  for (int r = threadIdx.x; r < dp; r += blockDim.x) {  // node-major row r = j n + ca
    const int j = r / n, ca = r % n;
    const double v = ok ? big_border_col(a, ws, WL, PhiE, eq, E, n, col, ca, j) : NAN;
    Hb[(size_t)r * ld + dp + col] = v;
    Hb[(size_t)(dp + col) * ld + r] = v;
  }
  for (int c = threadIdx.x; c < K; c += blockDim.x)  // S's lower triangle, as k_big_border's LDL^T reads it
    Hb[(size_t)(dp + col) * ld + dp + c] = ok ? big_border_s(a, ws, WL, E, col >= c ? col : c, col >= c ? c : col) : NAN;
  if (threadIdx.x == 0) gout[(size_t)b * ld + dp + col] = ok ? -big_border_rhs(a, ws, WL, eq, eqr, X, E, col) : NAN;
}

// the caller's dense node-major H (lower triangle read; leading dp x dp block of a ld x ld
// matrix) and g into the tiles and BV = -g; grid (lower tiles, batch), one thread per
// tile element
__global__ void k_big_import_hg(BigArgs a, int batch, int ld, const double* Hin, const double* gin) {
  const int b = blockIdx.y;
  const BigWs WL = big_ws_layout(a.P, a.M, a.n, a.NT, a.nz, a.nc);
  double* ws = a.ws + (size_t)b * a.ws_stride;
  int t = blockIdx.x, J = 0;  // tile t -> (I, J), I >= J, column-major over the lower triangle
  while (t >= a.NT - J) {
    t -= a.NT - J;
    ++J;
  }
  const int I = J + t;
  const int tr = threadIdx.x >> 4, tc = threadIdx.x & 15;
  const int R = 16 * I + tr, C = 16 * J + tc;  // component-major
  const int r = (R % a.Pp) * a.n + R / a.Pp, c = (C % a.Pp) * a.n + C / a.Pp;
  const int hi = r >= c ? r : c, lo = r >= c ? c : r;  // node-major, lower triangle
  const double v = Hin[((size_t)b * ld + hi) * ld + lo];
  ws[WL.H + (size_t)blockIdx.x * 256 + threadIdx.x] = v;
  if (I == J && tr == 0) ws[WL.BV + 16 * I + tc] = -gin[(size_t)b * ld + (C % a.Pp) * a.n + C / a.Pp];
  if (MHE_BIG_ENV && __syncthreads_or(v != 0.0) && threadIdx.x == 0) {  // component pair flags (envelope)
    int* EM = big_env_mask(ws, WL);
    const int ca = I / a.NTc, cb = J / a.NTc;
    EM[ca * a.n + cb] = 1;
    EM[cb * a.n + ca] = 1;
  }
}

// The caller's KKT border (rows dp .. dp + K - 1 of a ld = dp + K system, lower part read:
// B^T and S) into the workspace k_big_border reads with border_import set: the columns
// of B component-major in BM and ZM (the panel padding columns K .. KP - 1 zero), S and
// r = -g_tail in KS; grid (KP, batch)
__global__ void k_big_import_border(BigArgs a, int batch, const double* Hin, const double* gin) {
  const int b = blockIdx.y, col = blockIdx.x;
  const int n = a.n, dp = n * a.Pp, K = a.nz + a.nc, ld = dp + K;
  const BigWs WL = big_ws_layout(a.P, a.M, n, a.NT, a.nz, a.nc);
  double* ws = a.ws + (size_t)b * a.ws_stride;
  const double* Hb = Hin + (size_t)b * ld * ld;
  for (int R = threadIdx.x; R < dp; R += blockDim.x) {  // component-major row R = ca Pp + j
    const int r = (R % a.Pp) * n + R / a.Pp;
    const double v = col < K ? Hb[(size_t)(dp + col) * ld + r] : 0.0;
    if (col < K) ws[WL.BM + (size_t)col * dp + R] = v;
    ws[WL.ZM + (size_t)col * dp + R] = v;
  }
  if (col < K) {
    for (int c = threadIdx.x; c < K; c += blockDim.x) {  // lower triangle of S, mirrored
      const int hi = col >= c ? col : c, lo = col >= c ? c : col;
      ws[WL.KS + (size_t)col * K + c] = Hb[(size_t)(dp + hi) * ld + dp + lo];
    }
    if (threadIdx.x == 0) ws[WL.KS + (size_t)K * K + col] = -gin[(size_t)b * ld + dp + col];
  }
}

// delta (node-major) from YV (component-major), then the border unknowns w = [dz; lambda]
// of the bordered step (K > 0); ld = dp + K per trajectory
__global__ void k_big_export_delta(BigArgs a, int batch, int ld, double* delta) {
  const int dp = a.n * a.Pp;
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (long long)batch * ld) return;
  const int b = (int)(e / ld), r = (int)(e % ld);
  const BigWs WL = big_ws_layout(a.P, a.M, a.n, a.NT, a.nz, a.nc);
  const double* ws = a.ws + (size_t)b * a.ws_stride;
  const int K = a.nz + a.nc;
  const double v = r < dp ? ws[WL.YV + big_cm(r, a.n, a.Pp)] : ws[WL.KS + (size_t)K * K + K + (r - dp)];
  delta[e] = a.state[b] == BIG_RUNNING ? v : NAN;
}

}  // namespace mhe

#ifdef MHE_DIAG
extern "C" void mhe_diag_set_buffer(void* p) { g_dbg = (unsigned long long*)p; }
#endif

extern "C" {

int32_t mhe_set_option(int32_t option, int32_t value) {
  int* slot = option == MHE_OPT_BIG_RIGHT_LOOKING ? &g_opt_big_right_looking
              : option == MHE_OPT_DEBUG_SMEM_PAD  ? &g_opt_smem_pad
                                                  : nullptr;
  if (!slot || value < 0 || (option == MHE_OPT_DEBUG_SMEM_PAD && value > 160 * 1024)) return MHE_ERR_DIMS;
  const int old = *slot;
  *slot = value;
  return old;
}

const char* mhe_version(void) { return "libmhe 0.3 (gfx950, register-tiled fp64 MFMA Cholesky)"; }

int32_t mhe_padded_dim(const mhe_dims* dims) {
  int NT = 0;
  if (check_dims(dims, &NT) != MHE_OK) return -1;
  return 16 * NT;  // big path: n * Pp (component-major)
}

size_t mhe_workspace_bytes(const mhe_dims* dims, int32_t batch) {
  int NT = 0;
  if (check_dims(dims, &NT) != MHE_OK || batch < 0) return 0;
  if (!is_big(dims)) return 0;
  return sizeof(double) * big_ws_doubles(dims, NT) * (size_t)batch;
}

size_t mhe_const_bytes(const mhe_dims* dims) {
  int NT = 0;
  if (check_dims(dims, &NT) != MHE_OK) return 0;
  return const_total_bytes(dims, NT);
}

int mhe_build_constants(const mhe_dims* dims, const double* D, const double* cw, const double* Phi,
                        const double* Qw, const double* Rw, const double* Pw, void* const_buf, void* stream) {
  int NT = 0;
  int rc = check_dims(dims, &NT);
  if (rc != MHE_OK) return rc;
  if (!D || !cw || !Qw || !const_buf || (dims->M > 0 && (!Phi || !Rw)) || (dims->has_prior && !Pw))
    return MHE_ERR_NULL;
  const PairOps* ops = find_pair(dims);
  if (!ops) return MHE_ERR_UNSUPPORTED;
  hipStream_t st = (hipStream_t)stream;
  char* cb = (char*)const_buf;
  if (is_big(dims)) {
    rc = build_big_consts(dims, D, cw, Phi, Qw, Rw, Pw, cb, st);
  } else {
    hipLaunchKernelGGL(k_copy_consts, dim3(256), dim3(256), 0, st, dims->N + 1, dims->M, dims->n, dims->p, NT, D,
                       cw, Phi, Qw, Rw, Pw, cb);
    rc = ops->build_cc(dims, NT, D, cw, Phi, Qw, Rw, Pw, cb, st);
  }
  if (rc != MHE_OK) return rc;
  hipLaunchKernelGGL(k_write_tag, dim3(1), dim3(1), 0, st, (unsigned long long*)cb, const_tag(dims, NT));
  return hipGetLastError() == hipSuccess ? MHE_OK : MHE_ERR_HIP;
}

int mhe_gn_solve(const mhe_dims* dims, const void* const_buf, int32_t batch, const double* X0, double* X_out,
                 const double* U, int64_t u_bstride, const double* Y, const double* PAR, int64_t par_bstride,
                 const double* x0, double* cost_out, int32_t* iters_out, int32_t* status_out, int32_t max_iter,
                 double tol, void* stream) {
  return mhe_gn_solve_ws(dims, const_buf, batch, X0, X_out, U, u_bstride, Y, PAR, par_bstride, x0, cost_out,
                         iters_out, status_out, max_iter, tol, nullptr, 0, stream);
}

int mhe_gn_solve_ws(const mhe_dims* dims, const void* const_buf, int32_t batch, const double* X0, double* X_out,
                    const double* U, int64_t u_bstride, const double* Y, const double* PAR, int64_t par_bstride,
                    const double* x0, double* cost_out, int32_t* iters_out, int32_t* status_out, int32_t max_iter,
                    double tol, void* workspace, size_t workspace_bytes, void* stream) {
  return mhe_gn_solve_ext(dims, const_buf, batch, X0, X_out, nullptr, nullptr, U, u_bstride, Y, PAR, par_bstride, x0,
                          cost_out, iters_out, status_out, max_iter, tol, workspace, workspace_bytes, stream);
}

int mhe_gn_solve_ext(const mhe_dims* dims, const void* const_buf, int32_t batch, const double* X0, double* X_out,
                     const double* Z0, double* Z_out, const double* U, int64_t u_bstride, const double* Y,
                     const double* PAR, int64_t par_bstride, const double* x0, double* cost_out, int32_t* iters_out,
                     int32_t* status_out, int32_t max_iter, double tol, void* workspace, size_t workspace_bytes,
                     void* stream) {
  mhe_solve_args g = {};
  g.struct_size = (int32_t)sizeof(mhe_solve_args);
  g.batch = batch; g.X0 = X0; g.X_out = X_out; g.Z0 = Z0; g.Z_out = Z_out; g.U = U; g.u_bstride = u_bstride;
  g.Y = Y; g.PAR = PAR; g.par_bstride = par_bstride; g.Rw = nullptr; g.rw_bstride = 0; g.x0 = x0;
  g.cost_out = cost_out; g.iters_out = iters_out; g.status_out = status_out; g.max_iter = max_iter; g.tol = tol;
  g.workspace = workspace; g.workspace_bytes = workspace_bytes;
  return mhe_solve(dims, const_buf, &g, stream);
}

int mhe_solve(const mhe_dims* dims, const void* const_buf, const mhe_solve_args* g, void* stream) {
  int NT = 0;
  int rc = check_dims(dims, &NT);
  if (rc != MHE_OK) return rc;
  if (!g) return MHE_ERR_NULL;
  if (g->struct_size != (int32_t)sizeof(mhe_solve_args)) return MHE_ERR_DIMS;
  const int batch = g->batch;
  if (batch < 0 || g->max_iter < 0) return MHE_ERR_DIMS;
  if (batch == 0) return MHE_OK;
  if (!const_buf || !g->X0 || !g->X_out || !g->cost_out || !g->iters_out || !g->status_out ||
      (dims->M > 0 && !g->Y) || (dims->m > 0 && !g->U) || (dims->q > 0 && !g->PAR) || (dims->has_prior && !g->x0) ||
      (dims->n_extra > 0 && (!g->Z0 || !g->Z_out)))
    return MHE_ERR_NULL;
  if (g->Rw) {  // per-solve weights: nonlinear measurement models only (a linear h folds Rw into Cc)
    int p, q;
    bool lin;
    meas_info(dims->meas_model, dims->n, p, q, lin);
    if (lin) return MHE_ERR_UNSUPPORTED;
  }
  const PairOps* ops = find_pair(dims);
  if (!ops) return MHE_ERR_UNSUPPORTED;
  hipStream_t st = (hipStream_t)stream;
  if (is_big(dims)) {
    if (!g->workspace || g->workspace_bytes < mhe_workspace_bytes(dims, batch)) return MHE_ERR_NULL;
    BigArgs A = make_big_args(dims, const_buf, NT, g->workspace);
    A.U = g->U; A.ustride = g->u_bstride; A.Y = g->Y; A.PAR = g->PAR; A.pstride = g->par_bstride; A.x0 = g->x0;
    A.Rw = g->Rw; A.rwstride = g->rw_bstride;
    A.X = g->X_out; A.cost = g->cost_out; A.iters = g->iters_out; A.state = g->status_out; A.tol = g->tol;
    A.Z = g->Z_out;
    A.lam = dims->n_eq > 0 ? g->lambda_out : nullptr;
    if (A.X != g->X0 &&
        hipMemcpyAsync(A.X, g->X0, sizeof(double) * batch * A.P * A.n, hipMemcpyDeviceToDevice, st) != hipSuccess)
      return MHE_ERR_HIP;
    if (A.nz > 0 && g->Z0 != A.Z &&
        hipMemcpyAsync(A.Z, g->Z0, sizeof(double) * batch * A.nz, hipMemcpyDeviceToDevice, st) != hipSuccess)
      return MHE_ERR_HIP;
    hipLaunchKernelGGL(k_big_init, dim3((batch + 255) / 256), dim3(256), 0, st, A, batch);
    rc = ops->big(dims, A, batch, g->max_iter, st);
    if (rc != MHE_OK) return rc;
    hipLaunchKernelGGL(k_big_finish, dim3((batch + 255) / 256), dim3(256), 0, st, batch, A.state);
    return hipGetLastError() == hipSuccess ? MHE_OK : MHE_ERR_HIP;
  }
  GnArgs a = make_args(dims, const_buf, NT);
  a.X0 = g->X0; a.Xout = g->X_out; a.U = g->U; a.ustride = g->u_bstride; a.Y = g->Y; a.PAR = g->PAR;
  a.pstride = g->par_bstride; a.x0 = g->x0; a.cost = g->cost_out; a.iters = g->iters_out; a.status = g->status_out;
  a.max_iter = g->max_iter; a.tol = g->tol; a.Rw = g->Rw; a.rwstride = g->rw_bstride;
  return ops->gn(dims, a, batch, MODE_SOLVE, st);
}

int mhe_resjac(const mhe_dims* dims, const void* const_buf, int32_t batch, const double* X, const double* U,
               int64_t u_bstride, const double* Y, const double* PAR, int64_t par_bstride, double* W, double* F,
               double* E, double* Hm, void* stream) {
  int NT = 0;
  int rc = check_dims(dims, &NT);
  if (rc != MHE_OK) return rc;
  if (dims->meas_model == MHE_MEAS_MIXED) return MHE_ERR_UNSUPPORTED;
  if (batch <= 0) return batch == 0 ? MHE_OK : MHE_ERR_DIMS;
  if (!const_buf || !X || (dims->m > 0 && !U) || (dims->M > 0 && E && !Y) || (dims->q > 0 && dims->M > 0 && !PAR))
    return MHE_ERR_NULL;
  const PairOps* ops = find_pair(dims);
  if (!ops) return MHE_ERR_UNSUPPORTED;
  ResjacArgs a = {};
  a.cbuf = (const char*)const_buf;
  a.P = dims->N + 1; a.M = dims->M; a.big = is_big(dims) ? 1 : 0; a.alpha = 2.0 / dims->T;
  a.X = X; a.U = U; a.ustride = u_bstride; a.Y = Y; a.PAR = PAR; a.pstride = par_bstride;
  a.W = W; a.F = F; a.E = E; a.Hm = Hm;
  for (int i = 0; i < 8; ++i) {
    a.idx[i] = dims->meas_idx[i];
    a.dpar[i] = dims->dyn_par[i];
  }
  a.tag = const_tag(dims, NT);
  return ops->resjac(a, batch, (hipStream_t)stream);
}

int mhe_assemble(const mhe_dims* dims, const void* const_buf, int32_t batch, const double* X, const double* U,
                 int64_t u_bstride, const double* Y, const double* PAR, int64_t par_bstride, const double* x0,
                 double* H, double* g, double* cost, void* stream) {
  int NT = 0;
  int rc = check_dims(dims, &NT);
  if (rc != MHE_OK) return rc;
  if (is_big(dims)) return MHE_ERR_UNSUPPORTED;  // kernel-level parity APIs: register path only
  if (batch <= 0) return batch == 0 ? MHE_OK : MHE_ERR_DIMS;
  if (!const_buf || !X || !H || !g || !cost || (dims->M > 0 && !Y) || (dims->m > 0 && !U) ||
      (dims->q > 0 && !PAR) || (dims->has_prior && !x0))
    return MHE_ERR_NULL;
  const PairOps* ops = find_pair(dims);
  if (!ops) return MHE_ERR_UNSUPPORTED;
  GnArgs a = make_args(dims, const_buf, NT);
  a.X0 = X; a.U = U; a.ustride = u_bstride; a.Y = Y; a.PAR = PAR; a.pstride = par_bstride; a.x0 = x0;
  a.Hout = H; a.gout = g; a.cost = cost;
  return ops->gn(dims, a, batch, MODE_ASSEMBLE, (hipStream_t)stream);
}

int mhe_chol_solve(const mhe_dims* dims, const void* const_buf, int32_t batch, const double* H, const double* g,
                   double* delta, int32_t* status, void* stream) {
  int NT = 0;
  int rc = check_dims(dims, &NT);
  if (rc != MHE_OK) return rc;
  if (is_big(dims)) return MHE_ERR_UNSUPPORTED;  // kernel-level parity APIs: register path only
  if (batch <= 0) return batch == 0 ? MHE_OK : MHE_ERR_DIMS;
  if (!const_buf || !H || !g || !delta || !status) return MHE_ERR_NULL;
  const PairOps* ops = find_pair(dims);
  if (!ops) return MHE_ERR_UNSUPPORTED;
  GnArgs a = make_args(dims, const_buf, NT);
  a.Hin = H; a.gin = g; a.dout = delta; a.status = status;
  return ops->gn(dims, a, batch, MODE_LINSOLVE, (hipStream_t)stream);
}

int mhe_assemble_ws(const mhe_dims* dims, const void* const_buf, int32_t batch, const double* X, const double* U,
                    int64_t u_bstride, const double* Y, const double* PAR, int64_t par_bstride, const double* x0,
                    double* H, double* g, double* cost, int32_t* status, void* workspace, size_t workspace_bytes,
                    void* stream) {
  return mhe_assemble_kkt_ws(dims, const_buf, batch, X, nullptr, U, u_bstride, Y, PAR, par_bstride, x0, H, g, cost,
                             status, workspace, workspace_bytes, stream);
}

int32_t mhe_solve_kernel_name(const mhe_dims* dims, int32_t batch, void* stream, char* buf, int32_t len) {
  int NT = 0;
  const int rc = check_dims(dims, &NT);
  if (rc != MHE_OK) return rc;
  if (!buf || len <= 0) return MHE_ERR_NULL;
  if (is_big(dims)) {
    BigArgs A = make_big_args(dims, nullptr, NT, nullptr);
    const bool wide = A.NT >= BIG_WIDE_NT, split = g_opt_big_right_looking == 0 && (MHE_BIG_SPLIT == 1 ||
                                                                                      (MHE_BIG_SPLIT == 2 && wide));
    snprintf(buf, len, "large-system path (dyn %d, meas %d, NT %d): k_big_resid, k_big_assemble, %s%s, k_big_%s",
             dims->dyn_model, dims->meas_model, NT,
             split ? "k_big_chol<8|4, LL, split stages> + k_big_rows" : (wide ? "k_big_chol<8" : "k_big_chol<4"),
             split ? "" : (g_opt_big_right_looking ? ">" : ", LL>"), dims->n_bounds > 0 ? "linesearch" : "update");
    return MHE_OK;
  }
  const GnChoice c = gn_choice(dims, NT, batch, MODE_SOLVE, (hipStream_t)stream);
  if (c.smem > REG_LDS_LIMIT) return MHE_ERR_UNSUPPORTED;
  snprintf(buf, len, "mhe::%s<dyn %d, meas %d, SLOTS=%d, MODE_SOLVE, HUBER=%d%s>%s", c.bounded ? "k_gn_bounded" : "k_gn",
           dims->dyn_model, dims->meas_model, c.sb ? SB_SLOTS : MAX_SLOTS, c.huber ? 1 : 0,
           c.sb ? ", MINW=2, SB=true" : "", c.sb ? " (small-batch factorization: batch <= CUs)" : " (two workgroups per CU)");
  return MHE_OK;
}

int32_t mhe_big_envelope(const mhe_dims* dims, const void* workspace, size_t workspace_bytes, int32_t traj,
                         int32_t* first_col, int32_t n_out, void* stream) {
  int NT = 0;
  const int rc = check_dims(dims, &NT);
  if (rc != MHE_OK) return rc;
  if (!is_big(dims) || !MHE_BIG_ENV) return MHE_ERR_UNSUPPORTED;
  if (!workspace || !first_col) return MHE_ERR_NULL;
  if (n_out < NT || traj < 0) return MHE_ERR_DIMS;
  const BigArgs A = make_big_args(dims, nullptr, NT, const_cast<void*>(workspace));
  if ((size_t)(traj + 1) * A.ws_stride * sizeof(double) > workspace_bytes) return MHE_ERR_DIMS;
  const BigWs WL = big_ws_layout(A.P, A.M, A.n, A.NT, A.nz, A.nc);
  const int* src = (const int*)(A.ws + (size_t)traj * A.ws_stride + WL.ENV) + A.n * A.n;
  hipStream_t st = (hipStream_t)stream;
  if (hipMemcpyAsync(first_col, src, (size_t)NT * sizeof(int32_t), hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess)
    return MHE_ERR_HIP;
  return NT;
}

int32_t mhe_kkt_dim(const mhe_dims* dims) {
  const int32_t dp = mhe_padded_dim(dims);
  return dp < 0 ? dp : dp + dims->n_extra + dims->n_eq;
}

int mhe_assemble_kkt_ws(const mhe_dims* dims, const void* const_buf, int32_t batch, const double* X, const double* Z,
                        const double* U, int64_t u_bstride, const double* Y, const double* PAR, int64_t par_bstride,
                        const double* x0, double* H, double* g, double* cost, int32_t* status, void* workspace,
                        size_t workspace_bytes, void* stream) {
  int NT = 0;
  int rc = check_dims(dims, &NT);
  if (rc != MHE_OK) return rc;
  hipStream_t st = (hipStream_t)stream;
  if (!is_big(dims)) {
    rc = mhe_assemble(dims, const_buf, batch, X, U, u_bstride, Y, PAR, par_bstride, x0, H, g, cost, stream);
    if (rc == MHE_OK && status && batch > 0 && hipMemsetAsync(status, 0, sizeof(int32_t) * batch, st) != hipSuccess)
      return MHE_ERR_HIP;
    return rc;
  }
  if (batch <= 0) return batch == 0 ? MHE_OK : MHE_ERR_DIMS;
  if (!const_buf || !X || !H || !g || !cost || !status || (dims->M > 0 && !Y) || (dims->m > 0 && !U) ||
      (dims->q > 0 && !PAR) || (dims->has_prior && !x0) || (dims->n_extra > 0 && !Z))
    return MHE_ERR_NULL;
  if (!workspace || workspace_bytes < mhe_workspace_bytes(dims, batch)) return MHE_ERR_NULL;
  const PairOps* ops = find_pair(dims);
  if (!ops) return MHE_ERR_UNSUPPORTED;
  BigArgs A = make_big_args(dims, const_buf, NT, workspace);
  A.n_bounds = 0;  // the plain GN system: the projected method's reduction belongs to the solve
  A.U = U; A.ustride = u_bstride; A.Y = Y; A.PAR = PAR; A.pstride = par_bstride; A.x0 = x0;
  A.X = const_cast<double*>(X);  // read only by k_big_resid / k_big_assemble
  A.Z = const_cast<double*>(Z);  // read only by k_big_resid
  A.cost = cost; A.state = status;
  const int nb = (batch + 255) / 256;
  hipLaunchKernelGGL(k_big_parity_init, dim3(nb), dim3(256), 0, st, A, batch);
  rc = ops->big_stage(dims, A, batch, BIG_STAGE_ASSEMBLE, st);
  if (rc != MHE_OK) return rc;
  const size_t dp = (size_t)A.n * A.Pp;
  const int K = A.nz + A.nc;
  const size_t gx0 = (dp * dp + 255) / 256;
  const unsigned gx = (unsigned)(gx0 < 8192 ? gx0 : 8192);
  hipLaunchKernelGGL(k_big_export_hg, dim3(gx, batch), dim3(256), 0, st, A, batch, (int)dp + K, H, g);
  if (K > 0) hipLaunchKernelGGL(k_big_export_border, dim3(K, batch), dim3(256), 0, st, A, batch, dims->p, H, g);
  hipLaunchKernelGGL(k_big_parity_finish, dim3(nb), dim3(256), 0, st, batch, status);
  return hipGetLastError() == hipSuccess ? MHE_OK : MHE_ERR_HIP;
}

int mhe_chol_solve_ws(const mhe_dims* dims, const void* const_buf, int32_t batch, const double* H, const double* g,
                      double* delta, int32_t* status, void* workspace, size_t workspace_bytes, void* stream) {
  int NT = 0;
  int rc = check_dims(dims, &NT);
  if (rc != MHE_OK) return rc;
  if (!is_big(dims)) return mhe_chol_solve(dims, const_buf, batch, H, g, delta, status, stream);
  if (batch <= 0) return batch == 0 ? MHE_OK : MHE_ERR_DIMS;
  if (!const_buf || !H || !g || !delta || !status) return MHE_ERR_NULL;
  if (!workspace || workspace_bytes < mhe_workspace_bytes(dims, batch)) return MHE_ERR_NULL;
  const PairOps* ops = find_pair(dims);
  if (!ops) return MHE_ERR_UNSUPPORTED;
  hipStream_t st = (hipStream_t)stream;
  BigArgs A = make_big_args(dims, const_buf, NT, workspace);
  A.n_bounds = 0;
  A.state = status;
  A.border_import = 1;  // K > 0: the caller's border, not one formed at an iterate
  A.lam = nullptr;
  const int K = A.nz + A.nc, ld = A.n * A.Pp + K;
  const int nb = (batch + 255) / 256;
  hipLaunchKernelGGL(k_big_parity_init, dim3(nb), dim3(256), 0, st, A, batch);
  hipLaunchKernelGGL(k_big_import_hg, dim3(NT * (NT + 1) / 2, batch), dim3(256), 0, st, A, batch, ld, H, g);
  if (K > 0) hipLaunchKernelGGL(k_big_import_border, dim3((K + 15) / 16 * 16, batch), dim3(256), 0, st, A, batch, H, g);
  rc = ops->big_stage(dims, A, batch, BIG_STAGE_FACTOR, st);
  if (rc != MHE_OK) return rc;
  const long long ne = (long long)batch * ld;
  hipLaunchKernelGGL(k_big_export_delta, dim3((unsigned)((ne + 255) / 256)), dim3(256), 0, st, A, batch, ld, delta);
  hipLaunchKernelGGL(k_big_parity_finish, dim3(nb), dim3(256), 0, st, batch, status);
  return hipGetLastError() == hipSuccess ? MHE_OK : MHE_ERR_HIP;
}

}  // extern "C"
