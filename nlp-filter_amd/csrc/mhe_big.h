// libmhe: large-system Gauss-Newton path (padded system beyond the register-
// resident limit, i.e. C3-C5: d = 1005 / 3006 / 8040).  Included by mhe_gn.hip
// inside namespace mhe; shares the model functors and the panel / reduction
// helpers with the register-resident kernel.
//
// Same iteration as k_gn (nlp/nlp.py:202-286 objective, GN with W eliminated),
// run as a stream-ordered sequence of kernels per iteration over a caller-owned
// workspace:
//   k_big_resid    residuals, dynamics Jacobians, epoch-grouped measurement
//                  terms G_e = sum_{i in e} H_i^T R_i H_i, gradient, cost
//   k_big_assemble lower tiles of H in COMPONENT-MAJOR order (index a*Pp + j):
//                  the (a,b) block is the P x P matrix
//                    a^2 Qw_ab (D^T C D) - a (D^T diag(E_ab) + diag(E_ba) D)
//                    + diag(FtE_ab) + Phi_E^T diag(G_ab) Phi_E
//                  whose measurement part is an MFMA GEMM over the epochs
//   k_big_chol     blocked right-looking Cholesky on HBM-resident 16x16 tiles
//                  (diagonal blocks through the same single-wave panel as k_gn,
//                  MFMA TRSM and trailing updates, block column cached in LDS
//                  when it fits) + forward and backward solves
//   k_big_border   (extra variables z / equality constraints)
//                  bordered KKT step through the factor: H Z = [H_xz C^T] by a
//                  16-column MFMA forward/backward substitution, Schur complement
//                  S - B^T Z, LDL^T (quasi-definite: z pivots > 0, constraint
//                  pivots < 0), delta -= Z w
//   k_big_update   X += delta (back to node-major), z += dz, convergence / status
// Converged or failed trajectories are frozen by a per-trajectory state word,
// so the host loop only enqueues (no synchronisation).

#ifndef MHE_BIG_DIAG_DB
#define MHE_BIG_DIAG_DB 1  // split diagonal stage: KC = 2 double-buffered slabs (C3 +0.8 %, C4 0)
#endif
#ifndef MHE_BIG_ENV
#define MHE_BIG_ENV 1  // split form: skip the tiles outside the factor's envelope (component-pair sparsity; C5 5.8x, C3 +8 %)
#endif
#ifndef MHE_BIG_WSKIP
#define MHE_BIG_WSKIP 1  // envelope: a row's wave skips the left-looking chunks left of its own f (k_big_rows: C5 +2.5 %, C3 +2.7 %)
#endif
#ifndef MHE_BIG_WSKIP_DIAG
#define MHE_BIG_WSKIP_DIAG 0  // the same for the diagonal stage's rows (neutral to -1 %; with the rows' skip C4 -4 %)
#endif
#ifndef MHE_BIG_ASM_ZSKIP
#define MHE_BIG_ASM_ZSKIP 1  // envelope: k_big_assemble skips storing zero tiles the previous factorization left zero (C5 +2.8 %)
#endif
#ifndef MHE_BIG_RESID_SLOTS
#define MHE_BIG_RESID_SLOTS 1  // k_big_resid, mixed rows: per-slot gradients (MeasMixed::eval_slots), scratch 752 -> 352 B/lane (C5 +1.8 %)
#endif
#ifndef MHE_BIG_DIAG_AKPF
#define MHE_BIG_DIAG_AKPF 1  // diagonal block: the next diagonal tile loaded one column ahead (+0.3 %)
#endif
#ifndef MHE_BIG_RESID_LDS
#define MHE_BIG_RESID_LDS 1  // k_big_resid: X staged in LDS for the node / epoch dot products (C3 +0.7 %)
#endif
constexpr int BIG_NW = 8;
constexpr int BIG_NTHREADS = BIG_NW * 64;
constexpr int BIG_RUNNING = -1;

__host__ __device__ inline int big_pp(int P) { return 16 * ((P + 15) / 16); }

struct BigConst {  // byte offsets into the constants buffer
  size_t D, Dt, DCD, cw, Qw, Pw, Rw, PhiE, PhiET, erow, ne, flag, eq, eqr, total;
};

__host__ __device__ inline BigConst big_const_layout(int P, int M, int n, int p, int nc = 0) {
  BigConst L;
  size_t o = CONST_HEADER;  // the layout stamp (mhe_core.h)
  const int Mr = M > 0 ? M : 1;
  L.D = o;     o = align256(o + sizeof(double) * P * P);
  L.Dt = o;    o = align256(o + sizeof(double) * P * P);
  L.DCD = o;   o = align256(o + sizeof(double) * P * P);
  L.cw = o;    o = align256(o + sizeof(double) * P);
  L.Qw = o;    o = align256(o + sizeof(double) * n * n);
  L.Pw = o;    o = align256(o + sizeof(double) * n * n);
  L.Rw = o;    o = align256(o + sizeof(double) * Mr * p * p);
  L.PhiE = o;  o = align256(o + sizeof(double) * Mr * P);   // unique measurement rows (epochs) x P
  L.PhiET = o; o = align256(o + sizeof(double) * P * Mr);   // P x E (stride Mr)
  L.erow = o;  o = align256(o + sizeof(int) * (Mr + 1));    // first row of each epoch, erow[E] = M
  L.ne = o;    o = align256(o + sizeof(int));               // E
  L.flag = o;  o = align256(o + sizeof(int) * Mr);          // scratch: row starts a new epoch
  L.eq = o;    o = align256(o + sizeof(int) * 2 * (nc > 0 ? nc : 1));  // equality-constraint index pairs
  L.eqr = o;   o = align256(o + sizeof(double) * (nc > 0 ? nc : 1));   // their constants: v[a] - v[b] = r
  L.total = o;
  return L;
}

struct BigWs {  // per-trajectory workspace offsets in doubles
  size_t H, LT, BV, YV, XE, GEe, Ge, Es, FtE, Vs, FtV, GZe, HZZe, GZVe, BM, ZM, DZ, ACT, GV, NZ, LAM, KS, ENV, total;
};

// nz extra variables, nc equality constraints (border of the KKT system)
__host__ __device__ inline BigWs big_ws_layout(int P, int M, int n, int NT, int nz = 0, int nc = 0) {
  BigWs W;
  size_t o = 0;
  const size_t ntiles = (size_t)NT * (NT + 1) / 2;
  const int Mr = M > 0 ? M : 1;
  const int dp = 16 * NT;
  auto al = [](size_t x) { return (x + 31) & ~size_t(31); };  // 256-B alignment
  W.H = o;   o = al(o + ntiles * 256);
  W.LT = o;  o = al(o + (size_t)NT * DTS);
  W.BV = o;  o = al(o + dp);
  W.YV = o;  o = al(o + dp);
  W.XE = o;  o = al(o + (size_t)Mr * n);
  W.GEe = o; o = al(o + (size_t)Mr * n);
  W.Ge = o;  o = al(o + (size_t)Mr * n * n);
  W.Es = o;  o = al(o + (size_t)P * n * n);  // E_k = c_k Qw F_k, component-major [(a n + b) P + k]
  W.FtE = o; o = al(o + (size_t)P * n * n);
  W.Vs = o;  o = al(o + (size_t)P * n);
  W.FtV = o; o = al(o + (size_t)P * n);
  const int NZX = nz > 0 ? MHE_MAX_EXTRA : 0, K = nz + nc;
  W.GZe = o;  o = al(o + (size_t)(nz > 0 ? Mr : 0) * n * NZX);   // per epoch  sum H_x^T R H_z
  W.HZZe = o; o = al(o + (size_t)(nz > 0 ? Mr : 0) * NZX * NZX); //            sum H_z^T R H_z
  W.GZVe = o; o = al(o + (size_t)(nz > 0 ? Mr : 0) * NZX);       //            sum H_z^T R e
  W.BM = o;   o = al(o + (size_t)K * dp);                        // border columns [H_xz C^T]
  W.ZM = o;   o = al(o + (size_t)((K + 15) / 16) * 16 * dp);     // H^-1 [H_xz C^T] (16-col panels)
  W.DZ = o;   o = al(o + (size_t)NZX);                           // z step
  W.ACT = o;  o = al(o + (size_t)dp / 2);                        // bounds: epsilon-active set (int per unknown)
  W.GV = o;   o = al(o + (size_t)dp);                            // bounds: -g at the iterate (k_big_chol
                                                                 // overwrites BV with the forward solve)
  W.NZ = o;   o = al(o + 1);                                     // bounds: the cost's rounding level at X
  W.LAM = o;  o = al(o + (size_t)P * n);                         // Huber IRLS weights c_k lambda_ka
  W.KS = o;   o = al(o + (size_t)K * K + 2 * K);                 // border: S (K x K), r, w of the last
                                                                 // bordered step (kernel-level KKT parity)
  W.ENV = o;  o = al(o + ((size_t)n * n + NT + 1) / 2);          // envelope (ints): n x n component-pair
                                                                 // nonzero flags, then each tile row's
                                                                 // first nonzero tile column (big_env_*)
  W.total = o;
  return W;
}
// The envelope of the split factorization.  k_big_assemble (or the kernel-level import)
// flags every component pair (a, b) whose block of H has a nonzero element; tile row I of
// component a then has no nonzero tile left of f(I) = NTc * min{b : (a, b) flagged}, and
// neither has the Cholesky factor (fill stays inside the envelope of A's rows), so the
// left-looking updates start at the rows' f, and the backward solve skips the tiles left
// of them.  Skipped terms are products with exact zeros: the iterates are those of the
// dense forms (C5's eight receivers: a receiver's components couple to its own and, by
// the range rows, to the previous receiver's positions -- 1/17 of the dense work).
__device__ __forceinline__ int* big_env_mask(const double* ws, const BigWs& WL) {
  return (int*)const_cast<double*>(ws + WL.ENV);
}
__device__ __forceinline__ int* big_env_first(const double* ws, const BigWs& WL, int n) { return big_env_mask(ws, WL) + n * n; }

constexpr int BIG_MAX_PAIRS = 44 * 45 / 2;  // component pairs (ca >= cb) of the largest model (n = 40 + z)

struct BigArgs {
  const char* cbuf;
  int P, M, n, Pp, NTc, NT, q, has_prior;
  int idx[8];
  double alpha;
  const double* U;
  long long ustride;
  const double* Y;
  const double* PAR;
  long long pstride;
  const double* x0;
  double* X;       // (B, P, n) current iterate (X_out)
  double* cost;
  int* iters;
  int* state;      // BIG_RUNNING or final MHE_STATUS_*
  double tol;
  double* ws;      // workspace base
  size_t ws_stride;  // doubles per trajectory
  int n_bounds;      // addVarBounds: projected Newton (k_big_linesearch)
  int bidx[8];
  double blb[8], bub[8];
  int nz, nc;        // extra variables / equality constraints (f4)
  double* Z;         // (B, nz) current extra variables (Z_out)
  double* lam;       // (B, nc) or NULL: multipliers of the constraint rows, last bordered step
  unsigned long long tag;  // layout stamp expected at offset 0 of the constants buffer
  // component pairs (ca >= cb) of the measurement contraction, those whose G_e can be
  // nonzero first ("live": both components in the measurement Jacobian's support),
  // and the k_big_assemble chunking over them (BigPairPlan)
  int npr, nlive, nchl, pchl, nch;
  unsigned char pa[BIG_MAX_PAIRS], pb[BIG_MAX_PAIRS];
  double dpar[8];    // mhe_dims.dyn_par (dynamics plug-in params)
  const double* Rw;  // per-solve measurement weights (B|1, M, p, p) or NULL = the constants' Rw
  long long rwstride;
  int huber;         // MHE_COST_HUBER: IRLS weights (k_big_resid), D^T diag(c lambda) D blocks (k_big_assemble)
  double huber_delta;
  int border_import;  // k_big_border: the border B, S and r were imported into BM / ZM / KS
                      // (mhe_chol_solve_ws on a KKT system) instead of formed at X
  int asm_zskip;      // k_big_assemble: tiles left of the envelope the previous iteration's
                      // factorization used hold zeros (iterations >= 1 of one launch_big)
};

// measurement weights of trajectory b: the per-solve array when given, else the constants'
__device__ __forceinline__ const double* big_rw(const BigArgs& a, const double* Rc, int b) {
  return a.Rw ? a.Rw + (long long)b * a.rwstride : Rc;
}

__device__ __forceinline__ int big_tile_index(int I, int J, int NT) { return J * NT - J * (J - 1) / 2 + (I - J); }

// ------------------------------------------------------------ bounds
// addVarBounds as the projected Newton method of k_gn_bounded (mhe_gn.hip; oracle
// gauss_newton_bounded): k_big_resid marks the epsilon-active set, k_big_assemble
// reduces the active rows / columns of H to their diagonal, k_big_linesearch runs
// the Armijo search along the projection arc and the stopping test.
__device__ __forceinline__ void big_box(const BigArgs& a, int c, double& lo, double& hi) {
  lo = -INFINITY;
  hi = INFINITY;
  for (int i = 0; i < a.n_bounds; ++i)
    if (a.bidx[i] == c) {
      lo = fmax(lo, a.blb[i]);
      hi = fmin(hi, a.bub[i]);
    }
}

// block max of two values (BIG_NTHREADS threads, red >= 2 BIG_NW doubles), broadcast
__device__ __forceinline__ void big_max2(double* red, double& x, double& y) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  x = wave_max(x);
  y = wave_max(y);
  __syncthreads();
  if (lane == 0) {
    red[wave] = x;
    red[BIG_NW + wave] = y;
  }
  __syncthreads();
  x = red[0];
  y = red[BIG_NW];
  for (int w = 1; w < BIG_NW; ++w) {
    x = fmax(x, red[w]);
    y = fmax(y, red[BIG_NW + w]);
  }
  __syncthreads();
}

// ACT[c Pp + j] = 1 for the epsilon-active unknowns at X (node-major) with the
// gradient -BV (component-major); called by every thread of the trajectory's block
template <int n>
__device__ void big_active_set(const BigArgs& a, const double* X, const double* BV, int* ACT, double* red) {
  double w = 0.0, xm = 0.0;
  for (int t = threadIdx.x; t < a.P * n; t += BIG_NTHREADS) {
    const int j = t / n, c = t % n;
    double lo, hi;
    big_box(a, c, lo, hi);
    const double x = X[t], g = -BV[c * a.Pp + j];
    xm = fmax(xm, fabs(x));
    if (lo > -INFINITY || hi < INFINITY) w = fmax(w, fabs(x - fmin(fmax(x - g, lo), hi)));
  }
  big_max2(red, w, xm);
  const double eps = fmin(EPS_ACT * (1.0 + xm), w);
  for (int t = threadIdx.x; t < n * a.Pp; t += BIG_NTHREADS) {
    const int c = t / a.Pp, j = t % a.Pp;
    int act = 0;
    if (j < a.P) {
      double lo, hi;
      big_box(a, c, lo, hi);
      const double x = X[j * n + c], g = -BV[t];
      act = (lo > -INFINITY || hi < INFINITY) && ((x <= lo + eps && g > 0.0) || (x >= hi - eps && g < 0.0));
    }
    ACT[t] = act;
  }
}

// ------------------------------------------------------------ residuals
// Node terms for a SPARSE dynamics Jacobian (DynGnssReceivers: n = 40): E = c Qw F,
// F^T V and F^T E accumulated from the (row, col, value) triples straight into the
// workspace -- no n x n private array (it would live in scratch memory).
template <class DYN>
__device__ void big_nodes_sparse(const BigArgs& a, const BigConst& CL, const BigWs& WL, double* ws, const double* X,
                                 int b, double& cost) {
  constexpr int n = DYN::n, m = DYN::m, NNZ = DYN::NNZ;
  const double* Dt = (const double*)(a.cbuf + CL.Dt);
  const double* cw = (const double*)(a.cbuf + CL.cw);
  const double* Qw = (const double*)(a.cbuf + CL.Qw);
  for (int k = threadIdx.x; k < a.P; k += BIG_NTHREADS) {
    double W[n], f[n], Fv[NNZ], uk[m > 0 ? m : 1];
    for (int c = 0; c < n; ++c) W[c] = 0.0;
    constexpr int UJ = n <= 8 ? 8 : 2;  // loads in flight; n = 40 (C5) would spill at 8
#pragma unroll UJ
    for (int j = 0; j < a.P; ++j) {
      const double dv = Dt[(size_t)j * a.P + k];
      for (int c = 0; c < n; ++c) W[c] += dv * X[j * n + c];
    }
    if (m > 0) {
      const double* Up = a.U + (long long)b * a.ustride + (long long)k * m;
      for (int c = 0; c < m; ++c) uk[c] = Up[c];
    }
    DYN::eval_sparse(X + k * n, uk, a.dpar, f, Fv);
    for (int c = 0; c < n; ++c) W[c] = a.alpha * W[c] - f[c];
    const double ck = cw[k];
    double* Ek = ws + WL.Es + k;  // component-major: E_k[r][c] at (r n + c) P + k
    double* Vk = ws + WL.Vs + (size_t)k * n;
    double* FtV = ws + WL.FtV + (size_t)k * n;
    double* FtE = ws + WL.FtE + (size_t)k * n * n;
    const size_t P_ = a.P;
    for (int c = 0; c < n * n; ++c) {
      Ek[c * P_] = 0.0;
      FtE[c] = 0.0;
    }
    for (int r = 0; r < n; ++r) {
      double v;
      if (a.huber) {
        const double q = Qw[r * n + r], dl = a.huber_delta;
        const double sr = sqrt(1.0 + W[r] * W[r] / (dl * dl));
        const double lam = ck * (q / sr);
        v = lam * W[r];
        cost += ck * (2.0 * q * dl * dl * (sr - 1.0));
        ws[WL.LAM + k * n + r] = lam;
        for (int z = 0; z < NNZ; ++z)
          if (DYN::frow(z) == r) Ek[(r * n + DYN::fcol(z)) * P_] = lam * Fv[z];
      } else {
        double s = 0.0;
        for (int c = 0; c < n; ++c) s += Qw[r * n + c] * W[c];
        v = ck * s;
        cost += W[r] * v;
        for (int z = 0; z < NNZ; ++z) Ek[(r * n + DYN::fcol(z)) * P_] += ck * Qw[r * n + DYN::frow(z)] * Fv[z];
      }
      Vk[r] = v;
      FtV[r] = 0.0;
    }
    for (int z = 0; z < NNZ; ++z) {
      const int t = DYN::frow(z), r = DYN::fcol(z);
      FtV[r] += Fv[z] * Vk[t];
      for (int c = 0; c < n; ++c) FtE[r * n + c] += Fv[z] * Ek[(t * n + c) * P_];
    }
  }
}

template <class DYN, class MEAS>
__global__ __launch_bounds__(BIG_NTHREADS) void k_big_resid(BigArgs a, int final_pass) {
  constexpr int n = DYN::n, m = DYN::m, p = MEAS::p, q = MEAS::q;
  const int b = blockIdx.x;
  if (!final_pass && a.state[b] != BIG_RUNNING) return;
  if (a.state[b] == MHE_STATUS_BAD_CONSTANTS) return;
  const BigConst CL = big_const_layout(a.P, a.M, n, p, a.nc);
  const BigWs WL = big_ws_layout(a.P, a.M, n, a.NT, a.nz, a.nc);
  double* ws = a.ws + (size_t)b * a.ws_stride;
  // MHE_BIG_ENV: which component pairs (a, b) have a nonzero block of H at this iterate --
  // from the E, F^T E and G_e values formed below (one coalesced pass over each, flags in
  // LDS), Qw and Pw; k_big_assemble skips the others' epoch GEMM and writes their tiles as
  // zeros, the split factorization derives its envelope from them
  __shared__ int pflag[MHE_BIG_ENV ? n * n : 1];
  if (MHE_BIG_ENV)
    for (int t = threadIdx.x; t < n * n; t += BIG_NTHREADS) pflag[t] = 0;
  const double* D = (const double*)(a.cbuf + CL.D);
  const double* Dt = (const double*)(a.cbuf + CL.Dt);
  const double* cw = (const double*)(a.cbuf + CL.cw);
  const double* Qw = (const double*)(a.cbuf + CL.Qw);
  const double* Pw = (const double*)(a.cbuf + CL.Pw);
  const double* Rw = big_rw(a, (const double*)(a.cbuf + CL.Rw), b);
  const double* PhiE = (const double*)(a.cbuf + CL.PhiE);
  const double* PhiET = (const double*)(a.cbuf + CL.PhiET);
  const int* erow = (const int*)(a.cbuf + CL.erow);
  const int E = a.M > 0 ? *(const int*)(a.cbuf + CL.ne) : 0;
  const int Mr = a.M > 0 ? a.M : 1;
  // X staged in LDS (MHE_BIG_RESID_LDS; dynamic LDS of P n doubles): every thread's node
  // and epoch dot products read all of X, as LDS broadcasts instead of L1/L2 loads
  extern __shared__ __attribute__((aligned(16))) double xl_dyn[];
  const double* Xg = a.X + (size_t)b * a.P * n;
  if (MHE_BIG_RESID_LDS) {
    for (int t = threadIdx.x; t < a.P * n; t += BIG_NTHREADS) xl_dyn[t] = Xg[t];
    __syncthreads();
  }
  const double* X = MHE_BIG_RESID_LDS ? xl_dyn : Xg;
  __shared__ double red[2 * BIG_NW];
  double cost = 0.0, noise = 0.0;  // noise: the cost's rounding level (bounded problems' line search)
  // interpolated states at the epochs: x_e = sum_j Phi_E[e][j] X_j
  for (int e = threadIdx.x; e < E; e += BIG_NTHREADS) {
    double xe[n];
    for (int c = 0; c < n; ++c) xe[c] = 0.0;
    #pragma unroll 8
    for (int j = 0; j < a.P; ++j) {
      const double ph = PhiET[(size_t)j * Mr + e];
      for (int c = 0; c < n; ++c) xe[c] += ph * X[j * n + c];
    }
    for (int c = 0; c < n; ++c) ws[WL.XE + e * n + c] = xe[c];
  }
  // nodes (nlp/nlp.py:225-245)
  if constexpr (dyn_sparse<DYN>::value) {
    big_nodes_sparse<DYN>(a, CL, WL, ws, X, b, cost);
  } else
  for (int k = threadIdx.x; k < a.P; k += BIG_NTHREADS) {
    double dx[n], xk[n], uk[m > 0 ? m : 1], f[n], F[n * n];
    for (int c = 0; c < n; ++c) dx[c] = 0.0;
    #pragma unroll 8
    for (int j = 0; j < a.P; ++j) {
      const double dv = Dt[(size_t)j * a.P + k];
      for (int c = 0; c < n; ++c) dx[c] += dv * X[j * n + c];
    }
    for (int c = 0; c < n; ++c) xk[c] = X[k * n + c];
    if (m > 0) {
      const double* Up = a.U + (long long)b * a.ustride + (long long)k * m;
      for (int c = 0; c < m; ++c) uk[c] = Up[c];
    }
    DYN::eval(xk, uk, a.dpar, f, F);
    double W[n], V[n];
    for (int c = 0; c < n; ++c) W[c] = a.alpha * dx[c] - f[c];
    const double ck = cw[k];
    double* Ek = ws + WL.Es + k;  // component-major: E_k[r][c] at (r n + c) P + k
    const size_t P_ = a.P;
    if (a.huber) {
      // pseudo_huber_loss (cost_functions.py:25-31) by IRLS, as k_gn: lambda = c q / sqrt(1 +
      // W^2 / delta^2) per component (only diag(Qw) enters), V = lambda W, E = diag(lambda) F
      const double dl = a.huber_delta;
      for (int r = 0; r < n; ++r) {
        const double q = Qw[r * n + r];
        const double sr = sqrt(1.0 + W[r] * W[r] / (dl * dl));
        const double lam = ck * (q / sr);
        V[r] = lam * W[r];
        cost += ck * (2.0 * q * dl * dl * (sr - 1.0));
        ws[WL.LAM + k * n + r] = lam;
        for (int c = 0; c < n; ++c) Ek[(r * n + c) * P_] = lam * F[r * n + c];
      }
    } else {
      for (int r = 0; r < n; ++r) {
        double s = 0.0;
        for (int c = 0; c < n; ++c) s += Qw[r * n + c] * W[c];
        V[r] = ck * s;
        cost += W[r] * V[r];
        for (int c = 0; c < n; ++c) {
          double e = 0.0;
          for (int t = 0; t < n; ++t) e += Qw[r * n + t] * F[t * n + c];
          Ek[(r * n + c) * P_] = ck * e;
        }
      }
    }
    for (int r = 0; r < n; ++r) {
      ws[WL.Vs + k * n + r] = V[r];
      double s = 0.0;
      for (int t = 0; t < n; ++t) s += F[t * n + r] * V[t];
      ws[WL.FtV + k * n + r] = s;
    }
    // F^T E (E read back from this thread's own writes)
    for (int r = 0; r < n; ++r)
      for (int c = 0; c < n; ++c) {
        double u = 0.0;
        for (int t = 0; t < n; ++t) u += F[t * n + r] * Ek[(t * n + c) * P_];
        ws[WL.FtE + (k * n + r) * n + c] = u;
      }
  }
  __syncthreads();
  // measurement rows grouped by epoch (nlp/nlp.py:264-273)
  if constexpr (MEAS::MIXED) {
    // scalar rows of several plug-ins over [x(t_e) ; z]; the z couplings are
    // accumulated per epoch for k_big_border.  A row's gradient has at most 8 nonzeros
    // (MHE_ROW_* codes), so its outer product is scattered straight into the epoch's
    // blocks in the workspace (no n x n private array: n = 40 for the 8-receiver C5)
    constexpr int NA = MEAS::NA, NZX = MHE_MAX_EXTRA;
    const int nz = a.nz;
    for (int e = threadIdx.x; e < E; e += BIG_NTHREADS) {
      double* G = ws + WL.Ge + (size_t)e * n * n;
      double* ge = ws + WL.GEe + (size_t)e * n;
      double* Gz = ws + WL.GZe + (size_t)e * n * NZX;
      double* Hzz = ws + WL.HZZe + (size_t)e * NZX * NZX;
      double* gz = ws + WL.GZVe + (size_t)e * NZX;
      double xt[MHE_BIG_RESID_SLOTS ? 1 : NA];
      for (int c = 0; c < n; ++c) {
        if (!MHE_BIG_RESID_SLOTS) xt[c] = ws[WL.XE + e * n + c];
        ge[c] = 0.0;
      }
      if (!MHE_BIG_RESID_SLOTS)
        for (int c = 0; c < NZX; ++c) xt[n + c] = c < nz ? a.Z[(size_t)b * nz + c] : 0.0;
      for (int c = 0; c < n * n; ++c) G[c] = 0.0;
      if (nz > 0) {
        for (int c = 0; c < n * NZX; ++c) Gz[c] = 0.0;
        for (int c = 0; c < NZX * NZX; ++c) Hzz[c] = 0.0;
        for (int c = 0; c < NZX; ++c) gz[c] = 0.0;
      }
      for (int i = erow[e]; i < erow[e + 1]; ++i) {
        const double* PR = a.PAR + (long long)b * a.pstride + (long long)i * q;
        const double R = Rw[i];
        if (R == 0.0) continue;  // R = 0 masks the row (empty satellite slot, autonomous-car.py:260-263)
        if constexpr (MHE_BIG_RESID_SLOTS) {
          // per-slot gradient: a component in two slots gets their sum (two terms: the same
          // value as the dense accumulation), zero gradients dropped -- the dense form's
          // nonzero set; each (ia, ib) entry is still added once per row, so G_e, g_e and
          // the z blocks take the same values
          double h, gs[7];
          int id[7];
          MEAS::eval_slots([&](int c) { return c < n ? ws[WL.XE + e * n + c] : a.Z[(size_t)b * nz + (c - n)]; }, PR, nz, h,
                           id, gs);
#pragma unroll
          for (int k1 = 0; k1 < 7; ++k1)
#pragma unroll
            for (int k2 = k1 + 1; k2 < 7; ++k2)
              if (id[k1] >= 0 && id[k2] == id[k1]) {
                gs[k1] += gs[k2];
                id[k2] = -1;
              }
#pragma unroll
          for (int k1 = 0; k1 < 7; ++k1)
            if (gs[k1] == 0.0) id[k1] = -1;
          const double yv = a.Y[(long long)b * a.M + i], ev = yv - h, Re = R * ev;
          cost += ev * Re;
          noise += fabs(Re) * (fabs(yv) + fabs(h));
#pragma unroll
          for (int u = 0; u < 7; ++u) {
            if (id[u] < 0) continue;
            const int ia = id[u];
            const double ga = gs[u];
            if (ia < n) ge[ia] += ga * Re;
            else gz[ia - n] += ga * Re;
#pragma unroll
            for (int v = 0; v < 7; ++v) {
              if (id[v] < 0) continue;
              const int ib = id[v];
              const double w2 = ga * R * gs[v];
              if (ia < n && ib < n) G[ia * n + ib] += w2;
              else if (ia < n) Gz[ia * NZX + (ib - n)] += w2;
              else if (ib >= n) Hzz[(ia - n) * NZX + (ib - n)] += w2;
            }
          }
          continue;
        }
        double h, Gr[NA];
        MEAS::eval(xt, PR, nz, h, Gr);
        const double yv = a.Y[(long long)b * a.M + i], ev = yv - h, Re = R * ev;
        cost += ev * Re;
        noise += fabs(Re) * (fabs(yv) + fabs(h));
        int id[8], k = 0;
        for (int c = 0; c < NA && k < 8; ++c)
          if (Gr[c] != 0.0) id[k++] = c;
        for (int u = 0; u < k; ++u) {
          const int ia = id[u];
          const double ga = Gr[ia];
          if (ia < n) ge[ia] += ga * Re;
          else gz[ia - n] += ga * Re;
          for (int v = 0; v < k; ++v) {
            const int ib = id[v];
            const double w2 = ga * R * Gr[ib];
            if (ia < n && ib < n) G[ia * n + ib] += w2;
            else if (ia < n) Gz[ia * NZX + (ib - n)] += w2;
            else if (ib >= n) Hzz[(ia - n) * NZX + (ib - n)] += w2;
          }
        }
      }
    }
  } else
  for (int e = threadIdx.x; e < E; e += BIG_NTHREADS) {
    double xe[n], ge[n], G[n * n];
    for (int c = 0; c < n; ++c) {
      xe[c] = ws[WL.XE + e * n + c];
      ge[c] = 0.0;
    }
    for (int c = 0; c < n * n; ++c) G[c] = 0.0;
    for (int i = erow[e]; i < erow[e + 1]; ++i) {
      double par[q > 0 ? q : 1];
      if (q > 0) {
        const double* PR = a.PAR + (long long)b * a.pstride + (long long)i * q;
        for (int c = 0; c < q; ++c) par[c] = PR[c];
      }
      const double* R = Rw + (size_t)i * p * p;
      if (masked_row<p>(R)) continue;  // R = 0 masks the row (autonomous-car.py:260-263)
      double h[p], Hm[p * n];
      MEAS::eval(xe, par, a.idx, h, Hm);
      const double* yi = a.Y + ((long long)b * a.M + i) * p;
      double ev[p], Re[p];
      for (int r = 0; r < p; ++r) ev[r] = yi[r] - h[r];
      for (int r = 0; r < p; ++r) {
        double s = 0.0;
        for (int c = 0; c < p; ++c) s += R[r * p + c] * ev[c];
        Re[r] = s;
        cost += ev[r] * s;
        noise += fabs(s) * (fabs(yi[r]) + fabs(h[r]));
      }
      for (int c = 0; c < n; ++c) {
        double s = 0.0;
        for (int r = 0; r < p; ++r) s += Hm[r * n + c] * Re[r];
        ge[c] += s;
      }
      for (int r = 0; r < n; ++r)
        for (int c = 0; c < n; ++c) {
          double s = 0.0;
          for (int t = 0; t < p; ++t) {
            double rh = 0.0;
            for (int t2 = 0; t2 < p; ++t2) rh += R[t * p + t2] * Hm[t2 * n + c];
            s += Hm[t * n + r] * rh;
          }
          G[r * n + c] += s;
        }
    }
    for (int c = 0; c < n; ++c) ws[WL.GEe + e * n + c] = ge[c];
    for (int c = 0; c < n * n; ++c) ws[WL.Ge + e * n * n + c] = G[c];
  }
  __syncthreads();
  // gradient, component-major: BV[a*Pp + j] = -g_(j,a)
  for (int t = threadIdx.x; t < n * a.Pp; t += BIG_NTHREADS) {
    const int c = t / a.Pp, j = t % a.Pp;
    double gv = 0.0;
    if (j < a.P) {
      double s = 0.0;
      #pragma unroll 8
      for (int k = 0; k < a.P; ++k) s += D[(size_t)k * a.P + j] * ws[WL.Vs + k * n + c];
      double o = 0.0;
      #pragma unroll 8
      for (int e = 0; e < E; ++e) o += PhiE[(size_t)e * a.P + j] * ws[WL.GEe + e * n + c];
      gv = a.alpha * s - ws[WL.FtV + j * n + c] - o;
      if (a.has_prior && j == 0) {
        double t2 = 0.0;
        for (int cc = 0; cc < n; ++cc) t2 += Pw[c * n + cc] * (X[cc] - a.x0[(long long)b * n + cc]);
        gv += t2;
      }
    }
    ws[WL.BV + t] = -gv;
  }
  if (a.has_prior && threadIdx.x == 0) {
    for (int r = 0; r < n; ++r) {
      double t2 = 0.0;
      for (int c = 0; c < n; ++c) t2 += Pw[r * n + c] * (X[c] - a.x0[(long long)b * n + c]);
      cost += (X[r] - a.x0[(long long)b * n + r]) * t2;
    }
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  cost = wave_sum(cost);
  noise = wave_sum(noise);
  if (lane == 0) {
    red[wave] = cost;
    red[BIG_NW + wave] = noise;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double c = 0.0, z = 0.0;
    for (int w = 0; w < BIG_NW; ++w) {
      c += red[w];
      z += red[BIG_NW + w];
    }
    a.cost[b] = c;
    if (a.n_bounds > 0) ws[WL.NZ] = COST_NOISE * __DBL_EPSILON__ * z;
  }
  if (MHE_BIG_ENV && !final_pass) {
    // (the barrier above ordered every thread's E, F^T E and G_e writes before these reads)
    const size_t nes = (size_t)n * n * a.P, nge = (size_t)E * n * n;
    for (size_t t = threadIdx.x; t < nes; t += BIG_NTHREADS) {
      if (ws[WL.Es + t] != 0.0) pflag[t / a.P] = 1;                     // [(r n + c) P + k]
      if (ws[WL.FtE + t] != 0.0) pflag[t % (n * n)] = 1;                // [(k n + r) n + c]
    }
    for (size_t t = threadIdx.x; t < nge; t += BIG_NTHREADS)
      if (ws[WL.Ge + t] != 0.0) pflag[t % (n * n)] = 1;                 // [(e n + r) n + c]
    __syncthreads();
    int* EM = big_env_mask(ws, WL);
    for (int t = threadIdx.x; t < n * n; t += BIG_NTHREADS) {
      const int ca = t / n, cb = t % n, tt = cb * n + ca;
      const bool nzq = ca == cb || pflag[t] || pflag[tt] || (!a.huber && (Qw[t] != 0.0 || Qw[tt] != 0.0)) ||
                       (a.has_prior && (Pw[t] != 0.0 || Pw[tt] != 0.0));
      EM[t] = nzq ? 1 : 0;
    }
  }
  if (a.n_bounds > 0 && !final_pass) {
    big_active_set<n>(a, X, ws + WL.BV, (int*)(ws + WL.ACT), red);
    for (int t = threadIdx.x; t < n * a.Pp; t += BIG_NTHREADS) ws[WL.GV + t] = ws[WL.BV + t];  // for the line search
  }
}

// ------------------------------------------------------------ assembly
// Block (a, b) of H (component-major) is the P x P matrix
//   a^2 Qw_ab (D^T C D) - a (D^T diag(E_ab) + diag(E_ba) D) + diag(FtE_ab)
//   + M_ab,   M_ab = Phi_E^T diag(G_ab) Phi_E   (G_e = sum_{i in e} H_i^T R_i H_i)
// M_ab is a GEMM over the E epochs, symmetric (M_ab = M_ab^T = M_ba), and all
// component pairs share the same operands Phi_E: one wave takes one tile position
// (it >= jt) and a chunk of up to BIG_PCH pairs (ca >= cb) -- one MFMA accumulator per
// pair -- so each K step of 4 epochs loads 2 Phi_E values (L2-resident, shared by
// every trajectory) and feeds up to 5 MFMAs (G_e[ca][cb] read per lane; 5
// accumulators: 96 VGPRs, no spills).  Pairs outside the measurement Jacobian's
// support (BigGSupport) skip the GEMM: their chunks only write.  The
// dynamics terms are added elementwise at the write; an off-diagonal pair also
// writes the transposed tile (jt, it) from the same accumulator.
// State components a measurement row's Jacobian can touch (bit c: component c);
// G_e[a][b] = sum H_i^T R_i H_i can be nonzero only when both bits are set.
// Conservative (all components) unless the model says otherwise.
template <class MEAS>
struct BigGSupport {
  static unsigned long long get(const int*, int n) { return n >= 64 ? ~0ull : (1ull << n) - 1ull; }
};
template <int N>
struct BigGSupport<MeasPseudorange<N>> {  // h = |x[idx0..2] - sat| + x[idx3]
  static unsigned long long get(const int* idx, int) {
    return 1ull << idx[0] | 1ull << idx[1] | 1ull << idx[2] | 1ull << idx[3];
  }
};
template <>
struct BigGSupport<MeasVehiclePseudorange> {  // h = |x[0, 1, 8] - sat| + x[6]
  static unsigned long long get(const int*, int) { return 1ull << 0 | 1ull << 1 | 1ull << 8 | 1ull << 6; }
};

constexpr int BIG_PCH = 5;  // pair accumulators per wave (96 VGPRs, no spills)

// Pair table and chunking of k_big_assemble: the live pairs are split into
// nchl chunks of <= pchl (balanced, <= BIG_PCH) that run the epoch GEMM; the
// pairs whose contraction is zero (e.g. the clock-drift component under
// pseudoranges) get chunks of BIG_PCH that only write the dynamics terms.
inline void big_pair_plan(BigArgs& A, unsigned long long support) {  // bit c: component c (n <= 44)
  const int n = A.n;
  int k = 0;
  for (int pass = 0; pass < 2; ++pass)
    for (int ca = 0; ca < n; ++ca)
      for (int cb = 0; cb <= ca; ++cb) {
        const bool live = (support >> ca & 1ull) && (support >> cb & 1ull);
        if (live == (pass == 0)) {
          A.pa[k] = (unsigned char)ca;
          A.pb[k] = (unsigned char)cb;
          ++k;
        }
      }
  A.npr = k;
  int nl = 0;
  for (int ca = 0; ca < n; ++ca)
    for (int cb = 0; cb <= ca; ++cb) nl += (support >> ca & 1ull) && (support >> cb & 1ull);
  A.nlive = nl;
  A.nchl = (nl + BIG_PCH - 1) / BIG_PCH;
  A.pchl = A.nchl ? (nl + A.nchl - 1) / A.nchl : 0;
  A.nch = A.nchl + (A.npr - nl + BIG_PCH - 1) / BIG_PCH;
}

// Epoch-GEMM staging of k_big_assemble: BIG_AKC epochs per chunk, double-buffered in LDS --
// the two 16-row Phi_E column blocks of the tile position and G_e[pair] of every pair the
// workgroup's waves contract (WPB waves x BIG_PCH pairs)
constexpr int BIG_AKC = 32;
__host__ __device__ constexpr int big_asm_lds(int wpb) { return 2 * (2 * BIG_AKC * 16 + wpb * BIG_PCH * BIG_AKC); }  // doubles

// Work items are (tile position (it, jt), pair chunk), one wave each. The chunks with
// measurement-coupled ("live") pairs come first: a workgroup of WPB waves takes one
// position and WPB live chunks, so the waves share the position's Phi_E rows -- per chunk
// of BIG_AKC epochs the workgroup stages Phi_E[e][16 it + r], Phi_E[e][16 jt + r] and its
// pairs' G_e into LDS with global loads issued one chunk ahead (their latency hides under
// the current chunk's MFMAs), and each wave's K steps read their operands from LDS (round
// 3: every wave streamed its own operands from L2/HBM, two K steps ahead -- MFMA busy
// ~25 %). The remaining blocks take the chunks without an epoch GEMM, WPB consecutive
// (position, chunk) items per workgroup, no barriers.
template <class DYN, class MEAS>
__global__ __launch_bounds__(256, 4) void k_big_assemble(BigArgs a) {
  constexpr int n = DYN::n, p = MEAS::p;
  const int b = blockIdx.y;
  if (a.state[b] != BIG_RUNNING) return;
  const BigConst CL = big_const_layout(a.P, a.M, n, p, a.nc);
  const BigWs WL = big_ws_layout(a.P, a.M, n, a.NT, a.nz, a.nc);
  const double* ws = a.ws + (size_t)b * a.ws_stride;
  double* H = a.ws + (size_t)b * a.ws_stride + WL.H;
  const double* D = (const double*)(a.cbuf + CL.D);
  const double* DCD = (const double*)(a.cbuf + CL.DCD);
  const double* Qw = (const double*)(a.cbuf + CL.Qw);
  const double* Pw = (const double*)(a.cbuf + CL.Pw);
  const double* PhiE = (const double*)(a.cbuf + CL.PhiE);
  const int E = a.M > 0 ? *(const int*)(a.cbuf + CL.ne) : 0;
  // wave-uniform work decomposition (SGPRs: the tile position, pair chunk and table reads are scalar)
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int WPB = blockDim.x >> 6, nthr = blockDim.x;
  const int NTc = a.NTc, P = a.P, NCH = a.nch;
  const int npos = NTc * (NTc + 1) / 2;
  const int nlg = (a.nchl + WPB - 1) / WPB;  // live groups per position
  const bool gblock = (int)blockIdx.x < npos * nlg;
  int grp = 0, pos, ch;
  if (gblock) {
    grp = blockIdx.x % nlg;
    pos = blockIdx.x / nlg;
    ch = grp * WPB + wave;
  } else {
    const int nd = NCH - a.nchl, item = ((int)blockIdx.x - npos * nlg) * WPB + wave;
    pos = item / nd;
    ch = a.nchl + item % nd;
    if (pos >= npos) return;  // tail of the last block (no barriers on this side)
  }
  int it = 0;  // pos -> (it, jt), jt <= it
  while (pos > it) {
    pos -= it + 1;
    ++it;
  }
  const int jt = pos;
  const bool valid = ch < NCH && (!gblock || ch < a.nchl);
  // this wave's pairs: table entries [q0, q0 + np) (BigPairPlan)
  const bool live = valid && ch < a.nchl;
  const int q0 = !valid ? 0 : live ? ch * a.pchl : a.nlive + (ch - a.nchl) * BIG_PCH;
  const int np = !valid ? 0 : min(live ? a.pchl : BIG_PCH, (live ? a.nlive : a.npr) - q0);
  // MHE_BIG_ENV: bit q set when pair q's block of H can be nonzero at this iterate (k_big_resid's
  // flags); the others skip the epoch GEMM (their G_e are zero) and write zero tiles
  int lqm = 0;
#pragma unroll
  for (int q = 0; q < BIG_PCH; ++q)
    if (q < np && (!MHE_BIG_ENV || big_env_mask(ws, WL)[a.pa[q0 + q] * n + a.pb[q0 + q]] != 0)) lqm |= 1 << q;
  d4 acc[BIG_PCH];
#pragma unroll
  for (int q = 0; q < BIG_PCH; ++q) acc[q] = d4{0.0, 0.0, 0.0, 0.0};
  const double* Ge = ws + WL.Ge;
  // workgroup-uniform; MHE_BIG_ENV: a workgroup none of whose pairs has a nonzero term
  // skips the whole epoch loop (its staging and barriers, not only the MFMAs)
  if (gblock && E > 0 && (!MHE_BIG_ENV || __syncthreads_or(lqm != 0))) {
    extern __shared__ __attribute__((aligned(16))) double sm[];
    constexpr int KC = BIG_AKC, SA = KC * 16, SGW = BIG_PCH * KC;
    const int SBUF = 2 * SA + WPB * SGW;
    // staging sources: raw buffer loads with the hardware bounds check -- a slot past the
    // last epoch, on a padding row / column, or of an absent pair reads 0
    const __amdgpu_buffer_rsrc_t rp = __builtin_amdgcn_make_buffer_rsrc((void*)PhiE, (short)0, E * P * 8, 0x00020000);
    const __amdgpu_buffer_rsrc_t rg = __builtin_amdgcn_make_buffer_rsrc((void*)Ge, (short)0, E * n * n * 8, 0x00020000);
    constexpr int OOB = 0x40000000;
    // Phi_E rows: shared by the workgroup, element idx = t + nthr k of [2][KC][16];
    // G_e: private to the wave, element g = lane + 64 k of [BIG_PCH][KC]
    constexpr int NAB = 2 * SA / 64, NG = (SGW + 63) / 64;
    int gsrc[NG];  // pair offset within one epoch's G_e, or OOB
#pragma unroll
    for (int k = 0; k < NG; ++k) {
      const int g = lane + 64 * k, q = g / KC;
      gsrc[k] = (g < SGW && q < np && live && ((lqm >> q) & 1)) ? (a.pa[q0 + q] * n + a.pb[q0 + q]) * 8 : OOB;
    }
    const int nchk = (E + KC - 1) / KC;
    double sab[NAB], sg[NG];
    auto fetch = [&](int c) {
#pragma unroll
      for (int k = 0; k < NAB; ++k) {
        const int idx = threadIdx.x + nthr * k;
        if (idx < 2 * SA) {
          const int rem = idx & (SA - 1), rowc = 16 * (idx >= SA ? jt : it) + (rem & 15);
          sab[k] = bload(rp, rowc < P ? ((c * KC + (rem >> 4)) * P + rowc) * 8 : OOB, 0);
        }
      }
#pragma unroll
      for (int k = 0; k < NG; ++k) {
        const int e = c * KC + (lane + 64 * k) % KC;
        sg[k] = bload(rg, gsrc[k] >= OOB ? OOB : e * n * n * 8 + gsrc[k], 0);
      }
    };
    auto deposit = [&](int buf) {
      double* s0 = sm + buf * SBUF;
#pragma unroll
      for (int k = 0; k < NAB; ++k) {
        const int idx = threadIdx.x + nthr * k;
        if (idx < 2 * SA) s0[idx] = sab[k];
      }
#pragma unroll
      for (int k = 0; k < NG; ++k) {
        const int g = lane + 64 * k;
        if (g < SGW) s0[2 * SA + wave * SGW + g] = sg[k];
      }
    };
    fetch(0);
    deposit(0);
    __syncthreads();
    const int eg = lane >> 4, r16 = lane & 15;
#pragma unroll 1
    for (int c = 0; c < nchk; ++c) {
      const int buf = c & 1;
      if (c + 1 < nchk) fetch(c + 1);  // in flight during this chunk's MFMAs
      if (live) {
        const double* sA = sm + buf * SBUF;
        const double* sB = sA + SA;
        const double* sG = sA + 2 * SA + wave * SGW;
        // two K steps per trip (the MFMAs are convergent: no remainder loop); a step past
        // the last epoch reads the zeros staged for it
        const int ks = min(KC, E - c * KC);
#pragma unroll 1
        for (int e0 = 0; e0 < ks; e0 += 8) {
#pragma unroll
          for (int h = 0; h < 8; h += 4) {
            const int e = e0 + h + eg;
            const double a0 = sA[e * 16 + r16], b0 = sB[e * 16 + r16];
#pragma unroll
            for (int q = 0; q < BIG_PCH; ++q)
              if ((lqm >> q) & 1) acc[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0 * sG[q * KC + e], b0, acc[q], 0, 0, 0);
          }
        }
      }
      if (c + 1 < nchk) deposit(buf ^ 1);
      __syncthreads();
    }
  }
  if (!valid) return;
  const int row = 16 * it + (lane & 15), col = 16 * jt + (lane & 15);
  const bool vr = row < P, vc = col < P;
  if (a.huber) {
    // pseudo-Huber IRLS: the dynamics part a^2 (D^T C D) (x) Qw is no longer constant --
    // block (ca, ca) gets a^2 D^T diag(c lambda_ca) D (k_big_resid's weights), a GEMM
    // over the P nodes with the same operand layout as the epoch contraction
    const double* LAM = ws + WL.LAM;
    const double a2 = a.alpha * a.alpha;
    int lo[BIG_PCH];  // lambda offset of a diagonal pair, -1 otherwise
#pragma unroll
    for (int q = 0; q < BIG_PCH; ++q) lo[q] = (q < np && a.pa[q0 + q] == a.pb[q0 + q]) ? a.pa[q0 + q] : -1;
#pragma unroll 1
    for (int k0 = 0; k0 < P; k0 += 4) {
      const int k = k0 + (lane >> 4);
      const int kc = k < P ? k : P - 1;
      const double dv = (k < P && vr) ? D[(size_t)kc * P + row] : 0.0;
      const double ev = (k < P && vc) ? D[(size_t)kc * P + col] : 0.0;
#pragma unroll
      for (int q = 0; q < BIG_PCH; ++q)
        if (lo[q] >= 0) acc[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(dv * (a2 * LAM[kc * n + lo[q]]), ev, acc[q], 0, 0, 0);
    }
  }
  // element writes: raw buffer loads / stores with 32-bit offsets (one resource each over
  // the constants, this trajectory's workspace and its H tiles), wave-uniform parts of
  // every offset in SGPRs -- no 64-bit address arithmetic per element
  const __amdgpu_buffer_rsrc_t rc = cbuf_rsrc(a.cbuf, CL.total);
  const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc((void*)ws, (short)0, (int)(WL.total * 8), 0x00020000);
  const __amdgpu_buffer_rsrc_t rh =
      __builtin_amdgcn_make_buffer_rsrc((void*)H, (short)0, (int)((size_t)a.NT * (a.NT + 1) / 2 * 256 * 8), 0x00020000);
#pragma unroll
  for (int q = 0; q < BIG_PCH; ++q) {
    if (q < np) {
      const int ca = a.pa[q0 + q], cb = a.pb[q0 + q];
      const double qab = a.huber ? 0.0 : a.alpha * a.alpha * Qw[ca * n + cb];
      const double pw = a.has_prior ? Pw[ca * n + cb] : 0.0;
      // E_l[ca][cb] and E_j[cb][ca] (component-major: node index fastest)
      const int sE1 = (int)((WL.Es + (size_t)(ca * n + cb) * P) * 8), sE2 = (int)((WL.Es + (size_t)(cb * n + ca) * P) * 8);
      const int sF = (int)(WL.FtE * 8) + (ca * n + cb) * 8;
      if (MHE_BIG_ASM_ZSKIP && !((lqm >> q) & 1)) {
        // a pair without a nonzero term: zero tiles, not stored where the previous
        // factorization's envelope already left zeros (a tile left of its row's f: A was 0
        // there, and the factorization wrote nothing but zeros left of f)
        const int* FIp = big_env_first(ws, WL, n);
#pragma unroll
        for (int tp = 0; tp < 2; ++tp) {
          if (tp == 1 && (ca == cb || it == jt)) break;
          const int I = ca * NTc + (tp ? jt : it), J = cb * NTc + (tp ? it : jt);
          if (a.asm_zskip && J < FIp[I]) continue;
          const int sT = big_tile_index(I, J, a.NT) * 256 * 8;
#pragma unroll
          for (int r = 0; r < 4; ++r)
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(mhe_u2, 0.0), rh, (64 * r + lane) * 8, sT, 0);
        }
        continue;
      }
      // tile (it, jt) of block (ca, cb) and, off the diagonal pair, its transpose into (jt, it)
#pragma unroll
      for (int tp = 0; tp < 2; ++tp) {
        if (tp == 1 && (ca == cb || it == jt)) break;
        const int ti = tp ? jt : it, tj = tp ? it : jt;
        const int I = ca * NTc + ti, J = cb * NTc + tj;
        const int sT = big_tile_index(I, J, a.NT) * 256 * 8;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int cr = (lane >> 4) + 4 * r, cc = lane & 15;  // accumulator element (cr, cc) of tile (it, jt)
          const int tr = tp ? cc : cr, tc = tp ? cr : cc;       // position in the written tile
          const int j = 16 * ti + tr, l = 16 * tj + tc;
          double v;
          if (!((lqm >> q) & 1)) {
            v = 0.0;  // a pair without a nonzero term (never a diagonal pair: no identity padding)
          } else if (j < P && l < P) {
            // every operand read along the lane-varying index (l for the tile, j for its
            // transpose): D_lj from D^T or D, D_jl from D or D^T, the exactly symmetric
            // D^T C D either way, E component-major -- coalesced, not P- or n^2-strided
            const int jl = (j * P + l) * 8, lj = (l * P + j) * 8;
            const double dcd = bload(rc, tp ? lj : jl, (int)CL.DCD);
            const double d_lj = tp ? bload(rc, lj, (int)CL.D) : bload(rc, jl, (int)CL.Dt);
            const double d_jl = tp ? bload(rc, lj, (int)CL.Dt) : bload(rc, jl, (int)CL.D);
            v = acc[q][r] + qab * dcd - a.alpha * (d_lj * bload(rw, l * 8, sE1) + d_jl * bload(rw, j * 8, sE2));
            if (j == l) v += bload(rw, j * n * n * 8, sF);
            if (j == 0 && l == 0) v += pw;
          } else {
            v = (I == J && tr == tc) ? 1.0 : 0.0;
          }
          if (a.n_bounds > 0) {  // active rows / columns reduced to the diagonal (projected Newton)
            const int* ACT = (const int*)(ws + WL.ACT);
            const int gr = 16 * I + tr, gc = 16 * J + tc;
            if ((ACT[gr] | ACT[gc]) && gr != gc) v = 0.0;
          }
          __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(mhe_u2, v), rh, (tr * 16 + tc) * 8, sT, 0);
        }
      }
    }
  }
}

// ------------------------------------------------------------ factor + solve
// Blocked right-looking Cholesky over super-blocks of BIG_KB tile columns
// (nb = 16 BIG_KB).  Per super-block:
//   diagonal block  the BIG_KB x BIG_KB tiles of the block's own rows, 16 columns at
//                 a time: single-wave diagonal panel (L_kk^-T, y_k), in-block updates
//                 left-looking from LDS, MFMA TRSM -- two workgroup barriers per k;
//   rows below    every row I >= block end independently (one wave per row, no
//                 barriers): its BIG_KB tiles A_Ik are read once, the in-block
//                 updates and the TRSMs run from registers (the row's L_Ik' stay in
//                 VGPRs, L_kk' and L_kk^-1 come from LDS), L_Ik written once, and
//                 b_I -= L_Ik y_k;
//   trailing      A_IJ -= sum_{k in block} L_Ik L_Jk^T for all J >= block end:
//                 K = nb per tile visit, so every trailing tile is read and
//                 written once per nb columns instead of once per 16 (the 16-wide
//                 right-looking form moved ~4x the HBM bytes for the same flops).
//                 L_J of JB tile columns is staged in LDS (B operands, shared by
//                 all waves); each wave walks tile rows I, holds L_I (A operands)
//                 in registers and updates the row's (up to) JB tiles.
constexpr int BIG_KB = 8;      // tile columns per super-block
// Tile columns per LDS-staged trailing slab: every row visit reads its BIG_KB L_Ik
// tiles once for JB output tiles, so the L traffic of the trailing update goes as
// 1 / JB.  JB = 8 (128 KB slab, one workgroup per CU) for wide systems (NT >=
// BIG_WIDE_NT, C4: HBM-bound there), JB = 4 (64 KB, two workgroups per CU, whose
// overlap the latency-bound panel phase of narrower systems needs) otherwise.
#ifndef MHE_BIG_WIDE_NT
#define MHE_BIG_WIDE_NT 128
#endif
constexpr int BIG_WIDE_NT = MHE_BIG_WIDE_NT;
#ifndef MHE_BIG_LLR8
#define MHE_BIG_LLR8 2  // rows per wave of the left-looking update, 8-wide slab instance
#endif
#ifndef MHE_BIG_SPLIT
#define MHE_BIG_SPLIT 1  // the left-looking factorization as per-block-column launches (k_big_chol SPLIT,
                         // k_big_rows): 1 = always (round 6: C3 too), 2 = for wide systems only (NT >=
                         // BIG_WIDE_NT: C4, C5; the round-5 default), 0 = never
#endif
#ifndef MHE_BIG_TWO_STREAMS
#define MHE_BIG_TWO_STREAMS 1  // split factorization: the batch's two halves on two streams (envelope build: C5 +6.2 %, C3 +1.5 %, C4 0)
#endif
#ifndef MHE_BIG_DIAG_REG
#define MHE_BIG_DIAG_REG 1  // split diagonal stage: its rows' left-looking update register-resident (as k_big_rows)
#endif
#ifndef MHE_BIG_DIAG_SKIP
#define MHE_BIG_DIAG_SKIP 1  // split diagonal stage: skip the MFMAs of tiles past a row's diagonal, SIMD-balanced rows
#endif
#ifndef MHE_BIG_DIAG_LROW
#define MHE_BIG_DIAG_LROW 1  // split diagonal stage: the rows' own L_Ik from the staged slab (LDS), not HBM
#endif
#ifndef MHE_BIG_BWD_PF
#define MHE_BIG_BWD_PF 2  // split solve launch: tiles of the next column each wave has in flight (5: slower at C3)
#endif
#ifndef MHE_BIG_ROWS_SKIP
#define MHE_BIG_ROWS_SKIP 1  // k_big_rows: row-less waves skip the left-looking MFMAs
#endif
#ifndef MHE_BIG_BWD_COAL
#define MHE_BIG_BWD_COAL 1  // backward solve: coalesced tile loads, one DPP row reduction per step (C3 +3.7 %, C4 +2.1 %)
#endif
#ifndef MHE_BIG_ROWS_TLDS
#define MHE_BIG_ROWS_TLDS 1  // k_big_rows: the row's A_Ik^T read coalesced and transposed through LDS (C3 +1.8 %, C4 +1.1 %)
#endif
#ifndef MHE_BIG_ROWS_LBDMA
#define MHE_BIG_ROWS_LBDMA 1  // k_big_rows: the in-block L tiles and L_kk^-T staged by LDS-DMA (C3 +2.4 %, C4 0)
#endif
#ifndef MHE_BIG_ROWS_KC
#define MHE_BIG_ROWS_KC 2  // k_big_rows: k tiles per staged slab
#endif
#ifndef MHE_BIG_ROWS_DB
#define MHE_BIG_ROWS_DB 1  // k_big_rows: slabs double-buffered (the next in flight during this one's MFMAs)
#endif
#ifndef MHE_BIG_ROWS_RPF
#define MHE_BIG_ROWS_RPF 1  // k_big_rows: the row's L_Ik loaded a whole slab chunk ahead
#endif
#ifndef MHE_BIG_ROWS_XCD
#define MHE_BIG_ROWS_XCD 1  // k_big_rows: a trajectory's row groups on one XCD (batch % 8 == 0)
#endif
#ifndef MHE_BIG_KO
#define MHE_BIG_KO 0  // knock-out mask for timing probes only (tools/ko_big.sh): 1 trailing / left-looking
                      // update, 2 in-block, 4 TRSM, 8 the left-looking update's slab staging,
                      // 16 the rows below the diagonal block, 32 the backward solve; any
                      // nonzero mask also freezes X (k_big_update), 64 only that (the baseline)
#endif
#ifndef MHE_BIG_HEAD
#define MHE_BIG_HEAD 1  // split form: the NT % 8 leftover tile columns as the FIRST block column, so every
                        // rows launch has whole groups of 8 rows (C3: NT = 65; +9.8 %)
#endif
constexpr int BIG_LB_TILES = BIG_KB * (BIG_KB - 1) / 2;
// End of the split form's block column that starts at k0.  Block columns are 8 wide; with
// MHE_BIG_HEAD the NT % 8 leftover columns form the first one instead of the last, so the
// rows below every block column are a multiple of 8 (k_big_rows: one workgroup per 8 rows;
// at C3, NT = 65, a trailing 1-wide block left one row in the last group of EVERY rows
// launch).  Tile results do not depend on the partition: each tile's updates accumulate
// in ascending k in every form.
__host__ __device__ inline int big_split_kend(int k0, int NT) {
  const int h = MHE_BIG_HEAD ? NT % BIG_KB : 0;
  return (k0 == 0 && h != 0) ? h : (k0 + BIG_KB < NT ? k0 + BIG_KB : NT);
}
// the LJ region: the trailing slab, or (panel phase) the in-block L tiles LB and the
// block's L_kk^-T matrices LTs
__host__ __device__ constexpr int big_slab_doubles(int JB) {
  return JB * BIG_KB * 256 > BIG_LB_TILES * 256 + BIG_KB * DTS ? JB * BIG_KB * 256 : BIG_LB_TILES * 256 + BIG_KB * DTS;
}
__host__ __device__ constexpr int big_chol_lds(int JB) { return DTS + BIG_NW * 16 + 16 + 2 + UNITS + big_slab_doubles(JB); }  // doubles

// Stage the slab of L tiles (J0 + jj, k0 + kk), jj < jb, kk < kb, into LDS as
// [jj][kk][256]: 16-byte loads, 8 in flight per thread before any LDS store (one
// memory round trip per 64 KB instead of one per 4 KB).
__device__ __forceinline__ void stage_slab(double* LJ, const double* H, int J0, int jb, int k0, int kb, int NT) {
  const int nch = jb * kb * 128;  // 16-B chunks
  for (int c0 = threadIdx.x; c0 < nch; c0 += 8 * BIG_NTHREADS) {
    double vx[8], vy[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int c = min(c0 + u * BIG_NTHREADS, nch - 1);  // clamped: always a valid slab chunk
      const int t = c >> 7, jj = t / kb, kk = t - jj * kb;
      const double2 w = *(const double2*)(H + (size_t)big_tile_index(J0 + jj, k0 + kk, NT) * 256 + 2 * (c & 127));
      vx[u] = w.x;
      vy[u] = w.y;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int c = c0 + u * BIG_NTHREADS;
      if (c < nch) *(double2*)(LJ + 2 * c) = make_double2(vx[u], vy[u]);
    }
  }
}

// stage_slab by LDS-DMA (global_load_lds_dwordx4): no VGPR holds the data, so a pass
// with its accumulators in registers (FR) can stage without spilling them.  One wave
// instruction moves 64 consecutive 16-B chunks (half a tile) to consecutive LDS.  The
// caller's __syncthreads() after the vmcnt(0) makes the slab visible (wait = false: the
// caller waits, e.g. one chunk later).
__device__ __forceinline__ void stage_slab_lds(double* LJ, const double* H, int J0, int jb, int k0, int kb, int NT,
                                               bool wait = true) {
  const int nch = jb * kb * 128;  // 16-B chunks, a multiple of 64
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int c0 = wave * 64; c0 < nch; c0 += BIG_NTHREADS) {
    const int t = c0 >> 7, jj = t / kb, kk = t - jj * kb;
    const double* src = H + (size_t)big_tile_index(J0 + jj, k0 + kk, NT) * 256 + 2 * ((c0 & 127) + lane);
    __builtin_amdgcn_global_load_lds((const void*)src, (__attribute__((address_space(3))) void*)(LJ + 2 * c0), 16, 0, 0);
  }
  if (wait) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// Block column k0 of the left-looking factorization up to its diagonal block: the
// left-looking update of the column's tiles (rows < rowend: all rows in the one-launch
// form, the block's own rows in the split one), then the diagonal block (panels on wave 0,
// in-block updates and TRSM on the others; L_Ik to H and LB, L_kk^-T to LT and LTs, y_k to
// YV, b_I updated).  LDS as k_big_chol's (DT, flag, UN, LJ); a non-SPD pivot sets *flag.
template <int BIG_JB, bool LL, bool SPLITROWS>
__device__ __forceinline__ void big_diag_block(const BigArgs& a, int k0, int kend, double* H, double* LTg, double* BV,
                                               double* YV, double* sm, int lane, int wave, const int* FI = nullptr) {
  double* DT = sm;
  int* flag = (int*)(sm + DTS + BIG_NW * 16 + 16);
  double* UN = sm + DTS + BIG_NW * 16 + 16 + 2;
  double* LJ = UN + UNITS;
  const int NT = a.NT;
  if constexpr (LL && SPLITROWS && MHE_BIG_DIAG_REG) {
    // ---- split form: the left-looking update of the block's own <= 8 rows, one row per
    // wave with its (up to 8) block-column tiles as accumulators, the kb x 4 slab of L_Jk
    // staged by LDS-DMA and shared by the 8 rows -- as k_big_rows, but in the tiles' own
    // orientation (the diagonal block below reads them from H).  Branch-free: tiles past
    // the row's diagonal and waves without a row compute on clamped tiles, stores only.
    // Same operations and order per element as the pass below.
    // MHE_BIG_DIAG_DB: KC = 2 slabs double-buffered (the next chunk's LDS-DMA in flight
    // during this one's MFMAs; 2 x 32 KB in the LJ region), else KC = 4 single-buffered
    constexpr bool DDB = MHE_BIG_DIAG_DB != 0;
    constexpr int KC = DDB ? 2 : 4;
    constexpr int SLABD = BIG_KB * KC * 256;
    static_assert(!DDB || 2 * SLABD <= BIG_LB_TILES * 256 + BIG_KB * DTS, "both slabs fit the LJ region");
    static_assert(!MHE_BIG_HEAD || KC <= 2, "k0 need not be a multiple of KC: a chunk's tiles must stay below the diagonal");
    const int kb = kend - k0;
    if (k0 > 0 && !(MHE_BIG_KO & 1)) {
      const int wv = __builtin_amdgcn_readfirstlane(wave);
      // Row k0 + o needs only its o + 1 tiles up to the diagonal: the MFMAs of tiles past it
      // (and every MFMA of a wave without a row) are skipped by wave-uniform branches
      // (MHE_BIG_DIAG_SKIP), and the rows are dealt so that the two waves sharing a SIMD
      // (w, w + 4) take rows o and 7 - o: 9 tiles per SIMD instead of up to 16.
      const int o = (MHE_BIG_DIAG_SKIP && wv >= 4) ? 11 - wv : wv;
      const int I = k0 + o;
      const bool act = I < kend;
      const int Ic = act ? I : kend - 1, jlast = Ic - k0;
      const int jdo = MHE_BIG_DIAG_SKIP ? (act ? jlast : -1) : BIG_KB - 1;  // last tile computed
      d4 acc[BIG_KB];
#pragma unroll
      for (int jj = 0; jj < BIG_KB; ++jj) {
        const double* C = H + (size_t)big_tile_index(Ic, k0 + min(jj, jlast), NT) * 256;
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[jj][r] = C[64 * r + lane];
      }
      // MHE_BIG_ENV: the update starts at the block rows' first nonzero tile column (their
      // L_Jk left of it are zero), rounded down to a chunk
      int kst = 0;
      if (MHE_BIG_ENV && FI) {
        kst = k0;
        for (int J = k0; J < kend; ++J) kst = min(kst, FI[J]);
        kst &= ~(KC - 1);
      }
      if (DDB && kst < k0) stage_slab_lds(LJ, H, k0, kb, kst, KC, NT, false);
      for (int kc = kst; kc < k0; kc += KC) {
        const int ci = (kc - kst) / KC;  // chunk index: slab buffer ci & 1
        double* S = LJ + (DDB ? (ci & 1) * SLABD : 0);
        if (DDB) {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this chunk's slab has landed
          __syncthreads();  // ... for every wave; the other buffer's readers are done
          if (kc + KC < k0) stage_slab_lds(LJ + ((ci + 1) & 1) * SLABD, H, k0, kb, kc + KC, KC, NT, false);
        } else {
          __syncthreads();  // the previous slab is consumed
          stage_slab_lds(LJ, H, k0, kb, kc, KC, NT);  // L_Jk, J = k0 + jj, k = kc + kk
          __syncthreads();
        }
        if (MHE_BIG_WSKIP_DIAG && FI && act && kc + KC <= FI[Ic]) continue;  // the row's L_Ik here are zero
        // the row's own L_Ik are slab tiles too (I is one of the block's rows J): read from
        // LDS (MHE_BIG_DIAG_LROW) instead of a second time from HBM
        auto lrow = [&](int kk) {
          return MHE_BIG_DIAG_LROW ? S + (jlast * KC + kk) * 256 : H + (size_t)big_tile_index(Ic, kc + kk, NT) * 256;
        };
        double an[4];
        const double* L0 = lrow(0);
#pragma unroll
        for (int r = 0; r < 4; ++r) an[r] = L0[64 * r + lane];
#pragma unroll
        for (int kk = 0; kk < KC; ++kk) {
          if (MHE_BIG_HEAD && kc + kk >= k0) break;  // k0 odd (MHE_BIG_HEAD): the chunk's last tile is past it
          double av[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) av[r] = an[r];  // negated by the MFMA
          if (kk + 1 < KC) {
            const double* Ln = lrow(kk + 1);
#pragma unroll
            for (int r = 0; r < 4; ++r) an[r] = Ln[64 * r + lane];
          }
#pragma unroll
          for (int jj = 0; jj < BIG_KB; ++jj) {
            if (jj <= jdo) {  // wave-uniform
              const double* Bt = S + (min(jj, jlast) * KC + kk) * 256;
#pragma unroll
              for (int r = 0; r < 4; ++r)
                acc[jj] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[r], Bt[64 * r + lane], acc[jj], 0, 0, MFMA_NEG_A);
            }
          }
        }
      }
#pragma unroll
      for (int jj = 0; jj < BIG_KB; ++jj) {
        if (act && jj <= jlast) {
          double* C = H + (size_t)big_tile_index(I, k0 + jj, NT) * 256;
#pragma unroll
          for (int r = 0; r < 4; ++r) C[64 * r + lane] = acc[jj][r];
        }
      }
    }
    __syncthreads();  // the block column's tiles are up to date; LJ is free for LB / LTs
  } else if constexpr (LL) {
    // ---- left-looking update of block column k0 by all previous columns: a wave
    // takes LLR rows (g0 + wave + 8 q), so one staged slab serves 8 LLR rows
    constexpr int LLR = BIG_JB == 8 ? MHE_BIG_LLR8 : 2;
    for (int jh = 0; jh < kend - k0 && k0 > 0 && !(MHE_BIG_KO & 1); jh += BIG_JB) {
      const int jw = min(BIG_JB, kend - k0 - jh), Jb = k0 + jh;
      const int rowend = SPLITROWS ? kend : NT;  // split: the rows below get theirs in k_big_rows
      for (int g0 = Jb; g0 < rowend; g0 += BIG_NW * LLR) {
        int Iq[LLR], jm[LLR];
        d4 c[LLR][BIG_JB];
#pragma unroll
        for (int q = 0; q < LLR; ++q) {
          Iq[q] = g0 + wave + BIG_NW * q;
          jm[q] = Iq[q] < rowend ? min(jw, Iq[q] - Jb + 1) : 0;
#pragma unroll
          for (int jj = 0; jj < BIG_JB; ++jj) {
            if (jj < jm[q]) {
              const double* C = H + (size_t)big_tile_index(Iq[q], Jb + jj, NT) * 256;
#pragma unroll
              for (int r = 0; r < 4; ++r) c[q][jj][r] = C[64 * r + lane];
            }
          }
        }
        for (int kc = 0; kc < k0; kc += BIG_KB) {
          __syncthreads();  // the previous chunk's slab is consumed
          if (!(MHE_BIG_KO & 8)) stage_slab(LJ, H, Jb, jw, kc, BIG_KB, NT);  // L_Jk, jj < jw, kk < BIG_KB
          __syncthreads();
          // both rows share each staged B operand (one LDS read per 2 x 4 MFMAs); the
          // rows' next L_Ik tiles are loaded one k step ahead
          double av[LLR][4];
#pragma unroll
          for (int q = 0; q < LLR; ++q) {
            const double* LI0 = H + (size_t)big_tile_index(jm[q] > 0 ? Iq[q] : Jb, kc, NT) * 256;
#pragma unroll
            for (int r = 0; r < 4; ++r) av[q][r] = LI0[64 * r + lane];  // negated by the MFMA
          }
#pragma unroll 1
          for (int kk = 0; kk < BIG_KB; ++kk) {
            double an[LLR][4];
#pragma unroll
            for (int q = 0; q < LLR; ++q) {
              const double* LIn =
                  H + (size_t)big_tile_index(jm[q] > 0 ? Iq[q] : Jb, kc + min(kk + 1, BIG_KB - 1), NT) * 256;
#pragma unroll
              for (int r = 0; r < 4; ++r) an[q][r] = LIn[64 * r + lane];
            }
#pragma unroll
            for (int jj = 0; jj < BIG_JB; ++jj) {
              if (jj < jm[0]) {  // rows ascend with q: jm[0] <= jm[1]
                const double* Bt = LJ + (jj * BIG_KB + kk) * 256;
                double bv[4];
#pragma unroll
                for (int r = 0; r < 4; ++r) bv[r] = Bt[64 * r + lane];
#pragma unroll
                for (int q = 0; q < LLR; ++q) {
                  if (jj < jm[q]) {
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                      c[q][jj] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[q][r], bv[r], c[q][jj], 0, 0, MFMA_NEG_A);
                  }
                }
              } else if (jj < jm[LLR - 1]) {
                const double* Bt = LJ + (jj * BIG_KB + kk) * 256;
                double bv[4];
#pragma unroll
                for (int r = 0; r < 4; ++r) bv[r] = Bt[64 * r + lane];
#pragma unroll
                for (int r = 0; r < 4; ++r)
                  c[LLR - 1][jj] =
                      __builtin_amdgcn_mfma_f64_16x16x4f64(av[LLR - 1][r], bv[r], c[LLR - 1][jj], 0, 0, MFMA_NEG_A);
              }
            }
#pragma unroll
            for (int q = 0; q < LLR; ++q)
#pragma unroll
              for (int r = 0; r < 4; ++r) av[q][r] = an[q][r];
          }
        }
#pragma unroll
        for (int q = 0; q < LLR; ++q) {
#pragma unroll
          for (int jj = 0; jj < BIG_JB; ++jj) {
            if (jj < jm[q]) {
              double* C = H + (size_t)big_tile_index(Iq[q], Jb + jj, NT) * 256;
#pragma unroll
              for (int r = 0; r < 4; ++r) C[64 * r + lane] = c[q][jj][r];
            }
          }
        }
      }
    }
    __syncthreads();  // the block column is up to date; LJ is free for LB / LTs
  }
  // ---- diagonal block, left-looking inside the block column: at step k every tile
  // (I, k), k <= I < kend, gets all of its in-block updates in ONE pass (K = 16 (k - k0),
  // L_kk' operands from LDS), then the TRSM.  Two workgroup barriers per k.
  // LB (= the LJ region, free until the trailing phase): L_Ik' for k0 <= k' < I < kend, packed
  // strictly-lower: slot (I - k0)(I - k0 - 1)/2 + (k' - k0); LTs: L_kk^-T of the block's k.
  double* LB = LJ;
  double* LTs = LJ + BIG_LB_TILES * 256;
  // wave 0's next diagonal tile is loaded one column ahead (MHE_BIG_DIAG_AKPF): A_kk is not
  // written in the column loop before its own column, so its load latency leaves the chain
  d4 akn;
  if (MHE_BIG_DIAG_AKPF && wave == 0) {
    const double* A0 = H + (size_t)big_tile_index(k0, k0, NT) * 256;
#pragma unroll
    for (int r = 0; r < 4; ++r) akn[r] = A0[64 * r + lane];
  }
  for (int k = k0; k < kend; ++k) {
    const int nk = k - k0;
    if (wave == 0) {
      // diagonal tile: A_kk - sum L_kk' L_kk'^T -> DT, panel, y_k
      const double* Akk = H + (size_t)big_tile_index(k, k, NT) * 256;
      d4 c;
      if (MHE_BIG_DIAG_AKPF) {
        c = akn;
        if (k + 1 < kend) {
          const double* An = H + (size_t)big_tile_index(k + 1, k + 1, NT) * 256;
#pragma unroll
          for (int r = 0; r < 4; ++r) akn[r] = An[64 * r + lane];
        }
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) c[r] = Akk[64 * r + lane];
      }
      for (int kk = 0; kk < nk && !(MHE_BIG_KO & 2); ++kk) {
        const double* Lt = LB + (nk * (nk - 1) / 2 + kk) * 256;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const double v = Lt[64 * r + lane];
          c = __builtin_amdgcn_mfma_f64_16x16x4f64(v, v, c, 0, 0, MFMA_NEG_A);
        }
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) DT[64 * r + lane] = c[r];
      wave_lds_sync();
      const bool bad = panel(DT, UN, lane);
      if (bad && lane == 0 && !MHE_BIG_KO) *flag = 1;  // probes keep every trajectory running
      wave_lds_sync();
      block_fwd(DT, BV + 16 * k, YV + 16 * k, lane);  // y_k = L_kk^-1 b_k
      for (int e = lane; e < DTS; e += 64) {
        LTg[(size_t)k * DTS + e] = DT[e];
        LTs[nk * DTS + e] = DT[e];
      }
    } else {
      // block rows k < I < kend: c' = A_Ik^T - sum_k' L_kk' L_Ik'^T, stored k-major in place (= A_Ik^T row-major)
      for (int I = k + wave; I < kend; I += BIG_NW - 1) {
        double* Ak = H + (size_t)big_tile_index(I, k, NT) * 256;
        d4 c;
#pragma unroll
        for (int r = 0; r < 4; ++r) c[r] = Ak[(lane & 15) * 16 + 4 * r + (lane >> 4)];
        for (int kk = 0; kk < nk && !(MHE_BIG_KO & 2); ++kk) {
          const double* Lk = LB + (nk * (nk - 1) / 2 + kk) * 256;
          const double* LI = LB + ((I - k0) * (I - k0 - 1) / 2 + kk) * 256;
#pragma unroll
          for (int r = 0; r < 4; ++r)
            c = __builtin_amdgcn_mfma_f64_16x16x4f64(Lk[64 * r + lane], LI[64 * r + lane], c, 0, 0, MFMA_NEG_A);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) Ak[64 * r + lane] = c[r];
      }
    }
    __syncthreads();
    if (*flag) break;
    // TRSM: L_Ik^T = L_kk^-1 A_Ik^T (k-major result) for the block rows, b_I -= L_Ik y_k; L_Ik also to LB
    const double yk = YV[16 * k + (lane >> 4)], yk1 = YV[16 * k + 4 + (lane >> 4)],
                 yk2 = YV[16 * k + 8 + (lane >> 4)], yk3 = YV[16 * k + 12 + (lane >> 4)];
    for (int I = k + 1 + wave; I < kend && !(MHE_BIG_KO & 4); I += BIG_NW) {
      double* Ak = H + (size_t)big_tile_index(I, k, NT) * 256;
      double av[4], bv[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        av[r] = DT[(4 * r + (lane >> 4)) * LIS + (lane & 15)];  // L_kk^-1 [lane & 15][4r + (lane >> 4)]
        bv[r] = Ak[64 * r + lane];
      }
      d4 u = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int r = 0; r < 4; ++r) u = __builtin_amdgcn_mfma_f64_16x16x4f64(av[r], bv[r], u, 0, 0, 0);
      // u[r] = L_Ik[lane & 15][(lane >> 4) + 4 r]
      double* LBs = LB + ((I - k0) * (I - k0 - 1) / 2 + nk) * 256;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        Ak[64 * r + lane] = u[r];
        LBs[64 * r + lane] = u[r];
      }
      double s = u[0] * yk + u[1] * yk1 + u[2] * yk2 + u[3] * yk3;
      s += __shfl_xor(s, 16);
      s += __shfl_xor(s, 32);
      if (lane < 16) BV[16 * I + lane] -= s;
    }
    __syncthreads();
  }
}

// LL = true: LEFT-looking updates instead of the trailing update.  Before block column
// k0 is factored, its tiles (I, k0 .. kend-1), I >= k0, receive all their updates
// sum_{k < k0} L_Ik L_Jk^T in one visit: a wave keeps one row's BIG_JB accumulators in
// registers while the block column's L_Jk are staged through LDS BIG_KB tile columns at
// a time.  Every tile is then read and written ONCE per factorization (the right-looking
// update reads and writes it once per super-block above it); L_Ik is read once per block
// column (as before) and the staged L_Jk once per group of 8 rows.
// SPLIT (left-looking only) runs the factorization as one launch per stage instead of one
// per trajectory: SPLIT = 1 is block column kfirst's diagonal stage (the left-looking update
// of the block's own rows, then the diagonal block), k_big_rows the rows below it (a launch
// of its own, one workgroup per 8 rows), SPLIT = 2 the backward solve.  SPLIT = 0: the whole
// factorization and solve in one launch (the right-looking form, and the A/B baseline).
template <int BIG_JB, bool LL = false, int SPLIT = 0>
__global__ __launch_bounds__(BIG_NTHREADS, BIG_JB == 8 ? 2 : 4) void k_big_chol(BigArgs a, int kfirst) {
  static_assert(SPLIT == 0 || LL, "the split stages are the left-looking factorization's");
  const int b = blockIdx.x;
  if (a.state[b] != BIG_RUNNING) return;
  const BigWs WL = big_ws_layout(a.P, a.M, a.n, a.NT, a.nz, a.nc);
  double* ws = a.ws + (size_t)b * a.ws_stride;
  double* H = ws + WL.H;
  double* LTg = ws + WL.LT;
  double* BV = ws + WL.BV;
  double* YV = ws + WL.YV;
  extern __shared__ __attribute__((aligned(16))) double sm[];
  double* DT = sm;                 // DTS: A_kk, then L_kk^-T
  double* PART = sm + DTS;         // BIG_NW x 16 partial sums (backward)
  double* YL = PART + BIG_NW * 16; // 16: block right-hand side (backward)
  int* flag = (int*)(YL + 16);
  double* UN = sm + DTS + BIG_NW * 16 + 16 + 2;  // identity rows for the panel (unit_row)
  double* LJ = UN + UNITS;                        // staged L_Jk tiles [jj][kk][256], row-major
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int NT = a.NT;
  if (threadIdx.x == 0) *flag = 0;
  init_units(UN);
  // MHE_BIG_ENV: each tile row's first nonzero tile column from k_big_assemble's component-pair
  // flags, once per factorization (the first diagonal stage; read by the later stages)
  int* FIw = MHE_BIG_ENV && SPLIT != 0 ? big_env_first(ws, WL, a.n) : nullptr;
  const int* FI = FIw;
  if constexpr (MHE_BIG_ENV && SPLIT == 1) {
    if (kfirst == 0) {
      const int* EM = big_env_mask(ws, WL);
      for (int t = threadIdx.x; t < NT; t += BIG_NTHREADS) {
        const int ca = t / a.NTc;
        int bm = ca;
        for (int cb = 0; cb < ca; ++cb) {
          if (EM[ca * a.n + cb] | EM[cb * a.n + ca]) {
            bm = cb;
            break;
          }
        }
        FIw[t] = bm * a.NTc;
      }
    }
  }
  const int kbeg = SPLIT == 1 ? kfirst : 0, kstop = SPLIT == 1 ? big_split_kend(kfirst, NT) : (SPLIT == 2 ? 0 : NT);
  for (int k0 = kbeg; k0 < kstop; k0 += BIG_KB) {
    const int kend = SPLIT == 1 ? kstop : min(k0 + BIG_KB, NT);
    big_diag_block<BIG_JB, LL, SPLIT != 0>(a, k0, kend, H, LTg, BV, YV, sm, lane, wave, FI);
    double* LB = LJ;  // the diagonal block's L_Ik' and L_kk^-T (big_diag_block)
    double* LTs = LJ + BIG_LB_TILES * 256;
    if (*flag) break;
    // ---- rows below the block, one wave per row: the same operations per element as
    // the diagonal block's (in-block updates in k' order, TRSM, b_I update in k order),
    // without barriers; the row's L_Ik' are re-read right after this wave wrote them
    // (L2 hits: the old form re-read them after a sweep over every row)
    const int kb = kend - k0;
    // 8-wide instance: two rows per wave (I, I + 8), independent MFMA chains and their
    // L_Ik' loads in flight together, the block's L_kk' read once from LDS for both (C4
    // +2 %, C5 +0.7 %); the 4-wide one keeps one row per wave (the second row's registers
    // spill there: C3 -0.9 %).  Unused second-row work is dead code at JB = 4.
    constexpr int RPW = BIG_JB == 8 ? 2 : 1;
    // 8-wide instance: loads one step ahead -- the rows' next A_Ik tiles during tile kk, the
    // next L_Ik' during in-block step kp (C4 -0.4 %); the 4-wide one loads at the point of
    // use (the prefetch registers add spills there: C3 +1.6 %, profiles/r04_ab_big_rows_prefetch.txt).
    constexpr bool RPF = BIG_JB == 8;
    for (int I = kend + wave; I < NT && !SPLIT && !(MHE_BIG_KO & 16); I += RPW * BIG_NW) {
      const bool two = RPW == 2 && I + BIG_NW < NT;
      const int I2 = two ? I + BIG_NW : I;
      d4 an, an2;  // A_Ik^T of the next tile, k-major (= row-major A_Ik read transposed)
      auto load_a = [&](int kk) {
        const double* A1 = H + (size_t)big_tile_index(I, k0 + kk, NT) * 256;
        const double* A2 = H + (size_t)big_tile_index(I2, k0 + kk, NT) * 256;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          an[r] = A1[(lane & 15) * 16 + 4 * r + (lane >> 4)];
          an2[r] = A2[(lane & 15) * 16 + 4 * r + (lane >> 4)];
        }
      };
      if (RPF) load_a(0);
      for (int kk = 0; kk < kb; ++kk) {
        double* Ak = H + (size_t)big_tile_index(I, k0 + kk, NT) * 256;
        double* Ak2 = H + (size_t)big_tile_index(I2, k0 + kk, NT) * 256;
        if (!RPF) load_a(kk);
        d4 c = an, c2 = an2;
        if (RPF && kk + 1 < kb) load_a(kk + 1);
        double ln[4], ln2[4];  // L_Ik' of the next in-block step
        auto load_l = [&](int kp) {
          const double* L1 = H + (size_t)big_tile_index(I, k0 + kp, NT) * 256;
          const double* L2 = H + (size_t)big_tile_index(I2, k0 + kp, NT) * 256;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            ln[r] = L1[64 * r + lane];
            ln2[r] = L2[64 * r + lane];
          }
        };
        if (RPF && kk > 0) load_l(0);
        for (int kp = 0; kp < kk && !(MHE_BIG_KO & 2); ++kp) {
          const double* Lk = LB + (kk * (kk - 1) / 2 + kp) * 256;
          double lk[4], li[4], li2[4];
          if (!RPF) load_l(kp);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            li[r] = ln[r];
            li2[r] = ln2[r];
            lk[r] = Lk[64 * r + lane];
          }
          if (RPF && kp + 1 < kk) load_l(kp + 1);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            c = __builtin_amdgcn_mfma_f64_16x16x4f64(lk[r], li[r], c, 0, 0, MFMA_NEG_A);
            c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(lk[r], li2[r], c2, 0, 0, MFMA_NEG_A);
          }
        }
        const double* LT = LTs + kk * DTS;
        d4 t = {0.0, 0.0, 0.0, 0.0}, t2 = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const double lv = LT[(4 * r + (lane >> 4)) * LIS + (lane & 15)];
          t = __builtin_amdgcn_mfma_f64_16x16x4f64(lv, c[r], t, 0, 0, 0);
          t2 = __builtin_amdgcn_mfma_f64_16x16x4f64(lv, c2[r], t2, 0, 0, 0);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) Ak[64 * r + lane] = t[r];
        if (two) {
#pragma unroll
          for (int r = 0; r < 4; ++r) Ak2[64 * r + lane] = t2[r];
        }
        const int k = k0 + kk;
        const double y0 = YV[16 * k + (lane >> 4)], y1 = YV[16 * k + 4 + (lane >> 4)],
                     y2 = YV[16 * k + 8 + (lane >> 4)], y3 = YV[16 * k + 12 + (lane >> 4)];
        double s = t[0] * y0 + t[1] * y1 + t[2] * y2 + t[3] * y3;
        double s2 = t2[0] * y0 + t2[1] * y1 + t2[2] * y2 + t2[3] * y3;
        s += __shfl_xor(s, 16);
        s += __shfl_xor(s, 32);
        s2 += __shfl_xor(s2, 16);
        s2 += __shfl_xor(s2, 32);
        if (lane < 16) {
          BV[16 * I + lane] -= s;
          if (two) BV[16 * I2 + lane] -= s2;
        }
      }
    }
    __syncthreads();
    // ---- trailing update with K = (kend - k0) tiles (right-looking form only)
    for (int J0 = kend; J0 < NT && !LL && !(MHE_BIG_KO & 1); J0 += BIG_JB) {
      const int jb = min(BIG_JB, NT - J0);
      stage_slab(LJ, H, J0, jb, k0, kb, NT);  // L_Jk (jb x kb tiles) into LDS
      __syncthreads();
      for (int I = J0 + wave; I < NT; I += BIG_NW) {
        // row I of the slab: up to BIG_JB accumulators (jmax: the triangle's rows
        // stop at the diagonal), L_Ik operands streamed one k tile ahead and read
        // once per row visit
        const int jmax = min(jb, I - J0 + 1);
        d4 c[BIG_JB];
#pragma unroll
        for (int jj = 0; jj < BIG_JB; ++jj) {
          if (jj < jmax) {
            const double* C = H + (size_t)big_tile_index(I, J0 + jj, NT) * 256;
#pragma unroll
            for (int r = 0; r < 4; ++r) c[jj][r] = C[64 * r + lane];
          }
        }
        const double* LI0 = H + (size_t)big_tile_index(I, k0, NT) * 256;
        double av[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) av[r] = LI0[64 * r + lane];  // negated by the MFMA (MFMA_NEG_A)
#pragma unroll 1
        for (int kk = 0; kk < kb; ++kk) {
          double an[4];
          const double* LIn = H + (size_t)big_tile_index(I, k0 + min(kk + 1, kb - 1), NT) * 256;
#pragma unroll
          for (int r = 0; r < 4; ++r) an[r] = LIn[64 * r + lane];
#pragma unroll
          for (int jj = 0; jj < BIG_JB; ++jj) {
            if (jj < jmax) {
              const double* Bt = LJ + (jj * kb + kk) * 256;
#pragma unroll
              for (int r = 0; r < 4; ++r)
                c[jj] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[r], Bt[64 * r + lane], c[jj], 0, 0, MFMA_NEG_A);
            }
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) av[r] = an[r];
        }
#pragma unroll
        for (int jj = 0; jj < BIG_JB; ++jj) {
          if (jj < jmax) {
            double* C = H + (size_t)big_tile_index(I, J0 + jj, NT) * 256;
#pragma unroll
            for (int r = 0; r < 4; ++r) C[64 * r + lane] = c[jj][r];
          }
        }
      }
      __syncthreads();
    }
  }
  // SPLIT = 2 (the backward solve alone) runs no block column, so nothing orders thread
  // 0's flag reset before the other waves' reads: it must not read the flag at all.  A
  // non-SPD pivot was recorded in a.state by its diagonal stage (SPLIT = 1 launch), and
  // such a trajectory returned at the state test above.
  if constexpr (SPLIT != 2) {
    if (*flag) {
      if (threadIdx.x == 0) a.state[b] = MHE_STATUS_NOT_SPD;
      return;
    }
  }
  if constexpr (SPLIT == 1) return;  // the rows below and the solve are launches of their own
  // backward: delta_k = L_kk^-T (y_k - sum_{I>k} L_Ik^T delta_I), delta in place in YV.
  // A chain of NT steps with two barriers each, so nothing on it waits for HBM: every
  // wave loads its first BWD_PF tiles of column k - 1 (and wave 0 its four L_kk^-T
  // entries per lane) during step k; y / delta live in LDS (the slab region, free now)
  // when they fit, the global YV copy is written alongside for k_big_update.
  // the split form's solve launch (SPLIT = 2) runs nothing else, so its registers can hold
  // a whole column's tiles for this wave at C3 (NT = 65: <= 8 per wave) -- every tile of
  // column k - 1 in flight during step k instead of two (MHE_BIG_BWD_PF)
  constexpr int BWD_PF = SPLIT == 2 ? MHE_BIG_BWD_PF : (BIG_JB == 8 ? 4 : 2);
  const bool yl = NT * 16 <= big_slab_doubles(BIG_JB);
  double* yb = yl ? LJ : YV;
  if (yl) {
    for (int e = threadIdx.x; e < NT * 16; e += BIG_NTHREADS) LJ[e] = YV[e];
    __syncthreads();
  }
  const int bc = lane & 15, bg = lane >> 4;
  double cur[BWD_PF][4], nxt[BWD_PF][4], lt[4], ltn[4];
  auto load_col = [&](int k, double (&dst)[BWD_PF][4], double (&l4)[4]) {
#pragma unroll
    for (int m = 0; m < BWD_PF; ++m) {
      const int I = k + 1 + wave + BIG_NW * m;
      if (I < NT && FI && FI[I] > k) {  // outside the envelope (MHE_BIG_ENV): L_Ik = 0, not read
#pragma unroll
        for (int r = 0; r < 4; ++r) dst[m][r] = 0.0;
      } else if (I < NT) {
        const double* L = H + (size_t)big_tile_index(I, k, NT) * 256;
#pragma unroll
        for (int r = 0; r < 4; ++r)  // L_Ik[tr][bc], k-major tile; coalesced: element (4r + bg) * 16 + bc
          dst[m][r] = MHE_BIG_BWD_COAL ? L[64 * r + lane] : L[bc * 16 + bg + 4 * r];
      }
    }
    if (wave == 0) {
#pragma unroll
      for (int i = 0; i < 4; ++i) l4[i] = LTg[(size_t)k * DTS + bc * LIS + 4 * bg + i];
    }
  };
  if (!(MHE_BIG_KO & 32)) load_col(NT - 1, cur, lt);
  for (int k = NT - 1; k >= 0 && !(MHE_BIG_KO & 32); --k) {
    if (k > 0) load_col(k - 1, nxt, ltn);  // in flight during this step
    double pv = 0.0;
    double pq[4] = {0.0, 0.0, 0.0, 0.0};  // MHE_BIG_BWD_COAL: output column 4r + bg, this lane's row bc
#pragma unroll
    for (int m = 0; m < BWD_PF; ++m) {
      const int I = k + 1 + wave + BIG_NW * m;
      if (I < NT) {
        if (MHE_BIG_BWD_COAL) {
          const double dI = yb[16 * I + bc];
#pragma unroll
          for (int r = 0; r < 4; ++r) pq[r] += cur[m][r] * dI;
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r) pv += cur[m][r] * yb[16 * I + bg + 4 * r];
        }
      }
    }
    for (int I = k + 1 + wave + BIG_NW * BWD_PF; I < NT; I += BIG_NW) {  // past the prefetched tiles (C4, C5)
      // (issuing these loads four at a time measured slower: the solve launch 1.23 -> 1.45 ms at C3)
      if (FI && FI[I] > k) continue;  // outside the envelope
      const double* L = H + (size_t)big_tile_index(I, k, NT) * 256;
      if (MHE_BIG_BWD_COAL) {
        const double dI = yb[16 * I + bc];
#pragma unroll
        for (int r = 0; r < 4; ++r) pq[r] += L[64 * r + lane] * dI;
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) pv += L[bc * 16 + bg + 4 * r] * yb[16 * I + bg + 4 * r];
      }
    }
    if (MHE_BIG_BWD_COAL) {
      // the 16 rows of each output column are the 16 lanes of a DPP row: lane (bc, bg) ends
      // with column 4 r(bc) + bg, r(bc) = 2 (bc >> 3) + ((bc >> 2) & 1)
      const double z = row16_sum4(pq, bc);
      if ((bc & 3) == 0) PART[wave * 16 + 4 * (2 * (bc >> 3) + ((bc >> 2) & 1)) + bg] = z;
    } else {
      pv += __shfl_xor(pv, 16);
      pv += __shfl_xor(pv, 32);
      if (lane < 16) PART[wave * 16 + lane] = pv;
    }
    __syncthreads();
    if (wave == 0) {
      if (lane < 16) {
        double rhs = yb[16 * k + lane];
        for (int w = 0; w < BIG_NW; ++w) rhs -= PART[w * 16 + lane];
        YL[lane] = rhs;
      }
      wave_lds_sync();
      // delta_k = L_kk^-T rhs: lane (c, g) the four terms 4g .. 4g + 3 of row c
      double sd = 0.0;
#pragma unroll
      for (int i = 0; i < 4; ++i) sd = fma(lt[i], YL[4 * bg + i], sd);
      const double dv = rows4_sum(sd);
      if (lane < 16) {
        yb[16 * k + lane] = dv;
        if (yl) YV[16 * k + lane] = dv;
      }
    }
    __syncthreads();
#pragma unroll
    for (int m = 0; m < BWD_PF; ++m)
#pragma unroll
      for (int r = 0; r < 4; ++r) cur[m][r] = nxt[m][r];
#pragma unroll
    for (int i = 0; i < 4; ++i) lt[i] = ltn[i];
  }
}


// The rows below block column k0 of the split left-looking factorization (k_big_chol
// SPLIT = 1 has factored the block's diagonal tiles, L_kk^-T in LT, y_k in YV): one
// workgroup per BIG_NW rows (one row per wave).  Each row's kb block-column tiles are
// accumulated transposed in registers, c^T = A_Ik^T - sum_{k<k0} L_Jk L_Ik^T (the staged
// L_Jk as the MFMA A operand, the row's L_Ik streamed as B), then the in-block updates and
// the TRSM run on those registers: every L_Ik (k < k0) is read once per block column and
// L_Ik is written once.  Same operations in the same order per element as the one-launch
// form's left-looking pass + rows pass.
//   staging  the kb x KC slab of L_Jk by LDS-DMA, double-buffered: chunk i + 1 is in flight
//            while chunk i's MFMAs run (one barrier per chunk);
//   XCD      a batch that is a multiple of 8 is remapped so all groups of a trajectory land
//            on one XCD (dispatch is round-robin over the 8 XCDs by linear workgroup id):
//            the slab and LB tiles every group of the trajectory stages come from that L2.
// LDS: two slabs, then (same region) the block's in-block L tiles LB and L_kk^-T.
__host__ __device__ constexpr int big_rows_lds() { return BIG_LB_TILES * 256 + BIG_KB * DTS; }  // doubles
// One group of BIG_NW rows below block column k0 (rows kend + 8 grp + wave): the body of
// k_big_rows.  sm: the LDS region of the slabs, LB and LTs (big_rows_lds() doubles).
template <int KC, bool DB>
__device__ __forceinline__ void big_rows_group(double* H, const double* LTg, double* BV, const double* YV,
                                               double* sm, int NT, int k0, int grp, const int* FI = nullptr) {
  static_assert((DB ? 2 : 1) * BIG_KB * KC * 256 <= big_rows_lds(), "the slabs fit the LDS region");
  static_assert(!MHE_BIG_HEAD || KC <= 2, "k0 need not be a multiple of KC: a chunk's tiles must stay below the diagonal");
  double* LB = sm;
  double* LTs = sm + BIG_LB_TILES * 256;
  const int kend = big_split_kend(k0, NT), kb = kend - k0;
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4, c = lane & 15;
  // Branch-free over the accumulators (a conditionally updated accumulator costs phi copies
  // of all of them): a wave without a row (I >= NT) and the columns past kb of the last
  // block column compute on clamped, valid tiles; only stores are predicated.
  const int I = kend + BIG_NW * grp + wave;
  const bool act = I < NT;
  const int Ic = act ? I : NT - 1;
  // MHE_BIG_ENV: the group's left-looking update starts at its rows' first nonzero tile
  // column (rounded down to a chunk); a group whose rows are all zero in this block column
  // has nothing to do (its tiles hold A_Ik = 0 = L_Ik, and b_I -= L_Ik y_k is no change)
  int kst = 0;
  if (MHE_BIG_ENV && FI) {
    kst = NT;
    for (int w = 0; w < BIG_NW; ++w) {
      const int Iw = kend + BIG_NW * grp + w;
      if (Iw < NT) kst = min(kst, FI[Iw]);
    }
    if (kst >= kend) return;
    kst = min(kst, k0) & ~(KC - 1);
  }
  const int fI = (MHE_BIG_ENV && MHE_BIG_WSKIP && FI) ? FI[Ic] : 0;  // this wave's row's first nonzero tile column
  d4 acc[BIG_KB];
  constexpr int SLAB = BIG_KB * KC * 256;
  if constexpr (MHE_BIG_ROWS_TLDS && DB) {
    // A_Ik^T through LDS: the tiles read coalesced (element 64 r + lane = A[4r + g][c]), then
    // transposed through this wave's padded 16 x 17 scratch in the second slab buffer (first
    // staged at chunk 1, after a barrier) -- the per-lane transposed global reads touched 16
    // cache lines per instruction
#pragma unroll
    for (int kk = 0; kk < BIG_KB; ++kk) {
      const double* A = H + (size_t)big_tile_index(Ic, k0 + min(kk, kb - 1), NT) * 256;
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[kk][r] = A[64 * r + lane];
    }
    double* T = sm + SLAB + wave * 272;
#pragma unroll
    for (int kk = 0; kk < BIG_KB; ++kk) {
#pragma unroll
      for (int r = 0; r < 4; ++r) T[(4 * r + g) * 17 + c] = acc[kk][r];
      wave_lds_sync();
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[kk][r] = T[c * 17 + g + 4 * r];  // A_Ik^T, k-major
      wave_lds_sync();
    }
  } else {
#pragma unroll
    for (int kk = 0; kk < BIG_KB; ++kk) {
      const double* A = H + (size_t)big_tile_index(Ic, k0 + min(kk, kb - 1), NT) * 256;
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[kk][r] = A[c * 16 + 4 * r + g];  // A_Ik^T, k-major
    }
  }
  if (kst < k0 && !(MHE_BIG_KO & 1)) stage_slab_lds(sm, H, k0, kb, kst, KC, NT, false);
#if MHE_BIG_ROWS_RPF
  // The row's L_Ik (B operands) a whole chunk ahead: tile kc + kk is loaded into bq[kk]
  // right after chunk kc - KC's MFMAs have read bq[kk], so its HBM latency is covered by
  // a chunk of MFMAs (and the slab wait) instead of by one k step.
  double bq[KC][4];
  if (kst < k0 && !(MHE_BIG_KO & 1)) {
#pragma unroll
    for (int kk = 0; kk < KC; ++kk) {
      const double* L0 = H + (size_t)big_tile_index(Ic, kst + kk, NT) * 256;
#pragma unroll
      for (int r = 0; r < 4; ++r) bq[kk][r] = L0[64 * r + lane];
    }
  }
  for (int kc = kst; kc < k0 && !(MHE_BIG_KO & 1); kc += KC) {
    const int ci = (kc - kst) / KC;  // chunk index: slab buffer ci & 1 (the first in buffer 0)
    const double* LJ = sm + (DB ? (ci & 1) * SLAB : 0);
    if (!DB && kc > kst) {
      __syncthreads();  // the previous chunk's readers are done
      stage_slab_lds(sm, H, k0, kb, kc, KC, NT, false);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this chunk's slab (and row tiles) have landed
    __syncthreads();
    if (DB && kc + KC < k0) stage_slab_lds(sm + ((ci + 1) & 1) * SLAB, H, k0, kb, kc + KC, KC, NT, false);
    // a wave without a row (I >= NT: the last group of every launch) skips the MFMAs by a
    // wave-uniform branch around the whole chunk (MHE_BIG_ROWS_SKIP); it still stages and
    // meets the barriers
    if (MHE_BIG_ROWS_SKIP && !act) continue;
    if (MHE_BIG_WSKIP && kc + KC <= fI) {
      // the row's L_Ik of this chunk are zero (left of its f): no MFMAs; the next chunk's
      // B operands are loaded here when that chunk is the row's first nonzero one
      if (kc + KC < k0 && kc + 2 * KC > fI) {
#pragma unroll
        for (int kk = 0; kk < KC; ++kk) {
          const double* Ln = H + (size_t)big_tile_index(Ic, kc + KC + kk, NT) * 256;
#pragma unroll
          for (int r = 0; r < 4; ++r) bq[kk][r] = Ln[64 * r + lane];
        }
      }
      continue;
    }
#pragma unroll
    for (int kk = 0; kk < KC; ++kk) {
      if (MHE_BIG_HEAD && kc + kk >= k0) break;  // k0 odd (MHE_BIG_HEAD): no next chunk either
      double a0[4], a1[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) a0[r] = LJ[kk * 256 + 64 * r + lane];
#pragma unroll
      for (int jj = 0; jj < BIG_KB; ++jj) {
        if (jj + 1 < BIG_KB) {
          const int jn = min(jj + 1, kb - 1);
#pragma unroll
          for (int r = 0; r < 4; ++r) a1[r] = LJ[(jn * KC + kk) * 256 + 64 * r + lane];
        }
#pragma unroll
        for (int r = 0; r < 4; ++r)
          acc[jj] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0[r], bq[kk][r], acc[jj], 0, 0, MFMA_NEG_A);
#pragma unroll
        for (int r = 0; r < 4; ++r) a0[r] = a1[r];
      }
      if (kc + KC < k0) {  // the next chunk's tile kk (its MFMAs above have read bq[kk])
        const double* Ln = H + (size_t)big_tile_index(Ic, kc + KC + kk, NT) * 256;
#pragma unroll
        for (int r = 0; r < 4; ++r) bq[kk][r] = Ln[64 * r + lane];
      }
    }
  }
#else
  for (int kc = kst; kc < k0 && !(MHE_BIG_KO & 1); kc += KC) {
    const int ci = (kc - kst) / KC;
    const double* LJ = sm + (DB ? (ci & 1) * SLAB : 0);
    if (!DB && kc > kst) {
      __syncthreads();  // the previous chunk's readers are done
      stage_slab_lds(sm, H, k0, kb, kc, KC, NT, false);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this chunk's slab has landed
    __syncthreads();  // ... for every wave, and the other buffer's last readers are done
    if (DB && kc + KC < k0) stage_slab_lds(sm + ((ci + 1) & 1) * SLAB, H, k0, kb, kc + KC, KC, NT, false);
    double bn[4];
    const double* L0 = H + (size_t)big_tile_index(Ic, kc, NT) * 256;
#pragma unroll
    for (int r = 0; r < 4; ++r) bn[r] = L0[64 * r + lane];  // (kc >= kst)
#pragma unroll
    for (int kk = 0; kk < KC; ++kk) {
      if (MHE_BIG_HEAD && kc + kk >= k0) break;
      double bv[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) bv[r] = bn[r];
      if (kk + 1 < KC) {
        const double* Ln = H + (size_t)big_tile_index(Ic, kc + kk + 1, NT) * 256;
#pragma unroll
        for (int r = 0; r < 4; ++r) bn[r] = Ln[64 * r + lane];
      }
      // the staged A operands one tile ahead
      double a0[4], a1[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) a0[r] = LJ[kk * 256 + 64 * r + lane];
#pragma unroll
      for (int jj = 0; jj < BIG_KB; ++jj) {
        if (jj + 1 < BIG_KB) {
          const int jn = min(jj + 1, kb - 1);
#pragma unroll
          for (int r = 0; r < 4; ++r) a1[r] = LJ[(jn * KC + kk) * 256 + 64 * r + lane];
        }
#pragma unroll
        for (int r = 0; r < 4; ++r)
          acc[jj] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0[r], bv[r], acc[jj], 0, 0, MFMA_NEG_A);
#pragma unroll
        for (int r = 0; r < 4; ++r) a0[r] = a1[r];
      }
    }
  }
#endif
  // the block's in-block L tiles and L_kk^-T into LDS (over the slabs)
  __syncthreads();
  if constexpr (MHE_BIG_ROWS_LBDMA) {
    // by LDS-DMA, every wave's share issued at once and waited for once (the load -> store
    // loop made one L2 round trip per 8 KB: ~19 of them before the in-block chain could start)
    const int nlb = kb * (kb - 1) / 2 * 2;  // half tiles (1 KB: one wave instruction each)
    for (int h = wave; h < nlb; h += BIG_NW) {
      const int slot = h >> 1;
      int ii = 1;  // slot = ii (ii - 1) / 2 + kp, kp < ii
      while (ii * (ii + 1) / 2 <= slot) ++ii;
      const int kp = slot - ii * (ii - 1) / 2;
      const double* src = H + (size_t)big_tile_index(k0 + ii, k0 + kp, NT) * 256 + 128 * (h & 1) + 2 * lane;
      __builtin_amdgcn_global_load_lds((const void*)src, (__attribute__((address_space(3))) void*)(LB + 256 * slot + 128 * (h & 1)),
                                       16, 0, 0);
    }
    const int nlt = (kb * DTS) / 2;  // 16-B chunks of the block's L_kk^-T (kb * DTS is even)
    for (int c0 = wave * 64; c0 < nlt; c0 += BIG_NTHREADS) {
      if (c0 + lane < nlt)
        __builtin_amdgcn_global_load_lds((const void*)(LTg + (size_t)k0 * DTS + 2 * (c0 + lane)),
                                         (__attribute__((address_space(3))) void*)(LTs + 2 * c0), 16, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else {
    for (int e = threadIdx.x; e < (kb * (kb - 1) / 2) * 128; e += BIG_NTHREADS) {
      const int slot = e >> 7;
      int ii = 1;  // slot = ii (ii - 1) / 2 + kp, kp < ii
      while (ii * (ii + 1) / 2 <= slot) ++ii;
      const int kp = slot - ii * (ii - 1) / 2;
      const double2 w = *(const double2*)(H + (size_t)big_tile_index(k0 + ii, k0 + kp, NT) * 256 + 2 * (e & 127));
      *(double2*)(LB + 256 * slot + 2 * (e & 127)) = w;
    }
    for (int e = threadIdx.x; e < kb * DTS; e += BIG_NTHREADS) LTs[e] = LTg[(size_t)k0 * DTS + e];
  }
  __syncthreads();
#pragma unroll
  for (int kk = 0; kk < BIG_KB; ++kk) {
    if (MHE_BIG_HEAD && kk >= kb) break;  // a narrow (head) block: no work past its columns
    d4 cc = acc[kk];
#pragma unroll
    for (int kp = 0; kp < kk; ++kp) {
      const double* Lk = LB + (kk * (kk - 1) / 2 + kp) * 256;
#pragma unroll
      for (int r = 0; r < 4; ++r)
        cc = __builtin_amdgcn_mfma_f64_16x16x4f64(Lk[64 * r + lane], acc[kp][r], cc, 0, 0, MFMA_NEG_A);
    }
    const double* LT = LTs + kk * DTS;
    d4 t = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int r = 0; r < 4; ++r) t = __builtin_amdgcn_mfma_f64_16x16x4f64(LT[(4 * r + g) * LIS + c], cc[r], t, 0, 0, 0);
    acc[kk] = t;
    const int k = k0 + min(kk, kb - 1);
    int go = g;  // opaque per step: the y addresses are not hoisted (8 x 4 of them)
    asm volatile("" : "+v"(go));
    const double* yk = YV + 16 * k;
    const double y0 = yk[go], y1 = yk[go + 4], y2 = yk[go + 8], y3 = yk[go + 12];
    double s = t[0] * y0 + t[1] * y1 + t[2] * y2 + t[3] * y3;
    s += __shfl_xor(s, 16);
    s += __shfl_xor(s, 32);
    if (act && kk < kb) {
      double* Ak = H + (size_t)big_tile_index(I, k0 + kk, NT) * 256;
#pragma unroll
      for (int r = 0; r < 4; ++r) Ak[64 * r + lane] = t[r];
      if (lane < 16) BV[16 * I + lane] -= s;
    }
  }
}

template <int KC = MHE_BIG_ROWS_KC, bool DB = MHE_BIG_ROWS_DB != 0>
__global__ __launch_bounds__(BIG_NTHREADS, 4) void k_big_rows(BigArgs a, int k0) {
  const int G = gridDim.x;
  int b = blockIdx.y, grp = blockIdx.x;
  if (MHE_BIG_ROWS_XCD && (gridDim.y & 7) == 0) {
    const int L = blockIdx.x + G * blockIdx.y, x = L & 7, j = L >> 3;
    b = 8 * (j / G) + x;
    grp = j - G * (j / G);
  }
  if (a.state[b] != BIG_RUNNING) return;
  const BigWs WL = big_ws_layout(a.P, a.M, a.n, a.NT, a.nz, a.nc);
  double* ws = a.ws + (size_t)b * a.ws_stride;
  extern __shared__ __attribute__((aligned(16))) double sm[];
  big_rows_group<KC, DB>(ws + WL.H, ws + WL.LT, ws + WL.BV, ws + WL.YV, sm, a.NT, k0, grp,
                         MHE_BIG_ENV ? big_env_first(ws, WL, a.n) : nullptr);
}

// ------------------------------------------------------------ border (f4)
// Bordered Gauss-Newton step for extra variables z and equality constraints
// C v = r (include/mhe.h; r = 0 for addEqConstraint rows, the bound or constant of
// a row the host's active set imposes).  Runs after k_big_chol, which left the factor
// H = L L^T (L_Ik tiles in place, L_kk^-T in LT) and the unconstrained step
// du = -H^-1 g in YV.  With B = [H_xz  C^T] (dp x K), S = [H_zz 0; 0 0]:
//   Z = H^-1 B                 (16-column panels: MFMA forward/backward substitution)
//   (S - B^T Z) w = r - B^T du,  r = [-g_z ; -c(v)]
//   dx = du - Z w,  dz = w[0:nz],  lambda = w[nz:K]  (H dx + C^T lambda = -g: the
//   multipliers of L = J + lambda^T (C v - r), written to a.lam when given)
// The Schur matrix is quasi-definite (z block SPD, constraint block negative
// definite), so LDL^T without pivoting is stable; a z component no row depends on
// (zero pivot with a zero row) is held fixed (dz = 0), the minimum-norm choice.
// Dynamic LDS: K*K (Schur) + 2K (rhs / w, pivot column) doubles.
// Border of the KKT system at the iterate, shared by k_big_border and the kernel-level
// KKT export (mhe_assemble_kkt_ws), so both see the same values:
//   column col < nz of B at component-major row (ca, j): (H_xz)_{(j,ca), col}
//     = sum_e PhiE[e][j] GZe[e][ca][col]  (epoch order);
//   column nz + k: the constraint row k's coefficients (+1 at eq[2k], -1 at eq[2k+1]);
//   S[r][c] = sum_e HZZe[e][r][c] for r, c < nz (the constraint block 0);
//   rhs r[i] = -g_z[i] = sum_e GZVe[e][i] (i < nz), -c(v) = -(v[a] - v[b] - r_k) else.
__device__ __forceinline__ double big_border_col(const BigArgs& a, const double* ws, const BigWs& WL,
                                                 const double* PhiE, const int* eq, int E, int n, int col, int ca,
                                                 int j) {
  constexpr int NZX = MHE_MAX_EXTRA;
  double v = 0.0;
  if (j < a.P && col < a.nz + a.nc) {
    if (col < a.nz) {
      for (int e = 0; e < E; ++e) v += PhiE[(size_t)e * a.P + j] * ws[WL.GZe + ((size_t)e * n + ca) * NZX + col];
    } else {
      const int fi = j * n + ca;  // node-major index of this row
      if (eq[2 * (col - a.nz)] == fi) v += 1.0;
      if (eq[2 * (col - a.nz) + 1] == fi) v -= 1.0;
    }
  }
  return v;
}
__device__ __forceinline__ double big_border_s(const BigArgs& a, const double* ws, const BigWs& WL, int E, int r,
                                               int c) {
  constexpr int NZX = MHE_MAX_EXTRA;
  double sv = 0.0;
  if (r < a.nz && c < a.nz)
    for (int e = 0; e < E; ++e) sv += ws[WL.HZZe + (size_t)e * NZX * NZX + r * NZX + c];
  return sv;
}
__device__ __forceinline__ double big_border_rhs(const BigArgs& a, const double* ws, const BigWs& WL, const int* eq,
                                                 const double* eqr, const double* X, int E, int r) {
  constexpr int NZX = MHE_MAX_EXTRA;
  double base = 0.0;
  if (r < a.nz) {  // -g_z = sum H_z^T R e
    for (int e = 0; e < E; ++e) base += ws[WL.GZVe + (size_t)e * NZX + r];
  } else {  // -c(v)
    const int ia = eq[2 * (r - a.nz)], ib = eq[2 * (r - a.nz) + 1];
    base = -(X[ia] - (ib >= 0 ? X[ib] : 0.0) - eqr[r - a.nz]);
  }
  return base;
}

template <int n, int p>
__global__ __launch_bounds__(BIG_NTHREADS) void k_big_border(BigArgs a) {
  constexpr int NZX = MHE_MAX_EXTRA;
  const int b = blockIdx.x;
  if (a.state[b] != BIG_RUNNING) return;
  const BigConst CL = big_const_layout(a.P, a.M, n, p, a.nc);  // p: the Rw section size
  const BigWs WL = big_ws_layout(a.P, a.M, n, a.NT, a.nz, a.nc);
  double* ws = a.ws + (size_t)b * a.ws_stride;
  const double* H = ws + WL.H;
  const double* LT = ws + WL.LT;
  double* YV = ws + WL.YV;
  double* BM = ws + WL.BM;
  double* ZM = ws + WL.ZM;
  const double* PhiE = (const double*)(a.cbuf + CL.PhiE);
  const int* eq = (const int*)(a.cbuf + CL.eq);
  const double* eqr = (const double*)(a.cbuf + CL.eqr);
  const int E = a.M > 0 ? *(const int*)(a.cbuf + CL.ne) : 0;
  const int nz = a.nz, nc = a.nc, K = nz + nc, KP = (K + 15) / 16 * 16;
  const int NT = a.NT, Pp = a.Pp, dp = 16 * NT;
  const double* X = a.X + (size_t)b * a.P * n;
  extern __shared__ __attribute__((aligned(16))) double sm[];
  double* Ms = sm;            // K x K Schur complement, then its LDL^T
  double* rw = sm + K * K;    // K: right-hand side, then w
  double* lc = rw + K;        // K: pivot column of the current LDL^T step
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;

  // (1) border columns, component-major rows r = c*Pp + j (padding rows 0);
  //     ZM columns K..KP-1 are zero (inert panel columns).  Imported (KKT parity): BM and
  //     ZM hold the caller's columns already.
  if (!a.border_import) {
    for (int t = threadIdx.x; t < KP * dp; t += BIG_NTHREADS) {
      const int col = t / dp, r = t % dp, ca = r / Pp, j = r % Pp;
      const double v = big_border_col(a, ws, WL, PhiE, eq, E, n, col, ca, j);
      if (col < K) BM[(size_t)col * dp + r] = v;
      ZM[(size_t)col * dp + r] = v;
    }
    __syncthreads();
  }

  // (2) Z = H^-1 B in place in ZM, one 16-column panel at a time.  MFMA operand
  //     layout as in k_big_chol: A[i = l&15][m = 4r + (l>>4)], B[m][j = l&15],
  //     C[(l>>4) + 4r][l&15].  ZM is column-major (col*dp + row).
  const int ii = lane & 15, mg = lane >> 4;
  for (int p0 = 0; p0 < K; p0 += 16) {
    double* Zp = ZM + (size_t)p0 * dp;
    auto zload = [&](int blk, int r) { return Zp[(size_t)ii * dp + 16 * blk + 4 * r + mg]; };       // B[m][j]
    for (int k = 0; k < NT; ++k) {  // forward: Y_k = L_kk^-1 Z_k;  Z_I -= L_Ik Y_k
      if (wave == 0) {
        d4 c = {0.0, 0.0, 0.0, 0.0};
        double av[4], bv[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          av[r] = LT[(size_t)k * DTS + (4 * r + mg) * LIS + ii];  // (L^-1)[i][m] = (L^-T)[m][i]
          bv[r] = zload(k, r);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) c = __builtin_amdgcn_mfma_f64_16x16x4f64(av[r], bv[r], c, 0, 0, 0);
#pragma unroll
        for (int r = 0; r < 4; ++r) Zp[(size_t)ii * dp + 16 * k + mg + 4 * r] = c[r];
      }
      __syncthreads();
      for (int I = k + 1 + wave; I < NT; I += BIG_NW) {
        const double* L = H + (size_t)big_tile_index(I, k, NT) * 256;
        d4 c;
        double av[4], bv[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          c[r] = Zp[(size_t)ii * dp + 16 * I + mg + 4 * r];
          av[r] = L[(4 * r + mg) * 16 + ii];  // L_Ik[i][m], k-major tile (negated by the MFMA)
          bv[r] = zload(k, r);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) c = __builtin_amdgcn_mfma_f64_16x16x4f64(av[r], bv[r], c, 0, 0, MFMA_NEG_A);
#pragma unroll
        for (int r = 0; r < 4; ++r) Zp[(size_t)ii * dp + 16 * I + mg + 4 * r] = c[r];
      }
      __syncthreads();
    }
    for (int k = NT - 1; k >= 0; --k) {  // backward: Z_k = L_kk^-T Y_k;  Y_J -= L_kJ^T Z_k
      if (wave == 0) {
        d4 c = {0.0, 0.0, 0.0, 0.0};
        double av[4], bv[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          av[r] = LT[(size_t)k * DTS + ii * LIS + 4 * r + mg];  // (L^-T)[i][m]
          bv[r] = zload(k, r);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) c = __builtin_amdgcn_mfma_f64_16x16x4f64(av[r], bv[r], c, 0, 0, 0);
#pragma unroll
        for (int r = 0; r < 4; ++r) Zp[(size_t)ii * dp + 16 * k + mg + 4 * r] = c[r];
      }
      __syncthreads();
      for (int J = wave; J < k; J += BIG_NW) {
        const double* L = H + (size_t)big_tile_index(k, J, NT) * 256;
        d4 c;
        double av[4], bv[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          c[r] = Zp[(size_t)ii * dp + 16 * J + mg + 4 * r];
          av[r] = L[ii * 16 + 4 * r + mg];  // (L_kJ^T)[i][m] = L_kJ[m][i], k-major tile (negated by the MFMA)
          bv[r] = zload(k, r);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) c = __builtin_amdgcn_mfma_f64_16x16x4f64(av[r], bv[r], c, 0, 0, MFMA_NEG_A);
#pragma unroll
        for (int r = 0; r < 4; ++r) Zp[(size_t)ii * dp + 16 * J + mg + 4 * r] = c[r];
      }
      __syncthreads();
    }
  }

  // (3) Schur complement and right-hand side (one wave per entry, lanes over rows)
  for (int t = wave; t < K * K + K; t += BIG_NW) {
    const bool isr = t >= K * K;
    const int r = isr ? t - K * K : t / K, c = isr ? 0 : t % K;
    const double* x = BM + (size_t)r * dp;
    const double* y = isr ? YV : ZM + (size_t)c * dp;
    double s = 0.0;
    for (int i = lane; i < dp; i += 64) s += x[i] * y[i];
    s = wave_sum(s);
    if (lane == 0) {
      const double* KS = ws + WL.KS;  // imported S (K x K) and r (K)
      if (isr) {
        const double base = a.border_import ? KS[K * K + r] : big_border_rhs(a, ws, WL, eq, eqr, X, E, r);
        rw[r] = base - s;
      } else {
        const double sv = a.border_import ? KS[r * K + c] : big_border_s(a, ws, WL, E, r, c);
        Ms[r * K + c] = sv - s;
      }
    }
  }
  __syncthreads();

  // (4) LDL^T (right-looking, lanes over rows) and the solve, wave 0
  if (wave == 0) {
    // lower triangle only; the pivot column is snapshotted into lc before the
    // rank-1 update so no lane reads an entry another lane has already scaled
    for (int j = 0; j < K; ++j) {
      const double d = Ms[j * K + j];
      // exactly zero pivot: an extra variable no residual depends on (its row and
      // column are exactly zero) -- held fixed.  A NaN pivot propagates into the
      // step and the trajectory fails the finiteness test in k_big_update.
      const bool skip = d == 0.0;
      for (int i = j + 1 + lane; i < K; i += 64) lc[i] = Ms[i * K + j];
      wave_lds_sync();
      for (int i = j + 1 + lane; i < K; i += 64) {
        const double l = skip ? 0.0 : lc[i] / d;
        for (int c = j + 1; c <= i; ++c) Ms[i * K + c] -= l * lc[c];
        Ms[i * K + j] = l;  // unit-lower L below the diagonal
      }
      if (lane == 0 && skip) Ms[j * K + j] = 0.0;  // D_j = 0 marks a held variable
      wave_lds_sync();
    }
    if (lane == 0) {
      for (int i = 0; i < K; ++i)  // L y = r
        for (int c = 0; c < i; ++c) rw[i] -= Ms[i * K + c] * rw[c];
      for (int i = 0; i < K; ++i) rw[i] = Ms[i * K + i] != 0.0 ? rw[i] / Ms[i * K + i] : 0.0;
      for (int i = K - 1; i >= 0; --i)  // L^T w = y
        for (int c = i + 1; c < K; ++c) rw[i] -= Ms[c * K + i] * rw[c];
    }
  }
  __syncthreads();

  // (5) dx = du - Z w,  dz = w[0:nz]
  for (int i = threadIdx.x; i < dp; i += BIG_NTHREADS) {
    double s = YV[i];
    for (int c = 0; c < K; ++c) s -= ZM[(size_t)c * dp + i] * rw[c];
    YV[i] = s;
  }
  if (threadIdx.x < NZX) ws[WL.DZ + threadIdx.x] = threadIdx.x < nz ? rw[threadIdx.x] : 0.0;
  for (int i = threadIdx.x; i < K; i += BIG_NTHREADS) ws[WL.KS + K * K + K + i] = rw[i];  // w = [dz; lambda]
  if (a.lam)
    for (int i = threadIdx.x; i < nc; i += BIG_NTHREADS) a.lam[(size_t)b * nc + i] = rw[nz + i];
}

// ------------------------------------------------------------ update
// Unbounded problems (bounded ones run k_big_linesearch instead).
template <int n>
__global__ __launch_bounds__(256) void k_big_update(BigArgs a) {
  const int b = blockIdx.x;
  if (a.state[b] != BIG_RUNNING || MHE_BIG_KO) return;  // (timing probes: X frozen)
  const BigWs WL = big_ws_layout(a.P, a.M, n, a.NT, a.nz, a.nc);
  const double* YV = a.ws + (size_t)b * a.ws_stride + WL.YV;
  double* X = a.X + (size_t)b * a.P * n;
  __shared__ double red[8];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  double dmax = 0.0, fin = 0.0;
  const double* DZ = a.ws + (size_t)b * a.ws_stride + WL.DZ;
  if (threadIdx.x < a.nz) {  // extra variables (f4): same stopping rule
    const double dv = DZ[threadIdx.x];
    if (!isfinite(dv)) fin = 1.0;
    dmax = fabs(dv);
  }
  for (int t = threadIdx.x; t < a.P * n; t += 256) {
    const int j = t / n, c = t % n;
    const double dv = YV[c * a.Pp + j];
    if (!isfinite(dv)) fin = 1.0;
    dmax = fmax(dmax, fabs(dv));
  }
  dmax = wave_max(dmax);
  fin = wave_max(fin);
  if (lane == 0) {
    red[wave] = dmax;
    red[4 + wave] = fin;
  }
  __syncthreads();
  dmax = fmax(fmax(red[0], red[1]), fmax(red[2], red[3]));
  fin = fmax(fmax(red[4], red[5]), fmax(red[6], red[7]));
  __syncthreads();
  if (fin != 0.0) {
    if (threadIdx.x == 0) a.state[b] = MHE_STATUS_NONFINITE;
    return;
  }
  double xmax = 0.0;
  if (threadIdx.x < a.nz) {
    double* zp = a.Z + (size_t)b * a.nz + threadIdx.x;
    *zp += DZ[threadIdx.x];
    xmax = fabs(*zp);
  }
  for (int t = threadIdx.x; t < a.P * n; t += 256) {
    const int j = t / n, c = t % n;
    const double xv = X[t] + YV[c * a.Pp + j];
    X[t] = xv;
    xmax = fmax(xmax, fabs(xv));
  }
  xmax = wave_max(xmax);
  if (lane == 0) red[wave] = xmax;
  __syncthreads();
  xmax = fmax(fmax(red[0], red[1]), fmax(red[2], red[3]));
  if (threadIdx.x == 0) {
    a.iters[b] += 1;
    if (dmax <= a.tol * (1.0 + xmax)) a.state[b] = MHE_STATUS_CONVERGED;
  }
}

// Objective at X (node-major, any memory; the extra variables z of mixed rows are
// not supported with bounds): the sums of k_big_resid without Jacobians.  Every
// thread of the block calls it; returns the block total in every thread.
template <class MEAS, int n, bool = MEAS::MIXED>
struct MeasArgLen {  // length of the argument vector h reads: x (n), or [x ; z] for mixed rows
  static constexpr int v = n;
};
template <class MEAS, int n>
struct MeasArgLen<MEAS, n, true> {
  static constexpr int v = MEAS::NA;
};

template <class DYN, class MEAS>
__device__ double big_cost(const BigArgs& a, const double* X, int b, double* red, double& nz_out) {
  constexpr int n = DYN::n, m = DYN::m, p = MEAS::p, q = MEAS::q, NAX = MeasArgLen<MEAS, n>::v;
  const BigConst CL = big_const_layout(a.P, a.M, n, p, a.nc);
  const double* Dt = (const double*)(a.cbuf + CL.Dt);
  const double* cw = (const double*)(a.cbuf + CL.cw);
  const double* Qw = (const double*)(a.cbuf + CL.Qw);
  const double* Pw = (const double*)(a.cbuf + CL.Pw);
  const double* Rw = big_rw(a, (const double*)(a.cbuf + CL.Rw), b);
  const double* PhiET = (const double*)(a.cbuf + CL.PhiET);
  const int* erow = (const int*)(a.cbuf + CL.erow);
  const int E = a.M > 0 ? *(const int*)(a.cbuf + CL.ne) : 0;
  const int Mr = a.M > 0 ? a.M : 1;
  double cost = 0.0, noise = 0.0;
  for (int k = threadIdx.x; k < a.P; k += BIG_NTHREADS) {
    double dx[n], xk[n], uk[m > 0 ? m : 1], f[n];
    for (int c = 0; c < n; ++c) dx[c] = 0.0;
    constexpr int UJ = n <= 8 ? 8 : 2;  // loads in flight; n = 40 (C5) would spill at 8
#pragma unroll UJ
    for (int j = 0; j < a.P; ++j) {
      const double dv = Dt[(size_t)j * a.P + k];
      for (int c = 0; c < n; ++c) dx[c] += dv * X[j * n + c];
    }
    for (int c = 0; c < n; ++c) xk[c] = X[k * n + c];
    if (m > 0) {
      const double* Up = a.U + (long long)b * a.ustride + (long long)k * m;
      for (int c = 0; c < m; ++c) uk[c] = Up[c];
    }
    if constexpr (dyn_sparse<DYN>::value) {
      double Fv[DYN::NNZ];
      DYN::eval_sparse(xk, uk, a.dpar, f, Fv);
    } else {
      double F[n * n];
      DYN::eval(xk, uk, a.dpar, f, F);
    }
    double W[n];
    for (int c = 0; c < n; ++c) W[c] = a.alpha * dx[c] - f[c];
    const double ck = cw[k];
    for (int r = 0; r < n; ++r) {
      if (a.huber) {  // pseudo_huber_loss (cost_functions.py:25-31), as k_big_resid
        const double q = Qw[r * n + r], dl = a.huber_delta;
        cost += ck * (2.0 * q * dl * dl * (sqrt(1.0 + W[r] * W[r] / (dl * dl)) - 1.0));
        continue;
      }
      double s = 0.0;
      for (int c = 0; c < n; ++c) s += Qw[r * n + c] * W[c];
      cost += W[r] * (ck * s);
    }
  }
  for (int e = threadIdx.x; e < E; e += BIG_NTHREADS) {
    double xe[NAX];
    for (int c = 0; c < NAX; ++c) xe[c] = 0.0;
    constexpr int UJ = n <= 8 ? 8 : 2;  // loads in flight; n = 40 (C5) would spill at 8
#pragma unroll UJ
    for (int j = 0; j < a.P; ++j) {
      const double ph = PhiET[(size_t)j * Mr + e];
      for (int c = 0; c < n; ++c) xe[c] += ph * X[j * n + c];
    }
    for (int i = erow[e]; i < erow[e + 1]; ++i) {
      if constexpr (MEAS::MIXED) {
        const double* PR = a.PAR + (long long)b * a.pstride + (long long)i * q;
        const double R = Rw[i];
        if (R == 0.0) continue;
        double h, Gr[NAX];
        MEAS::eval(xe, PR, 0, h, Gr);
        const double yv = a.Y[(long long)b * a.M + i], ev = yv - h;
        cost += ev * (R * ev);
        noise += fabs(R * ev) * (fabs(yv) + fabs(h));
      } else {
        double par[q > 0 ? q : 1];
        if (q > 0) {
          const double* PR = a.PAR + (long long)b * a.pstride + (long long)i * q;
          for (int c = 0; c < q; ++c) par[c] = PR[c];
        }
        const double* R = Rw + (size_t)i * p * p;
        if (masked_row<p>(R)) continue;
        double h[p], Hm[p * n];
        MEAS::eval(xe, par, a.idx, h, Hm);
        const double* yi = a.Y + ((long long)b * a.M + i) * p;
        double ev[p];
        for (int r = 0; r < p; ++r) ev[r] = yi[r] - h[r];
        for (int r = 0; r < p; ++r) {
          double s = 0.0;
          for (int c = 0; c < p; ++c) s += R[r * p + c] * ev[c];
          cost += ev[r] * s;
          noise += fabs(s) * (fabs(yi[r]) + fabs(h[r]));
        }
      }
    }
  }
  if (a.has_prior && threadIdx.x == 0) {
    for (int r = 0; r < n; ++r) {
      double t2 = 0.0;
      for (int c = 0; c < n; ++c) t2 += Pw[r * n + c] * (X[c] - a.x0[(long long)b * n + c]);
      cost += (X[r] - a.x0[(long long)b * n + r]) * t2;
    }
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  cost = wave_sum(cost);
  noise = wave_sum(noise);
  __syncthreads();
  if (lane == 0) {
    red[wave] = cost;
    red[BIG_NW + wave] = noise;
  }
  __syncthreads();
  double c = 0.0, z = 0.0;
  for (int w = 0; w < BIG_NW; ++w) {
    c += red[w];
    z += red[BIG_NW + w];
  }
  __syncthreads();
  nz_out = COST_NOISE * __DBL_EPSILON__ * z;
  return c;
}

// Bounded problems: replaces k_big_update.  Stationarity measure s = P(X + d) - X,
// Armijo search along P(X + a d) (trial iterates in LDS, cost by big_cost), X <-
// accepted trial, convergence max|s| <= tol (1 + max|X|).  Constants as k_gn_bounded.
template <class DYN, class MEAS>
__global__ __launch_bounds__(BIG_NTHREADS) void k_big_linesearch(BigArgs a) {
  constexpr int n = DYN::n;
  const int b = blockIdx.x;
  if (a.state[b] != BIG_RUNNING) return;
  const BigWs WL = big_ws_layout(a.P, a.M, n, a.NT, a.nz, a.nc);
  const double* ws = a.ws + (size_t)b * a.ws_stride;
  const double* YV = ws + WL.YV;
  const double* GV = ws + WL.GV;  // -g at X (k_big_resid; BV now holds the forward solve)
  const int* ACT = (const int*)(ws + WL.ACT);
  double* X = a.X + (size_t)b * a.P * n;
  extern __shared__ __attribute__((aligned(16))) double xt[];  // trial iterate (P, n)
  __shared__ double red[2 * BIG_NW];
  double smax = 0.0, fin = 0.0;
  for (int t = threadIdx.x; t < a.P * n; t += BIG_NTHREADS) {
    const int j = t / n, c = t % n;
    double lo, hi;
    big_box(a, c, lo, hi);
    const double x = X[t], dv = YV[c * a.Pp + j];
    if (!isfinite(dv)) fin = 1.0;
    smax = fmax(smax, fabs(fmin(fmax(x + dv, lo), hi) - x));
  }
  big_max2(red, smax, fin);
  if (fin != 0.0) {
    if (threadIdx.x == 0) a.state[b] = MHE_STATUS_NONFINITE;
    return;
  }
  const double cost0 = a.cost[b];  // k_big_resid at X
  const double nz0 = ws[WL.NZ];    // its rounding level (Armijo slack, as k_gn_bounded)
  double alpha = 1.0;
  for (int ls = 0;;) {
    double pred = 0.0;
    for (int t = threadIdx.x; t < a.P * n; t += BIG_NTHREADS) {
      const int j = t / n, c = t % n;
      double lo, hi;
      big_box(a, c, lo, hi);
      const int u = c * a.Pp + j;
      const double x = X[t], dv = YV[u], g = -GV[u];
      const double xv = fmin(fmax(x + alpha * dv, lo), hi);
      pred += ACT[u] ? g * (xv - x) : alpha * g * dv;
      xt[t] = xv;
    }
    __syncthreads();
    double nzt;
    const double ct = big_cost<DYN, MEAS>(a, xt, b, red, nzt);
    pred = wave_sum(pred);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = pred;
    __syncthreads();
    pred = 0.0;
    for (int w = 0; w < BIG_NW; ++w) pred += red[w];
    __syncthreads();
    ++ls;
    if (ct <= cost0 + 2.0 * ARMIJO_SIGMA * pred + nz0 + nzt + COST_SLACK * fabs(cost0) || ls >= LS_MAX) break;
    alpha *= 0.5;
  }
  double xn = 0.0, z = 0.0;
  for (int t = threadIdx.x; t < a.P * n; t += BIG_NTHREADS) {
    X[t] = xt[t];
    xn = fmax(xn, fabs(xt[t]));
  }
  big_max2(red, xn, z);
  if (threadIdx.x == 0) {
    a.iters[b] += 1;
    if (smax <= a.tol * (1.0 + xn)) a.state[b] = MHE_STATUS_CONVERGED;
  }
}

// X <- P(X) (bounded problems: the projected Newton method starts inside the box)
template <int n>
__global__ void k_big_project(BigArgs a, int batch) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (size_t)batch * a.P * n || a.state[t / ((size_t)a.P * n)] != BIG_RUNNING) return;
  double lo, hi;
  big_box(a, (int)(t % n), lo, hi);
  a.X[t] = fmin(fmax(a.X[t], lo), hi);
}
