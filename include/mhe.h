/*
 * mhe.h -- C-ABI of libmhe.so, the MI355X (gfx950) batched collocation
 * Gauss-Newton estimator.
 *
 * This is the drop-in boundary under the reference's solver facade:
 *
 *   reference                                   replaced by
 *   ------------------------------------------  -----------------------------------
 *   NLP.build()      nlp/nlp.py:61-69           mhe_const_bytes + mhe_build_constants
 *   NLP.solve()      nlp/nlp.py:76-83           mhe_gn_solve  (CasADi Opti + IPOPT ->
 *                                               hand-written HIP Gauss-Newton)
 *   addDynamics/addDynamicsCost/addResidualCost/addInitialCost
 *                    nlp/nlp.py:202-286         the objective those calls record is
 *                                               what mhe_gn_solve minimises; its pieces
 *                                               are exported for kernel-level parity:
 *                                               mhe_assemble (J^T W J, J^T W r, cost)
 *                                               mhe_chol_solve (dense SPD solve)
 *   extractSolution  nlp/nlp.py:99-119          host side (Lagrange interpolation)
 *
 * Conventions
 *   - every pointer argument except `dims` and the host-side constant tables
 *     of mhe_build_constants is a DEVICE pointer owned by the caller (torch
 *     tensors in the Python host; hipMalloc'd memory from C);
 *   - fp64 everywhere, row-major, batch outermost; a batch stride of 0 means
 *     "shared by every trajectory";
 *   - no hidden allocation, no host synchronisation: every call only enqueues
 *     work on `stream` (graph-capturable);
 *   - returns MHE_OK (0) or a negative MHE_ERR_* code; per-trajectory solver
 *     outcomes are reported in `status_out` (MHE_STATUS_*), never by aborting
 *     the batch;
 *   - calls that share a constants buffer may run concurrently on different
 *     streams; a constants buffer is read-only after mhe_build_constants.
 */
#ifndef MHE_H
#define MHE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* return codes */
#define MHE_OK 0
#define MHE_ERR_DIMS (-1)        /* dims inconsistent with the models / limits */
#define MHE_ERR_MODEL (-2)       /* unknown dynamics or measurement model id   */
#define MHE_ERR_HIP (-3)         /* a HIP runtime call failed                  */
#define MHE_ERR_UNSUPPORTED (-4) /* valid request this build does not handle   */
#define MHE_ERR_NULL (-5)        /* required pointer is NULL                   */

/* per-trajectory solver status (status_out) */
#define MHE_STATUS_CONVERGED 0   /* max|delta| <= tol * (1 + max|X|)           */
#define MHE_STATUS_MAX_ITER 1    /* max_iter Gauss-Newton steps taken          */
#define MHE_STATUS_NOT_SPD 2     /* Cholesky pivot <= 0 (J^T W J not SPD)      */
#define MHE_STATUS_NONFINITE 3   /* NaN/Inf in the step                        */
#define MHE_STATUS_BAD_CONSTANTS 4 /* const_buf was not built for these dims (its tag
                                      differs): nothing was computed, X_out = X0     */

/* dynamics plug-ins (reference nlp/dynamics.py) */
#define MHE_DYN_SINGLE_INTEGRATOR 1      /* :4-8    n=1  m=1 */
#define MHE_DYN_SINGLE_INTEGRATOR_2D 2   /* :10-17  n=2  m=2 */
#define MHE_DYN_SINGLE_INTEGRATOR_3D 3   /* :19-27  n=3  m=3 */
#define MHE_DYN_DOUBLE_INTEGRATOR 4      /* :29-38  n=4  m=2 */
#define MHE_DYN_VAN_DER_POL 5            /* :61-66  n=2  m=1 */
#define MHE_DYN_GNSS_POS_AND_BIAS 6      /* :68-79  n=5  m=3 */
#define MHE_DYN_MULTI_RECEIVER 7         /* :81-96  n=8  m=0 */
#define MHE_DYN_GNSS_TWO_RECEIVER 8      /* :98-115 n=10 m=6 */
#define MHE_DYN_KINEMATIC_BICYCLE 9      /* :117-136 n=6 m=2 (kinematic_bycicle_and_bias) */
#define MHE_DYN_GNSS_8_RECEIVERS 11      /* 8 receivers x the :98-115 block [x,y,z,b,alpha]:
                                            n=40 m=24 */
#define MHE_DYN_VEHICLE_GNSS 10          /* :148-174 n=9 m=2 (vehicle_dynamics_and_gnss);
                                            dyn_par = params["car_params"] as
                                            [C_AF, C_AR, M, D_F, D_R, I_Z] */

/* measurement plug-ins (reference nlp/measurements.py) */
#define MHE_MEAS_FULL_STATE 1            /* :4-5   p=n, linear            */
#define MHE_MEAS_PSEUDORANGE 2           /* :56-70 p=1, q=3 (sat_pos), idx[4] */
#define MHE_MEAS_VEHICLE_PSEUDORANGE 3   /* :81-88 p=1, q=3 (x[0], x[1], x[8]; bias x[6]) */
#define MHE_MEAS_RANGE_3D 4              /* :39-54 p=1, q=3 ("y" form), idx[3] */
#define MHE_MEAS_MIXED 5                 /* several scalar plug-ins in one problem (one
                                            addResidualCost call each, nlp/nlp.py:258-277):
                                            p=1, q=MHE_MIXED_Q, every row names its model */

/* MHE_MEAS_MIXED rows: PAR row = [code, i0..i6, v0..v5] (q = 14).  Indices point
 * into the augmented vector [x(t_i) (n) ; z (n_extra)] -- z are the extra decision
 * variables (addVariables beyond the state, e.g. XA in multi-receiver.py:73,99);
 * -1 = unused term.  h per code (reference nlp/measurements.py):
 *   PSEUDORANGE       :56-70  |x[i0..i2] - v0..2| + x[i3]
 *   PSEUDORANGE_RATE  :72-79  (v3..5 - x[i3..i5]) . (v0..2 - x[i0..i2]) / |.| + x[i6]
 *   RANGE_2D          :7-20   sqrt(sum_k (x[i_k] - x[i_{k+2}] - v_k)^2 + 1e-6), k < 2
 *   RANGE_3D          :39-54  sqrt(sum_k (x[i_k] - x[i_{k+3}] - v_k)^2 + 1e-6), k < 3
 *                             (both forms: "idxA/idxB" -> i = A, B; "y" -> i = idx, -1
 *                             and v = y, or with y a decision variable i = idx, n + j)
 *   HEADING_2D        :22-37  atan2(x[i0] - x[i1] + v0, x[i2] - x[i3] + v1)
 *   COMPONENT         :4-5    x[i0] (full_state as scalar rows)
 *   NONE                      h = 0 (padding row; give it R = 0) */
#define MHE_MIXED_Q 14
#define MHE_ROW_NONE 0
#define MHE_ROW_PSEUDORANGE 1
#define MHE_ROW_PSEUDORANGE_RATE 2
#define MHE_ROW_RANGE_2D 3
#define MHE_ROW_RANGE_3D 4
#define MHE_ROW_HEADING_2D 5
#define MHE_ROW_COMPONENT 6
#define MHE_MAX_EXTRA 4   /* extra decision variables per trajectory */
#define MHE_MAX_EQ 48     /* n_extra + n_eq */

/* Every dims struct starts with struct_size: the caller sets it to sizeof() of
 * the struct it declares, and every entry point returns MHE_ERR_DIMS (0 / -1 for
 * the size queries) unless it equals this build's sizeof -- a binding that
 * declares an older or truncated struct is refused before any later field is
 * read.  (mhe/_lib.py sets it in the ctypes constructors.) */
#define MHE_ABI_VERSION 7

typedef struct mhe_dims {
  int32_t struct_size;  /* = sizeof(mhe_dims)                                */
  int32_t N;            /* collocation order; P = N + 1 CGL nodes            */
  int32_t n;            /* state dimension   (must equal the model's)        */
  int32_t m;            /* control dimension (must equal the model's)        */
  int32_t p;            /* rows of one measurement (model's)                 */
  int32_t M;            /* number of measurement times in the window         */
  int32_t q;            /* per-row measurement parameters (0 if none)        */
  int32_t dyn_model;    /* MHE_DYN_*                                         */
  int32_t meas_model;   /* MHE_MEAS_*                                        */
  int32_t has_prior;    /* 1: addInitialCost term present                    */
  int32_t meas_idx[8];  /* static index params (params["idx"]), model-defined */
  double T;             /* window length; node times tau2t(tau)              */
  int32_t dyn_cost;     /* MHE_COST_L2 (weighted_l2_norm) or MHE_COST_HUBER  */
  int32_t n_bounds;     /* addVarBounds: number of bounded state components  */
  double huber_delta;   /* pseudo_huber_loss params["delta"]                 */
  int32_t bound_idx[8]; /* bounded component indices (< n)                   */
  double bound_lb[8];   /* lower / upper bounds (+-inf allowed), every node  */
  double bound_ub[8];
  int32_t n_extra;      /* extra decision variables z (<= MHE_MAX_EXTRA); they
                           enter MHE_MEAS_MIXED rows only                        */
  int32_t n_eq;         /* addEqConstraint(equality_constaint, [a, b]) rows
                           (nlp/nlp.py:52-53, nlp/constraints.py): v[a] - v[b] = 0 */
  const int32_t* eq_idx;/* HOST pointer, 2*n_eq entries (a, b) into the flattened
                           state vector v = X (P*n, node-major: j*n + c); b = -1
                           means v[a] = 0.  Copied into the constants buffer at
                           build time and part of its layout stamp (with eq_rhs):
                           solving with other rows than the buffer was built with
                           returns MHE_STATUS_BAD_CONSTANTS -- rebuild instead.     */
  int32_t force_large;  /* 1: take the large-system path even when the problem fits
                           the register-resident kernel (parity tests of the two
                           paths on identical inputs).  The path is a function of
                           dims alone; mhe_build_constants stamps it (with the
                           layout-defining dims) into the constants buffer and every
                           solve checks that stamp on the device.                 */
  double dyn_par[8];    /* static dynamics parameters (model-defined, e.g.
                           MHE_DYN_VEHICLE_GNSS); 0 for the parameter-free models   */
  const double* eq_rhs; /* HOST pointer, n_eq constants r_i of the rows
                           v[a] - v[b] = r_i, or NULL (all 0: addEqConstraint rows).
                           Non-zero r: the rows an active set imposes (bounds and
                           inequality constraints held at equality by the host) */
} mhe_dims;

/* Dynamics cost (addDynamicsCost, nlp/nlp.py:242-245): */
#define MHE_COST_L2 0     /* cost_functions.weighted_l2_norm  (cost_functions.py:20-22) */
#define MHE_COST_HUBER 1  /* cost_functions.pseudo_huber_loss (cost_functions.py:25-31): IRLS
                             weights q_a / sqrt(1 + W_a^2 / delta^2), only diag(Qw) enters */
/* Bounds (addVarBounds, nlp/nlp.py:314-317) are enforced by a projected Newton
 * method on the GN model (Bertsekas 1982): the iterate starts projected onto the
 * box, each step is the GN step reduced to the free unknowns (epsilon-active set)
 * followed by an Armijo search along the projection arc; MHE_STATUS_CONVERGED
 * then means a KKT point of the bounded problem (max|P(X + d) - X| <= tol (1 + max|X|)).
 * Extra variables and equality constraints run on the
 * large-system path: each GN step solves the bordered (KKT) system
 *   [ H    H_xz  C^T ] [dx]   [-g  ]
 *   [ H_zx H_zz  0   ] [dz] = [-g_z]
 *   [ C    0     0   ] [l ]   [-c  ]
 * through the Cholesky factor of H (one multi-RHS solve of the border columns,
 * a small quasi-definite LDL^T of the Schur complement).  Linear constraints are
 * therefore met exactly after every step.  Bounds and constraints together are
 * not supported (MHE_ERR_UNSUPPORTED). */

/* Process-wide A/B options, for measurements and tests only; nothing else (no
 * environment variable) changes what a solve runs.  Returns the previous value, or
 * MHE_ERR_DIMS for an unknown option or a value out of range.
 *   MHE_OPT_BIG_RIGHT_LOOKING  1: the large-system factorization's right-looking
 *                              trailing-update form (bitwise-identical iterates,
 *                              slower); 0 (default): left-looking block columns
 *   MHE_OPT_DEBUG_SMEM_PAD     bytes of LDS added to the fused kernel's launch
 *                              (forces lower occupancy; default 0)
 * Not thread-safe against concurrent launches: set it before enqueueing work. */
#define MHE_OPT_BIG_RIGHT_LOOKING 1
#define MHE_OPT_DEBUG_SMEM_PAD 2
int32_t mhe_set_option(int32_t option, int32_t value);

/* Size in bytes of the device constants buffer for `dims` (0 on bad dims).  The
 * first 256 bytes are a header holding the layout stamp written by
 * mhe_build_constants (offset 0: every solve checks it in bounds). */
size_t mhe_const_bytes(const mhe_dims* dims);

/*
 * Build the per-problem device constants (one-time, NLP.build()).
 *   D    (P,P)    negated CGL differentiation matrix   (collocation.py:42-64)
 *   cw   (P)      (T/2) * w_k, w the reference weights   (nlp/nlp.py:245)
 *   Phi  (M,P)    Lagrange basis at the measurement times (nlp/nlp.py:266)
 *   Qw   (n,n)    dynamics-cost weight = params["Q"] of weighted_l2_norm
 *   Rw   (M,p,p)  measurement information R passed to addResidualCost
 *   Pw   (n,n)    prior weight (may be NULL when !has_prior)
 * All six are DEVICE pointers; `const_buf` is a caller-owned device buffer of
 * mhe_const_bytes(dims) bytes.
 */
int mhe_build_constants(const mhe_dims* dims, const double* D, const double* cw,
                        const double* Phi, const double* Qw, const double* Rw,
                        const double* Pw, void* const_buf, void* stream);

/*
 * Batched Gauss-Newton solve (NLP.solve()).  One trajectory per workgroup;
 * the whole GN loop (residual + Jacobian, J^T W J / J^T W r assembly,
 * Cholesky, triangular solves, update) runs inside one launch.
 *   X0     (B,P,n)    initial iterate (warm start = previous solution)
 *   X_out  (B,P,n)    solution (may alias X0)
 *   U      (B|1,P,m)  controls at the nodes (setControl, nlp/nlp.py:304-308);
 *                     NULL when m == 0
 *   Y      (B,M,p)    measurements
 *   PAR    (B|1,M,q)  per-row measurement params (sat_pos ...); NULL if q == 0
 *   x0     (B,n)      prior mean (addInitialCost); NULL when !has_prior
 *   cost_out (B) objective at X_out; iters_out (B) GN steps; status_out (B)
 */
int mhe_gn_solve(const mhe_dims* dims, const void* const_buf, int32_t batch,
                 const double* X0, double* X_out,
                 const double* U, int64_t u_bstride,
                 const double* Y,
                 const double* PAR, int64_t par_bstride,
                 const double* x0,
                 double* cost_out, int32_t* iters_out, int32_t* status_out,
                 int32_t max_iter, double tol, void* stream);

/* Padded system size used by the kernels: 16 * ceil(P*n / 16) on the
 * register-resident path (<= 208); n * 16 * ceil(P / 16) (component-major
 * ordering) on the large-system path. */
int32_t mhe_padded_dim(const mhe_dims* dims);

/*
 * Workspace the large-system path needs for `batch` trajectories (bytes; 0 when
 * the problem fits the register-resident kernel, which needs none).  Holds the
 * per-trajectory H tiles, L_kk^-T blocks and iteration scratch.
 */
size_t mhe_workspace_bytes(const mhe_dims* dims, int32_t batch);

/*
 * mhe_gn_solve with a caller-owned device workspace of >= mhe_workspace_bytes
 * (required when the padded system exceeds the register-resident limit: C3-C5,
 * d = 1005 / 3006 / 8040).  Same arguments and results as mhe_gn_solve, which is
 * this call with workspace = NULL (and returns MHE_ERR_NULL for such problems).
 * Enqueues max_iter iterations of stream-ordered kernels; trajectories that
 * converge or fail are frozen on the device, so no host synchronisation occurs.
 */
int mhe_gn_solve_ws(const mhe_dims* dims, const void* const_buf, int32_t batch,
                    const double* X0, double* X_out,
                    const double* U, int64_t u_bstride,
                    const double* Y, const double* PAR, int64_t par_bstride,
                    const double* x0,
                    double* cost_out, int32_t* iters_out, int32_t* status_out,
                    int32_t max_iter, double tol, void* workspace, size_t workspace_bytes,
                    void* stream);

/*
 * mhe_gn_solve_ws with extra decision variables: Z0 / Z_out (B, n_extra) device
 * arrays (initial values / solution; NULL when n_extra == 0).  Problems with
 * n_extra > 0, n_eq > 0 or MHE_MEAS_MIXED always take the large-system path
 * (workspace required).  The stopping rule covers z too:
 * max|(dx, dz)| <= tol * (1 + max|(X, z)|).
 */
int mhe_gn_solve_ext(const mhe_dims* dims, const void* const_buf, int32_t batch,
                     const double* X0, double* X_out, const double* Z0, double* Z_out,
                     const double* U, int64_t u_bstride,
                     const double* Y, const double* PAR, int64_t par_bstride,
                     const double* x0,
                     double* cost_out, int32_t* iters_out, int32_t* status_out,
                     int32_t max_iter, double tol, void* workspace, size_t workspace_bytes,
                     void* stream);

/*
 * All solve inputs and outputs in one struct (the entry point new bindings use;
 * mhe_gn_solve / _ws / _ext are this call with Rw = NULL).  Pointers as
 * mhe_gn_solve_ext, plus
 *   Rw  (B|1, M, p, p)  per-solve measurement information, overriding the Rw the
 *                       constants were built with (batch stride rw_bstride, 0 =
 *                       shared; M scalars per trajectory for MHE_MEAS_MIXED).  The
 *                       reference's MHE windows re-set R every window (R = 0 masks
 *                       empty satellite slots, autonomous-car.py:250-263,
 *                       gnss-multi-receiver.py:186-204): passing it here keeps one
 *                       constants buffer for all windows.  Nonlinear measurement
 *                       models only (a linear h has Rw folded into the constant
 *                       part of J^T W J): MHE_ERR_UNSUPPORTED otherwise.
 */
typedef struct mhe_solve_args {
  int32_t struct_size;     /* = sizeof(mhe_solve_args) */
  int32_t batch;
  const double* X0;
  double* X_out;
  const double* Z0;        /* extra variables (n_extra > 0), else NULL */
  double* Z_out;
  const double* U;
  int64_t u_bstride;
  const double* Y;
  const double* PAR;
  int64_t par_bstride;
  const double* Rw;        /* optional, see above */
  int64_t rw_bstride;
  const double* x0;
  double* cost_out;
  int32_t* iters_out;
  int32_t* status_out;
  int32_t max_iter;
  double tol;
  void* workspace;         /* large-system path: >= mhe_workspace_bytes(dims, batch) */
  size_t workspace_bytes;
  double* lambda_out;      /* optional (B, n_eq): multipliers of the constraint rows from the
                              last bordered step, L = J + lambda^T (C v - r) (their signs
                              drive the host's active set), or NULL */
} mhe_solve_args;

int mhe_solve(const mhe_dims* dims, const void* const_buf, const mhe_solve_args* args, void* stream);

/*
 * Kernel-level parity of the per-collocation-point evaluation (SURVEY §8(a) a5-a7,
 * nlp/nlp.py:225-235 and :264-273): at X (B,P,n) with the solve's device functors,
 *   W  (B,P,n)    W_k = (2/T) sum_j D_kj X_j - f(X_k, U_k)   (the eliminated defects)
 *   F  (B,P,n,n)  df/dx at (X_k, U_k)
 *   E  (B,M,p)    e_i = y_i - h(x(t_i)),  x(t_i) = sum_j Phi_ij X_j
 *   Hm (B,M,p,n)  dh/dx at x(t_i)
 * Any output may be NULL.  Both paths; not for MHE_MEAS_MIXED (MHE_ERR_UNSUPPORTED).
 * A constants buffer built for other dims leaves the outputs untouched.
 */
int mhe_resjac(const mhe_dims* dims, const void* const_buf, int32_t batch, const double* X, const double* U,
               int64_t u_bstride, const double* Y, const double* PAR, int64_t par_bstride, double* W,
               double* F, double* E, double* Hm, void* stream);

/*
 * Kernel-level parity: assemble the GN normal equations at X.
 *   H (B,dp,dp) full symmetric (dp = mhe_padded_dim; padding rows = identity),
 *   g (B,dp) gradient J^T W r (padding 0), cost (B).
 * Register-resident path only (MHE_ERR_UNSUPPORTED on the large-system path, which
 * needs a workspace: mhe_assemble_ws / mhe_chol_solve_ws below).
 */
int mhe_assemble(const mhe_dims* dims, const void* const_buf, int32_t batch,
                 const double* X, const double* U, int64_t u_bstride,
                 const double* Y, const double* PAR, int64_t par_bstride,
                 const double* x0, double* H, double* g, double* cost, void* stream);

/*
 * Kernel-level parity: solve H delta = -g for a batch of SPD matrices with the
 * solver's register-tiled Cholesky.  H (B,dp,dp) (lower triangle read),
 * g (B,dp), delta (B,dp), status (B).  `const_buf` is any constants buffer
 * built for `dims` (only its tile table is read).
 */
int mhe_chol_solve(const mhe_dims* dims, const void* const_buf, int32_t batch,
                   const double* H, const double* g, double* delta, int32_t* status,
                   void* stream);

/*
 * Both kernel-level parity entry points for EVERY path (ABI v5+): on the register-
 * resident path they are mhe_assemble / mhe_chol_solve (workspace ignored, status
 * set to 0 by the assembly); on the large-system path (C3-C5, mhe_workspace_bytes > 0)
 * they run the solve's own kernels over a caller-owned workspace of
 * >= mhe_workspace_bytes(dims, batch) bytes:
 *   mhe_assemble_ws    k_big_resid + k_big_assemble at X, then H and g copied out of
 *                      the kernels' component-major tiles into the SAME dense node-major
 *                      layout as mhe_assemble: H (B,dp,dp), g (B,dp), dp = mhe_padded_dim
 *                      = n * Pp, row j*n + c for node j < Pp (the first P*n rows are the
 *                      oracle's order; padding nodes last: identity block, zero coupling,
 *                      zero gradient), cost (B), status (B): 0, or
 *                      MHE_STATUS_BAD_CONSTANTS (outputs NaN).  The plain GN system
 *                      (bounds are a solve-time reduction).  n_extra / n_eq > 0: the
 *                      bordered KKT system of mhe_assemble_kkt_ws below (Z = NULL, so
 *                      n_extra > 0 returns MHE_ERR_NULL here: use the _kkt_ form).
 *   mhe_chol_solve_ws  H (lower triangle read, node-major as above) and g into the
 *                      tiles, k_big_chol (blocked Cholesky + both triangular solves),
 *                      delta = -H^-1 g (B,dp) node-major; status 0, MHE_STATUS_NOT_SPD
 *                      (non-positive or non-finite pivot; delta NaN) or BAD_CONSTANTS.
 *                      n_extra / n_eq > 0 (ABI v6): H, g, delta are the KKT system of
 *                      mhe_kkt_dim rows below, solved as every bordered GN step is
 *                      (k_big_chol on the leading block, then k_big_border: the border
 *                      columns through the factor, LDL^T of the Schur complement);
 *                      delta = [dx; dz; lambda].
 */
int mhe_assemble_ws(const mhe_dims* dims, const void* const_buf, int32_t batch,
                    const double* X, const double* U, int64_t u_bstride,
                    const double* Y, const double* PAR, int64_t par_bstride,
                    const double* x0, double* H, double* g, double* cost, int32_t* status,
                    void* workspace, size_t workspace_bytes, void* stream);
int mhe_chol_solve_ws(const mhe_dims* dims, const void* const_buf, int32_t batch,
                      const double* H, const double* g, double* delta, int32_t* status,
                      void* workspace, size_t workspace_bytes, void* stream);

/*
 * Kernel-level parity of the BORDERED system (ABI v6; SURVEY §8 f4: extra decision
 * variables z, nlp/nlp.py:40-47 addVariables used by multi-receiver.py:73,99, and
 * addEqConstraint rows, nlp/nlp.py:49-53 / gnss-multi-receiver.py:76-78).  Each
 * bordered GN step solves, with K = n_extra + n_eq and dk = mhe_kkt_dim = dp + K,
 *   [ H    H_xz  C^T ] [dx]     [ g_x       ]
 *   [ H_zx H_zz  0   ] [dz] = - [ g_z       ]     (rows C v - r of the constraints)
 *   [ C    0     0   ] [l ]     [ C v - r   ]
 * mhe_assemble_kkt_ws exports that matrix (B,dk,dk) and right-hand side g (B,dk) at
 * (X, Z): the leading dp x dp block is mhe_assemble_ws's node-major H, then the z rows,
 * then the constraint rows, in the values the solve's own k_big_resid / k_big_border
 * form (Z (B, n_extra) device array; NULL when n_extra == 0).  K = 0: exactly
 * mhe_assemble_ws.  mhe_chol_solve_ws takes the same shapes back (see above).
 */
int32_t mhe_kkt_dim(const mhe_dims* dims);

/* The kernel(s) a solve of `batch` trajectories on `stream` would run, as text into buf
 * (len bytes, NUL-terminated): the register path's k_gn instance -- chosen by the same
 * function as the launch (batch vs the stream device's CUs, Huber, bounds, LDS fit) --
 * or the large-system path's kernel sequence.  Host-only query; launches nothing.
 * (bench.py names the roofline record's kernel with it.) */
int32_t mhe_solve_kernel_name(const mhe_dims* dims, int32_t batch, void* stream, char* buf, int32_t len);

/* The envelope the large-system path's split factorization used (ABI v7): for
 * trajectory `traj` of the last solve / mhe_chol_solve_ws run on `workspace`
 * (workspace_bytes as passed there), the first nonzero tile column of each of its
 * NT = dp / 16 component-major tile rows (the factor has no nonzero tile left of it;
 * the left-looking updates and the backward solve skip those tiles), NT int32 into
 * first_col (n_out >= NT).  Formed on the device from the component pairs whose block
 * of H has a nonzero element at the iterate.  Synchronises `stream` (a copy to the
 * host); returns NT, MHE_ERR_UNSUPPORTED on the register path or in a build without
 * the envelope (every column then starts at 0), MHE_ERR_NULL / MHE_ERR_DIMS on bad
 * arguments.  Used by tools/bench_big.py for the executed flop count. */
int32_t mhe_big_envelope(const mhe_dims* dims, const void* workspace, size_t workspace_bytes, int32_t traj,
                         int32_t* first_col, int32_t n_out, void* stream);
int mhe_assemble_kkt_ws(const mhe_dims* dims, const void* const_buf, int32_t batch,
                        const double* X, const double* Z, const double* U, int64_t u_bstride,
                        const double* Y, const double* PAR, int64_t par_bstride,
                        const double* x0, double* H, double* g, double* cost, int32_t* status,
                        void* workspace, size_t workspace_bytes, void* stream);

/* ------------------------------------------------------------------------
 * Batched extended Kalman filter.
 * Replaces utils/ekf.py:20-61 (EKF.update / predict / correct) with the
 * utils/gnss.py plug-ins, for `batch` independent filter instances, `steps`
 * updates each, in one launch (one wavefront per instance).
 * ------------------------------------------------------------------------ */
#define MHE_EKF_DYN_GNSS_POS_AND_BIAS 1          /* utils/gnss.py:79-90 (n=5, m=3, params dt) */
#define MHE_EKF_MEAS_MULTI_PSEUDORANGE 1         /* utils/gnss.py:27-45 (q=3: sat ENU position) */
#define MHE_EKF_MEAS_MULTI_PSEUDORANGE_AND_BIAS 2 /* utils/gnss.py:48-61 (last row: bias, zero Jacobian row) */
/* the autonomous-car script's own EKF plug-ins (autonomous-car.py:18-77) */
#define MHE_EKF_DYN_DISCRETE_VEHICLE 2           /* discrete_vehicle_dynamics :18-52 (n=9, m=2; params dt,
                                                    car_params -> dyn_par = [C_AF, C_AR, M, D_F, D_R, I_Z]) */
#define MHE_EKF_MEAS_VEHICLE_SENSORS 3           /* vehicle_sensors_model :54-77 (q=3: sat ENU position;
                                                    rows of multi_pseudorange on x[0, 1, 8, 6, 7]) */

typedef struct mhe_ekf_dims {
  int32_t struct_size; /* = sizeof(mhe_ekf_dims) */
  int32_t n, m;        /* state and control sizes of the dynamics model */
  int32_t pmax;        /* row capacity of Z / PAR / R per step (<= 32) */
  int32_t q;           /* parameters per measurement row (3) */
  int32_t dyn_model;   /* MHE_EKF_DYN_* */
  int32_t meas_model;  /* MHE_EKF_MEAS_* */
  double dt;           /* dyn_func_params["dt"] */
  int32_t r_diag;      /* 1: the caller guarantees every step's R block is diagonal -> the
                          correction runs as sequential scalar updates, one filter per lane
                          (same result as the batch update up to rounding); 0: general R,
                          one wavefront per filter with an augmented Cholesky sweep */
  int32_t hist_batch_inner; /* 1: mu_hist is (steps, n, B) and S_hist (steps, n, n, B) --
                               batch innermost, so a wavefront's history stores coalesce;
                               0: (B, steps, n) / (B, steps, n, n) as below */
  int32_t in_batch_inner;   /* 1: U (steps, m, B), Z (steps, pmax, B), nz (steps, B), PAR
                               (steps, pmax, q, B) -- batch innermost (coalesced reads; the
                               *_bstride arguments are ignored); 0: the layouts below */
  double dyn_par[8];        /* static dynamics parameters (MHE_EKF_DYN_DISCRETE_VEHICLE: the car
                               constants; unused by gnss_pos_and_bias) */
} mhe_ekf_dims;

/*
 * All pointers are device pointers; a batch stride of 0 broadcasts one array to
 * every instance.  Per instance b and step k:
 *   U   (steps, m)                      at U   + b*u_bstride
 *   Z   (steps, pmax), rows 0..nz-1     at Z   + b*z_bstride   (z, utils/ekf.py:20)
 *   nz  (steps) valid rows; 0 = no measurement (predict only, utils/ekf.py:30-38)
 *   PAR (steps, pmax, q)                at PAR + b*par_bstride (meas_func_params)
 *   R   leading nz x nz block of (pmax, pmax) at R + b*r_bstride + k*r_sstride
 *   Q   (n, n) shared.
 * mu (B,n) and S (B,n,n) hold the prior on entry and the final state on exit;
 * mu_hist (B,steps,n) / S_hist (B,steps,n,n) (optional) receive the state after
 * every update; status (B, optional): 0 ok, 1 innovation covariance not SPD,
 * 2 nz > 32.  Returns MHE_OK or a negative MHE_ERR_*.
 */
int mhe_ekf_run(const mhe_ekf_dims* dims, int32_t batch, int32_t steps, double* mu, double* S,
                const double* U, int64_t u_bstride, const double* Z, int64_t z_bstride,
                const int32_t* nz, int64_t nz_bstride, const double* PAR, int64_t par_bstride,
                const double* Q, const double* R, int64_t r_bstride, int64_t r_sstride,
                double* mu_hist, double* S_hist, int32_t* status, void* stream);

/* ------------------------------------------------------------------------
 * Batched GNSS least-squares fixes (the MHE initialiser).
 * Replaces utils/leastsquares.py:19-42 (iterativeLeastSquares),
 * :45-63 (iterativeLeastSquaresVel) and the per-epoch loop of
 * runLeastSquares (:97-141) for `chains` logs of `epochs` epochs each.
 * ------------------------------------------------------------------------ */
typedef struct mhe_ls_dims {
  int32_t struct_size; /* = sizeof(mhe_ls_dims) */
  int32_t slots;     /* satellite slots per epoch in the arrays (<= 64) */
  int32_t max_iter;  /* maxiter of iterativeLeastSquares (reference default 100); 0 = no position
                        iterations (velocity at x_init: iterativeLeastSquaresVel alone) */
  int32_t warm;      /* 1: epochs of a chain run in order, each starting from the previous fix
                        (the reference's shared default x, utils/leastsquares.py:19,34);
                        0: every epoch starts from x_init (all epochs in parallel) */
  int32_t with_vel;  /* 1: also the velocity / bias-rate solve (utils/leastsquares.py:45-63) */
  double tol;        /* stop when ||dx|| < tol (reference: 1e-7) */
} mhe_ls_dims;

/*
 * Device pointers.  Per chain c and epoch k (e = c*epochs + k):
 *   sat_pos (C,T,slots,3) ECEF, pr (C,T,slots), nsat (C,T): rows 0..nsat-1 valid
 *   sat_vel (C,T,slots,3), pr_rate (C,T,slots): only with with_vel
 *   x_init (C,3): starting position (b starts at 0 every epoch, as the reference)
 * Outputs: x_out (C,T,3), b_out (C,T), v_out (C,T,3) / bd_out (C,T) with with_vel
 * (NaN where the velocity system is singular: velocity failure alone leaves
 * iters_out untouched), iters_out (C,T) position GN steps taken (-1: fewer than 4
 * independent satellites for the position fix),
 * x_last (C,3, optional, warm only) the chain's final position (the value the
 * reference's shared default holds afterwards).  Returns MHE_OK or MHE_ERR_*.
 */
int mhe_ls_run(const mhe_ls_dims* dims, int32_t chains, int32_t epochs, const double* sat_pos,
               const double* pr, const int32_t* nsat, const double* sat_vel, const double* pr_rate,
               const double* x_init, double* x_out, double* b_out, double* v_out, double* bd_out,
               int32_t* iters_out, double* x_last, void* stream);

/* Library version string. */
const char* mhe_version(void);

#ifdef __cplusplus
}
#endif
#endif /* MHE_H */
