// libmhe core: the kernels of the batched collocation Gauss-Newton estimator
// (register-resident path k_gn / k_gn_bounded, large-system path mhe_big.h)
// and the host-side launch templates, shared by the translation units that
// instantiate them per (dynamics, measurement) plug-in pair (pair_*.hip).
// The C-ABI itself (include/mhe.h) lives in mhe_gn.hip.
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
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <mutex>
#include <stdint.h>
#include <stdlib.h>

#include "mhe.h"
#include "mhe_models.h"

namespace mhe {

typedef double d4 __attribute__((ext_vector_type(4)));

// waves per workgroup (one trajectory).  -DMHE_NW=16 builds the one-workgroup-per-CU
// shape (5 slots per wave, 99 VGPRs, no scratch; bitwise-identical iterates) for A/B
// runs -- measured 5 % slower at B = 128 and 256, 38 % at 1024
// min waves per SIMD of the fused kernels' launch bounds: 4 = two 8-wave workgroups per
// CU (128 VGPRs); 2 = one per CU with 256 VGPRs (A/B variant for small batches)
#ifndef MHE_GN_MINW
#define MHE_GN_MINW 4
#endif
#ifndef MHE_NW
#define MHE_NW 8
#endif
#ifndef MHE_SB_DIAG_BUILD
#define MHE_SB_DIAG_BUILD 0  // A/B: small-batch instance's diagonal tiles built by waves 0 and 4 only
#endif
constexpr int NW = MHE_NW;
constexpr int NTHREADS = NW * 64;
constexpr int MAX_NT = 13;         // padded system <= 208 (register-resident path)
// The NT(NT-1)/2 off-diagonal tiles live in MFMA accumulator registers (20
// slots per wave at NT = 13, 160 VGPRs); the NT diagonal tiles live in LDS.
// Holding all 91 tiles in registers (23 slots) left too few registers for the
// rest of the kernel and the allocator spilled tiles to scratch.
constexpr int MAX_SLOTS = (MAX_NT * (MAX_NT - 1) / 2 + NW - 1) / NW;  // 10 at 8 waves

enum Mode { MODE_SOLVE = 0, MODE_ASSEMBLE = 1, MODE_LINSOLVE = 2 };

// Process-wide A/B options (defined in mhe_gn.hip, set only through the explicit
// mhe_set_option call of include/mhe.h -- never from the environment): the
// right-looking large-path factorization and an LDS pad that forces occupancy.
extern int g_opt_big_right_looking;
extern int g_opt_smem_pad;

// ------------------------------------------------------------ layouts
struct ConstLayout {
  size_t D, Dt, Phi, PhiT, cw, Qw, Pw, Rw, Cc, DA, DB, DAc, DBc, total;  // byte offsets
};

__host__ __device__ inline size_t align256(size_t x) { return (x + 255) & ~size_t(255); }

// Every constants buffer starts with this header: the layout stamp at offset 0.
constexpr size_t CONST_HEADER = 256;

__host__ __device__ inline ConstLayout const_layout(int P, int M, int n, int p, int NT) {
  ConstLayout L;
  size_t o = CONST_HEADER;
  const size_t ntiles = size_t(NT) * (NT + 1) / 2;
  L.D = o;    o = align256(o + sizeof(double) * P * P);
  L.Dt = o;   o = align256(o + sizeof(double) * P * P);
  L.Phi = o;  o = align256(o + sizeof(double) * M * P);
  L.PhiT = o; o = align256(o + sizeof(double) * M * P);
  L.cw = o;   o = align256(o + sizeof(double) * P);
  L.Qw = o;   o = align256(o + sizeof(double) * n * n);
  L.Pw = o;   o = align256(o + sizeof(double) * n * n);
  L.Rw = o;   o = align256(o + sizeof(double) * M * p * p);
  L.Cc = o;   o = align256(o + sizeof(double) * ntiles * 256);  // constant part of J^T W J
  L.DA = o;   o = align256(o + sizeof(double) * ntiles * 256);  // a * D[l][j] per tile element
  L.DB = o;   o = align256(o + sizeof(double) * ntiles * 256);  // a * D[j][l] per tile element
  // n = 2 only: the 8 x 8 node block of D behind each tile, a D[8I+cn][8J+rn] (DAc)
  // and a D[8J+rn][8I+cn] (DBc) -- 512 B per tile instead of 2 KB, one value per lane
  // in the layout that spread_dblock turns into the tile's C layout (VALU swaps)
  L.DAc = o;  o = align256(o + sizeof(double) * ntiles * 64);
  L.DBc = o;  o = align256(o + sizeof(double) * ntiles * 64);
  L.total = o;
  return L;
}

struct SmemLayout {  // offsets in doubles
  int Xs, Vs, FtV, Es, FtE, GE, G, LAM, BV, YV, PB, HB, BAND, ZT, DT, RED, ROWM, UN, XO, ACT, GV, total;
};

__host__ __device__ inline int rnd2(int x) { return (x + 1) & ~1; }  // keep 16-B alignment

constexpr int DTS = 272;  // diagonal-tile stride: A_kk row-major (256), then L_kk^-T with row stride 17
constexpr int LIS = 17;   // row stride of L_kk^-T (conflict-free row and column reads)
// Two unit vectors, e_16 in [0, 34) and e_51 in [34, 68): row i of the 16 x 16 identity
// is 16 consecutive doubles at an even (16-B aligned) offset, unit_row(i) (panel).
constexpr int UNITS = 68;
// blgp of v_mfma_f64 on gfx950 = neg modifiers [A, B, C]: bit 0 negates A
constexpr int MFMA_NEG_A = 1;
__host__ __device__ constexpr int unit_row(int i) { return (i & 1) ? 51 - i : 16 - i; }

// sb: the small-batch factorization (factor_forward_sb): U block rows double-buffered
// (PB) and the hand-off tile of the critical-path wave (HB, double-buffered)
__host__ __device__ inline SmemLayout smem_layout(int P, int M, int n, int NT, bool nonlinear, bool bounded = false,
                                                  bool sb = false) {
  SmemLayout S;
  int o = 0;
  const int dp = 16 * NT;
  S.Xs = o;   o += rnd2(P * n);
  S.Vs = o;   o += rnd2(P * n);
  S.FtV = o;  o += rnd2(P * n);
  S.Es = o;   o += rnd2(P * n * n);
  S.FtE = o;  o += rnd2(P * n * n);
  S.GE = o;   o += rnd2(M * n);
  S.G = o;    o += nonlinear ? rnd2(M * n * n) : 0;
  S.LAM = o;  o += rnd2(P * n);         // Huber IRLS weights c_k lambda_ka (MHE_COST_HUBER)
  S.BV = o;   o += dp;                  // right-hand side b = -g, updated block by block
  S.YV = o;   o += dp;                  // y = U^-T b, then delta = U^-1 y in place
  S.PB = o;   o += (sb ? 2 : 1) * (NT - 1) * 256;  // block row k of U (tiles U_kb, b > k), register order
  S.HB = o;   o += sb ? 2 * 256 : 0;
  S.BAND = o; o += sb ? (NT - 1) * 256 : 0;  // the band tiles U_{k,k+1} (backward_sb reads them here)
  S.ZT = o;   o += sb ? 256 : 0;             // a zero tile: operand loads of idle slots
  S.DT = o;   o += NT * DTS;            // diagonal blocks
  S.RED = o;  o += 4 * NW + 8;
  S.ROWM = o; o += NW * 8;              // per wave, per block row I: bit mask of its slots (I, J)
  S.UN = o;   o += UNITS;               // identity rows for the panel (unit_row)
  // bounded problems only (projected Newton, k_gn<..., BOUNDED>): the iterate the
  // line search starts from, and the epsilon-active set (one int per unknown)
  S.XO = o;   o += bounded ? rnd2(P * n) : 0;
  S.ACT = o;  o += bounded ? dp / 2 : 0;
  // -g at the iterate, kept for the Armijo test: factor_forward turns BV into the
  // forward-substituted right-hand side in place
  S.GV = o;   o += bounded ? dp : 0;
  S.total = o;
  return S;
}

struct GnArgs {
  const char* cbuf;
  int P, M, d, NT, ntiles, q, has_prior;
  int idx[8];
  double alpha;
  const double* X0;
  double* Xout;
  const double* U;
  long long ustride;
  const double* Y;
  const double* PAR;
  long long pstride;
  const double* x0;
  double* cost;
  int* iters;
  int* status;
  int max_iter;
  double tol;
  double* Hout;
  double* gout;
  const double* Hin;
  const double* gin;
  double* dout;
  unsigned long long* dbg;  // MHE_DIAG builds only: per-phase cycle sums
  double huber_delta;       // MHE_COST_HUBER only
  int n_bounds;             // addVarBounds: components bidx[i] in [blb, bub] (k_gn_bounded)
  unsigned long long tag;   // layout stamp expected at offset 0 of the constants buffer (mhe_build_constants)
  int bidx[8];
  double blb[8], bub[8];
  double dpar[8];           // mhe_dims.dyn_par (dynamics plug-in params)
  const double* Rw;         // per-solve measurement weights (B|1, M, p, p) or NULL = the constants' Rw
  long long rwstride;       //   (nonlinear measurement models only: a linear h folds Rw into Cc)
};

#ifdef MHE_DIAG
// Diagnostic build: s_memtime stamps at phase boundaries (wave 0), summed per
// workgroup.  Never compiled into the product library.
#define DIAG_DECL unsigned long long _dg[16] = {}; unsigned long long _dt = __builtin_amdgcn_s_memtime();
#define DIAG_MARK(i) do { const unsigned long long _n = __builtin_amdgcn_s_memtime(); _dg[i] += _n - _dt; _dt = _n; } while (0)
#define DIAG_FLUSH(b) do { if (threadIdx.x == 0 && a.dbg) for (int _i = 0; _i < 16; ++_i) a.dbg[(b) * 16 + _i] = _dg[_i]; } while (0)
#define DIAG_FDECL unsigned long long* _dg, unsigned long long& _dt
#define DIAG_FARGS _dg, _dt
#else
#define DIAG_DECL
#define DIAG_MARK(i) do { } while (0)
#define DIAG_FLUSH(b) do { } while (0)
#define DIAG_FDECL int
#define DIAG_FARGS 0
#endif

// Knock-out build (tools/ko_probe.py): -DMHE_KO=<mask> disables parts of the
// factorization to measure their cost; results are wrong.  Never in the product.
#ifndef MHE_KO
#define MHE_KO 0
#endif
#define KO(bit) ((MHE_KO >> (bit)) & 1)

// ------------------------------------------------------------ wave helpers
__device__ __forceinline__ double readlane_d(double v, int lane) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)b, lane);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), lane);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// Raw buffer loads from the constants buffer: one resource (SGPRs) over all of
// cbuf, a per-lane byte offset and a wave-uniform SGPR offset per unrolled term,
// so each table element costs one buffer_load and no 64-bit address VALU.
typedef unsigned int mhe_u2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t cbuf_rsrc(const char* cbuf, size_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)cbuf, (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ double bload(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
  const mhe_u2 v = __builtin_amdgcn_raw_buffer_load_b64(r, voff, soff, 0);
  return __builtin_bit_cast(double, v);
}

// Butterfly step over lanes within a DPP row: quad_perm xor 1 / xor 2,
// row_half_mirror, row_mirror -- each leaves every lane of the row holding the
// combined value of its partner set.  Then v_permlane16/32_swap across rows.
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_mov_dpp((int)b, CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), CTRL, 0xF, 0xF, false);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// The four alpha D values of a tile element's node pair for registers r = 0..3
// (n = 2 compact 8 x 8 node blocks, k_build_cc): lane l's value for register r
// is held by lane (l & ~0x11) | (r & 1) | (r >> 1) << 4, so two DPP quad
// broadcasts and two v_permlane16_swap pairs spread it -- VALU only, no LDS.
__device__ __forceinline__ void spread_dblock(double v, double (&o)[4]) {
  const double ev = dpp_d<0xA0>(v);  // quad_perm [0,0,2,2]: the even lane of each pair
  const double od = dpp_d<0xF5>(v);  // quad_perm [1,1,3,3]: the odd lane
  const long long be = __double_as_longlong(ev), bo = __double_as_longlong(od);
  const auto el = __builtin_amdgcn_permlane16_swap((int)be, (int)be, false, false);
  const auto eh = __builtin_amdgcn_permlane16_swap((int)(be >> 32), (int)(be >> 32), false, false);
  const auto ol = __builtin_amdgcn_permlane16_swap((int)bo, (int)bo, false, false);
  const auto oh = __builtin_amdgcn_permlane16_swap((int)(bo >> 32), (int)(bo >> 32), false, false);
  // [0]: the even 16-lane row of the pair, [1]: the odd one
  o[0] = __longlong_as_double(((long long)eh[0] << 32) | (unsigned int)el[0]);
  o[2] = __longlong_as_double(((long long)eh[1] << 32) | (unsigned int)el[1]);
  o[1] = __longlong_as_double(((long long)oh[0] << 32) | (unsigned int)ol[0]);
  o[3] = __longlong_as_double(((long long)oh[1] << 32) | (unsigned int)ol[1]);
}

// v_permlane16_swap (XOR16 = 1: row pairs) / v_permlane32_swap (2: wave halves)
// with the same register as both operands leaves the two members of each pair in
// [0] and [1] in every lane; OP combines them (sum / max).
template <int XOR16, bool MAX>
__device__ __forceinline__ double pair_combine(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = (int)b, hi = (int)(b >> 32);
  double x, y;
  if constexpr (XOR16 == 1) {
    auto l = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
    auto h = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
    x = __longlong_as_double(((long long)h[0] << 32) | (unsigned int)l[0]);
    y = __longlong_as_double(((long long)h[1] << 32) | (unsigned int)l[1]);
  } else {
    auto l = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
    auto h = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
    x = __longlong_as_double(((long long)h[0] << 32) | (unsigned int)l[0]);
    y = __longlong_as_double(((long long)h[1] << 32) | (unsigned int)l[1]);
  }
  return MAX ? fmax(x, y) : x + y;
}

__device__ __forceinline__ double wave_sum(double v) {
  v += dpp_d<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp_d<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_d<0x141>(v);  // row_half_mirror
  v += dpp_d<0x140>(v);  // row_mirror
  v = pair_combine<1, false>(v);
  return pair_combine<2, false>(v);
}

__device__ __forceinline__ double wave_max(double v) {
  v = fmax(v, dpp_d<0xB1>(v));
  v = fmax(v, dpp_d<0x4E>(v));
  v = fmax(v, dpp_d<0x141>(v));
  v = fmax(v, dpp_d<0x140>(v));
  v = pair_combine<1, true>(v);
  return pair_combine<2, true>(v);
}

// block-wide reduction of up to 2 values (sum or max), result broadcast
__device__ __forceinline__ void block_reduce2(double* red, double& a, double& b, bool is_max) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  a = is_max ? wave_max(a) : wave_sum(a);
  b = is_max ? wave_max(b) : wave_sum(b);
  if (lane == 0) {
    red[2 * wave] = a;
    red[2 * wave + 1] = b;
  }
  __syncthreads();
  double ra = red[0], rb = red[1];
#pragma unroll
  for (int w = 1; w < NW; ++w) {
    ra = is_max ? fmax(ra, red[2 * w]) : ra + red[2 * w];
    rb = is_max ? fmax(rb, red[2 * w + 1]) : rb + red[2 * w + 1];
  }
  __syncthreads();
  a = ra;
  b = rb;
}

// Slot table: lane s of every wave holds (I | J << 16) of the off-diagonal
// tile in its slot s (u = wave + NW*s over the tiles I > J, column-major), or
// -1.  A slot's coordinates are one v_readlane away (no memory round trip);
// callers pass an opaque per-step copy so LICM cannot hoist decoded values.
__device__ __forceinline__ int make_slot_table(int wave, int lane, int NT) {
  const int u = wave + NW * lane;
  if (lane >= MAX_SLOTS || u >= NT * (NT - 1) / 2) return -1;
  int J = 0, base = 0;
  while (u >= base + (NT - 1 - J)) {
    base += NT - 1 - J;
    ++J;
  }
  return (J + 1 + (u - base)) | (J << 16);
}

// linear index of tile (I, J), I >= J, in the column-major lower triangle (Cc/DA/DB layout)
__device__ __forceinline__ int tile_index(int I, int J, int NT) { return J * NT - J * (J - 1) / 2 + (I - J); }

__device__ __forceinline__ int slot_ij(int stab, int s) { return __builtin_amdgcn_readlane(stab, s); }

// Number of this wave's slots whose tile column is < j (slots are column-major,
// so the tiles of columns >= j are the slot suffix starting here).
__device__ __forceinline__ int slot_start(int j, int wave, int NT) {
  const int base = j * (NT - 1) - j * (j - 1) / 2;  // tiles in columns < j
  return base > wave ? (base - wave + NW - 1) / NW : 0;
}

// Per wave and block row I (< 16): the bit mask of the wave's slots holding a tile
// (I, J), written once per launch (the backward solve tests one bit per slot
// instead of decoding every slot's coordinates at every block step).
// the unit vectors behind unit_row, written by wave 0 alone (the big path's panel
// runs on wave 0 before any workgroup barrier)
__device__ __forceinline__ void init_units(double* un) {
  if (threadIdx.x < 64)
    for (int e = threadIdx.x; e < UNITS; e += 64) un[e] = (e == 16 || e == 51) ? 1.0 : 0.0;
}

template <int SLOTS = MAX_SLOTS>
__device__ __forceinline__ void init_rowmask(int* rowm, int wave, int lane, int stab) {
  unsigned m = 0;
#pragma unroll
  for (int s = 0; s < SLOTS; ++s) {
    const int IJ = slot_ij(stab, s);
    if (IJ >= 0 && (IJ & 0xffff) == lane) m |= 1u << s;
  }
  if (lane < 16) rowm[wave * 16 + lane] = (int)m;
}

// ------------------------------------------------------------ model phases
// Mat-vec phases use TPR threads per row (4 with 8 waves): each sums every
// TPR-th term of the row with an 8-deep unrolled loop (8 independent L2 loads
// in flight), the parts are combined with lane swaps.  The tables (D, D^T, Phi,
// Phi^T) are shared by every workgroup and L2-resident.
constexpr int TPR = NW >= 8 ? 4 : 2;

// threadIdx.x through an opaque move: values derived from it inside a phase
// are recomputed per phase instead of being hoisted out of the Gauss-Newton
// loop, where they would stay live across the register-hungry factorization.
__device__ __forceinline__ int opaque_tid() {
  int t = threadIdx.x;
  asm volatile("" : "+v"(t));
  return t;
}

template <int n>
__device__ __forceinline__ void dot_rows_part(const double* __restrict__ Mt, int ld, int row, int len, int part,
                                              const double* __restrict__ Xs, double (&acc)[n]) {
  // acc[c] = sum_j Mt[j*ld + row] * Xs[j*n + c], summed over the TPR lanes of the row
#pragma unroll
  for (int c = 0; c < n; ++c) acc[c] = 0.0;
  int j = part;
#pragma unroll 1
  for (; j + TPR * 7 < len; j += TPR * 8) {
    double m[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) m[u] = Mt[(j + TPR * u) * ld + row];
#pragma unroll
    for (int u = 0; u < 8; ++u)
#pragma unroll
      for (int c = 0; c < n; ++c) acc[c] += m[u] * Xs[(j + TPR * u) * n + c];
  }
  for (; j < len; j += TPR) {
    const double mv = Mt[j * ld + row];
#pragma unroll
    for (int c = 0; c < n; ++c) acc[c] += mv * Xs[j * n + c];
  }
  static_assert(TPR == 4, "quad reductions below assume 4 lanes per row");
#pragma unroll
  for (int c = 0; c < n; ++c) acc[c] += dpp_d<0xB1>(acc[c]);  // lane ^ 1 (DPP: no bpermute address registers)
#pragma unroll
  for (int c = 0; c < n; ++c) acc[c] += dpp_d<0x4E>(acc[c]);  // lane ^ 2
}

// Per-node dynamics quantities (nlp/nlp.py:225-245):
//   W_k = a * sum_j D_kj X_j - f(X_k, U_k);  V_k = c_k Qw W_k;  E_k = c_k Qw F_k;
//   FtE_k = F_k^T E_k;  FtV_k = F_k^T V_k;   cost += c_k W_k^T Qw W_k
template <class DYN, bool HUBER = false>
__device__ __forceinline__ double node_row(const GnArgs& a, const ConstLayout& CL, const SmemLayout& SL, double* sm,
                                           int b, int k, const double (&dx)[DYN::n]) {
  constexpr int n = DYN::n, m = DYN::m;
  const double* cw = (const double*)(a.cbuf + CL.cw);
  const double* Qw = (const double*)(a.cbuf + CL.Qw);
  const double* Xs = sm + SL.Xs;
  double cost = 0.0;
  {
    double xk[n], uk[m > 0 ? m : 1], f[n], F[n * n];
#pragma unroll
    for (int c = 0; c < n; ++c) xk[c] = Xs[k * n + c];
    if (m > 0) {
      const double* U = a.U + (long long)b * a.ustride + (long long)k * m;
#pragma unroll
      for (int c = 0; c < m; ++c) uk[c] = U[c];
    }
    DYN::eval(xk, uk, a.dpar, f, F);
    double W[n], V[n];
#pragma unroll
    for (int c = 0; c < n; ++c) W[c] = a.alpha * dx[c] - f[c];
    const double ck = cw[k];
    double E[n * n];
    if constexpr (HUBER) {
      // pseudo_huber_loss (cost_functions.py:25-31), IRLS: lambda = q / sqrt(1 + W^2/delta^2),
      // V = c lambda W (= c rho'/2), E = c diag(lambda) F
      const double dl = a.huber_delta;
#pragma unroll
      for (int r = 0; r < n; ++r) {
        const double q = Qw[r * n + r];
        const double sr = sqrt(1.0 + W[r] * W[r] / (dl * dl));
        const double lam = ck * (q / sr);
        V[r] = lam * W[r];
        cost += ck * (2.0 * q * dl * dl * (sr - 1.0));
        sm[SL.LAM + k * n + r] = lam;
#pragma unroll
        for (int c = 0; c < n; ++c) E[r * n + c] = lam * F[r * n + c];
      }
    } else {
#pragma unroll
      for (int r = 0; r < n; ++r) {
        double s = 0.0;
#pragma unroll
        for (int c = 0; c < n; ++c) s += Qw[r * n + c] * W[c];
        V[r] = ck * s;
        cost += W[r] * V[r];
      }
#pragma unroll
      for (int r = 0; r < n; ++r)
#pragma unroll
        for (int c = 0; c < n; ++c) {
          double s = 0.0;
#pragma unroll
          for (int t = 0; t < n; ++t) s += Qw[r * n + t] * F[t * n + c];
          E[r * n + c] = ck * s;
        }
    }
    double* Vs = sm + SL.Vs + k * n;
    double* FtV = sm + SL.FtV + k * n;
    double* Es = sm + SL.Es + k * n * n;
    double* FtE = sm + SL.FtE + k * n * n;
#pragma unroll
    for (int r = 0; r < n; ++r) {
      Vs[r] = V[r];
      double s = 0.0;
#pragma unroll
      for (int t = 0; t < n; ++t) s += F[t * n + r] * V[t];
      FtV[r] = s;
#pragma unroll
      for (int c = 0; c < n; ++c) {
        Es[r * n + c] = E[r * n + c];
        double u = 0.0;
#pragma unroll
        for (int t = 0; t < n; ++t) u += F[t * n + r] * E[t * n + c];
        FtE[r * n + c] = u;
      }
    }
  }
  return cost;
}

template <class DYN, bool HUBER = false>
__device__ __forceinline__ double node_phase(const GnArgs& a, const ConstLayout& CL, const SmemLayout& SL, double* sm, int b) {
  constexpr int n = DYN::n;
  const double* Dt = (const double*)(a.cbuf + CL.Dt);
  const double* Xs = sm + SL.Xs;
  double cost = 0.0;
  const int tid = opaque_tid();
  const int part = tid % TPR;
  for (int k0 = 0; k0 < a.P; k0 += NTHREADS / TPR) {
    const int k = k0 + tid / TPR;
    const int kk = k < a.P ? k : a.P - 1;
    double dx[n];
    dot_rows_part<n>(Dt, a.P, kk, a.P, part, Xs, dx);
    if (part || k >= a.P) continue;
    cost += node_row<DYN, HUBER>(a, CL, SL, sm, b, k, dx);
  }
  return cost;
}

// Per-measurement-row quantities (nlp/nlp.py:264-273):
//   x_i = sum_j Phi_ij X_j;  e_i = y_i - h(x_i);  GE_i = H_i^T Rw_i e_i;
//   (nonlinear) G_i = H_i^T Rw_i H_i;  cost += e_i^T Rw_i e_i
// NOISE (projected Newton's Armijo test only): also accumulate into *nzp the rounding
// level of this row's cost, COST_NOISE eps |R e| (|y| + |h|) -- e = y - h carries
// eps (|y| + |h|) of rounding in any evaluation order (oracle/gn.py cost_noise).
constexpr double COST_NOISE = 4.0;

template <class DYN, class MEAS, bool NOISE = false>
__device__ __forceinline__ double meas_row(const GnArgs& a, const ConstLayout& CL, const SmemLayout& SL, double* sm,
                                           int b, int i, const double (&xi)[DYN::n], double* nzp = nullptr) {
  constexpr int n = DYN::n, p = MEAS::p, q = MEAS::q;
  const double* Rw = (const double*)(a.cbuf + CL.Rw);
  double cost = 0.0;
  {
    double par[q > 0 ? q : 1];
    if (q > 0) {
      const double* PR = a.PAR + (long long)b * a.pstride + (long long)i * q;
#pragma unroll
      for (int c = 0; c < q; ++c) par[c] = PR[c];
    }
    const double* R = (!MEAS::LINEAR && a.Rw ? a.Rw + (long long)b * a.rwstride : Rw) + (long long)i * p * p;
    double h[p], H[p * n];
    MEAS::eval(xi, par, a.idx, h, H);
    const double* yi = a.Y + ((long long)b * a.M + i) * p;
    double e[p], Re[p];
#pragma unroll
    for (int r = 0; r < p; ++r) e[r] = yi[r] - h[r];
    const bool masked = masked_row<p>(R);
    if (masked) {  // R = 0 masks the row (autonomous-car.py:260-263): no NaN from h at a singular point
#pragma unroll
      for (int c = 0; c < p * n; ++c) H[c] = 0.0;
#pragma unroll
      for (int r = 0; r < p; ++r) e[r] = 0.0;
    }
#pragma unroll
    for (int r = 0; r < p; ++r) {
      double s = 0.0;
#pragma unroll
      for (int c = 0; c < p; ++c) s += R[r * p + c] * e[c];
      Re[r] = s;
      cost += e[r] * s;
    }
    if constexpr (NOISE) {
      if (!masked) {
        double t = 0.0;
#pragma unroll
        for (int r = 0; r < p; ++r) t += fabs(Re[r]) * (fabs(yi[r]) + fabs(h[r]));
        *nzp += COST_NOISE * __DBL_EPSILON__ * t;
      }
    }
    double* GE = sm + SL.GE + i * n;
#pragma unroll
    for (int c = 0; c < n; ++c) {
      double s = 0.0;
#pragma unroll
      for (int r = 0; r < p; ++r) s += H[r * n + c] * Re[r];
      GE[c] = s;
    }
    if (!MEAS::LINEAR) {
      double* G = sm + SL.G + i * n * n;
      double RH[p * n];
#pragma unroll
      for (int r = 0; r < p; ++r)
#pragma unroll
        for (int c = 0; c < n; ++c) {
          double s = 0.0;
#pragma unroll
          for (int t = 0; t < p; ++t) s += R[r * p + t] * H[t * n + c];
          RH[r * n + c] = s;
        }
#pragma unroll
      for (int r = 0; r < n; ++r)
#pragma unroll
        for (int c = 0; c < n; ++c) {
          double s = 0.0;
#pragma unroll
          for (int t = 0; t < p; ++t) s += H[t * n + r] * RH[t * n + c];
          G[r * n + c] = s;
        }
    }
  }
  return cost;
}

template <class DYN, class MEAS, bool NOISE = false>
__device__ __forceinline__ double meas_phase(const GnArgs& a, const ConstLayout& CL, const SmemLayout& SL, double* sm, int b,
                                             double* nzp = nullptr) {
  constexpr int n = DYN::n;
  const double* PhiT = (const double*)(a.cbuf + CL.PhiT);
  const double* Xs = sm + SL.Xs;
  double cost = 0.0;
  const int tid = opaque_tid();
  const int part = tid % TPR;
  for (int i0 = 0; i0 < a.M; i0 += NTHREADS / TPR) {
    const int i = i0 + tid / TPR;
    const int ii = i < a.M ? i : a.M - 1;
    double xi[n];
    dot_rows_part<n>(PhiT, a.M, ii, a.P, part, Xs, xi);
    if (part || i >= a.M) continue;
    cost += meas_row<DYN, MEAS, NOISE>(a, CL, SL, sm, b, i, xi, nzp);
  }
  return cost;
}

// v plus the value of the paired 16-lane row (rows 0+1, 2+3), in every lane
// (v_permlane16_swap; the sum is formed in the same order on both rows).
__device__ __forceinline__ double row_pair_sum(double v) {
  const long long b = __double_as_longlong(v);
  const auto l = __builtin_amdgcn_permlane16_swap((int)b, (int)b, false, false);
  const auto h = __builtin_amdgcn_permlane16_swap((int)(b >> 32), (int)(b >> 32), false, false);
  return __longlong_as_double(((long long)h[0] << 32) | (unsigned int)l[0]) +
         __longlong_as_double(((long long)h[1] << 32) | (unsigned int)l[1]);
}
// In lanes 0..31: the value of lane + 32 (v_permlane32_swap).
__device__ __forceinline__ double upper_half(double v) {
  const long long b = __double_as_longlong(v);
  const auto l = __builtin_amdgcn_permlane32_swap((int)b, (int)b, false, false);
  const auto h = __builtin_amdgcn_permlane32_swap((int)(b >> 32), (int)(b >> 32), false, false);
  return __longlong_as_double(((long long)h[1] << 32) | (unsigned int)l[1]);
}

// node_phase + meas_phase.  When both row counts fit one pass (P, M <= 128 with
// 4 lanes per row: C1, C2) each lane runs its D-row and Phi-row dots together,
// 16 L2 loads in flight instead of 8, halving the dependent round trips.
template <class DYN, class MEAS, bool HUBER = false, bool NOISE = false>
__device__ __forceinline__ double node_meas_phase(const GnArgs& a, const ConstLayout& CL, const SmemLayout& SL,
                                                  double* sm, int b, DIAG_FDECL, double* nzp = nullptr) {
  constexpr int n = DYN::n;
  constexpr int ROWS = NTHREADS / TPR;
  if (a.P > ROWS || a.M > ROWS)
    return node_phase<DYN, HUBER>(a, CL, SL, sm, b) + meas_phase<DYN, MEAS, NOISE>(a, CL, SL, sm, b, nzp);
  const __amdgpu_buffer_rsrc_t rs = cbuf_rsrc(a.cbuf, CL.total);
  const double* Xs = sm + SL.Xs;
  // the TPR = 4 parts of a row are the four 16-lane rows of a wave (row = 16 wave +
  // lane % 16): the 4 lanes of a quad read 4 consecutive rows of D^T / Phi^T, one
  // 32-B piece of one line (with the parts in a quad they touched 4 lines)
  const int tid = opaque_tid();
  const int part = (tid >> 4) & 3, r = (tid >> 6) * 16 + (tid & 15);
  const int kk = r < a.P ? r : a.P - 1, ii = r < a.M ? r : a.M - 1;
  double dx[n], xi[n];
#pragma unroll
  for (int c = 0; c < n; ++c) dx[c] = xi[c] = 0.0;
  const int len = a.P;
  // byte offsets of Dt[j][kk] and PhiT[j][ii]; per term u the uniform offsets u TPR ld 8
  int o1 = (int)CL.Dt + (part * a.P + kk) * 8, o2 = (int)CL.PhiT + (part * a.M + ii) * 8;
  const int s1 = TPR * a.P * 8, s2 = TPR * a.M * 8;
  int j = part;
#pragma unroll 1
  for (; j + TPR * 7 < len; j += TPR * 8) {
    double m1[8], m2[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      m1[u] = bload(rs, o1, u * s1);
      m2[u] = bload(rs, o2, u * s2);
    }
    o1 += 8 * s1;
    o2 += 8 * s2;
#pragma unroll
    for (int u = 0; u < 8; ++u)
#pragma unroll
      for (int c = 0; c < n; ++c) {
        const double x = Xs[(j + TPR * u) * n + c];
        dx[c] += m1[u] * x;
        xi[c] += m2[u] * x;
      }
  }
  for (; j < len; j += TPR) {
    const double m1 = bload(rs, o1, 0), m2 = bload(rs, o2, 0);
    o1 += s1;
    o2 += s2;
#pragma unroll
    for (int c = 0; c < n; ++c) {
      dx[c] += m1 * Xs[j * n + c];
      xi[c] += m2 * Xs[j * n + c];
    }
  }
  static_assert(TPR == 4, "the row reductions below assume 4 parts per row");
#pragma unroll
  for (int c = 0; c < n; ++c) {
    dx[c] = row_pair_sum(dx[c]);  // (part 0 + part 1), (part 2 + part 3)
    xi[c] = row_pair_sum(xi[c]);
  }
#pragma unroll
  for (int c = 0; c < n; ++c) {
    dx[c] += upper_half(dx[c]);  // complete in lanes 0..15 (part 0)
    xi[c] += upper_half(xi[c]);
  }
  DIAG_MARK(14);
  double cost = 0.0;
  if (part == 0) {
    if (r < a.P) cost += node_row<DYN, HUBER>(a, CL, SL, sm, b, r, dx);
    if (r < a.M) cost += meas_row<DYN, MEAS, NOISE>(a, CL, SL, sm, b, r, xi, nzp);
  }
  return cost;
}

template <class DYN, class MEAS, bool HUBER = false, bool NOISE = false>
__device__ __forceinline__ double node_meas_phase(const GnArgs& a, const ConstLayout& CL, const SmemLayout& SL,
                                                  double* sm, int b, double* nzp = nullptr) {
  DIAG_DECL
  return node_meas_phase<DYN, MEAS, HUBER, NOISE>(a, CL, SL, sm, b, DIAG_FARGS, nzp);
}

// Gradient g = J^T W r (nlp/nlp.py:242-286 objective); writes BV = -g (padding 0).
//   g_j = a sum_k D_kj V_k - F_j^T V_j - sum_i Phi_ij GE_i (+ Pw (X_0 - x0) at j = 0)
// TPR lanes per node: half sum the D column, half the Phi column.
template <class DYN>
__device__ __forceinline__ double grad_phase(const GnArgs& a, const ConstLayout& CL, const SmemLayout& SL, double* sm, int b) {
  constexpr int n = DYN::n;
  const __amdgpu_buffer_rsrc_t rs = cbuf_rsrc(a.cbuf, CL.total);
  const double* Pw = (const double*)(a.cbuf + CL.Pw);
  const double* Vs = sm + SL.Vs;
  const double* FtV = sm + SL.FtV;
  const double* GE = sm + SL.GE;
  const double* Xs = sm + SL.Xs;
  double* BV = sm + SL.BV;
  double cost = 0.0;
  const int dp = 16 * a.NT;
  const int tid = opaque_tid();
  // TPR lanes per node: the first half sums the D column (sum_k D[k][j] V_k), the
  // second half the Phi column (sum_i Phi[i][j] GE_i), each split over TPR/2 lanes
  // (the TPR lanes of a node are the four 16-lane rows of a wave, node = 16 wave +
  // lane % 16: a quad reads 4 consecutive columns of D / Phi, as in node_meas_phase)
  constexpr int HP = TPR / 2;
  const int q = (tid >> 4) & 3, sub = q % HP;
  const bool phi = q >= HP;
  for (int j0 = 0; j0 < a.P; j0 += NTHREADS / TPR) {
    const int j = j0 + (tid >> 6) * 16 + (tid & 15);
    const int jj = j < a.P ? j : a.P - 1;
    const double* vec = phi ? GE : Vs;
    const int len = phi ? a.M : a.P;
    double s[n];
#pragma unroll
    for (int c = 0; c < n; ++c) s[c] = 0.0;
    // D and Phi share the row stride P: byte offset of Mt[k][jj], uniform step per term
    int om = (int)(phi ? CL.Phi : CL.D) + (sub * a.P + jj) * 8;
    const int sm8 = HP * a.P * 8;
    int k = sub;
#pragma unroll 1
    for (; k + HP * 7 < len; k += HP * 8) {
      double mv[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) mv[u] = bload(rs, om, u * sm8);
      om += 8 * sm8;
#pragma unroll
      for (int u = 0; u < 8; ++u)
#pragma unroll
        for (int c = 0; c < n; ++c) s[c] += mv[u] * vec[(k + HP * u) * n + c];
    }
    for (; k < len; k += HP) {
      const double mv = bload(rs, om, 0);
      om += sm8;
#pragma unroll
      for (int c = 0; c < n; ++c) s[c] += mv * vec[k * n + c];
    }
    static_assert(HP == 2, "the row reductions below assume TPR == 4");
#pragma unroll
    for (int c = 0; c < n; ++c) s[c] = row_pair_sum(s[c]);  // rows 0+1: D column, rows 2+3: Phi column
    double o[n];
#pragma unroll
    for (int c = 0; c < n; ++c) o[c] = upper_half(s[c]);  // in row 0: the Phi column's sum
    if (q != 0 || j >= a.P) continue;
    double gv[n];
#pragma unroll
    for (int c = 0; c < n; ++c) gv[c] = a.alpha * s[c] - FtV[j * n + c] - o[c];
    if (a.has_prior && j == 0) {
      double r0[n];
#pragma unroll
      for (int c = 0; c < n; ++c) r0[c] = Xs[c] - a.x0[(long long)b * n + c];
#pragma unroll
      for (int r = 0; r < n; ++r) {
        double t2 = 0.0;
#pragma unroll
        for (int c = 0; c < n; ++c) t2 += Pw[r * n + c] * r0[c];
        gv[r] += t2;
        cost += r0[r] * t2;
      }
    }
#pragma unroll
    for (int c = 0; c < n; ++c) BV[j * n + c] = -gv[c];
  }
  for (int t = a.d + tid; t < dp; t += NTHREADS) BV[t] = 0.0;
  return cost;
}

// One 16x16 tile element of H at (row, col) in the MFMA C-layout position of
// this lane (see build_tiles).
template <class DYN, class MEAS, bool HUBER = false>
__device__ __forceinline__ double h_element(const GnArgs& a, const double* Phi, const double* Es,
                                            const double* FtE, const double* G, double v, double da,
                                            double db, int row, int col, const double* D = nullptr,
                                            const double* LAM = nullptr) {
  constexpr int n = DYN::n;
  if (row < a.d && col < a.d) {
    const int j = row / n, aa = row - j * n;
    const int l = col / n, bb = col - l * n;
    if constexpr (HUBER) {
      // a^2 sum_k D_kj c_k lambda_ka D_kl (a == b): the dynamics "constant" part with
      // iteration-dependent IRLS weights (excluded from Cc for MHE_COST_HUBER)
      if (aa == bb) {
        double s = 0.0;
        for (int k = 0; k < a.P; ++k) s += D[k * a.P + j] * LAM[k * n + aa] * D[k * a.P + l];
        v += a.alpha * a.alpha * s;
      }
    }
    v -= da * Es[(l * n + aa) * n + bb] + db * Es[(j * n + bb) * n + aa];
    if (j == l) v += FtE[(j * n + aa) * n + bb];
    if (!MEAS::LINEAR) {
      double s2 = 0.0;
      for (int i = 0; i < a.M; ++i) s2 += Phi[i * a.P + j] * Phi[i * a.P + l] * G[(i * n + aa) * n + bb];
      v += s2;
    }
  }
  return v;
}

// Off-diagonal slots for n = 2 with the L2 dynamics cost and linear measurements
// (C2's shape), software-pipelined: the six constant loads of slot s + 1 (Cc's
// four registers, the two compact alpha D blocks; raw buffer loads, one SGPR
// resource) are issued before slot s is formed, so the slots cost one L2 round
// trip in all instead of one per load.  Branch-free: an empty slot forms tile 0
// (never read); padding rows / columns keep -Cc by a select; with n | 16 no
// off-diagonal tile meets a node's own 2 x 2 block, so F^T E drops out.
template <int SLOTS, bool BOUNDED>
__device__ __forceinline__ void build_slots_n2(const GnArgs& a, const ConstLayout& CL, const SmemLayout& SL,
                                               double* sm, d4 (&acc)[SLOTS], int lane, int stab) {
  const __amdgpu_buffer_rsrc_t rs = cbuf_rsrc(a.cbuf, CL.total);
  const double* Es = sm + SL.Es;
  const int* ACT = (const int*)(sm + SL.ACT);
  double cn[4], an, bn;
  auto issue = [&](int s) {
    const int IJ = slot_ij(stab, s);
    const int ti = IJ < 0 ? 0 : tile_index(IJ & 0xffff, IJ >> 16, a.NT);
#pragma unroll
    for (int r = 0; r < 4; ++r) cn[r] = bload(rs, ti * 2048 + lane * 8, (int)CL.Cc + 512 * r);
    an = bload(rs, ti * 512 + lane * 8, (int)CL.DAc);
    bn = bload(rs, ti * 512 + lane * 8, (int)CL.DBc);
  };
  issue(0);
#pragma unroll
  for (int s = 0; s < SLOTS; ++s) {
    const double c[4] = {cn[0], cn[1], cn[2], cn[3]};
    const double av = an, bv = bn;
    if (s + 1 < SLOTS) issue(s + 1);
    const int IJ = slot_ij(stab, s);
    const int I = IJ < 0 ? 1 : IJ & 0xffff, J = IJ < 0 ? 0 : IJ >> 16;
    const int col = 16 * I + (lane & 15);
    const int cc = col < a.d ? col : a.d - 1;
    const int l = cc >> 1, bb = cc & 1;
    double dav[4], dbv[4];
    spread_dblock(av, dav);
    spread_dblock(bv, dbv);
    // the row's component aa = row & 1 is the same for the four registers (rows
    // differ by 4), so E_l[aa][bb] is one LDS read per slot; padding rows (row >= d)
    // read a clamped node and are replaced by -Cc below
    const int aa = (lane >> 4) & 1;
    const double el = Es[(l * 2 + aa) * 2 + bb];
    // off-diagonal tiles have no padding rows (16 J + 15 < 16 (NT - 1) < d): register
    // r's row 16 J + (lane >> 4) + 4 r is node 8 J + (lane >> 5) + 2 r, so the four
    // E_j[bb][aa] reads are one base address plus immediate offsets (8 doubles apart)
    const double* ej = Es + ((8 * J + (lane >> 5)) * 2 + bb) * 2 + aa;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = 16 * J + (lane >> 4) + 4 * r;
      const double t = dav[r] * el + dbv[r] * ej[8 * r];
      // padding lies only in the last tile column: a wave-uniform test, the
      // per-element select only there
      if (I == a.NT - 1)
        acc[s][r] = (row < a.d && col < a.d) ? t - c[r] : -c[r];
      else
        acc[s][r] = t - c[r];
      if (BOUNDED && (ACT[row] | ACT[col])) acc[s][r] = 0.0;
    }
    __builtin_amdgcn_sched_barrier(0);
  }
}

// Build the H tiles owned by this wave, NEGATED (the factorization accumulates
// +U^T U into -A, so no operand needs a sign flip).  Slot (I, J), I > J, holds
// the UPPER block H[J-block][I-block] in the MFMA C layout (lane l, register r: row
// (l>>4)+4r, column l&15); in that layout the tile is directly the B operand
// (and the transposed A operand) of v_mfma_f64_16x16x4f64 -- see factor_forward.
//   H = Cc (constant: a^2 (D^T C D) (x) Qw  + linear-measurement term + prior + padding I)
//     - a D_lj E_l[a,b] - a D_jl E_j[b,a] + delta_jl (F^T E)_j[a,b]      (dynamics, X-dependent)
//     + sum_i Phi_ij Phi_il G_i[a,b]                                      (nonlinear measurements)
// Cc, DA = a D_lj and DB = a D_jl are stored per tile element in the MFMA
// C-layout, so each is one coalesced 512-B load per register.  Off-diagonal
// tiles go to the accumulator slots, diagonal tiles (owner wave J % NW) to LDS.
// BOUNDED (projected Newton, k_gn_bounded): rows and columns of the epsilon-active
// unknowns (ACT) are replaced by their diagonal entries -- the reduced GN system on
// the free unknowns, a diagonally scaled gradient step on the active ones.
template <class DYN, class MEAS, int SLOTS, bool HUBER = false, bool BOUNDED = false, bool SB = false>
__device__ __forceinline__ void build_tiles(const GnArgs& a, const ConstLayout& CL, const SmemLayout& SL, double* sm,
                                            d4 (&acc)[SLOTS], int wave, int lane, int stab) {
  const int* ACT = (const int*)(sm + SL.ACT);
  const double* Dm = (const double*)(a.cbuf + CL.D);
  const double* LAM = sm + SL.LAM;
  const double* Cc = (const double*)(a.cbuf + CL.Cc);
  const double* DA = (const double*)(a.cbuf + CL.DA);
  const double* DB = (const double*)(a.cbuf + CL.DB);
  const double* Phi = (const double*)(a.cbuf + CL.Phi);
  const double* Es = sm + SL.Es;
  const double* FtE = sm + SL.FtE;
  const double* G = sm + SL.G;
  asm volatile("" : "+v"(lane));
  asm volatile("" : "+s"(wave));
  asm volatile("" : "+v"(stab));
  constexpr int n = DYN::n;
  // Off-diagonal tiles of the common case (L2 dynamics cost, linear measurements):
  // branch-free.  Padding rows / columns read clamped indices and keep Cc by a
  // select; when n divides 16 no off-diagonal tile meets a node's diagonal block,
  // so the F^T E term drops out.  (A per-element branch here costs an exec-mask
  // round trip and a wait on each LDS read.)
  constexpr bool FAST = !HUBER && MEAS::LINEAR;
  if constexpr (FAST && n == 2) build_slots_n2<SLOTS, BOUNDED>(a, CL, SL, sm, acc, lane, stab);
#pragma unroll
  for (int s = 0; s < (FAST && n == 2 ? 0 : SLOTS); ++s) {
    const int IJ = slot_ij(stab, s);
    if (IJ < 0) {
      // no tile: always define (keeps acc dead between iterations), but with an
      // opaque value -- a zero constant would be hoisted out of the Gauss-Newton
      // loop and kept live (spilled) across the factorization.  Never read.
      d4 junk;
      asm volatile("" : "=v"(junk));
      acc[s] = junk;
    } else {
      const int I = IJ & 0xffff, J = IJ >> 16;
      const int ti = tile_index(I, J, a.NT);
      const size_t off = (size_t)ti * 256 + lane;
      const int col = 16 * I + (lane & 15);
      if constexpr (FAST) {
        const int cc = col < a.d ? col : a.d - 1;
        const int l = cc / n, bb = cc - l * n;
        double dav[4], dbv[4];
        if constexpr (n == 2) {
          spread_dblock(((const double*)(a.cbuf + CL.DAc))[(size_t)ti * 64 + lane], dav);
          spread_dblock(((const double*)(a.cbuf + CL.DBc))[(size_t)ti * 64 + lane], dbv);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = 16 * J + (lane >> 4) + 4 * r;
          const int rr = row < a.d ? row : a.d - 1;
          const int j = rr / n, aa = rr - j * n;
          double da, db;
          if constexpr (n == 2) {
            da = dav[r];
            db = dbv[r];
          } else {
            da = DA[off + 64 * r];
            db = DB[off + 64 * r];
          }
          double t = da * Es[(l * n + aa) * n + bb] + db * Es[(j * n + bb) * n + aa];
          if constexpr (16 % n != 0) t -= j == l ? FtE[(j * n + aa) * n + bb] : 0.0;
          const double v = Cc[off + 64 * r];
          acc[s][r] = (row < a.d && col < a.d) ? t - v : -v;
          if (BOUNDED && (ACT[row] | ACT[col])) acc[s][r] = 0.0;
        }
      } else if constexpr (DYN::n == 2) {
        // a D_lj / a D_jl of element (row, col) = node pair (8I + cn, 8J + rn) of the
        // tile's 8 x 8 D block, cn = (lane & 15) >> 1, rn = (lane >> 5) + 2r:
        // one 512-B load per table, then a lane permute per register
        double dav[4], dbv[4];
        spread_dblock(((const double*)(a.cbuf + CL.DAc))[(size_t)ti * 64 + lane], dav);
        spread_dblock(((const double*)(a.cbuf + CL.DBc))[(size_t)ti * 64 + lane], dbv);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = 16 * J + (lane >> 4) + 4 * r;
          acc[s][r] = -h_element<DYN, MEAS, HUBER>(a, Phi, Es, FtE, G, Cc[off + 64 * r], dav[r], dbv[r], row,
                                                   col, Dm, LAM);
          if (BOUNDED && (ACT[row] | ACT[col])) acc[s][r] = 0.0;
        }
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = 16 * J + (lane >> 4) + 4 * r;
          acc[s][r] = -h_element<DYN, MEAS, HUBER>(a, Phi, Es, FtE, G, Cc[off + 64 * r], DA[off + 64 * r],
                                                   DB[off + 64 * r], row, col, Dm, LAM);
          if (BOUNDED && (ACT[row] | ACT[col])) acc[s][r] = 0.0;
        }
      }
    }
    // bound the scheduler's load hoisting to two slots (register pressure)
    if (s & 1) __builtin_amdgcn_sched_barrier(0);
  }
  double* DT = sm + SL.DT;
  // small-batch factorization: the diagonal tiles go to the two waves without slots (CP,
  // wave 0, and wave 4), alternately, instead of one or two to every wave -- the six
  // slot owners build only their off-diagonal tiles (MHE_SB_DIAG_BUILD)
  const bool sbd = SB && MHE_SB_DIAG_BUILD;
  const int j0 = sbd ? (wave == 0 ? 0 : wave == 4 ? 1 : a.NT) : wave, js = sbd ? 2 : NW;
  for (int J = j0; J < a.NT; J += js) {
    const int ti = tile_index(J, J, a.NT);
    const size_t off = (size_t)ti * 256 + lane;
    const int col = 16 * J + (lane & 15);
    double dav[4], dbv[4];
    if constexpr (DYN::n == 2) {
      spread_dblock(((const double*)(a.cbuf + CL.DAc))[(size_t)ti * 64 + lane], dav);
      spread_dblock(((const double*)(a.cbuf + CL.DBc))[(size_t)ti * 64 + lane], dbv);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int tr = (lane >> 4) + 4 * r;
      double da, db;
      if constexpr (DYN::n == 2) {
        da = dav[r];
        db = dbv[r];
      } else {
        da = DA[off + 64 * r];
        db = DB[off + 64 * r];
      }
      double v = h_element<DYN, MEAS, HUBER>(a, Phi, Es, FtE, G, Cc[off + 64 * r], da, db, 16 * J + tr, col, Dm, LAM);
      if (BOUNDED && (ACT[16 * J + tr] | ACT[col]) && 16 * J + tr != col) v = 0.0;
      DT[J * DTS + tr * 16 + (lane & 15)] = v;
    }
  }
}

// Load H tiles from a dense (dp x dp) matrix (MODE_LINSOLVE).
template <int SLOTS>
__device__ __forceinline__ void load_tiles(const GnArgs& a, const SmemLayout& SL, double* sm, const double* Hb,
                                           d4 (&acc)[SLOTS], int wave, int lane, int stab) {
  const int dp = 16 * a.NT;
#pragma unroll
  for (int s = 0; s < SLOTS; ++s) {
    const int IJ = slot_ij(stab, s);
    if (IJ < 0) {
      acc[s] = d4{0.0, 0.0, 0.0, 0.0};
    } else {
      const int I = IJ & 0xffff, J = IJ >> 16;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        // upper block (J, I) of the tile = transpose of the lower block read from H
        const int row = 16 * J + (lane >> 4) + 4 * r, col = 16 * I + (lane & 15);
        acc[s][r] = -Hb[(size_t)col * dp + row];
      }
    }
  }
  double* DT = sm + SL.DT;
  for (int J = wave; J < a.NT; J += NW)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int tr = (lane >> 4) + 4 * r;
      DT[J * DTS + tr * 16 + (lane & 15)] = Hb[(size_t)(16 * J + tr) * dp + 16 * J + (lane & 15)];
    }
}

// LDS ordering between lanes of ONE wave: LDS operations of a wave execute in
// order, so a compiler-level fence plus a wait on the wave's own stores suffices.
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Sum of v over the 16 lanes of a DPP row (lanes with equal l >> 4), result in
// every lane of the row: xor 1, xor 2 (quad_perm), half-mirror, mirror.
__device__ __forceinline__ double row16_sum(double v) {
#define MHE_DPP_ADD(ctrl)                                                                   \
  {                                                                                         \
    const long long bits = __double_as_longlong(v);                                         \
    const int lo = __builtin_amdgcn_mov_dpp((int)bits, ctrl, 0xF, 0xF, false);              \
    const int hi = __builtin_amdgcn_mov_dpp((int)(bits >> 32), ctrl, 0xF, 0xF, false);      \
    v += __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);                    \
  }
  MHE_DPP_ADD(0xB1)   // quad_perm [1,0,3,2]
  MHE_DPP_ADD(0x4E)   // quad_perm [2,3,0,1]
  MHE_DPP_ADD(0x141)  // row_half_mirror
  MHE_DPP_ADD(0x140)  // row_mirror
#undef MHE_DPP_ADD
  return v;
}

// Sums over the 16 lanes of a DPP row of four values at once: lane (c, g) ends with
// sum over its row of v[r], r = 2 (c >> 3) + ((c >> 2) & 1) (replicated over c & 3).
// The first two steps exchange half of the remaining values (row_ror:8 pairs c with
// c ^ 8, row_half_mirror c with 7 - c inside each half), the last two are plain
// butterflies: 6 DPP moves and 4 adds instead of 4 row16_sum's 16 and 16.
__device__ __forceinline__ double row16_sum4(const double (&v)[4], int c) {
  const bool b3 = c & 8, b2 = c & 4;
  const double k0 = b3 ? v[2] : v[0], k1 = b3 ? v[3] : v[1];
  const double s0 = b3 ? v[0] : v[2], s1 = b3 ? v[1] : v[3];
  const double w0 = k0 + dpp_d<0x128>(s0), w1 = k1 + dpp_d<0x128>(s1);  // row_ror:8
  const double k = b2 ? w1 : w0, t = b2 ? w0 : w1;
  double x = k + dpp_d<0x141>(t);  // row_half_mirror
  x += dpp_d<0x1B>(x);             // quad_perm [3,2,1,0]
  x += dpp_d<0xB1>(x);             // quad_perm [1,0,3,2]
  return x;
}

// acc -= (src0 of lane j of this 16-lane row) * src1: v_fmac_f64 with a negated DPP64
// row_newbcast source (one instruction; the compiler does not fuse a v_mov_b64_dpp
// into an f64 fma itself).  ISA hazard: a DPP source must not have been written by
// the two previous VALU instructions.  The first use after src0 was written
// (`fresh`) carries the wait states and passes src0 through as an output, so every
// later use depends on it and cannot be scheduled in front of it.
#define MHE_FMAC_BCAST(J)                                                                                  \
  case J:                                                                                                  \
    if (fresh)                                                                                             \
      asm("s_nop 1\n\tv_fmac_f64_dpp %0, -%1, %2 row_newbcast:" #J " row_mask:0xf bank_mask:0xf"          \
          : "+v"(acc), "+v"(src0) : "v"(src1));                                                            \
    else                                                                                                   \
      asm("v_fmac_f64_dpp %0, -%1, %2 row_newbcast:" #J " row_mask:0xf bank_mask:0xf"                       \
          : "+v"(acc) : "v"(src0), "v"(src1));                                                             \
    break;
__device__ __forceinline__ void fnmac_rowbcast(double& acc, double& src0, double src1, int j, bool fresh) {
  switch (j) {
    MHE_FMAC_BCAST(1) MHE_FMAC_BCAST(2) MHE_FMAC_BCAST(3) MHE_FMAC_BCAST(4) MHE_FMAC_BCAST(5)
    MHE_FMAC_BCAST(6) MHE_FMAC_BCAST(7) MHE_FMAC_BCAST(8) MHE_FMAC_BCAST(9) MHE_FMAC_BCAST(10)
    MHE_FMAC_BCAST(11) MHE_FMAC_BCAST(12) MHE_FMAC_BCAST(13) MHE_FMAC_BCAST(14) MHE_FMAC_BCAST(15)
    default: break;
  }
}
#undef MHE_FMAC_BCAST

// The value of the first 16-lane row (lanes 0..15) in the first two rows: element
// [0] of v_permlane16_swap over two copies of v (two 64-bit moves instead of four
// 32-bit ones: the copies are opaque, so the swaps consume them in place).
__device__ __forceinline__ double row0_both(double v) {
  double t1 = v, t2 = v;
  asm volatile("" : "+v"(t1), "+v"(t2));
  const long long b1 = __double_as_longlong(t1), b2 = __double_as_longlong(t2);
  const auto l = __builtin_amdgcn_permlane16_swap((int)b1, (int)b2, false, false);
  const auto h = __builtin_amdgcn_permlane16_swap((int)(b1 >> 32), (int)(b2 >> 32), false, false);
  return __longlong_as_double(((long long)h[0] << 32) | (unsigned int)l[0]);
}

// 1/sqrt(x) for a positive finite pivot: hardware v_rsq_f64 (~1e-9 relative)
// refined by one Newton step (error squared: ~1 ulp).  Non-positive or
// non-finite pivots are flagged by the caller and poison the factor anyway.
// (Writing the step as four instructions with the halving in the fma's output
// modifier needs inline asm, and then a wait state of its own after the rsq: no gain.)
__device__ __forceinline__ double rsqrt_pivot(double x) {
  const double r = __builtin_amdgcn_rsq(x);
  const double e = fma(-x * r, r, 1.0);  // 1 - x r^2
  return fma(0.5 * r, e, r);
}

// Panel of block k, run by ONE wave (look-ahead: during the previous step's
// trailing update).  On entry DT[k] holds the fully updated A_kk (row-major).
// One right-looking elimination in which the same register index j carries two
// things, one per lane role:
//   lanes  0..15  row i of A_kk:              v[j] = A'_ij
//   lanes 16..31  column t of the identity:   v[j] = E'_jt  (loaded from UN)
// Pivot c:  rs = 1 / sqrt(A'_cc);  q = v[c] rs  (= L_ic on row lanes, = (L^-1)_ct
// on the others, final at that point);  then for j > c
//   v[j] -= L_jc q   with L_jc = q of row lane j,
// i.e. ONE fma updates the Cholesky trailing row and the forward substitution
// L Y = I together: a v_fmac_f64 whose DPP64 row_newbcast source broadcasts L_jc
// from lane j of the row (the L column reaches the identity lanes' row by one
// v_permlane16_swap per pivot).  ~450 instructions, the wave's issue rate bounds it
// (every instruction counts, whatever its kind).  Stores L_kk^-T into DT[k] (row
// stride LIS).  The right-hand side is NOT carried here: y_k = L_kk^-1 b_k is formed
// later by another wave (off this critical chain).
// Returns true if a pivot was not positive and finite (wave-uniform; tested on the
// high word in scalar ALU: a pivot passes when its high word is in [1, 0x7FEFFFFF],
// i.e. positive, finite and >= 2^-1042 -- the larger subnormals pass, zero, the
// smallest subnormals, negatives, inf and NaN are flagged).
__device__ __forceinline__ bool panel(double* DTk, const double* UN, int lane) {
  const int i = lane & 15;
  const bool erow = (lane >= 16 && lane < 32);
  const double* src = erow ? UN + unit_row(i) : DTk + i * 16;
  double v[16];
#pragma unroll
  for (int c = 0; c < 16; c += 2) {
    const double2 a2 = *(const double2*)(src + c);
    v[c] = a2.x;
    v[c + 1] = a2.y;
  }
  unsigned bad = 0;
#pragma unroll
  for (int c = 0; c < 16; ++c) {
    const double piv = readlane_d(v[c], c);
    bad |= (unsigned)__double2hiint(piv) - 1u >= 0x7FEFFFFFu;  // high word not in [1, 0x7FEFFFFF]
    double q = v[c] * rsqrt_pivot(piv);
    v[c] = q;
    if (c < 15) {
      // L column c (the row lanes' q) into both 16-lane rows, then for j > c
      // v[j] -= L_jc q with L_jc broadcast from lane j of the row by the fma itself
      double lq = row0_both(q);
#pragma unroll
      for (int j = c + 1; j < 16; ++j) fnmac_rowbcast(v[j], lq, q, j, j == c + 1);
    }
  }
  if (erow) {
#pragma unroll
    for (int j = 0; j < 16; ++j) DTk[i * LIS + j] = v[j];  // (L^-T)[t][j] = (L^-1)[j][t]
  }
  return bad != 0;
}

// y = L^-1 b for one block (L^-T stored with row stride LIS), by a whole wave:
// lane (c, g = l >> 4) sums the terms s = 4g..4g+3 of row c of L^-1, i.e. column
// c of L^-T, rows4_sum completes the dot.  Lanes 0..15 write y[c].
__device__ __forceinline__ void block_fwd(const double* LT, const double* b, double* y, int lane);

// Right-looking blocked Cholesky H = U^T U (U = L^T) with the forward solve
// U^T y = b (b = -g in BV) fused.  Slot (I, J), I > J, holds the upper block
// H[J][I] in C layout; after step J it holds U_JI.  Per block row k:
//   T(k)  owners of the tiles (k, b), b > k:  U_kb = L_kk^-1 A_kb  (4 MFMAs, the
//         tile is the B operand straight from its registers, L_kk^-1 the A
//         operand from LDS); U_kb -> PB in register order (= row-major).
//   U(k)  trailing update A_ab -= U_ka^T U_kb (a <= b) with both operands read
//         row-major from PB, and b_b -= U_kb^T y_k from PB (VALU); the panel
//         wave (k+1) % NW first finishes b_{k+1} and the diagonal block k+1,
//         then runs panel(k+1) while the other waves do the remaining tiles
//         (look-ahead: no separate panel phase).
// Two workgroup barriers per block row.  Returns false on a bad pivot.
template <int SLOTS>
__device__ __forceinline__ bool factor_forward(const GnArgs& a, const SmemLayout& SL, double* sm,
                                               d4 (&acc)[SLOTS], int wave, int lane, int stab, DIAG_FDECL) {
  double* BV = sm + SL.BV;
  double* YV = sm + SL.YV;
  double* PB = sm + SL.PB;
  double* DT = sm + SL.DT;
  int* flag = (int*)(sm + SL.RED + 4 * NW);
  const int NT = a.NT;
  bool bad = false;
  // k = -1 is the prologue: panel(0) only
#pragma unroll 1
  for (int k = -1; k + 1 < NT; ++k) {
    // opaque per-step copies: keep LICM from hoisting decoded slots and lane
    // masks out of the step loop (they would spill)
    int lane_o = lane, wave_o = wave, stab_o = stab;
    asm volatile("" : "+v"(lane_o));
    asm volatile("" : "+s"(wave_o));
    asm volatile("" : "+v"(stab_o));
    // ---- T(k): U_kb = L_kk^-1 A_kb for the tiles (k, b) of this wave, slots [sT, sU)
    const int sT = slot_start(k < 0 ? 0 : k, wave_o, NT), sU = slot_start(k + 1, wave_o, NT);
    const int nS = slot_start(NT - 1, wave_o, NT);
    // the slot ranges [sT, sU) and [sU, nS) as wave-uniform bit masks: one bit test
    // per unrolled slot instead of two compares and their combination
    const unsigned mT = (1u << sU) - (1u << sT), mU = (1u << nS) - (1u << sU);
    if (k >= 0 && wave_o == (k + 2) % NW)  // forward solve, one block behind the factorization
      block_fwd(DT + k * DTS, BV + 16 * k, YV + 16 * k, lane_o);
    if (k >= 0) {
      const double* LT = DT + k * DTS;
      double la[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) la[r] = LT[(4 * r + (lane_o >> 4)) * LIS + (lane_o & 15)];  // L^-1[l&15][4r+(l>>4)], negated by the MFMA
#pragma unroll
      for (int s = 0; s < SLOTS; ++s) {
        if ((mT >> s) & 1u) {
          d4 u = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
          for (int r = 0; r < 4; ++r) u = __builtin_amdgcn_mfma_f64_16x16x4f64(la[r], acc[s][r], u, 0, 0, MFMA_NEG_A);
          if (!KO(0)) acc[s] = u;
          const int I = slot_ij(stab_o, s) & 0xffff;
#pragma unroll
          for (int r = 0; r < 4; ++r) PB[(I - k - 1) * 256 + r * 64 + lane_o] = u[r];
        }
      }
    }
    DIAG_MARK(8);
    __syncthreads();
    DIAG_MARK(9);
    // ---- U(k)
    const int pw = (k + 1) % NW;  // panel wave of this step
    if (wave_o == pw) {
      // the panel is the serial critical path of the factorization: issue it ahead
      // of the co-resident waves (the other workgroup's and this one's MFMA work)
      __builtin_amdgcn_s_setprio(3);
      double* DTn = DT + (k + 1) * DTS;
      if (k >= 0) {
        d4 t;
        double v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          t[r] = DTn[r * 64 + lane_o];
          v[r] = PB[r * 64 + lane_o];
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) t = __builtin_amdgcn_mfma_f64_16x16x4f64(v[r], v[r], t, 0, 0, MFMA_NEG_A);
#pragma unroll
        for (int r = 0; r < 4; ++r) DTn[r * 64 + lane_o] = t[r];
        wave_lds_sync();
      }
      if (!KO(3)) bad |= panel(DTn, sm + SL.UN, lane_o);
      __builtin_amdgcn_s_setprio(0);
    } else if (k >= 0 && !KO(4)) {
      // b_b -= U_kb^T y_k for b >= k + 1: one output per lane of the other waves
      const int vt = ((wave_o - pw - 1 + NW) % NW) * 64 + lane_o;
      const int bq = k + 1 + (vt >> 4), c = vt & 15;
      if (bq < NT) {
        const double* ub = PB + (bq - k - 1) * 256 + c;
        double s0 = 0.0, s1 = 0.0;
#pragma unroll
        for (int q = 0; q < 16; q += 2) {
          s0 += ub[q * 16] * YV[16 * k + q];
          s1 += ub[(q + 1) * 16] * YV[16 * k + q + 1];
        }
        BV[16 * bq + c] -= s0 + s1;
      }
    }
    DIAG_MARK(12);
    // off-diagonal trailing update over the slot suffix [sU, nS)
    if (k >= 0 && !KO(1)) {
#pragma unroll
      for (int s = 0; s < SLOTS; ++s) {
        if ((mU >> s) & 1u) {
          const int IJ = slot_ij(stab_o, s);
          const double* ua = PB + ((IJ >> 16) - k - 1) * 256 + lane_o;
          const double* ub = PB + ((IJ & 0xffff) - k - 1) * 256 + lane_o;
          double av[4], bv[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            av[r] = ua[64 * r];
            bv[r] = ub[64 * r];
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[s] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[r], bv[r], acc[s], 0, 0, 0);
        }
      }
    }
    DIAG_MARK(13);
    // remaining diagonal blocks J > k + 1 of this wave
    for (int J = wave_o; J < NT; J += NW) {
      if (J <= k + 1 || k < 0 || KO(2)) continue;
      double* DTj = DT + J * DTS;
      d4 t;
      double v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        t[r] = DTj[r * 64 + lane_o];
        v[r] = PB[(J - k - 1) * 256 + r * 64 + lane_o];
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) t = __builtin_amdgcn_mfma_f64_16x16x4f64(v[r], v[r], t, 0, 0, MFMA_NEG_A);
#pragma unroll
      for (int r = 0; r < 4; ++r) DTj[r * 64 + lane_o] = t[r];
    }
    DIAG_MARK(10);
    __syncthreads();  // PB is single-buffered; DT[k+1] / y_{k+1} complete
    DIAG_MARK(11);
  }
  if (bad && lane == 0) flag[0] = 1;  // flag was zeroed at kernel start
  __syncthreads();
  return flag[0] == 0;
}

// ------------------------------------------------------------ small-batch factorization
// When the batch gives each CU at most one trajectory (C2 strong scaling at 4 and 8
// GPUs: 256 / 128 per GPU) a trajectory's GN iteration is a latency chain, and in the
// factorization above every block step costs panel + two workgroup barriers + the T
// and diagonal-update MFMAs of the next critical tile, one after another.
// factor_forward_sb takes the critical chain P(k) -> T(k, k+1) -> D_{k+1} -> P(k+1) off
// the workgroup barriers: ONE wave (CP, wave 0) runs it alone, one barrier per block
// step, while six worker waves own the 78 off-diagonal tiles (13 slots each: the
// one-workgroup-per-CU instance may use 256 VGPRs) and CP's SIMD partner (wave 4; waves
// w and w + 4 share a SIMD) does only the forward substitution, so no MFMA of theirs
// competes with the panel for that SIMD.  Interval k (between barriers k and k + 1):
//   CP       A_{k,k+1} (handed over by its owner, updated through step k - 2)
//              -= U_{k-1,k}^T U_{k-1,k+1};  U_{k,k+1} = L_kk^-1 A_{k,k+1} -> PB_k;
//            D_{k+1} -= U_{k,k+1}^T U_{k,k+1};  panel(k + 1)
//   workers  every owned tile (J, I), J >= k, other than (k, k+1): the deferred trailing
//            update of step k - 1, A_JI -= U_{k-1,J}^T U_{k-1,I} (from PB_{k-1});
//            row k tiles then T(k) -> PB_k and D_I -= U_kI^T U_kI (their own D_I);
//            tile (k+1, k+2) is handed to CP (HB); CP keeps the band tiles U_{k,k+1} in
//            LDS (BAND), where backward_sb reads them (their owners' registers go stale)
//   wave 4   y_{k-1} = L^-1 b_{k-1}, b_b -= U_{k-1,b}^T y_{k-1}  (b >= k)
// PB (rows k - 1 and k of U) and HB are double-buffered, so one barrier per interval
// orders every hand-off.  Every tile still receives its trailing updates in k order (the
// deferral moves WHEN step k - 1's update is applied, not its order), so the factor --
// and the iterates -- are bitwise those of factor_forward (the two-workgroups-per-CU
// instance): tests/test_gpu_parity.py::test_small_batch_instance_matches_full_occupancy_instance
// and ::test_full_occupancy_instance_iterates_match_oracle assert it, which is what keeps
// results independent of the GPU count a strong split runs on.
#ifndef MHE_SB_WEIGHTED
#define MHE_SB_WEIGHTED 0  // A/B: 7:6 weighted tile shares (factorization -10 %, build / backward slower: -3 % overall)
#endif
#ifndef MHE_GN_SB
#define MHE_GN_SB 1  // 0: no small-batch factorization (A/B builds only: the round-4 small-batch instance)
#endif
constexpr int SB_WORKERS = 6;
// Waves w and w + 4 share a SIMD, and the older one (1, 2, 3) wins the issue arbitration
// of every pair, so with equal shares the younger one (5, 6, 7) finished an interval
// ~20 % later.  The tiles are dealt by smooth weighted round robin, weights 7 : 6 for the
// older / younger workers (0-2 = waves 1-3, 3-5 = waves 5-7): 14 and 12 tiles, and every
// interval's active tiles split about 7 : 6 as well.
constexpr int SB_SLOTS = MHE_SB_WEIGHTED ? 14 : (MAX_NT * (MAX_NT - 1) / 2 + SB_WORKERS - 1) / SB_WORKERS;
__constant__ const unsigned char SB_OWNER[MAX_NT * (MAX_NT - 1) / 2] = {
    0, 1, 2, 3, 4, 5, 0, 1, 2, 3, 4, 5, 0, 1, 2, 3, 4, 5, 0, 1, 2, 3, 4, 5, 0, 1, 2, 3, 4, 5, 0, 1, 2, 3, 4, 5, 0, 1, 2,
    0, 1, 2, 3, 4, 5, 0, 1, 2, 3, 4, 5, 0, 1, 2, 3, 4, 5, 0, 1, 2, 3, 4, 5, 0, 1, 2, 3, 4, 5, 0, 1, 2, 3, 4, 5, 0, 1, 2};

__device__ __forceinline__ int sb_worker(int wave) { return (wave == 0 || wave == 4) ? -1 : wave < 4 ? wave - 1 : wave - 2; }

__device__ __forceinline__ int sb_owner(int u) { return MHE_SB_WEIGHTED ? SB_OWNER[u] : u % SB_WORKERS; }

// slot table of factor_forward_sb: the s-th tile (column-major over I > J) that this
// wave's worker owns
__device__ __forceinline__ int make_slot_table_sb(int wave, int lane, int NT) {
  const int w = sb_worker(wave);
  if (w < 0 || lane >= SB_SLOTS) return -1;
  const int ntl = NT * (NT - 1) / 2;
  int u = 0, seen = 0;
  for (; u < ntl; ++u)
    if (sb_owner(u) == w && seen++ == lane) break;
  if (u >= ntl) return -1;
  int J = 0, base = 0;
  while (u >= base + (NT - 1 - J)) {
    base += NT - 1 - J;
    ++J;
  }
  return (J + 1 + (u - base)) | (J << 16);
}

// The slot masks of every interval of factor_forward_sb, lane k holding interval k's:
// computed once per launch from the slot table (the GN loop then reads them with one
// v_readlane each per interval).
struct SbMasks {
  unsigned A, T, H;
};
template <int SLOTS>
__device__ __forceinline__ SbMasks sb_masks(int lane, int stab, int NT) {
  SbMasks m = {0u, 0u, 0u};
  const int k = lane;
#pragma unroll
  for (int s = 0; s < SLOTS; ++s) {
    const int IJ = slot_ij(stab, s);
    const int I = IJ & 0xffff, J = IJ >> 16;
    const bool ok = IJ >= 0 && k < NT;
    const bool band = J == k && I == k + 1;
    m.A |= (ok && k >= 1 && J >= k && !band) ? 1u << s : 0u;  // deferred update of step k - 1
    m.T |= (ok && J == k && !band) ? 1u << s : 0u;             // T(k) and D_I
    m.H |= (ok && J == k + 1 && I == k + 2) ? 1u << s : 0u;    // next band tile to CP
  }
  return m;
}

template <int SLOTS>
__device__ __forceinline__ bool factor_forward_sb(const GnArgs& a, const SmemLayout& SL, double* sm,
                                                  d4 (&acc)[SLOTS], int wave, int lane, int stab, SbMasks mv,
                                                  DIAG_FDECL) {
  double* BV = sm + SL.BV;
  double* YV = sm + SL.YV;
  double* DT = sm + SL.DT;
  double* PB0 = sm + SL.PB;
  double* HB0 = sm + SL.HB;
  int* flag = (int*)(sm + SL.RED + 4 * NW);
  const int NT = a.NT;
  const int PBS = (NT - 1) * 256;
  bool bad = false;
  // prologue: panel(0) on CP; the owner of tile (0, 1) hands it over
  if (wave == 0) {
    __builtin_amdgcn_s_setprio(3);
    bad |= panel(DT, sm + SL.UN, lane);
    __builtin_amdgcn_s_setprio(0);
  } else {
#pragma unroll
    for (int s = 0; s < SLOTS; ++s)
      if (slot_ij(stab, s) == 1)  // tile (I, J) = (1, 0)
#pragma unroll
        for (int r = 0; r < 4; ++r) HB0[r * 64 + lane] = acc[s][r];
  }
  __syncthreads();
#ifdef MHE_DIAG
  // every wave's busy time per interval (diagnostic build only), in the ZT region
  unsigned long long wt0 = __builtin_amdgcn_s_memtime();
  unsigned long long* busy = (unsigned long long*)(sm + SL.ZT);  // [wave][k], k < 16
#endif
#pragma unroll 1
  for (int k = 0; k < NT; ++k) {
    int lane_o = lane, stab_o = stab;
    asm volatile("" : "+v"(lane_o));
    asm volatile("" : "+v"(stab_o));
    const double* PBp = PB0 + ((k + 1) & 1) * PBS;  // U block row k - 1
    double* PBk = PB0 + (k & 1) * PBS;              // U block row k
    if (wave == 0) {
      if (k + 1 < NT) {
        __builtin_amdgcn_s_setprio(3);
        const double* hb = HB0 + (k & 1) * 256;
        d4 t;
#pragma unroll
        for (int r = 0; r < 4; ++r) t[r] = hb[r * 64 + lane_o];
        if (k >= 1) {
          double av[4], bv[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            av[r] = PBp[r * 64 + lane_o];        // U_{k-1,k}
            bv[r] = PBp[256 + r * 64 + lane_o];  // U_{k-1,k+1}
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) t = __builtin_amdgcn_mfma_f64_16x16x4f64(av[r], bv[r], t, 0, 0, 0);
        }
        const double* LT = DT + k * DTS;
        double la[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) la[r] = LT[(4 * r + (lane_o >> 4)) * LIS + (lane_o & 15)];
        double* DTn = DT + (k + 1) * DTS;
        d4 dn;
#pragma unroll
        for (int r = 0; r < 4; ++r) dn[r] = DTn[r * 64 + lane_o];
        d4 u = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int r = 0; r < 4; ++r) u = __builtin_amdgcn_mfma_f64_16x16x4f64(la[r], t[r], u, 0, 0, MFMA_NEG_A);
#pragma unroll
        for (int r = 0; r < 4; ++r) dn = __builtin_amdgcn_mfma_f64_16x16x4f64(u[r], u[r], dn, 0, 0, MFMA_NEG_A);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          PBk[r * 64 + lane_o] = u[r];
          DTn[r * 64 + lane_o] = dn[r];
          sm[SL.BAND + k * 256 + r * 64 + lane_o] = u[r];
        }
        wave_lds_sync();
        DIAG_MARK(8);
        if (!KO(3)) bad |= panel(DTn, sm + SL.UN, lane_o);
        __builtin_amdgcn_s_setprio(0);
        DIAG_MARK(12);
      }
    } else if (wave == 4) {
      if (k >= 1) {
        block_fwd(DT + (k - 1) * DTS, BV + 16 * (k - 1), YV + 16 * (k - 1), lane_o);
        wave_lds_sync();
        for (int v = lane_o; v < 16 * (NT - k); v += 64) {
          const int bq = k + (v >> 4), c = v & 15;
          const double* ub = PBp + (bq - k) * 256 + c;
          double s0 = 0.0, s1 = 0.0;
#pragma unroll
          for (int q = 0; q < 16; q += 2) {
            s0 += ub[q * 16] * YV[16 * (k - 1) + q];
            s1 += ub[(q + 1) * 16] * YV[16 * (k - 1) + q + 1];
          }
          BV[16 * bq + c] -= s0 + s1;
        }
      }
    }
    {
      // the workers' slot work, outside the role branches (CP and wave 4 own no slots:
      // their masks are 0), so the accumulators are only ever modified under per-slot
      // bits -- a role branch around them made the compiler keep a second copy of all
      // 13 slots and copy it back every interval.  Roles of this interval's slots
      // (worker w owns tiles u = w + 6 s, column-major; row J starts at u = base(J)):
      //   mA  tiles of rows >= k but the band tile (k, k+1): deferred update of step k-1
      //   mT  row k but the band tile: T(k) and D_I
      //   mH  tile (k+1, k+2): handed to CP
#ifdef MHE_DIAG_SUB
      unsigned long long st0 = __builtin_amdgcn_s_memtime();
      if (wave == 1 && lane == 0 && k < 16) busy[7 * 16 + k] = st0 - wt0;
#endif
      const int w = sb_worker(wave);
      const unsigned mA = __builtin_amdgcn_readlane(mv.A, k), mT = __builtin_amdgcn_readlane(mv.T, k),
                     mH = __builtin_amdgcn_readlane(mv.H, k);
#ifdef MHE_DIAG_SUB
      unsigned long long st1 = __builtin_amdgcn_s_memtime();
      if (wave == 1 && lane == 0 && k < 16) busy[2 * 16 + k] = st1 - st0;
#endif
      if (w >= 0) {
      const double* LT = DT + k * DTS;
      double la[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) la[r] = LT[(4 * r + (lane_o >> 4)) * LIS + (lane_o & 15)];
      // three passes (the deferred updates, then T, then the hand-off) rather than one
      // per slot: every update accumulates into its slot in place; a slot that T
      // rewrites in the same pass as its update made the compiler keep the whole
      // accumulator array in temporaries and copy it back every interval
      auto upd_ops = [&](int s, double (&av)[4], double (&bv)[4]) {
        const int IJ = slot_ij(stab_o, s);
        const double* ua = PBp + ((IJ >> 16) - k) * 256 + lane_o;
        const double* ub = PBp + ((IJ & 0xffff) - k) * 256 + lane_o;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          av[r] = ua[64 * r];
          bv[r] = ub[64 * r];
        }
      };
#pragma unroll
      for (int s = 0; s < SLOTS; ++s) {
        if (((mA >> s) & 1u) && !KO(1)) {
          double av[4], bv[4];
          upd_ops(s, av, bv);
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[s] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[r], bv[r], acc[s], 0, 0, 0);
        }
      }
#ifdef MHE_DIAG_SUB
      __builtin_amdgcn_s_waitcnt(0);
      unsigned long long st2 = __builtin_amdgcn_s_memtime();
      if (wave == 1 && lane == 0 && k < 16) busy[3 * 16 + k] = st2 - st1;
#endif
#pragma unroll
      for (int s = 0; s < SLOTS; ++s) {
        if ((mT >> s) & 1u) {
          const int I = slot_ij(stab_o, s) & 0xffff;
          d4 u = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
          for (int r = 0; r < 4; ++r) u = __builtin_amdgcn_mfma_f64_16x16x4f64(la[r], acc[s][r], u, 0, 0, MFMA_NEG_A);
          if (!KO(0)) acc[s] = u;
          double* DTi = DT + I * DTS;
          d4 di;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            PBk[(I - k - 1) * 256 + r * 64 + lane_o] = u[r];
            di[r] = DTi[r * 64 + lane_o];
          }
          if (!KO(2)) {
#pragma unroll
            for (int r = 0; r < 4; ++r) di = __builtin_amdgcn_mfma_f64_16x16x4f64(u[r], u[r], di, 0, 0, MFMA_NEG_A);
#pragma unroll
            for (int r = 0; r < 4; ++r) DTi[r * 64 + lane_o] = di[r];
          }
        }
      }
#ifdef MHE_DIAG_SUB
      __builtin_amdgcn_s_waitcnt(0);
      unsigned long long st3 = __builtin_amdgcn_s_memtime();
      if (wave == 1 && lane == 0 && k < 16) busy[5 * 16 + k] = st3 - st2;
#endif
#pragma unroll
      for (int s = 0; s < SLOTS; ++s) {
        if ((mH >> s) & 1u) {
#pragma unroll
          for (int r = 0; r < 4; ++r) HB0[((k + 1) & 1) * 256 + r * 64 + lane_o] = acc[s][r];
        }
      }
      }
    }
    DIAG_MARK(13);
#ifdef MHE_DIAG
#ifdef MHE_DIAG_SUB
    if ((wave == 0 || wave == 1 || wave == 4) && lane == 0 && k < 16) busy[wave * 16 + k] = __builtin_amdgcn_s_memtime() - wt0;
#else
    if (lane == 0 && k < 16) busy[wave * 16 + k] = __builtin_amdgcn_s_memtime() - wt0;
#endif
#endif
    __syncthreads();
#ifdef MHE_DIAG
    wt0 = __builtin_amdgcn_s_memtime();
#endif
    DIAG_MARK(11);
  }
#ifdef MHE_DIAG
  __syncthreads();
  if (threadIdx.x == 0) {
    // 9: sum over intervals of the slowest worker's busy time; 10: of its excess over
    // CP's; 13: wave 4's (forward substitution) busy time
    for (int k = 0; k < NT && k < 16; ++k) {
      unsigned long long mx = 0;
      for (int w = 1; w < NW; ++w)
        if (w != 4 && busy[w * 16 + k] > mx) mx = busy[w * 16 + k];
      _dg[9] += mx;
      _dg[10] += mx > busy[k] ? mx - busy[k] : 0;
      _dg[13] += busy[4 * 16 + k];
    }
    if (blockIdx.x == 0 && a.dbg)  // block 0's matrix after the per-block stats (diag_phases.py)
      for (int t = 0; t < 8 * 16; ++t) a.dbg[(size_t)gridDim.x * 16 + t] += busy[t];
  }
  __syncthreads();
  for (int t = threadIdx.x; t < 256; t += NTHREADS) sm[SL.ZT + t] = 0.0;  // the zero tile again
  __syncthreads();
#endif
  if (bad && lane == 0) flag[0] = 1;  // flag was zeroed at kernel start
  __syncthreads();
  return flag[0] == 0;
}

// Sum over the four 16-lane rows of a wave (v_permlane16/32_swap), result in every row.
__device__ __forceinline__ double rows4_sum(double v) {
  long long b = __double_as_longlong(v);
  int lo = (int)b, hi = (int)(b >> 32);
  auto l1 = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
  auto h1 = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
  v = __longlong_as_double(((long long)h1[0] << 32) | (unsigned int)l1[0]) +
      __longlong_as_double(((long long)h1[1] << 32) | (unsigned int)l1[1]);
  b = __double_as_longlong(v);
  lo = (int)b;
  hi = (int)(b >> 32);
  auto l2 = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
  auto h2 = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
  return __longlong_as_double(((long long)h2[0] << 32) | (unsigned int)l2[0]) +
         __longlong_as_double(((long long)h2[1] << 32) | (unsigned int)l2[1]);
}

__device__ __forceinline__ void block_fwd(const double* LT, const double* b, double* y, int lane) {
  asm volatile("" : "+v"(lane));  // derive c, g here: a kernel-wide copy of them is what spilled
  const int c = lane & 15, g = lane >> 4;
  const double2 b01 = *(const double2*)(b + 4 * g);
  const double2 b23 = *(const double2*)(b + 4 * g + 2);
  const double* lt = LT + 4 * g * LIS + c;  // (L^-1)[c][s] = (L^-T)[s][c]
  double s = lt[0] * b01.x;
  s = fma(lt[LIS], b01.y, s);
  s = fma(lt[2 * LIS], b23.x, s);
  s = fma(lt[3 * LIS], b23.y, s);
  const double yv = rows4_sum(s);
  if (lane < 16) y[c] = yv;
}

// delta_k = L_kk^-T y_k, in place, by one whole wave: lane (c, g = l >> 4) sums
// the four terms q = 4g..4g+3 of row c of L^-T, rows4_sum completes the dot.
__device__ __forceinline__ void block_back(const double* LT, double* yv, int lane) {
  asm volatile("" : "+v"(lane));  // as block_fwd: no kernel-wide copy of c, g
  const int c = lane & 15, g = lane >> 4;
  const double2 y01 = *(const double2*)(yv + 4 * g);
  const double2 y23 = *(const double2*)(yv + 4 * g + 2);
  const double* lt = LT + c * LIS + 4 * g;
  double s = lt[0] * y01.x;
  s = fma(lt[1], y01.y, s);
  s = fma(lt[2], y23.x, s);
  s = fma(lt[3], y23.y, s);
  const double dv = rows4_sum(s);
  wave_lds_sync();  // every lane has read y before any lane overwrites it
  if (lane < 16) yv[c] = dv;
}

// Backward solve U delta = y (YV, in place), right-looking over block columns:
// once delta_b is known, the owners of the tiles (J, b), J < b, subtract
// U_Jb delta_b from y_J (row sums over the 16 lanes of a DPP row); the owner of
// (b-1, b) then finishes y_{b-1} and forms delta_{b-1} = L^-T y_{b-1} itself.
// One workgroup barrier per block.
template <int SLOTS>
__device__ __forceinline__ void backward(const GnArgs& a, const SmemLayout& SL, double* sm,
                                         d4 (&acc)[SLOTS], int wave, int lane, int stab) {
  const double* DT = sm + SL.DT;
  double* DV = sm + SL.YV;
  const int NT = a.NT;
  if (wave == (NT - 1) % NW) {
    const double* BV = sm + SL.BV;
    block_fwd(DT + (NT - 1) * DTS, BV + 16 * (NT - 1), DV + 16 * (NT - 1), lane);  // y_{NT-1}
    wave_lds_sync();
    block_back(DT + (NT - 1) * DTS, DV + 16 * (NT - 1), lane);
  }
  __syncthreads();
#pragma unroll 1
  for (int bb = NT - 1; bb >= 1 && !KO(5); --bb) {
    int lane_o = lane, stab_o = stab;
    asm volatile("" : "+v"(lane_o));
    asm volatile("" : "+v"(stab_o));
    const double db = DV[16 * bb + (lane_o & 15)];
    const unsigned rm = __builtin_amdgcn_readfirstlane(((const int*)(sm + SL.ROWM))[wave * 16 + bb]);
    // slots in DESCENDING order: within row bb the tile (bb, bb-1) has the largest
    // column-major index, and its owner's delta_{bb-1} is the critical chain
#pragma unroll
    for (int s = SLOTS - 1; s >= 0; --s) {
      if (!((rm >> s) & 1u)) continue;
      const int IJ = slot_ij(stab_o, s);
      const int J = IJ >> 16;
      if (!KO(6) || J == bb - 1) {
        const bool crit = J == bb - 1;
        double* yj = DV + 16 * J;
        const int g = lane_o >> 4, c = lane_o & 15;
        if (crit) {
          __builtin_amdgcn_s_setprio(3);
          double part[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) part[r] = row16_sum(acc[s][r] * db);
          // lane l of row group g = l>>4 holds the sums for rows g + 4r
          // delta_J = L_JJ^-T (y_J - U_{J,bb} delta_bb) straight from these registers:
          // lane (c, g) takes the rows g + 4r it already holds, rows4_sum completes the
          // dot -- no store / reload of y_J in between
          const double* LT = DT + J * DTS;
          double sd = 0.0;
#pragma unroll
          for (int r = 0; r < 4; ++r) sd += LT[c * LIS + g + 4 * r] * (yj[g + 4 * r] - part[r]);
          const double dv = rows4_sum(sd);
          if (lane_o < 16) yj[c] = dv;  // every lane has read y_J (rows4_sum depends on all of them)
          __builtin_amdgcn_s_setprio(0);
        } else {
          // the four row sums at once (row16_sum4): lane (c, g) holds row g + 4 r(c)'s
          const double v[4] = {acc[s][0] * db, acc[s][1] * db, acc[s][2] * db, acc[s][3] * db};
          const double z = row16_sum4(v, c);
          if ((c & 3) == 0) yj[g + 4 * (2 * (c >> 3) + ((c >> 2) & 1))] -= z;
        }
      }
    }
    __syncthreads();
  }
}

// backward() for factor_forward_sb: the critical tile of every block step is the band
// tile U_{bb-1,bb}, which CP kept in LDS (BAND) -- CP (wave 0, no tiles of its own)
// forms delta_{bb-1} from it while the workers subtract their tiles (J, bb), J < bb - 1,
// from y_J out of their registers.  Same operations and order per element as backward().
template <int SLOTS>
__device__ __forceinline__ void backward_sb(const GnArgs& a, const SmemLayout& SL, double* sm,
                                            d4 (&acc)[SLOTS], int wave, int lane, int stab) {
  const double* DT = sm + SL.DT;
  double* DV = sm + SL.YV;
  const int NT = a.NT;
  if (wave == 0) {
    const double* BV = sm + SL.BV;
    block_fwd(DT + (NT - 1) * DTS, BV + 16 * (NT - 1), DV + 16 * (NT - 1), lane);  // y_{NT-1}
    wave_lds_sync();
    block_back(DT + (NT - 1) * DTS, DV + 16 * (NT - 1), lane);
  }
  __syncthreads();
#pragma unroll 1
  for (int bb = NT - 1; bb >= 1 && !KO(5); --bb) {
    int lane_o = lane, stab_o = stab;
    asm volatile("" : "+v"(lane_o));
    asm volatile("" : "+v"(stab_o));
    const double db = DV[16 * bb + (lane_o & 15)];
    const int g = lane_o >> 4, c = lane_o & 15;
    if (wave == 0) {
      const int J = bb - 1;
      const double* ut = sm + SL.BAND + J * 256 + lane_o;
      double* yj = DV + 16 * J;
      double part[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) part[r] = row16_sum(ut[64 * r] * db);
      const double* LT = DT + J * DTS;
      double sd = 0.0;
#pragma unroll
      for (int r = 0; r < 4; ++r) sd += LT[c * LIS + g + 4 * r] * (yj[g + 4 * r] - part[r]);
      const double dv = rows4_sum(sd);
      if (lane_o < 16) yj[c] = dv;
    } else if (!KO(6)) {
      const unsigned rm = __builtin_amdgcn_readfirstlane(((const int*)(sm + SL.ROWM))[wave * 16 + bb]);
#pragma unroll
      for (int s = SLOTS - 1; s >= 0; --s) {
        if (!((rm >> s) & 1u)) continue;
        const int J = slot_ij(stab_o, s) >> 16;
        if (J == bb - 1) continue;  // the band tile: CP's, from LDS
        double* yj = DV + 16 * J;
        const double v[4] = {acc[s][0] * db, acc[s][1] * db, acc[s][2] * db, acc[s][3] * db};
        const double z = row16_sum4(v, c);
        if ((c & 3) == 0) yj[g + 4 * (2 * (c >> 3) + ((c >> 2) & 1))] -= z;
      }
    }
    __syncthreads();
  }
}

// The constants buffer starts with a 256-B header whose first word is a stamp of the
// dims that define its layout (const_tag); a solve whose dims disagree computes
// nothing and reports MHE_STATUS_BAD_CONSTANTS.  The stamp sits at offset 0, so the
// check itself is in bounds for any buffer mhe_build_constants produced, whatever
// dims it was built for.
__device__ __forceinline__ bool tag_ok(const GnArgs& a) {
  return *(const unsigned long long*)a.cbuf == a.tag;
}

__device__ inline void bad_constants(const GnArgs& a, int b, int mode) {
  if (mode == MODE_SOLVE)
    for (int t = threadIdx.x; t < a.d; t += blockDim.x) a.Xout[(size_t)b * a.d + t] = a.X0[(size_t)b * a.d + t];
  if (threadIdx.x == 0) {
    if (mode != MODE_ASSEMBLE) a.status[b] = MHE_STATUS_BAD_CONSTANTS;
    if (mode == MODE_SOLVE) a.iters[b] = 0;
    if (mode != MODE_LINSOLVE) a.cost[b] = NAN;
  }
}

// projected Newton constants (k_gn_bounded, k_big_linesearch; oracle/gn.py has the same)
constexpr double EPS_ACT = 1e-6;
constexpr double ARMIJO_SIGMA = 1e-4;
constexpr int LS_MAX = 30;
constexpr double COST_SLACK = 1e-12;

#include "mhe_big.h"

// Inside the Gauss-Newton loop every phase recomputes the layouts (and the
// table pointers derived from them) from opaque copies of the dimensions
// instead of keeping ~40 derived 64-bit offsets live in SGPRs across the
// factorization, whose broadcasts need the scalar registers (SGPR spills to
// VGPR lanes otherwise push VGPRs to scratch).
__device__ __forceinline__ int opaque_s(int x) {
  asm volatile("" : "+s"(x));
  return x;
}
#define FA a
#define FCL const_layout(opaque_s(a.P), opaque_s(a.M), n, MEAS::p, opaque_s(a.NT))
#define FSL smem_layout(opaque_s(a.P), opaque_s(a.M), n, opaque_s(a.NT), !MEAS::LINEAR, false, SB)

// MINW (launch bounds' 2nd argument): min waves per SIMD -- 4 = two workgroups (trajectories)
// per CU, 128 VGPRs; 2 = the small-batch instance (batch <= CUs: one workgroup per CU
// anyway), which may use 256 VGPRs
// SB: the small-batch factorization (factor_forward_sb, MODE_SOLVE with MINW = 2 only)
template <class DYN, class MEAS, int SLOTS, int mode, bool HUBER = false, int MINW = MHE_GN_MINW, bool SB = false>
__global__ __launch_bounds__(NTHREADS, MINW) void k_gn(GnArgs a) {
  constexpr int n = DYN::n;
  static_assert(!SB || (mode == MODE_SOLVE && MINW <= 2 && NW == 8), "small-batch factorization: one workgroup per CU");
  extern __shared__ __attribute__((aligned(16))) double sm[];
  const ConstLayout CL = const_layout(a.P, a.M, n, MEAS::p, a.NT);
  const SmemLayout SL = smem_layout(a.P, a.M, n, a.NT, !MEAS::LINEAR, false, SB);
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int b = blockIdx.x;
  const int stab = SB ? make_slot_table_sb(wave, lane, a.NT) : make_slot_table(wave, lane, a.NT);
  init_rowmask<SLOTS>((int*)(sm + SL.ROWM), wave, lane, stab);
  SbMasks sbm = {0u, 0u, 0u};
  if constexpr (SB) sbm = sb_masks<SLOTS>(lane, stab, a.NT);
  double* Xs = sm + SL.Xs;
  if (threadIdx.x == 0) *(int*)(sm + SL.RED + 4 * NW) = 0;  // NOT_SPD flag
  init_units(sm + SL.UN);
  if constexpr (SB)
    for (int t = threadIdx.x; t < 256; t += NTHREADS) sm[SL.ZT + t] = 0.0;
  double* DV = sm + SL.YV;  // delta after backward()
  double* RED = sm + SL.RED;
  d4 acc[SLOTS];
#pragma unroll
  for (int s = 0; s < SLOTS; ++s) acc[s] = d4{0.0, 0.0, 0.0, 0.0};
  if (!tag_ok(a)) {  // constants built for other dims: compute nothing
    bad_constants(a, b, mode);
    return;
  }

  __syncthreads();
  if constexpr (mode == MODE_LINSOLVE) {
    const int dp = 16 * a.NT;
    const double* Hb = a.Hin + (size_t)b * dp * dp;
    for (int t = threadIdx.x; t < dp; t += NTHREADS) sm[SL.BV + t] = -a.gin[(size_t)b * dp + t];
    load_tiles<SLOTS>(a, SL, sm, Hb, acc, wave, lane, stab);
    __syncthreads();
    DIAG_DECL
    const bool ok = factor_forward<SLOTS>(a, SL, sm, acc, wave, lane, stab, DIAG_FARGS);
    backward<SLOTS>(a, SL, sm, acc, wave, lane, stab);
    for (int t = threadIdx.x; t < dp; t += NTHREADS) a.dout[(size_t)b * dp + t] = DV[t];
    if (threadIdx.x == 0) a.status[b] = ok ? MHE_STATUS_CONVERGED : MHE_STATUS_NOT_SPD;
    return;
  }

  for (int t = threadIdx.x; t < a.d; t += NTHREADS) Xs[t] = a.X0[(size_t)b * a.d + t];
  __syncthreads();

  int status = MHE_STATUS_MAX_ITER;
  int it = 0;
  DIAG_DECL
  for (;;) {
    DIAG_MARK(7);
    double c1 = node_meas_phase<DYN, MEAS, HUBER>(FA, FCL, FSL, sm, opaque_s(b), DIAG_FARGS);
    DIAG_MARK(6);
    __syncthreads();
    DIAG_MARK(0);
    c1 += grad_phase<DYN>(FA, FCL, FSL, sm, opaque_s(b));
    {
      // park this wave's part of the cost in LDS (a live register across the
      // factorization would spill): read back if the loop exits at this iterate
      const double cwv = wave_sum(c1);
      if (lane == 0) RED[2 * NW + wave] = cwv;
    }
    DIAG_MARK(1);
    if constexpr (mode == MODE_ASSEMBLE) {
      double c2 = 0.0;
      block_reduce2(RED, c1, c2, false);
      build_tiles<DYN, MEAS, SLOTS, HUBER>(FA, FCL, FSL, sm, acc, wave, lane, stab);
      const int dp = 16 * a.NT;
      double* Hb = a.Hout + (size_t)b * dp * dp;
#pragma unroll
      for (int s = 0; s < SLOTS; ++s) {
        const int IJ = slot_ij(stab, s);
        if (IJ >= 0) {
          const int I = IJ & 0xffff, J = IJ >> 16;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int row = 16 * J + (lane >> 4) + 4 * r, col = 16 * I + (lane & 15);
            Hb[(size_t)row * dp + col] = -acc[s][r];
            if (I != J) Hb[(size_t)col * dp + row] = -acc[s][r];
          }
        }
      }
      __syncthreads();  // diagonal tiles (LDS) complete
      for (int t = threadIdx.x; t < a.NT * 256; t += NTHREADS) {
        const int J = t >> 8, tr = (t >> 4) & 15, tc = t & 15;
        Hb[(size_t)(16 * J + tr) * dp + 16 * J + tc] = sm[SL.DT + J * DTS + (t & 255)];
      }
      for (int t = threadIdx.x; t < dp; t += NTHREADS) a.gout[(size_t)b * dp + t] = -sm[SL.BV + t];
      if (threadIdx.x == 0) a.cost[b] = c1;
      return;
    }
    if (it >= a.max_iter) break;
    build_tiles<DYN, MEAS, SLOTS, HUBER, false, SB>(FA, FCL, FSL, sm, acc, wave, lane, stab);
    DIAG_MARK(15);
    __syncthreads();
    DIAG_MARK(2);
    bool ok;
    if constexpr (SB)
      ok = factor_forward_sb<SLOTS>(FA, FSL, sm, acc, wave, lane, stab, sbm, DIAG_FARGS);
    else
      ok = factor_forward<SLOTS>(FA, FSL, sm, acc, wave, lane, stab, DIAG_FARGS);
    DIAG_MARK(3);
    if (!ok) {
      status = MHE_STATUS_NOT_SPD;
      break;
    }
    if constexpr (SB)
      backward_sb<SLOTS>(FA, FSL, sm, acc, wave, lane, stab);
    else
      backward<SLOTS>(FA, FSL, sm, acc, wave, lane, stab);
    DIAG_MARK(4);
    // X += delta (bounded problems run k_gn_bounded).  A non-finite delta is flagged
    // as an infinite step (NONFINITE, X untouched).
    double dmax = 0.0, xmax = 0.0;
    const int tid_u = opaque_tid();
    for (int t = tid_u; t < a.d; t += NTHREADS) {
      const double dv = DV[t];
      dmax = isfinite(dv) ? fmax(dmax, fabs(dv)) : INFINITY;
      xmax = fmax(xmax, fabs(Xs[t] + dv));
    }
    block_reduce2(RED, dmax, xmax, true);
    if (dmax == INFINITY) {
      status = MHE_STATUS_NONFINITE;
      break;
    }
    for (int t = tid_u; t < a.d; t += NTHREADS) Xs[t] = Xs[t] + DV[t];
    __syncthreads();
    ++it;
    if (dmax <= a.tol * (1.0 + xmax)) {
      status = MHE_STATUS_CONVERGED;
      // final cost at the converged iterate
      double cf = node_meas_phase<DYN, MEAS, HUBER>(FA, FCL, FSL, sm, opaque_s(b));
      __syncthreads();
      cf += grad_phase<DYN>(FA, FCL, FSL, sm, opaque_s(b));
      double z = 0.0;
      block_reduce2(RED, cf, z, false);
      if (threadIdx.x == 0) a.cost[b] = cf;
      goto done;
    }
  }
  {
    // every other exit (max_iter, non-SPD pivot, non-finite step) leaves Xs at the
    // iterate of the loop's last residual pass: its cost is already summed
    __syncthreads();
    if (threadIdx.x == 0) {
      double cf = RED[2 * NW];
      for (int w = 1; w < NW; ++w) cf += RED[2 * NW + w];
      a.cost[b] = cf;
    }
  }
done:
  DIAG_MARK(5);
  DIAG_FLUSH(b);
  __syncthreads();
  for (int t = threadIdx.x; t < a.d; t += NTHREADS) a.Xout[(size_t)b * a.d + t] = Xs[t];
  if (threadIdx.x == 0) {
    a.iters[b] = it;
    a.status[b] = status;
  }
}
// ------------------------------------------------------------ bounds
// addVarBounds (nlp/nlp.py:314-317: lb <= x[idx] <= ub at every node) as a
// projected Newton method on the GN model (Bertsekas 1982), restated in
// oracle/gn.py:gauss_newton_bounded -- same constants, same decisions:
//   X <- P(X0); per iteration at X (g = J^T W r, half the cost gradient):
//   eps = min(EPS_ACT (1 + max|X|), max_bounded |X - P(X - g)|)
//   active: bounded, within eps of a bound, gradient pointing out of the box
//   d = -Ht^-1 g   (Ht: H with the active rows / columns reduced to the diagonal)
//   s = P(X + d) - X  (stationarity measure: 0 exactly at a KKT point)
//   Armijo along the projection arc X(a) = P(X + a d), a = 1, 1/2, ... (LS_MAX trials):
//     cost(X(a)) <= cost(X) + 2 sigma [sum_free a g d + sum_act g (X(a) - X)]
//                   + noise(X) + noise(X(a)) + slack |cost(X)|
//   (noise: the cost's rounding level, COST_NOISE eps sum |R e| (|y| + |h|) -- see meas_row)
//   converged when max|s| <= tol (1 + max|X(a)|).
// Limit points are KKT points of the bound-constrained problem (plain clipping of
// the GN step is not: its fixed points need not be).

// box of state component c: intersection of every addVarBounds entry for it
__device__ __forceinline__ void comp_box(const GnArgs& a, int c, double& lo, double& hi) {
  lo = -INFINITY;
  hi = INFINITY;
  for (int i = 0; i < a.n_bounds; ++i)
    if (a.bidx[i] == c) {
      lo = fmax(lo, a.blb[i]);
      hi = fmin(hi, a.bub[i]);
    }
}

// prior cost (X_0 - x0)^T Pw (X_0 - x0), same operation order as grad_phase
template <int n>
__device__ __forceinline__ double prior_cost(const GnArgs& a, const double* Pw, const double* Xs, int b) {
  double r0[n], cost = 0.0;
#pragma unroll
  for (int c = 0; c < n; ++c) r0[c] = Xs[c] - a.x0[(long long)b * n + c];
#pragma unroll
  for (int r = 0; r < n; ++r) {
    double t2 = 0.0;
#pragma unroll
    for (int c = 0; c < n; ++c) t2 += Pw[r * n + c] * r0[c];
    cost += r0[r] * t2;
  }
  return cost;
}

#define FSLB smem_layout(opaque_s(a.P), opaque_s(a.M), n, opaque_s(a.NT), !MEAS::LINEAR, true)

template <class DYN, class MEAS, int SLOTS, bool HUBER = false>
__global__ __launch_bounds__(NTHREADS, MHE_GN_MINW) void k_gn_bounded(GnArgs a) {
  constexpr int n = DYN::n;
  extern __shared__ __attribute__((aligned(16))) double sm[];
  const SmemLayout SL = smem_layout(a.P, a.M, n, a.NT, !MEAS::LINEAR, true);
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int b = blockIdx.x;
  const int stab = make_slot_table(wave, lane, a.NT);
  init_rowmask((int*)(sm + SL.ROWM), wave, lane, stab);
  double* Xs = sm + SL.Xs;
  double* XO = sm + SL.XO;
  int* ACT = (int*)(sm + SL.ACT);
  const double* BV = sm + SL.BV;  // -g at the current iterate (until factor_forward)
  double* GV = sm + SL.GV;        // copy of -g for the line search
  const double* DV = sm + SL.YV;  // step after backward()
  double* RED = sm + SL.RED;
  if (threadIdx.x == 0) *(int*)(sm + SL.RED + 4 * NW) = 0;  // NOT_SPD flag
  init_units(sm + SL.UN);
  d4 acc[SLOTS];
#pragma unroll
  for (int s = 0; s < SLOTS; ++s) acc[s] = d4{0.0, 0.0, 0.0, 0.0};
  if (!tag_ok(a)) {
    bad_constants(a, b, MODE_SOLVE);
    return;
  }
  for (int t = threadIdx.x; t < a.d; t += NTHREADS) {
    double lo, hi;
    comp_box(a, t % n, lo, hi);
    Xs[t] = fmin(fmax(a.X0[(size_t)b * a.d + t], lo), hi);  // X <- P(X0)
  }
  for (int t = threadIdx.x; t < 16 * a.NT; t += NTHREADS) ACT[t] = 0;
  __syncthreads();
  double nz0 = 0.0;  // rounding level of the cost at the iterate (Armijo slack, oracle cost_noise)
  double cost = node_meas_phase<DYN, MEAS, HUBER, true>(FA, FCL, FSLB, sm, opaque_s(b), &nz0);
  __syncthreads();
  cost += grad_phase<DYN>(FA, FCL, FSLB, sm, opaque_s(b));
  block_reduce2(RED, cost, nz0, false);
  int status = MHE_STATUS_MAX_ITER;
  int it = 0;
  DIAG_DECL
  for (;;) {
    if (it >= a.max_iter) break;
    // epsilon-active set
    double w = 0.0, xm = 0.0;
    for (int t = threadIdx.x; t < a.d; t += NTHREADS) {
      double lo, hi;
      comp_box(a, t % n, lo, hi);
      const double x = Xs[t], g = -BV[t];
      xm = fmax(xm, fabs(x));
      if (lo > -INFINITY || hi < INFINITY) w = fmax(w, fabs(x - fmin(fmax(x - g, lo), hi)));
    }
    block_reduce2(RED, w, xm, true);
    const double eps = fmin(EPS_ACT * (1.0 + xm), w);
    for (int t = threadIdx.x; t < a.d; t += NTHREADS) {
      double lo, hi;
      comp_box(a, t % n, lo, hi);
      const double x = Xs[t], g = -BV[t];
      ACT[t] = (lo > -INFINITY || hi < INFINITY) && ((x <= lo + eps && g > 0.0) || (x >= hi - eps && g < 0.0));
      GV[t] = BV[t];
    }
    __syncthreads();
    build_tiles<DYN, MEAS, SLOTS, HUBER, true>(FA, FCL, FSLB, sm, acc, wave, lane, stab);
    __syncthreads();
    const bool ok = factor_forward<SLOTS>(FA, FSLB, sm, acc, wave, lane, stab, DIAG_FARGS);
    if (!ok) {
      status = MHE_STATUS_NOT_SPD;
      break;
    }
    backward<SLOTS>(FA, FSLB, sm, acc, wave, lane, stab);
    // stationarity measure s = P(X + d) - X; keep X for the line search
    double smax = 0.0, fin = 0.0;
    for (int t = threadIdx.x; t < a.d; t += NTHREADS) {
      double lo, hi;
      comp_box(a, t % n, lo, hi);
      const double x = Xs[t], dv = DV[t];
      XO[t] = x;
      if (!isfinite(dv)) fin = 1.0;
      smax = fmax(smax, fabs(fmin(fmax(x + dv, lo), hi) - x));
    }
    block_reduce2(RED, smax, fin, true);
    if (fin != 0.0) {
      status = MHE_STATUS_NONFINITE;  // X untouched
      break;
    }
    // Armijo search along the projection arc (with the rounding levels of both costs as slack)
    double alpha = 1.0, ct = 0.0, nzt = 0.0;
    for (int ls = 0;;) {
      double pred = 0.0;
      for (int t = threadIdx.x; t < a.d; t += NTHREADS) {
        double lo, hi;
        comp_box(a, t % n, lo, hi);
        const double x = XO[t], dv = DV[t], g = -GV[t];
        const double xt = fmin(fmax(x + alpha * dv, lo), hi);
        pred += ACT[t] ? g * (xt - x) : alpha * g * dv;
        Xs[t] = xt;
      }
      __syncthreads();
      nzt = 0.0;
      ct = node_meas_phase<DYN, MEAS, HUBER, true>(FA, FCL, FSLB, sm, opaque_s(b), &nzt);
      if (threadIdx.x == 0 && a.has_prior)
        ct += prior_cost<n>(a, (const double*)(a.cbuf + FCL.Pw), Xs, b);
      block_reduce2(RED, ct, pred, false);
      {
        double z = 0.0;
        block_reduce2(RED, nzt, z, false);
      }
      ++ls;
      if (ct <= cost + 2.0 * ARMIJO_SIGMA * pred + nz0 + nzt + COST_SLACK * fabs(cost) || ls >= LS_MAX) break;
      alpha *= 0.5;
    }
    cost = ct;
    nz0 = nzt;
    ++it;
    double xn = 0.0, z = 0.0;
    for (int t = threadIdx.x; t < a.d; t += NTHREADS) xn = fmax(xn, fabs(Xs[t]));
    block_reduce2(RED, xn, z, true);
    if (smax <= a.tol * (1.0 + xn)) {
      status = MHE_STATUS_CONVERGED;
      break;
    }
    // gradient at the accepted iterate (its node / row quantities are in LDS from the
    // line search's last evaluation)
    grad_phase<DYN>(FA, FCL, FSLB, sm, opaque_s(b));
    __syncthreads();
  }
  __syncthreads();
  for (int t = threadIdx.x; t < a.d; t += NTHREADS) a.Xout[(size_t)b * a.d + t] = Xs[t];
  if (threadIdx.x == 0) {
    a.cost[b] = cost;
    a.iters[b] = it;
    a.status[b] = status;
  }
}
#undef FSLB
#undef FA
#undef FCL
#undef FSL

// ------------------------------------------------------------ constants
// Cc tile element (row, col) of the constant part of J^T W J.
template <class MEAS>
__global__ void k_build_cc(int P, int M, int n, int p, int NT, int has_prior, int huber, double alpha,
                           const double* D, const double* cw, const double* Phi, const double* Qw,
                           const double* Rw, const double* Pw, char* cbuf) {
  const ConstLayout CL = const_layout(P, M, n, p, NT);
  const int ntiles = NT * (NT + 1) / 2;
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= ntiles * 256) return;
  const int t = gid >> 8, e = gid & 255, r = e >> 6, lane = e & 63;
  // tile t -> (I, J): column-major over the lower triangle
  int J = 0, base = 0;
  while (t >= base + (NT - J)) {
    base += NT - J;
    ++J;
  }
  const int I = J + (t - base);
  // tile t = (I, J), I >= J, stores the upper block H[J-block][I-block] in C layout
  const int row = 16 * J + (lane >> 4) + 4 * r, col = 16 * I + (lane & 15);
  const int d = P * n;
  double v;
  if (row < d && col < d) {
    const int j = row / n, a = row % n, l = col / n, bb = col % n;
    double dcd = 0.0;
    for (int k = 0; k < P; ++k) dcd += D[k * P + j] * cw[k] * D[k * P + l];
    v = huber ? 0.0 : alpha * alpha * dcd * Qw[a * n + bb];  // Huber: rebuilt per iteration
    if (MEAS::LINEAR) {  // full_state: H_i = I, G_i = Rw_i
      double s = 0.0;
      for (int i = 0; i < M; ++i) s += Phi[i * P + j] * Phi[i * P + l] * Rw[(i * p + a) * p + bb];
      v += s;
    }
    if (has_prior && j == 0 && l == 0) v += Pw[a * n + bb];
  } else {
    v = (row == col) ? 1.0 : 0.0;
  }
  double* Cc = (double*)(cbuf + CL.Cc);
  Cc[(size_t)t * 256 + r * 64 + lane] = v;
  double da = 0.0, db = 0.0;
  if (row < d && col < d) {
    const int j = row / n, l = col / n;
    da = alpha * D[l * P + j];
    db = alpha * D[j * P + l];
  }
  ((double*)(cbuf + CL.DA))[(size_t)t * 256 + r * 64 + lane] = da;
  ((double*)(cbuf + CL.DB))[(size_t)t * 256 + r * 64 + lane] = db;
  if (r == 0) {
    // lane (c + 16 g) holds node pair (cn, rn) = (c >> 1, (g >> 1) + 2 (2 (g & 1) + (c & 1))):
    // the layout spread_dblock expects
    const int cn = (lane & 15) >> 1, rn = (lane >> 5) + 2 * (2 * ((lane >> 4) & 1) + (lane & 1));
    const int l = 8 * I + cn, j = 8 * J + rn;
    const bool ok = n == 2 && l < P && j < P;
    ((double*)(cbuf + CL.DAc))[(size_t)t * 64 + lane] = ok ? alpha * D[l * P + j] : 0.0;
    ((double*)(cbuf + CL.DBc))[(size_t)t * 64 + lane] = ok ? alpha * D[j * P + l] : 0.0;
  }
}

// ================================================================ host side
// Shared by the translation units: model tables, path selection, and the launch
// templates each pair_*.hip instantiates for its (dynamics, measurement) pairs.

inline bool dyn_info(int id, int& n, int& m) {
  switch (id) {
    case MHE_DYN_SINGLE_INTEGRATOR: n = 1; m = 1; return true;
    case MHE_DYN_SINGLE_INTEGRATOR_2D: n = 2; m = 2; return true;
    case MHE_DYN_SINGLE_INTEGRATOR_3D: n = 3; m = 3; return true;
    case MHE_DYN_DOUBLE_INTEGRATOR: n = 4; m = 2; return true;
    case MHE_DYN_VAN_DER_POL: n = 2; m = 1; return true;
    case MHE_DYN_GNSS_POS_AND_BIAS: n = 5; m = 3; return true;
    case MHE_DYN_MULTI_RECEIVER: n = 8; m = 0; return true;
    case MHE_DYN_GNSS_TWO_RECEIVER: n = 10; m = 6; return true;
    case MHE_DYN_KINEMATIC_BICYCLE: n = 6; m = 2; return true;
    case MHE_DYN_VEHICLE_GNSS: n = 9; m = 2; return true;
    case MHE_DYN_GNSS_8_RECEIVERS: n = 40; m = 24; return true;
  }
  return false;
}

inline bool meas_info(int id, int n, int& p, int& q, bool& linear) {
  switch (id) {
    case MHE_MEAS_FULL_STATE: p = n; q = 0; linear = true; return true;
    case MHE_MEAS_PSEUDORANGE: p = 1; q = 3; linear = false; return true;
    case MHE_MEAS_VEHICLE_PSEUDORANGE: p = 1; q = 3; linear = false; return true;
    case MHE_MEAS_RANGE_3D: p = 1; q = 3; linear = false; return true;
    case MHE_MEAS_MIXED: p = 1; q = MHE_MIXED_Q; linear = false; return true;
  }
  return false;
}

// Register-resident path iff the node-major padded system fits MAX_NT tiles --
// a function of dims alone.  dims->force_large (tests) routes a problem through
// the large-system path so both paths can be compared on identical inputs.
// Mixed-row problems, extra variables and equality constraints
// always take the large-system path (it carries the bordered KKT step).
inline int smem_bytes(const mhe_dims* dm, int NT, bool bounded = false, bool sb = false) {
  int p, q;
  bool lin;
  meas_info(dm->meas_model, dm->n, p, q, lin);
  return smem_layout(dm->N + 1, dm->M, dm->n, NT, !lin, bounded, sb).total * (int)sizeof(double);
}

// The register-resident kernel keeps per-row measurement blocks G_i (n x n) in LDS;
// when they do not fit (e.g. autonomous-car.py: 231 rows x 9 x 9) the problem takes
// the large-system path, which groups rows by epoch.
constexpr int REG_LDS_LIMIT = 160 * 1024;

inline bool is_big(const mhe_dims* dm) {
  if (dm->force_large) return true;
  if (dm->meas_model == MHE_MEAS_MIXED || dm->n_extra > 0 || dm->n_eq > 0) return true;
  const int NT = ((dm->N + 1) * dm->n + 15) / 16;
  if (NT > MAX_NT) return true;
  return smem_bytes(dm, NT, true) > REG_LDS_LIMIT;
}

inline size_t big_ws_doubles(const mhe_dims* dm, int NT) {
  return big_ws_layout(dm->N + 1, dm->M, dm->n, NT, dm->n_extra, dm->n_eq).total;
}

// ------------------------------------------------------------ resjac (kernel-level parity)
// Per-collocation-point residuals and Jacobians at X, one thread per
// (trajectory, node) and per (trajectory, row): W_k = a sum_j D_kj X_j - f(X_k, U_k),
// F_k = df/dx; e_i = y_i - h(x(t_i)), Hm_i = dh/dx at x(t_i) = sum_j Phi_ij X_j.  The
// same device functors and constants as the solve; Phi from the register layout or, on
// the large-system path, from the epoch-compressed rows (row i -> its epoch by erow).
struct ResjacArgs {
  const char* cbuf;
  int P, M, big;
  double alpha;
  const double *X, *U, *Y, *PAR;
  long long ustride, pstride;
  double *W, *F, *E, *Hm;
  int idx[8];
  double dpar[8];
  unsigned long long tag;
};

template <class DYN, class MEAS>
__global__ void k_resjac(ResjacArgs a, int batch) {
  constexpr int n = DYN::n, m = DYN::m, p = MEAS::p, q = MEAS::q;
  const int P = a.P, M = a.M;
  const long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= (long long)batch * (P + M)) return;
  if (*(const unsigned long long*)a.cbuf != a.tag) return;  // constants built for other dims
  const int b = (int)(gid / (P + M)), t = (int)(gid % (P + M));
  const double* X = a.X + (size_t)b * P * n;
  const double *D, *Phi = nullptr, *PhiE = nullptr;
  const int* erow = nullptr;
  int E = 0;
  if (a.big) {
    const BigConst CL = big_const_layout(P, M, n, p);
    D = (const double*)(a.cbuf + CL.D);
    PhiE = (const double*)(a.cbuf + CL.PhiE);
    erow = (const int*)(a.cbuf + CL.erow);
    E = M > 0 ? *(const int*)(a.cbuf + CL.ne) : 0;
  } else {
    const ConstLayout CL = const_layout(P, M, n, p, 1);
    D = (const double*)(a.cbuf + CL.D);
    Phi = (const double*)(a.cbuf + CL.Phi);
  }
  if (t < P) {
    const int k = t;
    double dx[n], xk[n], uk[m > 0 ? m : 1], f[n], F[n * n];
    for (int c = 0; c < n; ++c) dx[c] = 0.0;
    for (int j = 0; j < P; ++j)
      for (int c = 0; c < n; ++c) dx[c] += D[(size_t)k * P + j] * X[j * n + c];
    for (int c = 0; c < n; ++c) xk[c] = X[k * n + c];
    if (m > 0)
      for (int c = 0; c < m; ++c) uk[c] = a.U[(long long)b * a.ustride + (long long)k * m + c];
    DYN::eval(xk, uk, a.dpar, f, F);
    if (a.W)
      for (int c = 0; c < n; ++c) a.W[((size_t)b * P + k) * n + c] = a.alpha * dx[c] - f[c];
    if (a.F)
      for (int c = 0; c < n * n; ++c) a.F[((size_t)b * P + k) * n * n + c] = F[c];
    return;
  }
  const int i = t - P;
  const double* phi = Phi ? Phi + (size_t)i * P : nullptr;
  if (!phi) {  // large-system path: the row's epoch
    int lo = 0, hi = E - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) / 2;
      if (erow[mid] <= i) lo = mid; else hi = mid - 1;
    }
    phi = PhiE + (size_t)lo * P;
  }
  double xi[n], par[q > 0 ? q : 1], h[p], H[p * n];
  for (int c = 0; c < n; ++c) xi[c] = 0.0;
  for (int j = 0; j < P; ++j)
    for (int c = 0; c < n; ++c) xi[c] += phi[j] * X[j * n + c];
  for (int c = 0; c < q; ++c) par[c] = a.PAR[(long long)b * a.pstride + (long long)i * q + c];
  MEAS::eval(xi, par, a.idx, h, H);
  if (a.E)
    for (int r = 0; r < p; ++r) a.E[((size_t)b * M + i) * p + r] = a.Y[((size_t)b * M + i) * p + r] - h[r];
  if (a.Hm)
    for (int c = 0; c < p * n; ++c) a.Hm[((size_t)b * M + i) * p * n + c] = H[c];
}

template <class DYN, class MEAS>
int launch_resjac(ResjacArgs& a, int batch, hipStream_t st) {
  if constexpr (MEAS::MIXED) {
    return MHE_ERR_UNSUPPORTED;  // mixed rows: see mhe_solve parity tests
  } else {
    const long long nt = (long long)batch * (a.P + a.M);
    hipLaunchKernelGGL((k_resjac<DYN, MEAS>), dim3((unsigned)((nt + 255) / 256)), dim3(256), 0, st, a, batch);
    return hipGetLastError() == hipSuccess ? MHE_OK : MHE_ERR_HIP;
  }
}

// Per (dynamics, measurement) pair: the launches that depend on the model types.
struct PairOps {
  // register-resident path: the tile tables of the constants buffer (k_build_cc)
  int (*build_cc)(const mhe_dims* dm, int NT, const double* D, const double* cw, const double* Phi,
                  const double* Qw, const double* Rw, const double* Pw, char* cbuf, hipStream_t st);
  // register-resident path: one fused launch (MODE_SOLVE / ASSEMBLE / LINSOLVE)
  int (*gn)(const mhe_dims* dm, GnArgs& a, int batch, int mode, hipStream_t st);
  // large-system path: max_iter iterations of resid -> assemble -> chol (-> border)
  // -> update / line search, then the final residual pass (A.X holds X0 and the
  // state words are initialised by the caller)
  int (*big)(const mhe_dims* dm, BigArgs& A, int batch, int max_iter, hipStream_t st);
  // kernel-level parity: residuals and Jacobians per node / row (mhe_resjac)
  int (*resjac)(ResjacArgs& a, int batch, hipStream_t st);
  // kernel-level parity of the large-system path: one stage (BIG_STAGE_*) on the workspace
  int (*big_stage)(const mhe_dims* dm, BigArgs& A, int batch, int stage, hipStream_t st);
};

// compute units of the device the launch stream belongs to (not the calling thread's
// current device), cached per device; concurrent callers may both fill a slot, with
// the same value (relaxed atomics: no torn or racy plain accesses)
inline int device_cus(hipStream_t st) {
  static int cus[64] = {0};
  int dev = 0;
  if (hipStreamGetDevice(st, &dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  int c = __atomic_load_n(&cus[dev], __ATOMIC_RELAXED);
  if (c == 0) {
    int v = 0;
    c = hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0 ? v : 256;
    __atomic_store_n(&cus[dev], c, __ATOMIC_RELAXED);
  }
  return c;
}

// Which k_gn instance a register-path launch runs (launch_gn, and mhe_solve_kernel_name
// for the records that name it): a function of the dims, the mode and the batch against
// the launch stream's CU count only.
struct GnChoice {
  bool bounded, huber, sb;
  int smem;
};
inline GnChoice gn_choice(const mhe_dims* dm, int NT, int batch, int mode, hipStream_t st) {
  GnChoice c;
  c.bounded = mode == MODE_SOLVE && dm->n_bounds > 0;
  c.huber = dm->dyn_cost == MHE_COST_HUBER;
  // a batch that gives each CU at most one trajectory runs the small-batch instance:
  // 256 VGPRs (no two-workgroups-per-CU register cap) and factor_forward_sb (C2 strong
  // scaling at 4-8 GPUs: 256 / 128 per GPU)
  c.sb = MHE_GN_SB && mode == MODE_SOLVE && !c.bounded && !c.huber && batch <= device_cus(st) &&
         smem_bytes(dm, NT, false, true) + g_opt_smem_pad <= REG_LDS_LIMIT;
  c.smem = smem_bytes(dm, NT, c.bounded, c.sb) + g_opt_smem_pad;  // pad: mhe_set_option, occupancy A/B only
  return c;
}

template <class DYN, class MEAS>
int launch_gn(const mhe_dims* dm, GnArgs& a, int batch, int mode, hipStream_t st) {
  if constexpr (MEAS::MIXED) {
    return MHE_ERR_UNSUPPORTED;  // mixed rows: large-system path only
  } else {
    const GnChoice ch = gn_choice(dm, a.NT, batch, mode, st);
    const bool bounded = ch.bounded, huber = ch.huber, sb = ch.sb;
    const int smem = ch.smem;
    if (smem > REG_LDS_LIMIT) return MHE_ERR_UNSUPPORTED;
    void (*kern)(GnArgs) = nullptr;
    if (bounded) kern = huber ? k_gn_bounded<DYN, MEAS, MAX_SLOTS, true> : k_gn_bounded<DYN, MEAS, MAX_SLOTS>;
    else if (mode == MODE_SOLVE)
      kern = huber ? k_gn<DYN, MEAS, MAX_SLOTS, MODE_SOLVE, true>
             : sb  ? k_gn<DYN, MEAS, SB_SLOTS, MODE_SOLVE, false, 2, true>
                   : k_gn<DYN, MEAS, MAX_SLOTS, MODE_SOLVE>;
    else if (mode == MODE_ASSEMBLE)
      kern = huber ? k_gn<DYN, MEAS, MAX_SLOTS, MODE_ASSEMBLE, true> : k_gn<DYN, MEAS, MAX_SLOTS, MODE_ASSEMBLE>;
    else kern = k_gn<DYN, MEAS, MAX_SLOTS, MODE_LINSOLVE>;
    if (hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, smem) != hipSuccess)
      return MHE_ERR_HIP;
    hipLaunchKernelGGL(kern, dim3(batch), dim3(NTHREADS), smem, st, a);
    return hipGetLastError() == hipSuccess ? MHE_OK : MHE_ERR_HIP;
  }
}

template <class DYN, class MEAS>
int launch_build_cc(const mhe_dims* dm, int NT, const double* D, const double* cw, const double* Phi,
                    const double* Qw, const double* Rw, const double* Pw, char* cbuf, hipStream_t st) {
  if constexpr (MEAS::MIXED) {
    return MHE_ERR_UNSUPPORTED;
  } else {
    const int ntiles = NT * (NT + 1) / 2;
    hipLaunchKernelGGL(k_build_cc<MEAS>, dim3((ntiles * 256 + 255) / 256), dim3(256), 0, st, dm->N + 1, dm->M,
                       dm->n, dm->p, NT, dm->has_prior, dm->dyn_cost == MHE_COST_HUBER ? 1 : 0, 2.0 / dm->T, D, cw,
                       Phi, Qw, Rw, Pw, cbuf);
    return hipGetLastError() == hipSuccess ? MHE_OK : MHE_ERR_HIP;
  }
}

// The factorization of the large-system path: left-looking block-column updates (default;
// 38 % less HBM traffic than the right-looking trailing update, C3 +5 %, C4 +7.5 %, C5 +8 %);
// the right-looking form (bitwise-identical iterates, tests/test_gpu_big.py) only when a
// caller selected it with mhe_set_option(MHE_OPT_BIG_RIGHT_LOOKING, 1).  MHE_BIG_SPLIT: the
// left-looking form as launches per block column (k_big_chol SPLIT = 1, then k_big_rows over
// the rows below, one workgroup per 8 rows) and one for the solve (SPLIT = 2) -- for wide
// systems by default: C4 +8.9 %, C5 +8.2 %, but C3 -5 % (profiles/r05_ab_big_split.txt).
struct BigCholPlan {
  void (*mono)(BigArgs, int);
  void (*diag)(BigArgs, int);
  void (*bwd)(BigArgs, int);
  int smem, smem_rows, smem_diag;
  bool split;
};
inline int big_chol_plan(const BigArgs& A, BigCholPlan& p) {
  const bool wide = A.NT >= BIG_WIDE_NT;
  p.smem = big_chol_lds(wide ? 8 : 4) * (int)sizeof(double);
  p.smem_rows = big_rows_lds() * (int)sizeof(double);
  const bool ll = g_opt_big_right_looking == 0;
  p.split = ll && (MHE_BIG_SPLIT == 1 || (MHE_BIG_SPLIT == 2 && wide));
  p.mono = wide ? (ll ? k_big_chol<8, true> : k_big_chol<8>) : (ll ? k_big_chol<4, true> : k_big_chol<4>);
  // the split diagonal stage stages a kb x 4 slab at any width (MHE_BIG_DIAG_REG): the
  // 4-wide instance's LDS, two workgroups per CU
  const bool d4w = MHE_BIG_DIAG_REG != 0;
  p.diag = wide && !d4w ? k_big_chol<8, true, 1> : k_big_chol<4, true, 1>;
  p.smem_diag = big_chol_lds(wide && !d4w ? 8 : 4) * (int)sizeof(double);
  p.bwd = wide ? k_big_chol<8, true, 2> : k_big_chol<4, true, 2>;
  for (auto f : {p.mono, p.bwd})
    if (hipFuncSetAttribute((const void*)f, hipFuncAttributeMaxDynamicSharedMemorySize, p.smem) != hipSuccess)
      return -1;
  if (hipFuncSetAttribute((const void*)p.diag, hipFuncAttributeMaxDynamicSharedMemorySize, p.smem_diag) != hipSuccess)
    return -1;
  if (hipFuncSetAttribute((const void*)k_big_rows<>, hipFuncAttributeMaxDynamicSharedMemorySize, p.smem_rows) !=
      hipSuccess)
    return -1;
  return 0;
}
// One half of the batch through the split stages (trajectories boff .. boff + nb - 1);
// after_first (two-stream form): recorded on st after the first diagonal stage.
inline void launch_big_split(const BigCholPlan& p, BigArgs A, int boff, int nb, hipStream_t st,
                             hipEvent_t after_first = nullptr) {
  A.ws += (size_t)boff * A.ws_stride;  // the stages index trajectories by workgroup only
  A.state += boff;
  for (int k0 = 0, kend; k0 < A.NT; k0 = kend) {
    hipLaunchKernelGGL(p.diag, dim3(nb), dim3(BIG_NTHREADS), p.smem_diag, st, A, k0);
    if (k0 == 0 && after_first) (void)hipEventRecord(after_first, st);
    kend = big_split_kend(k0, A.NT);  // the same partition as the stages'

    if (kend < A.NT)
      hipLaunchKernelGGL(k_big_rows<>, dim3((A.NT - kend + BIG_NW - 1) / BIG_NW, nb), dim3(BIG_NTHREADS),
                         p.smem_rows, st, A, k0);
  }
  hipLaunchKernelGGL(p.bwd, dim3(nb), dim3(BIG_NTHREADS), p.smem, st, A, 0);
}

// The second stream and fork / join events of the two-stream split factorization, one set
// per device, created on first use (nullptr: run on one stream).  Concurrent callers:
// launch_big_factor holds `use` from its fork record to its join wait, so no other caller
// re-records the events in between (a stream wait captures the event's last record at
// enqueue time); their second halves share s2 (serialised, each behind its own fork).
struct BigAux {
  hipStream_t s2;
  hipEvent_t fork, join;
  std::mutex use;
};
inline BigAux* big_aux(hipStream_t st) {
  static BigAux aux[16];
  static int made[16] = {0};
  static std::mutex mu;
  int dev = 0, sdev = -1;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 16) return nullptr;
  // the second stream is created on the current device: only when the launch stream is on it
  if (hipStreamGetDevice(st, &sdev) != hipSuccess || sdev != dev) return nullptr;
  std::lock_guard<std::mutex> lock(mu);
  if (!made[dev]) {
    if (hipStreamCreateWithFlags(&aux[dev].s2, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&aux[dev].fork, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&aux[dev].join, hipEventDisableTiming) != hipSuccess)
      return nullptr;
    made[dev] = 1;
  }
  return &aux[dev];
}

// The factorization + solve.  Split: the two halves of the batch go through the stages on
// two streams, so one half's latency-bound diagonal stages and solve overlap the other
// half's row launches (what the one-launch kernel gets from trajectories at different
// phases) -- MHE_BIG_TWO_STREAMS.
inline void launch_big_factor(const BigCholPlan& p, const BigArgs& A, int batch, hipStream_t st) {
  if (!p.split) {
    hipLaunchKernelGGL(p.mono, dim3(batch), dim3(BIG_NTHREADS), p.smem, st, A, 0);
    return;
  }
  BigAux* aux = MHE_BIG_TWO_STREAMS && batch >= 16 ? big_aux(st) : nullptr;
  if (!aux) {
    launch_big_split(p, A, 0, batch, st);
    return;
  }
  std::lock_guard<std::mutex> hold(aux->use);  // this caller's record -> wait pairs, uninterleaved
  const int h = ((batch / 2) + 7) & ~7;  // a multiple of 8 (k_big_rows' XCD grouping)
  // the second half starts one diagonal stage behind the first, so that the halves'
  // latency-bound diagonal stages alternate with the other half's row launches
  launch_big_split(p, A, 0, h, st, aux->fork);
  if (hipStreamWaitEvent(aux->s2, aux->fork, 0) != hipSuccess) {
    (void)hipStreamSynchronize(st);
  }
  launch_big_split(p, A, h, batch - h, aux->s2);
  if (hipEventRecord(aux->join, aux->s2) != hipSuccess || hipStreamWaitEvent(st, aux->join, 0) != hipSuccess)
    (void)hipStreamSynchronize(aux->s2);  // the join failed: wait on the host instead
}

// k_big_assemble's launch shape: per tile position ceil(nchl / WPB) workgroups of WPB
// live pair chunks (the epoch GEMM's operands staged through LDS, big_asm_lds), then the
// other chunks WPB (position, chunk) items per workgroup
struct BigAsmShape {
  int wpb, blocks, lds;
};
inline BigAsmShape big_asm_shape(const BigArgs& A) {
  const int npos = A.NTc * (A.NTc + 1) / 2;
  BigAsmShape s;
  s.wpb = A.nchl > 0 ? (A.nchl < 4 ? A.nchl : 4) : (A.nch < 4 ? A.nch : 4);
  s.blocks = npos * ((A.nchl + s.wpb - 1) / s.wpb) + (npos * (A.nch - A.nchl) + s.wpb - 1) / s.wpb;
  s.lds = big_asm_lds(s.wpb) * (int)sizeof(double);
  return s;
}

// k_big_resid with its dynamic LDS (X staged when MHE_BIG_RESID_LDS: P n doubles; C5 64 KB)
template <class DYN, class MEAS>
inline int launch_big_resid(const BigArgs& A, int batch, int final_pass, hipStream_t st) {
  const int smem = MHE_BIG_RESID_LDS ? A.P * A.n * (int)sizeof(double) : 0;
  if (smem > 0 && hipFuncSetAttribute((const void*)k_big_resid<DYN, MEAS>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                      smem) != hipSuccess)
    return MHE_ERR_HIP;
  hipLaunchKernelGGL((k_big_resid<DYN, MEAS>), dim3(batch), dim3(BIG_NTHREADS), smem, st, A, final_pass);
  return MHE_OK;
}

// Kernel-level parity stages of the large-system path (mhe_assemble_ws /
// mhe_chol_solve_ws): BIG_STAGE_ASSEMBLE runs k_big_resid + k_big_assemble at A.X (H
// tiles and BV = -g in the workspace, cost; with z also the per-epoch border sums),
// BIG_STAGE_FACTOR runs k_big_chol on the workspace's tiles and BV (delta in YV) and,
// for a bordered system, k_big_border on the border the caller imported (w in KS).
// The state words are set by the caller.
constexpr int BIG_STAGE_ASSEMBLE = 0, BIG_STAGE_FACTOR = 1;
template <class DYN, class MEAS>
int launch_big_stage(const mhe_dims* dm, BigArgs& A, int batch, int stage, hipStream_t st) {
  (void)dm;
  if (stage == BIG_STAGE_ASSEMBLE) {
    big_pair_plan(A, BigGSupport<MEAS>::get(A.idx, A.n));
    const BigAsmShape sh = big_asm_shape(A);
    if (launch_big_resid<DYN, MEAS>(A, batch, 0, st) != MHE_OK) return MHE_ERR_HIP;
    hipLaunchKernelGGL((k_big_assemble<DYN, MEAS>), dim3(sh.blocks, batch), dim3(64 * sh.wpb), sh.lds, st, A);
  } else {
    BigCholPlan cp;
    if (big_chol_plan(A, cp) < 0) return MHE_ERR_HIP;
    launch_big_factor(cp, A, batch, st);
    const int K = A.nz + A.nc;  // the bordered (KKT) step through the factor, as the solve's
    if (K > 0) {
      const int smem_b = (K * K + 2 * K) * (int)sizeof(double);
      if (hipFuncSetAttribute((const void*)k_big_border<DYN::n, MEAS::p>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              smem_b) != hipSuccess)
        return MHE_ERR_HIP;
      hipLaunchKernelGGL((k_big_border<DYN::n, MEAS::p>), dim3(batch), dim3(BIG_NTHREADS), smem_b, st, A);
    }
  }
  return hipGetLastError() == hipSuccess ? MHE_OK : MHE_ERR_HIP;
}

template <class DYN, class MEAS>
int launch_big(const mhe_dims* dm, BigArgs& A, int batch, int max_iter, hipStream_t st) {
  big_pair_plan(A, BigGSupport<MEAS>::get(A.idx, A.n));
  BigCholPlan cp;
  if (big_chol_plan(A, cp) < 0) return MHE_ERR_HIP;
  const int K = A.nz + A.nc;
  const int smem_b = (K * K + 2 * K) * (int)sizeof(double);
  if (K > 0 && hipFuncSetAttribute((const void*)k_big_border<DYN::n, MEAS::p>,
                                   hipFuncAttributeMaxDynamicSharedMemorySize, smem_b) != hipSuccess)
    return MHE_ERR_HIP;
  const bool bounded = A.n_bounds > 0;
  const int smem_ls = A.P * A.n * (int)sizeof(double);
  if (bounded) {
    if (smem_ls > 128 * 1024) return MHE_ERR_UNSUPPORTED;
    if (hipFuncSetAttribute((const void*)k_big_linesearch<DYN, MEAS>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            smem_ls) != hipSuccess)
      return MHE_ERR_HIP;
    const size_t nx = (size_t)batch * A.P * A.n;
    hipLaunchKernelGGL(k_big_project<DYN::n>, dim3((unsigned)((nx + 255) / 256)), dim3(256), 0, st, A, batch);
  }
  const BigAsmShape sh = big_asm_shape(A);
  for (int it = 0; it < max_iter; ++it) {
    if (launch_big_resid<DYN, MEAS>(A, batch, 0, st) != MHE_OK) return MHE_ERR_HIP;
    A.asm_zskip = it > 0 && cp.split;  // the previous iteration's factorization left its envelope's zeros
    hipLaunchKernelGGL((k_big_assemble<DYN, MEAS>), dim3(sh.blocks, batch), dim3(64 * sh.wpb), sh.lds, st, A);
    A.asm_zskip = 0;
    launch_big_factor(cp, A, batch, st);
    if (K > 0) hipLaunchKernelGGL((k_big_border<DYN::n, MEAS::p>), dim3(batch), dim3(BIG_NTHREADS), smem_b, st, A);
    if (bounded)
      hipLaunchKernelGGL((k_big_linesearch<DYN, MEAS>), dim3(batch), dim3(BIG_NTHREADS), smem_ls, st, A);
    else
      hipLaunchKernelGGL((k_big_update<DYN::n>), dim3(batch), dim3(256), 0, st, A);
  }
  if (launch_big_resid<DYN, MEAS>(A, batch, 1, st) != MHE_OK) return MHE_ERR_HIP;
  return hipGetLastError() == hipSuccess ? MHE_OK : MHE_ERR_HIP;
}

template <class DYN, class MEAS>
const PairOps* pair_ops() {
  static const PairOps ops = {&launch_build_cc<DYN, MEAS>, &launch_gn<DYN, MEAS>, &launch_big<DYN, MEAS>,
                              &launch_resjac<DYN, MEAS>, &launch_big_stage<DYN, MEAS>};
  return &ops;
}

// Pair groups, one translation unit each (pair_*.hip): the ops of (dyn, meas) or nullptr.
const PairOps* pairs_vdp(int dyn, int meas);
const PairOps* pairs_integrators(int dyn, int meas);
const PairOps* pairs_gnss(int dyn, int meas);
const PairOps* pairs_vehicles(int dyn, int meas);
const PairOps* pairs_receivers(int dyn, int meas);

}  // namespace mhe
