// Microbenchmark of the diagonal-block panel (tools only; not part of the product).
// Includes the product source so the measured function is the shipped one.
#define MHE_FAST_BUILD
#include "../../nlp-filter_amd/csrc/mhe_gn.hip"

namespace probe {
using namespace mhe;

// variant 1: hardware v_rsq_f64 (no Newton refinement)
__device__ __forceinline__ bool panel_rawrsq(double* DTk, const double* bk, double* yk, int lane) {
  const int i = lane & 15;
  const bool erow = (lane >= 16 && lane < 32);
  double v[16];
#pragma unroll
  for (int c = 0; c < 16; c += 2) {
    const double2 a2 = *(const double2*)(DTk + i * 16 + c);
    const double2 b2 = *(const double2*)(bk + c);
    v[c] = (lane == 32) ? b2.x : (erow ? (c == i ? 1.0 : 0.0) : -a2.x);
    v[c + 1] = (lane == 32) ? b2.y : (erow ? (c + 1 == i ? 1.0 : 0.0) : -a2.y);
  }
  bool bad = false;
#pragma unroll
  for (int c = 0; c < 16; ++c) {
    const double piv = readlane_d(v[c], c);
    bad |= !(piv > 0.0 && piv < INFINITY);
    const double q = v[c] * __builtin_amdgcn_rsq(piv);
    v[c] = q;
#pragma unroll
    for (int j = c + 1; j < 16; ++j) v[j] -= q * readlane_d(q, j);
  }
  if (erow) {
#pragma unroll
    for (int j = 0; j < 16; ++j) DTk[i * LIS + j] = v[j];
  } else if (lane == 32) {
#pragma unroll
    for (int j = 0; j < 16; ++j) yk[j] = v[j];
  }
  return bad;
}

// variant 2: only the readlane+fma skeleton without pivots (instruction-cost floor)
__device__ __forceinline__ bool panel_skel(double* DTk, const double* bk, double* yk, int lane) {
  const int i = lane & 15;
  double v[16];
#pragma unroll
  for (int c = 0; c < 16; ++c) v[c] = DTk[i * 16 + c];
#pragma unroll
  for (int c = 0; c < 16; ++c) {
    const double q = v[c] * 0.5;
    v[c] = q;
#pragma unroll
    for (int j = c + 1; j < 16; ++j) v[j] -= q * readlane_d(q, j);
  }
#pragma unroll
  for (int j = 0; j < 16; ++j) DTk[i * LIS + j] = v[j];
  return false;
}


// variant 3: row layout (lane i: row i of A and of E = L^-1 work), 16-lane DPP
// row_newbcast broadcasts fused into v_fmac_f64 (one instruction per update)
template <int n>
__device__ __forceinline__ void fmac_bc(double& acc, double src, double m) {
  // acc += src(lane n of this 16-lane row) * m
  asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
               : "+v"(acc) : "v"(src), "v"(m), "i"(n));
}
template <int n>
__device__ __forceinline__ double mov_bc(double src) {
  double r;
  asm volatile("s_nop 1\n\tv_mov_b64_dpp %0, %1 row_newbcast:%2 row_mask:0xf bank_mask:0xf" : "=v"(r) : "v"(src), "i"(n));
  return r;
}
template <int c>
__device__ __forceinline__ void dpp_pivot(double (&a)[16], double (&e)[16], double& bb, double& idg, bool& bad, int i) {
  const double piv = mov_bc<c>(a[c]);
  bad |= !(piv > 0.0 && piv < INFINITY);
  const double rs = rsqrt(piv);
  const double q = a[c] * rs;        // lane j: L_jc
  const double nq = -q;
  const double nmm = (i > c) ? nq * rs : 0.0;   // -A'_ic / A'_cc
  idg = (i == c) ? rs : idg;
#pragma unroll
  for (int j = c + 1; j < 16; ++j) {
    // a[j] -= L_jc L_ic ; L_jc from lane j
    if (j == c + 1) fmac_bc<c + 1 < 16 ? c + 1 : 15>(a[j], q, nq);
    else if (j == c + 2) fmac_bc<c + 2 < 16 ? c + 2 : 15>(a[j], q, nq);
    else if (j == c + 3) fmac_bc<c + 3 < 16 ? c + 3 : 15>(a[j], q, nq);
    else if (j == c + 4) fmac_bc<c + 4 < 16 ? c + 4 : 15>(a[j], q, nq);
    else if (j == c + 5) fmac_bc<c + 5 < 16 ? c + 5 : 15>(a[j], q, nq);
    else if (j == c + 6) fmac_bc<c + 6 < 16 ? c + 6 : 15>(a[j], q, nq);
    else if (j == c + 7) fmac_bc<c + 7 < 16 ? c + 7 : 15>(a[j], q, nq);
    else if (j == c + 8) fmac_bc<c + 8 < 16 ? c + 8 : 15>(a[j], q, nq);
    else if (j == c + 9) fmac_bc<c + 9 < 16 ? c + 9 : 15>(a[j], q, nq);
    else if (j == c + 10) fmac_bc<c + 10 < 16 ? c + 10 : 15>(a[j], q, nq);
    else if (j == c + 11) fmac_bc<c + 11 < 16 ? c + 11 : 15>(a[j], q, nq);
    else if (j == c + 12) fmac_bc<c + 12 < 16 ? c + 12 : 15>(a[j], q, nq);
    else if (j == c + 13) fmac_bc<c + 13 < 16 ? c + 13 : 15>(a[j], q, nq);
    else if (j == c + 14) fmac_bc<c + 14 < 16 ? c + 14 : 15>(a[j], q, nq);
    else if (j == c + 15) fmac_bc<c + 15 < 16 ? c + 15 : 15>(a[j], q, nq);
  }
#pragma unroll
  for (int t = 0; t < c; ++t) fmac_bc<c>(e[t], e[t], nmm);   // E'_it -= m_i E'_ct
  e[c] = (i == c) ? 1.0 : nmm;
  fmac_bc<c>(bb, bb, nmm);
}
template <int c>
__device__ __forceinline__ void dpp_sweep(double (&a)[16], double (&e)[16], double& bb, double& idg, bool& bad, int i) {
  if constexpr (c < 16) {
    dpp_pivot<c>(a, e, bb, idg, bad, i);
    dpp_sweep<c + 1>(a, e, bb, idg, bad, i);
  }
}
__device__ __forceinline__ bool panel_dpp(double* DTk, const double* bk, double* yk, int lane) {
  const int i = lane & 15;
  double a[16], e[16];
#pragma unroll
  for (int c = 0; c < 16; c += 2) {
    const double2 a2 = *(const double2*)(DTk + i * 16 + c);
    a[c] = -a2.x;
    a[c + 1] = -a2.y;
    e[c] = 0.0;
    e[c + 1] = 0.0;
  }
  double bb = bk[i], idg = 0.0;
  bool bad = false;
  dpp_sweep<0>(a, e, bb, idg, bad, i);
  if (lane < 16) {
#pragma unroll
    for (int t = 0; t < 16; ++t) DTk[t * LIS + i] = (t <= i) ? e[t] * idg : 0.0;
    yk[i] = bb * idg;
  }
  return bad;
}

// variant 4: DPP skeleton, no s_nop, non-volatile (timing only)
template <int n>
__device__ __forceinline__ void fmac_bc_nn(double& acc, double src, double m) {
  asm("v_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf" : "+v"(acc) : "v"(src), "v"(m), "i"(n));
}
template <int c>
__device__ __forceinline__ void skel_dpp_pivot(double (&a)[16], int i) {
  const double q = a[c] * 0.5, nq = -q;
  a[c] = q;
#define SK(J) if constexpr (c + J < 16) fmac_bc_nn<(c + J < 16 ? c + J : 15)>(a[c + J < 16 ? c + J : 15], q, nq);
  SK(1) SK(2) SK(3) SK(4) SK(5) SK(6) SK(7) SK(8) SK(9) SK(10) SK(11) SK(12) SK(13) SK(14) SK(15)
#undef SK
}
template <int c>
__device__ __forceinline__ void skel_dpp(double (&a)[16], int i) {
  if constexpr (c < 16) { skel_dpp_pivot<c>(a, i); skel_dpp<c + 1>(a, i); }
}
__device__ __forceinline__ bool panel_skel_dpp(double* DTk, const double* bk, double* yk, int lane) {
  const int i = lane & 15;
  double a[16];
#pragma unroll
  for (int c = 0; c < 16; ++c) a[c] = DTk[i * 16 + c];
  skel_dpp<0>(a, i);
#pragma unroll
  for (int j = 0; j < 16; ++j) DTk[i * LIS + j] = a[j];
  return false;
}

template <int V>
__global__ __launch_bounds__(64) void k_panel_probe(double* out, unsigned long long* cyc, int reps) {
  __shared__ double DT[DTS];
  __shared__ double A0[256];
  __shared__ double bk[16], yk[16];
  const int lane = threadIdx.x;
  for (int t = lane; t < 256; t += 64) {
    const int r = t >> 4, c = t & 15;
    A0[t] = (r == c) ? 20.0 + r : 1.0 / (1.0 + (r > c ? r - c : c - r));
  }
  if (lane < 16) bk[lane] = 1.0 + lane;
  __syncthreads();
  unsigned long long tot = 0;
  bool bad = false;
  for (int rep = 0; rep < reps; ++rep) {
    for (int t = lane; t < 256; t += 64) DT[t] = -A0[t];
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    if (V == 0) bad |= panel(DT, lane);
    if (V == 1) bad |= panel_rawrsq(DT, bk, yk, lane);
    if (V == 2) bad |= panel_skel(DT, bk, yk, lane);
    if (V == 3) bad |= panel_dpp(DT, bk, yk, lane);
    if (V == 4) bad |= panel_skel_dpp(DT, bk, yk, lane);
    __syncthreads();
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    tot += t1 - t0;
  }
  for (int t = lane; t < DTS; t += 64) out[blockIdx.x * 288 + t] = DT[t];
  if (lane < 16) out[blockIdx.x * 288 + 272 + lane] = yk[lane] + (bad ? 1e30 : 0.0);
  if (lane == 0) cyc[blockIdx.x] = tot / reps;
}
}  // namespace probe

extern "C" int probe_panel(int variant, double* out, unsigned long long* cyc, int blocks, int reps) {
  if (variant == 0) hipLaunchKernelGGL(probe::k_panel_probe<0>, dim3(blocks), dim3(64), 0, 0, out, cyc, reps);
  if (variant == 1) hipLaunchKernelGGL(probe::k_panel_probe<1>, dim3(blocks), dim3(64), 0, 0, out, cyc, reps);
  if (variant == 2) hipLaunchKernelGGL(probe::k_panel_probe<2>, dim3(blocks), dim3(64), 0, 0, out, cyc, reps);
  if (variant == 3) hipLaunchKernelGGL(probe::k_panel_probe<3>, dim3(blocks), dim3(64), 0, 0, out, cyc, reps);
  if (variant == 4) hipLaunchKernelGGL(probe::k_panel_probe<4>, dim3(blocks), dim3(64), 0, 0, out, cyc, reps);
  return hipDeviceSynchronize() == hipSuccess ? 0 : -1;
}
