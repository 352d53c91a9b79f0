// Microbenchmark: cycles per diagonal-block panel, the shipped row sweep panel()
// vs an experimental C-layout blocked panel (panel_c, round 2, not shipped).  Tools only; not part of the product.
#define MHE_FAST_BUILD
#include "../../nlp-filter_amd/csrc/mhe_gn.hip"

namespace probe {
using namespace mhe;

__device__ __forceinline__ void gather_col4(double v, double (&o)[4]) {
  const long long bits = __double_as_longlong(v);
  const int lo = (int)bits, hi = (int)(bits >> 32);
  const auto l16 = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
  const auto h16 = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
  const auto la = __builtin_amdgcn_permlane32_swap(l16[0], l16[0], false, false);
  const auto ha = __builtin_amdgcn_permlane32_swap(h16[0], h16[0], false, false);
  const auto lb = __builtin_amdgcn_permlane32_swap(l16[1], l16[1], false, false);
  const auto hb = __builtin_amdgcn_permlane32_swap(h16[1], h16[1], false, false);
  o[0] = __longlong_as_double(((long long)ha[0] << 32) | (unsigned int)la[0]);
  o[2] = __longlong_as_double(((long long)ha[1] << 32) | (unsigned int)la[1]);
  o[1] = __longlong_as_double(((long long)hb[0] << 32) | (unsigned int)lb[0]);
  o[3] = __longlong_as_double(((long long)hb[1] << 32) | (unsigned int)lb[1]);
}
__device__ __forceinline__ double rcp_pivot(double x) {
  const double r = __builtin_amdgcn_rcp(x);
  return fma(r, fma(-x, r, 1.0), r);
}
// Experimental (round 2, not shipped): the panel from a C-layout tile in registers,
// blocked 4x4 right-looking Cholesky with MFMA trailing updates, then L^-1 by the
// same row operations on I.  Measured slower than the row sweep (mhe::panel).
__device__ __forceinline__ bool panel_c(d4 t, double* DTk, int lane) {
  const int col = lane & 15, g = lane >> 4;
  bool bad = false;
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    const int o = 4 * b;
    double x[4];
    gather_col4(t[b], x);
    const double s00 = -readlane_d(t[b], o), s01 = -readlane_d(t[b], o + 1);
    const double s02 = -readlane_d(t[b], o + 2), s03 = -readlane_d(t[b], o + 3);
    const double s11 = -readlane_d(t[b], o + 17), s12 = -readlane_d(t[b], o + 18);
    const double s13 = -readlane_d(t[b], o + 19), s22 = -readlane_d(t[b], o + 34);
    const double s23 = -readlane_d(t[b], o + 35), s33 = -readlane_d(t[b], o + 51);
    bad |= !(s00 > 0.0 && s00 < INFINITY);
    const double r0 = rsqrt_pivot(s00);
    const double v01 = s01 * r0, v02 = s02 * r0, v03 = s03 * r0;
    x[0] = -x[0] * r0;
    const double p1 = s11 - v01 * v01;
    bad |= !(p1 > 0.0 && p1 < INFINITY);
    const double r1 = rsqrt_pivot(p1);
    const double v12 = (s12 - v01 * v02) * r1, v13 = (s13 - v01 * v03) * r1;
    x[1] = (-x[1] - v01 * x[0]) * r1;
    const double p2 = s22 - v02 * v02 - v12 * v12;
    bad |= !(p2 > 0.0 && p2 < INFINITY);
    const double r2 = rsqrt_pivot(p2);
    const double v23 = (s23 - v02 * v03 - v12 * v13) * r2;
    x[2] = (-x[2] - v02 * x[0] - v12 * x[1]) * r2;
    const double p3 = s33 - v03 * v03 - v13 * v13 - v23 * v23;
    bad |= !(p3 > 0.0 && p3 < INFINITY);
    const double r3 = rsqrt_pivot(p3);
    x[3] = (-x[3] - v03 * x[0] - v13 * x[1] - v23 * x[2]) * r3;
    const double vb = g == 0 ? x[0] : g == 1 ? x[1] : g == 2 ? x[2] : x[3];
    t[b] = vb;
    if (b < 3) {
      const double vm = col >= o + 4 ? vb : 0.0;
      t = __builtin_amdgcn_mfma_f64_16x16x4f64(vm, vb, t, 0, 0, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  d4 z;
#pragma unroll
  for (int r = 0; r < 4; ++r) z[r] = (4 * r + g == col) ? 1.0 : 0.0;
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    const int o = 4 * b;
    const double v01 = readlane_d(t[b], o + 1), v02 = readlane_d(t[b], o + 2);
    const double v03 = readlane_d(t[b], o + 3), v12 = readlane_d(t[b], o + 18);
    const double v13 = readlane_d(t[b], o + 19), v23 = readlane_d(t[b], o + 35);
    const double r0 = rcp_pivot(readlane_d(t[b], o)), r1 = rcp_pivot(readlane_d(t[b], o + 17));
    const double r2 = rcp_pivot(readlane_d(t[b], o + 34)), r3 = rcp_pivot(readlane_d(t[b], o + 51));
    double y[4];
    gather_col4(z[b], y);
    y[0] = y[0] * r0;
    y[1] = (y[1] - v01 * y[0]) * r1;
    y[2] = (y[2] - v02 * y[0] - v12 * y[1]) * r2;
    y[3] = (y[3] - v03 * y[0] - v13 * y[1] - v23 * y[2]) * r3;
    const double zb = g == 0 ? y[0] : g == 1 ? y[1] : g == 2 ? y[2] : y[3];
    if (b < 3) {
      const double vm = col >= o + 4 ? t[b] : 0.0;
      z = __builtin_amdgcn_mfma_f64_16x16x4f64(-vm, zb, z, 0, 0, 0);
    }
    z[b] = zb;
    __builtin_amdgcn_sched_barrier(0);
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) DTk[col * LIS + 4 * r + g] = z[r];
  return bad;
}

// one wave per workgroup; A (16x16, row-major) -> -A in LDS; reps panels, each
// from the same -A (re-read from a second LDS copy so nothing is hoisted)
__global__ __launch_bounds__(64) void k_probe(int variant, const double* A, double* out,
                                              unsigned long long* cyc, int reps) {
  __shared__ double src[256];
  __shared__ double DT[DTS];
  const int lane = threadIdx.x;
  for (int e = lane; e < 256; e += 64) src[e] = -A[e];
  __syncthreads();
  unsigned long long total = 0;
  int bad = 0;
  for (int it = 0; it < reps; ++it) {
    int l = lane;
    asm volatile("" : "+v"(l));
    d4 t;
#pragma unroll
    for (int r = 0; r < 4; ++r) t[r] = src[r * 64 + l];  // C layout = row-major index r*64 + lane
    if (variant == 1)
      for (int e = l; e < 256; e += 64) DT[e] = src[e];
    wave_lds_sync();
    __builtin_amdgcn_s_waitcnt(0);
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    if (variant == 0)
      bad |= panel_c(t, DT, l);
    else
      bad |= panel(DT, l);
    wave_lds_sync();
    const double chk = DT[l];  // wait for the stores
    asm volatile("" ::"v"(chk));
    __builtin_amdgcn_s_waitcnt(0);
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    total += t1 - t0;
  }
  for (int e = lane; e < DTS; e += 64) out[(size_t)blockIdx.x * DTS + e] = DT[e];
  if (lane == 0) cyc[blockIdx.x] = total / reps + (bad ? (1ull << 40) : 0);
}
}  // namespace probe

extern "C" int probe_run(int variant, const double* A, double* out, unsigned long long* cyc, int blocks, int reps) {
  hipLaunchKernelGGL(probe::k_probe, dim3(blocks), dim3(64), 0, 0, variant, A, out, cyc, reps);
  return (int)hipDeviceSynchronize();
}
