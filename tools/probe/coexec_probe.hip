// Co-issue probe (tools only): do f64 MFMA and VALU from different waves of one
// SIMD overlap?  One workgroup of 8 waves (waves w and w + 4 share a SIMD):
// waves 0-3 run 8 interleaved v_mfma_f64_16x16x4f64 chains, waves 4-7 run 8
// interleaved f64 FMA (or int32 add) chains; each wave stamps its own cycles.
#include <hip/hip_runtime.h>
typedef double d4 __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(512) void k_coexec(double* out, long long* cyc, int mode, int iters) {
  const int wave = threadIdx.x >> 6;
  const long long t0 = __builtin_amdgcn_s_memtime();
  double r = 0.0;
  // mode bits: 1 MFMA on waves 0-3 (8 chains; 1 chain with bit 32), 2 f64 FMA on
  // waves 4-7 (also on waves 0-3 with bit 16), 4 int32 on waves 4-7, 8 s_setprio 3
  // on the VALU waves
  if ((mode & 8) && wave >= 4) __builtin_amdgcn_s_setprio(3);
  if (wave < 4 && (mode & 1) && (mode & 32)) {
    double a = threadIdx.x * 1e-3, b = 1.0 + threadIdx.x * 1e-4;
    d4 c = d4{0, 0, 0, 0};
    for (int it = 0; it < iters * 8; ++it) c = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
    r += c[0] + c[3];
  } else if (wave < 4 && (mode & 1)) {
    double a = threadIdx.x * 1e-3, b = 1.0 + threadIdx.x * 1e-4;
    d4 c[8];
    for (int i = 0; i < 8; ++i) c[i] = d4{0, 0, 0, 0};
    for (int it = 0; it < iters; ++it)
#pragma unroll
      for (int i = 0; i < 8; ++i) c[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c[i], 0, 0, 0);
    for (int i = 0; i < 8; ++i) r += c[i][0] + c[i][3];
  } else if ((wave >= 4 || (mode & 16)) && (mode & 2)) {
    double x[8];
    for (int i = 0; i < 8; ++i) x[i] = threadIdx.x * 1e-3 + i;
    const double m = 1.0 + 1e-9, q = 1e-7;
    for (int it = 0; it < iters * 16; ++it)
#pragma unroll
      for (int i = 0; i < 8; ++i) x[i] = fma(x[i], m, q);
    for (int i = 0; i < 8; ++i) r += x[i];
  } else if (wave >= 4 && (mode & 4)) {
    int x[8];
    for (int i = 0; i < 8; ++i) x[i] = threadIdx.x + i;
    for (int it = 0; it < iters * 16; ++it)
#pragma unroll
      for (int i = 0; i < 8; ++i) x[i] = x[i] * 3 + 1;
    for (int i = 0; i < 8; ++i) r += x[i];
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  out[threadIdx.x] = r;
  if ((threadIdx.x & 63) == 0) cyc[wave] = t1 - t0;
}
extern "C" int run(double* out, long long* cyc, int mode, int iters) {
  hipLaunchKernelGGL(k_coexec, 1, 512, 0, 0, out, cyc, mode, iters);
  return hipDeviceSynchronize();
}
