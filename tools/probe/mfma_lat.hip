// Latency probe: dependent f64 MFMA chains (1, 2, 4 interleaved) and LDS read->use, one wave.
#include <hip/hip_runtime.h>
typedef double d4 __attribute__((ext_vector_type(4)));
template <int CH>
__global__ void k_chain(double* out, long long* cyc, int iters) {
  double a = threadIdx.x * 1e-3, b = 1.0 + threadIdx.x * 1e-4;
  d4 c[CH];
  for (int i = 0; i < CH; ++i) c[i] = d4{0, 0, 0, 0};
  long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int i = 0; i < CH; ++i) c[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c[i], 0, 0, 0);
  }
  d4 s = c[0];
  for (int i = 1; i < CH; ++i) s += c[i];
  long long t1 = __builtin_amdgcn_s_memtime();
  out[threadIdx.x] = s[0] + s[1] + s[2] + s[3];
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}
__global__ void k_lds(double* out, long long* cyc, int iters) {
  __shared__ double buf[1024];
  for (int i = threadIdx.x; i < 1024; i += 64) buf[i] = i;
  __syncthreads();
  int idx = threadIdx.x;
  double acc = 0;
  long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
    double v = buf[idx];
    idx = ((int)v + 1) & 1023;  // dependent chain
    acc += v;
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  out[threadIdx.x] = acc;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}
extern "C" int run(int which, double* out, long long* cyc, int iters) {
  if (which == 1) hipLaunchKernelGGL(k_chain<1>, 1, 64, 0, 0, out, cyc, iters);
  if (which == 2) hipLaunchKernelGGL(k_chain<2>, 1, 64, 0, 0, out, cyc, iters);
  if (which == 4) hipLaunchKernelGGL(k_chain<4>, 1, 64, 0, 0, out, cyc, iters);
  if (which == 8) hipLaunchKernelGGL(k_chain<8>, 1, 64, 0, 0, out, cyc, iters);
  if (which == 0) hipLaunchKernelGGL(k_lds, 1, 64, 0, 0, out, cyc, iters);
  return hipDeviceSynchronize();
}
