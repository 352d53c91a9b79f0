// Hardware probe: f64 MFMA fragment layout + throughput, VALU f64 FMA throughput.
#include <hip/hip_runtime.h>
typedef double d4 __attribute__((ext_vector_type(4)));

__global__ void k_layout(const double* A, const double* B, double* D) {
  int l = threadIdx.x;
  // A is 16x4 row-major, B is 4x16 row-major
  double a = A[(l & 15) * 4 + (l >> 4)];
  double b = B[(l >> 4) * 16 + (l & 15)];
  d4 acc = {0, 0, 0, 0};
  acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
  for (int r = 0; r < 4; ++r) D[l * 4 + r] = acc[r];  // raw dump: lane, reg
}

__global__ void __launch_bounds__(256) k_mfma_rate(double* out, int iters, double s) {
  double a = s * threadIdx.x, b = s + threadIdx.x;
  d4 c0 = {0,0,0,0}, c1 = c0, c2 = c0, c3 = c0;
  for (int i = 0; i < iters; ++i) {
    c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c3, 0, 0, 0);
  }
  d4 t = c0 + c1 + c2 + c3;
  out[blockIdx.x * blockDim.x + threadIdx.x] = t[0] + t[1] + t[2] + t[3];
}

__global__ void __launch_bounds__(256) k_fma_rate(double* out, int iters, double s) {
  double x0 = s * threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5, x6 = x0 + 6, x7 = x0 + 7;
  double m = 0.999999, c = 1e-9;
  for (int i = 0; i < iters; ++i) {
    x0 = fma(x0, m, c); x1 = fma(x1, m, c); x2 = fma(x2, m, c); x3 = fma(x3, m, c);
    x4 = fma(x4, m, c); x5 = fma(x5, m, c); x6 = fma(x6, m, c); x7 = fma(x7, m, c);
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7;
}

extern "C" {
int probe_layout(const double* A, const double* B, double* D, void* stream) {
  hipLaunchKernelGGL(k_layout, dim3(1), dim3(64), 0, (hipStream_t)stream, A, B, D);
  return (int)hipGetLastError();
}
// returns elapsed ms
float probe_rate(int which, double* out, int blocks, int iters, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  hipEventRecord(e0, st);
  if (which == 0) hipLaunchKernelGGL(k_mfma_rate, dim3(blocks), dim3(256), 0, st, out, iters, 1e-3);
  else hipLaunchKernelGGL(k_fma_rate, dim3(blocks), dim3(256), 0, st, out, iters, 1e-3);
  hipEventRecord(e1, st); hipEventSynchronize(e1);
  float ms = 0; hipEventElapsedTime(&ms, e0, e1);
  hipEventDestroy(e0); hipEventDestroy(e1);
  return ms;
}
}
