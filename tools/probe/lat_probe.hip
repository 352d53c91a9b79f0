// Dependent-latency microbenchmarks of the primitives the panel is built from
// (tools only): one wave, a chain of 64 dependent ops, cycles per op.
#include <hip/hip_runtime.h>
#include <stdint.h>
typedef double d4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ double rl(double v, int lane) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)b, lane);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), lane);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

template <int which>
__global__ __launch_bounds__(64) void k_lat(double* out, unsigned long long* cyc) {
  const int lane = threadIdx.x;
  double x = 1.0 + lane * 1e-3, y = 0.999;
  asm volatile("" : "+v"(x), "+v"(y));
  d4 c = {x, x, x, x};
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int i = 0; i < 64; ++i) {
    if constexpr (which == 0) x = fma(x, y, 1e-9);                                  // f64 fma chain
    else if constexpr (which == 1) x = __builtin_amdgcn_rsq(x) + 0.5;               // rsq f64
    else if constexpr (which == 2) x = rl(x, i & 63) * y;                            // readlane pair + mul
    else if constexpr (which == 3) c = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, c, 0, 0, 0);  // MFMA acc chain
    else if constexpr (which == 4) { c = __builtin_amdgcn_mfma_f64_16x16x4f64(c[0], y, c, 0, 0, 0); }  // MFMA -> operand
    else if constexpr (which == 5) {                                                 // permlane16 swap pair
      const long long b = __double_as_longlong(x);
      auto l = __builtin_amdgcn_permlane16_swap((int)b, (int)b, false, false);
      auto h = __builtin_amdgcn_permlane16_swap((int)(b >> 32), (int)(b >> 32), false, false);
      x = __longlong_as_double(((long long)h[1] << 32) | (unsigned int)l[0]) * y;
    } else if constexpr (which == 6) x = x * y;                                      // f64 mul chain
    else if constexpr (which == 7) { x = __builtin_amdgcn_rcp(x) + 0.5; }           // rcp f64
    else if constexpr (which == 8) { c = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, c, 0, 0, 0); x = c[1] * y; }  // MFMA -> VALU -> MFMA
  }
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  asm volatile("" ::"v"(x), "v"(c));
  __builtin_amdgcn_sched_barrier(0);
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[lane] = x + c[0] + c[1] + c[2] + c[3];
  if (lane == 0) *cyc = t1 - t0;
}

extern "C" int lat_run(int which, double* out, unsigned long long* cyc) {
  switch (which) {
#define L(w) case w: hipLaunchKernelGGL(k_lat<w>, dim3(1), dim3(64), 0, 0, out, cyc); break;
    L(0) L(1) L(2) L(3) L(4) L(5) L(6) L(7) L(8)
#undef L
  }
  return (int)hipDeviceSynchronize();
}
