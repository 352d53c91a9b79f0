// Dependent-latency microbenchmarks of the primitives the panel is built from
// (tools only): one wave, a chain of 64 dependent ops, cycles per op; 9..13 are
// throughput (8 independent chains).
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
__global__ __launch_bounds__(1024) void k_lat(double* out, unsigned long long* cyc) {
  const int lane = threadIdx.x & 63;
  double x = 1.0 + lane * 1e-3, y = 0.999;
  asm volatile("" : "+v"(x), "+v"(y));
  d4 c = {x, x, x, x};
  double z[8];
  int w[8], sreg[8];
  unsigned long long sm64[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) { z[k] = x + k; w[k] = lane + k; sreg[k] = k; sm64[k] = 0; asm volatile("" : "+v"(z[k]), "+v"(w[k]), "+s"(sreg[k])); }
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
    else if constexpr (which == 9) { z[i & 7] = fma(z[i & 7], y, 1e-9); }          // 8 independent fma chains
    else if constexpr (which == 10) {                                               // 8 independent DPP64 fmac chains
      asm("v_fmac_f64_dpp %0, %1, %2 row_newbcast:3 row_mask:0xf bank_mask:0xf" : "+v"(z[i & 7]) : "v"(x), "v"(y));
    } else if constexpr (which == 11) {                                             // 8 independent non-DPP fmac (asm)
      asm("v_fmac_f64 %0, %1, %2" : "+v"(z[i & 7]) : "v"(x), "v"(y));
    } else if constexpr (which == 12) {                                             // DPP64 fmac, row_mask 0x1
      asm("v_fmac_f64_dpp %0, %1, %2 row_newbcast:3 row_mask:0x1 bank_mask:0xf" : "+v"(z[i & 7]) : "v"(x), "v"(y));
    } else if constexpr (which == 13) {                                             // 8 independent mul
      z[i & 7] = z[i & 7] * y;
    } else if constexpr (which == 14) {                                             // v_mov_b32
      asm volatile("v_mov_b32 %0, %1" : "=v"(w[i & 7]) : "v"(w[(i + 3) & 7]));
    } else if constexpr (which == 15) {                                             // v_mov_b64
      asm volatile("v_mov_b64 %0, %1" : "=v"(z[i & 7]) : "v"(z[(i + 3) & 7]));
    } else if constexpr (which == 16) {                                             // v_permlane16_swap
      asm volatile("v_permlane16_swap_b32 %0, %1" : "+v"(w[i & 7]), "+v"(w[(i + 4) & 7]));
    } else if constexpr (which == 17) {                                             // v_readlane
      asm volatile("v_readlane_b32 %0, %1, 5" : "=s"(sreg[i & 7]) : "v"(w[i & 7]));
    } else if constexpr (which == 18) {                                             // v_cmp_class_f64
      asm volatile("v_cmp_class_f64 %0, %1, %2" : "=s"(sm64[i & 7]) : "v"(z[i & 7]), "v"(w[0]));
    } else if constexpr (which == 19) {                                             // v_add_u32
      asm volatile("v_add_u32 %0, %1, %2" : "=v"(w[i & 7]) : "v"(w[(i + 3) & 7]), "v"(w[(i + 5) & 7]));
    } else if constexpr (which == 20) {                                             // s_add_u32
      asm volatile("s_add_u32 %0, %1, 7" : "=s"(sreg[i & 7]) : "s"(sreg[(i + 3) & 7]) : "scc");
    } else if constexpr (which == 21) {                                             // v_rsq_f64 independent
      z[i & 7] = __builtin_amdgcn_rsq(z[(i + 3) & 7]);
    } else if constexpr (which == 22) {                                             // v_mov_b32_dpp quad_perm
      w[i & 7] = __builtin_amdgcn_mov_dpp(w[(i + 3) & 7], 0xB1, 0xF, 0xF, false);
    } else if constexpr (which == 23) {                                             // s_nop 0
      asm volatile("s_nop 0");
    } else if constexpr (which == 24) {                                             // s_nop 1
      asm volatile("s_nop 1");
    } else if constexpr (which == 25) {                                             // v_mov_b32 + s_nop 1 pairs
      asm volatile("v_mov_b32 %0, %1\n\ts_nop 1" : "=v"(w[i & 7]) : "v"(w[(i + 3) & 7]));
    }
  }
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  asm volatile("" ::"v"(x), "v"(c));
#pragma unroll
  for (int k = 0; k < 8; ++k) asm volatile("" ::"v"(z[k]), "v"(w[k]), "s"(sreg[k]), "s"(sm64[k]));
  __builtin_amdgcn_sched_barrier(0);
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[threadIdx.x] = x + c[0] + c[1] + c[2] + c[3];
  if (lane == 0) cyc[threadIdx.x >> 6] = t1 - t0;
}

extern "C" int lat_run(int which, double* out, unsigned long long* cyc, int nthreads) {
  switch (which) {
#define L(w) case w: hipLaunchKernelGGL(k_lat<w>, dim3(1), dim3(nthreads), 0, 0, out, cyc); break;
    L(0) L(1) L(2) L(3) L(4) L(5) L(6) L(7) L(8) L(9) L(10) L(11) L(12) L(13) L(14) L(15) L(16) L(17) L(18) L(19) L(20) L(21) L(22) L(23) L(24) L(25)
#undef L
  }
  return (int)hipDeviceSynchronize();
}

// Dependent-load latency (pointer chase over `n` ints with stride `st`), one wave:
// cycles per load; n * 4 B > 32 KB misses the L1, < 4 MB hits the L2.
__global__ __launch_bounds__(64) void k_chase(const int* buf, int steps, int* out, unsigned long long* cyc) {
  int idx = threadIdx.x;
  for (int w = 0; w < 64; ++w) idx = buf[idx];  // warm
  __builtin_amdgcn_s_waitcnt(0);
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < steps; ++i) idx = buf[idx];
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[threadIdx.x] = idx;
  if (threadIdx.x == 0) *cyc = (t1 - t0) / steps;
}
extern "C" int chase_run(const int* buf, int steps, int* out, unsigned long long* cyc) {
  hipLaunchKernelGGL(k_chase, dim3(1), dim3(64), 0, 0, buf, steps, out, cyc);
  return (int)hipDeviceSynchronize();
}
