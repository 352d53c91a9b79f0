// Cycle costs of small code shapes used by the factorization (tools only).
#include <hip/hip_runtime.h>
typedef double d4 __attribute__((ext_vector_type(4)));
#define MF(a, b, c) __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0)

template <int V>
__global__ __launch_bounds__(256) void k_snip(double* out, unsigned long long* cyc, int reps) {
  __shared__ double L[8192];
  const int lane = threadIdx.x & 63;
  for (int t = threadIdx.x; t < 8192; t += blockDim.x) L[t] = 1.0 / (1 + (t & 31));
  __syncthreads();
  d4 acc[12];
#pragma unroll
  for (int s = 0; s < 12; ++s) acc[s] = d4{1.0 * s, 2.0, 3.0, 4.0};
  double la[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) la[r] = L[r * 64 + lane];
  unsigned long long tot = 0;
  for (int rep = 0; rep < reps; ++rep) {
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    if (V == 0) {  // 1 T tile: 4 dependent MFMAs, result -> LDS
      d4 u = {0, 0, 0, 0};
#pragma unroll
      for (int r = 0; r < 4; ++r) u = MF(la[r], acc[0][r], u);
      acc[0] = u;
#pragma unroll
      for (int r = 0; r < 4; ++r) L[4096 + r * 64 + lane] = u[r];
    } else if (V == 1) {  // 3 T tiles, MFMAs first then stores
#pragma unroll
      for (int s = 0; s < 3; ++s) {
        d4 u = {0, 0, 0, 0};
#pragma unroll
        for (int r = 0; r < 4; ++r) u = MF(la[r], acc[s][r], u);
        acc[s] = u;
      }
#pragma unroll
      for (int s = 0; s < 3; ++s)
#pragma unroll
        for (int r = 0; r < 4; ++r) L[4096 + s * 256 + r * 64 + lane] = acc[s][r];
    } else if (V == 2) {  // 10 U tiles, naive: load 8 then 4 MFMAs
#pragma unroll
      for (int s = 0; s < 10; ++s) {
        double av[4], bv[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          av[r] = L[(s % 4) * 256 + r * 64 + lane];
          bv[r] = L[1024 + ((s + 1) % 5) * 256 + r * 64 + lane];
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[s] = MF(av[r], bv[r], acc[s]);
        __builtin_amdgcn_sched_barrier(0);
      }
    } else if (V == 3) {  // 10 U tiles, 2 tiles interleaved
#pragma unroll
      for (int s = 0; s < 10; s += 2) {
        double av[4], bv[4], cv[4], dv[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          av[r] = L[(s % 4) * 256 + r * 64 + lane];
          bv[r] = L[1024 + ((s + 1) % 5) * 256 + r * 64 + lane];
          cv[r] = L[((s + 1) % 4) * 256 + r * 64 + lane];
          dv[r] = L[1024 + ((s + 2) % 5) * 256 + r * 64 + lane];
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          acc[s] = MF(av[r], bv[r], acc[s]);
          acc[s + 1] = MF(cv[r], dv[r], acc[s + 1]);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    } else if (V == 4) {  // 40 MFMAs back to back on 10 accumulators (pipe rate)
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int s = 0; s < 10; ++s) acc[s] = MF(la[r], la[(r + 1) & 3], acc[s]);
    } else if (V == 5) {  // 40 dependent MFMAs on one accumulator
#pragma unroll
      for (int r = 0; r < 40; ++r) acc[0] = MF(la[r & 3], la[(r + 1) & 3], acc[0]);
    } else if (V == 6) {  // LDS round trip: store then dependent load
      L[4096 + lane] = acc[0][0];
      __builtin_amdgcn_s_waitcnt(0xc07f);
      acc[0][1] = L[4096 + (lane ^ 1)];
      acc[0][2] += acc[0][1];
    } else if (V == 7) {  // 16 readlane pairs + 16 fma
      double x = acc[0][0];
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const long long b = __double_as_longlong(acc[1][j & 3] + j);
        const int lo = __builtin_amdgcn_readlane((int)b, j), hi = __builtin_amdgcn_readlane((int)(b >> 32), j);
        x = __builtin_fma(__longlong_as_double(((long long)hi << 32) | (unsigned)lo), acc[2][j & 3], x);
      }
      acc[0][0] = x;
    }
    __syncthreads();
    tot += __builtin_amdgcn_s_memtime() - t0;
  }
  double s = 0;
#pragma unroll
  for (int q = 0; q < 12; ++q) s += acc[q][0] + acc[q][1] + acc[q][2] + acc[q][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = tot / reps;
}

extern "C" int probe_snip(int v, int threads, double* out, unsigned long long* cyc, int blocks, int reps) {
#define L_(V) if (v == V) hipLaunchKernelGGL(k_snip<V>, dim3(blocks), dim3(threads), 0, 0, out, cyc, reps);
  L_(0) L_(1) L_(2) L_(3) L_(4) L_(5) L_(6) L_(7)
  return hipDeviceSynchronize() == hipSuccess ? 0 : -1;
}
