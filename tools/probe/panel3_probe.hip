// Microbenchmark: cycles per diagonal-block panel, the shipped row sweep panel()
// vs experimental variants (round 2, tools only; none shipped except what panel() is now).
#define MHE_FAST_BUILD
#include "../../nlp-filter_amd/csrc/mhe_gn.hip"

namespace probe {
using namespace mhe;

// acc -= bcast_J(src0) * src1 on the rows of RM
#define P3_FMAC(J)                                                                                   \
  case J:                                                                                            \
    if (fresh)                                                                                       \
      asm("s_nop 1\n\tv_fmac_f64_dpp %0, -%1, %2 row_newbcast:" #J " row_mask:%3 bank_mask:0xf"     \
          : "+v"(acc), "+v"(src0) : "v"(src1), "i"(RM));                                            \
    else                                                                                             \
      asm("v_fmac_f64_dpp %0, -%1, %2 row_newbcast:" #J " row_mask:%3 bank_mask:0xf"                  \
          : "+v"(acc) : "v"(src0), "v"(src1), "i"(RM));                                             \
    break;
template <int RM>
__device__ __forceinline__ void fnmac_rowbcast(double& acc, double& src0, double src1, int j, bool fresh) {
  switch (j) {
    P3_FMAC(1) P3_FMAC(2) P3_FMAC(3) P3_FMAC(4) P3_FMAC(5) P3_FMAC(6) P3_FMAC(7) P3_FMAC(8)
    P3_FMAC(9) P3_FMAC(10) P3_FMAC(11) P3_FMAC(12) P3_FMAC(13) P3_FMAC(14) P3_FMAC(15)
    default: break;
  }
}

template <int V>
__device__ __forceinline__ bool panel3(double* DTk, int lane) {
  const int i = lane & 15;
  const bool erow = (lane >= 16 && lane < 32);
  double v[16];
#pragma unroll
  for (int c = 0; c < 16; c += 2) {
    const double2 a2 = *(const double2*)(DTk + i * 16 + c);
    v[c] = a2.x;
    v[c + 1] = a2.y;
  }
#pragma unroll
  for (int c = 0; c < 16; ++c) asm volatile("" : "+v"(v[c]));
#pragma unroll
  for (int c = 0; c < 16; ++c) v[c] = erow ? (c == i ? 1.0 : 0.0) : -v[c];
  bool bad = false;
  double piv = readlane_d(v[0], 0);
#pragma unroll
  for (int c = 0; c < 16; ++c) {
    bad |= !(piv > 0.0 && piv < INFINITY);
    const double r = __builtin_amdgcn_rsq(piv);
    double q;
    if (V & 1) {  // refine q itself: q' = q + (q/2)(1 - x r^2)
      const double e = fma(-piv * r, r, 1.0);
      const double q0 = v[c] * r;
      q = fma(0.5 * q0, e, q0);
    } else {
      const double e = fma(-piv * r, r, 1.0);
      q = v[c] * fma(0.5 * r, e, r);
    }
    v[c] = q;
    if (c < 15) {
      if (V & 2) {
        // row 0 first, from q itself: the next pivot does not wait for the row swap
        fnmac_rowbcast<0x1>(v[c + 1], q, q, c + 1, true);
        piv = readlane_d(v[c + 1], c + 1);
        double lq = row0_both(q);
        fnmac_rowbcast<0xe>(v[c + 1], lq, q, c + 1, true);
#pragma unroll
        for (int j = c + 2; j < 16; ++j) fnmac_rowbcast<0xf>(v[j], lq, q, j, false);
      } else {
        double lq = row0_both(q);
#pragma unroll
        for (int j = c + 1; j < 16; ++j) fnmac_rowbcast<0xf>(v[j], lq, q, j, j == c + 1);
        piv = readlane_d(v[c + 1], c + 1);
      }
    }
  }
  if (erow) {
#pragma unroll
    for (int j = 0; j < 16; ++j) DTk[i * LIS + j] = v[j];
  }
  return bad;
}


// acc -= bcast_J(q) * q on the rows of RM, q written by the previous VALU
#define P5_FMAC(J)                                                                                   \
  case J:                                                                                            \
    asm("s_nop 1\n\tv_fmac_f64_dpp %0, -%1, %1 row_newbcast:" #J " row_mask:%2 bank_mask:0xf"       \
        : "+v"(acc) : "v"(q), "i"(RM));                                                            \
    break;
template <int RM>
__device__ __forceinline__ void fnmac_self(double& acc, double q, int j) {
  switch (j) {
    P5_FMAC(1) P5_FMAC(2) P5_FMAC(3) P5_FMAC(4) P5_FMAC(5) P5_FMAC(6) P5_FMAC(7) P5_FMAC(8)
    P5_FMAC(9) P5_FMAC(10) P5_FMAC(11) P5_FMAC(12) P5_FMAC(13) P5_FMAC(14) P5_FMAC(15)
    default: break;
  }
}
#define SB __builtin_amdgcn_sched_barrier(0)
// pivot c-1's deferred updates of v[J..END) (pivot c-1's L column lqp, its q qp)
template <int J, int END>
__device__ __forceinline__ void drain_range(double (&v)[16], double& lqp, double qp) {
  if constexpr (J < END && J < 16) {
    fnmac_rowbcast<0xf>(v[J], lqp, qp, J, false);
    drain_range<J + 1, END>(v, lqp, qp);
  }
}
struct P5 {
  double piv, r, lqp, qp;
  bool bad;
};
// Software-pipelined pivot C: its chain (1/sqrt, q, row-0 update of v[C+1], next
// pivot read) runs while pivot C-1's updates of v[C+2..15] are issued between its steps.
template <int C, int N0, int N1, int N2, int N3, int N4>
__device__ __forceinline__ void pivot5(double (&v)[16], P5& st) {
  constexpr bool DR = C >= 1;
  constexpr int d0 = C + 2, d1 = d0 + N0, d2 = d1 + N1, d3 = d2 + N2, d4_ = d3 + N3, d5 = d4_ + N4;
  SB;
  st.bad |= !(st.piv > 0.0 && st.piv < INFINITY);
  const double t = -st.piv * st.r;
  const double q0 = v[C] * st.r;
  SB;
  if constexpr (DR) drain_range<d0, d1>(v, st.lqp, st.qp);
  SB;
  const double e = fma(t, st.r, 1.0);
  const double h = 0.5 * q0;
  SB;
  if constexpr (DR) drain_range<d1, d2>(v, st.lqp, st.qp);
  SB;
  double q = fma(h, e, q0);
  v[C] = q;
  SB;
  if constexpr (DR) drain_range<d2, d3>(v, st.lqp, st.qp);
  SB;
  if constexpr (C < 15) {
    fnmac_self<0x1>(v[C + 1], q, C + 1);
    SB;
    if constexpr (DR) drain_range<d3, d4_>(v, st.lqp, st.qp);
    SB;
    st.piv = readlane_d(v[C + 1], C + 1);
    SB;
    if constexpr (DR) drain_range<d4_, d5>(v, st.lqp, st.qp);
    SB;
    st.r = __builtin_amdgcn_rsq(st.piv);
    SB;
    if constexpr (DR) drain_range<d5, 16>(v, st.lqp, st.qp);
    SB;
    double lq = row0_both(q);
    fnmac_rowbcast<0xe>(v[C + 1], lq, q, C + 1, true);
    if constexpr (C + 2 < 16) fnmac_rowbcast<0xf>(v[C + 2], lq, q, C + 2, false);
    st.lqp = lq;
    st.qp = q;
    pivot5<C + 1, N0, N1, N2, N3, N4>(v, st);
  }
}
template <int N0, int N1, int N2, int N3, int N4>
__device__ __forceinline__ bool panel5(double* DTk, int lane) {
  const int i = lane & 15;
  const bool erow = (lane >= 16 && lane < 32);
  double v[16];
#pragma unroll
  for (int c = 0; c < 16; c += 2) {
    const double2 a2 = *(const double2*)(DTk + i * 16 + c);
    v[c] = a2.x;
    v[c + 1] = a2.y;
  }
#pragma unroll
  for (int c = 0; c < 16; ++c) asm volatile("" : "+v"(v[c]));
#pragma unroll
  for (int c = 0; c < 16; ++c) v[c] = erow ? (c == i ? 1.0 : 0.0) : -v[c];
  P5 st;
  st.bad = false;
  st.piv = readlane_d(v[0], 0);
  st.r = __builtin_amdgcn_rsq(st.piv);
  st.lqp = st.qp = 0.0;
  pivot5<0, N0, N1, N2, N3, N4>(v, st);
  SB;
  if (erow) {
#pragma unroll
    for (int j = 0; j < 16; ++j) DTk[i * LIS + j] = v[j];
  }
  return st.bad;
}


// Panel with +A_kk in DT and the identity lanes loading rows of I from EYE (LDS).
template <bool ASMSWAP>
__device__ __forceinline__ bool panel6(double* DTk, const double* EYE, int lane) {
  const int i = lane & 15;
  const bool erow = (lane >= 16 && lane < 32);
  const double* src = (erow ? EYE : DTk) + i * 16;
  double v[16];
#pragma unroll
  for (int c = 0; c < 16; c += 2) {
    const double2 a2 = *(const double2*)(src + c);
    v[c] = a2.x;
    v[c + 1] = a2.y;
  }
  bool bad = false;
#pragma unroll
  for (int c = 0; c < 16; ++c) {
    const double piv = readlane_d(v[c], c);
    bad |= !(piv > 0.0 && piv < INFINITY);
    const double q = v[c] * rsqrt_pivot(piv);
    v[c] = q;
    if (c < 15) {
      double lq = row0_both(q);
#pragma unroll
      for (int j = c + 1; j < 16; ++j) fnmac_rowbcast<0xf>(v[j], lq, q, j, j == c + 1);
    }
  }
  if (erow) {
#pragma unroll
    for (int j = 0; j < 16; ++j) DTk[i * LIS + j] = v[j];
  }
  return bad;
}

__global__ __launch_bounds__(64) void k_probe(int variant, const double* A, double* out,
                                              unsigned long long* cyc, int reps) {
  __shared__ double src[256];
  __shared__ double DT[DTS];
  __shared__ double EYE[256];
  __shared__ __attribute__((aligned(16))) double UN[UNITS];
  init_units(UN);
  const int lane = threadIdx.x;
  for (int e = lane; e < 256; e += 64) src[e] = ((variant >= 9 || variant == 0) ? A[e] : -A[e]);
  for (int e = lane; e < 256; e += 64) EYE[e] = (e >> 4) == (e & 15) ? 1.0 : 0.0;
  __syncthreads();
  unsigned long long total = 0;
  int bad = 0;
  for (int it = 0; it < reps; ++it) {
    int l = lane;
    asm volatile("" : "+v"(l));
    for (int e = l; e < 256; e += 64) DT[e] = src[e];
    wave_lds_sync();
    __builtin_amdgcn_s_waitcnt(0);
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    switch (variant) {
      case 0: bad |= panel(DT, UN, l); break;
      case 1: bad |= panel3<0>(DT, l); break;
      case 2: bad |= panel3<1>(DT, l); break;
      case 3: bad |= panel3<2>(DT, l); break;
      case 4: bad |= panel3<3>(DT, l); break;
      case 5: bad |= panel5<2, 2, 1, 2, 2>(DT, l); break;
      case 6: bad |= panel5<1, 1, 1, 1, 1>(DT, l); break;
      case 7: bad |= panel5<0, 0, 0, 0, 0>(DT, l); break;
      case 8: bad |= panel5<3, 3, 2, 2, 2>(DT, l); break;
      case 9: bad |= panel6<false>(DT, EYE, l); break;
      default: bad |= panel6<true>(DT, EYE, l); break;
    }
    wave_lds_sync();
    const double chk = DT[l];
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
