// Shared helpers for the milwrm_amd HIP kernels (gfx950 / CDNA4, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <algorithm>
#include <stdint.h>
#include <string.h>
#include <stdio.h>

#include "../../include/milwrm_amd.h"

namespace mw {

// ---- error plumbing (thread-local last error, surfaced via mw_last_error) ----
void set_error(const char* fmt, ...);

#define MW_CHECK_ARG(cond, ...)            \
  do {                                     \
    if (!(cond)) {                         \
      ::mw::set_error(__VA_ARGS__);        \
      return MW_EINVAL;                    \
    }                                      \
  } while (0)

#define MW_HIP(call)                                                        \
  do {                                                                      \
    hipError_t e_ = (call);                                                 \
    if (e_ != hipSuccess) {                                                 \
      ::mw::set_error("%s: %s (%s:%d)", #call, hipGetErrorString(e_),       \
                      __FILE__, __LINE__);                                  \
      return MW_EHIP;                                                       \
    }                                                                       \
  } while (0)

// read-once loads of the row streams with the streaming (nt) cache policy
// (MW_STREAM_NT=0: the default policy, for same-box A/B builds).  Same-box
// A/B at config 2 (profiles/r06/nt_ab*/): k-means++ step pass 495 -> 457 us,
// Lloyd kind-1 pass 451 -> 399, label pass 2.74 -> 2.67 ms, gather -1 %; the
// blur and the nonzero statistics kept the default policy (nt: +2.5 / +3 %)
#ifndef MW_STREAM_NT
#define MW_STREAM_NT 1
#endif
template <typename T>
__device__ __forceinline__ T ld_stream(const T* p) {
  if constexpr (MW_STREAM_NT) return __builtin_nontemporal_load(p);
  else return *p;
}

#define MW_LAUNCH_CHECK()                                                   \
  do {                                                                      \
    hipError_t e_ = hipGetLastError();                                      \
    if (e_ != hipSuccess) {                                                 \
      ::mw::set_error("kernel launch: %s (%s:%d)", hipGetErrorString(e_),   \
                      __FILE__, __LINE__);                                  \
      return MW_EHIP;                                                       \
    }                                                                       \
  } while (0)

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

constexpr int kWave = 64;

// ---- wave64 reductions (DPP/shuffle through __shfl_xor, width 64) ----
template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Lane i of each 16-lane row takes lane i + N of the row (DPP row_shl:N; lanes
// past the row read 0: bound_ctrl).  Two 32-bit DPP moves for a double.
template <int N>
__device__ __forceinline__ double dpp_row_shl(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_mov_dpp((int)b, 0x100 + N, 0xF, 0xF, true);
  const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), 0x100 + N, 0xF, 0xF, true);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

// wave_sum's value in lane 0 only, bit for bit: at the level of offset o lane
// 0's tree needs lane i + o in lanes i < o, which is their xor partner, so the
// same additions happen in the same order; offsets 32 and 16 cross rows (LDS
// permutes, as wave_sum), 8, 4, 2, 1 are DPP row shifts (VALU, no LDS
// round trip in the dependent chain)
__device__ __forceinline__ double wave_sum_lane0(double v) {
  v += __shfl_xor(v, 32, 64);
  v += __shfl_xor(v, 16, 64);
  v += dpp_row_shl<8>(v);
  v += dpp_row_shl<4>(v);
  v += dpp_row_shl<2>(v);
  v += dpp_row_shl<1>(v);
  return v;
}

// v_permlane32_swap / v_permlane16_swap of a double pair (two dwords each):
// x32 exchanges the upper 32 lanes of `a` with the lower 32 lanes of `b`; x16
// the odd 16-lane rows of `a` with the even rows of `b`
__device__ __forceinline__ void pl_swap_d(double& a, double& b, bool x16) {
  const unsigned long long ua = (unsigned long long)__double_as_longlong(a);
  const unsigned long long ub = (unsigned long long)__double_as_longlong(b);
  unsigned a0 = (unsigned)ua, a1 = (unsigned)(ua >> 32), b0 = (unsigned)ub, b1 = (unsigned)(ub >> 32);
  if (x16) {
    const auto r0 = __builtin_amdgcn_permlane16_swap(a0, b0, false, false);
    const auto r1 = __builtin_amdgcn_permlane16_swap(a1, b1, false, false);
    a0 = r0[0]; b0 = r0[1]; a1 = r1[0]; b1 = r1[1];
  } else {
    const auto r0 = __builtin_amdgcn_permlane32_swap(a0, b0, false, false);
    const auto r1 = __builtin_amdgcn_permlane32_swap(a1, b1, false, false);
    a0 = r0[0]; b0 = r0[1]; a1 = r1[0]; b1 = r1[1];
  }
  a = __longlong_as_double((long long)(((unsigned long long)a1 << 32) | a0));
  b = __longlong_as_double((long long)(((unsigned long long)b1 << 32) | b0));
}

// wave_sum_lane0 of four values at once: v_r's sum lands in lane 16 r, bit
// for bit wave_sum_lane0(v_r)'s lane 0.  The l ^ 32 and l ^ 16 levels
// exchange register halves instead of LDS permutes, and each lane goes on
// with the one value its row keeps (lower half: v0, v1, upper: v2, v3; then
// row r: v_r): every level adds the same lane pairs as wave_sum_lane0's
// tree, so lane 16 r ends with lane 0's additions for v_r, in the same order
// (rows of 16 lanes then reduce by the same DPP row shifts)
__device__ __forceinline__ double wave_sum4_rows(double v0, double v1, double v2, double v3) {
  pl_swap_d(v0, v2, false);  // lower lanes: (own v0, v0 of l + 32); upper: (v2 of l - 32, own v2)
  pl_swap_d(v1, v3, false);
  double p = v0 + v2, q = v1 + v3;  // lower: v0, v1 pair sums; upper: v2, v3
  pl_swap_d(p, q, true);            // row 0: (p, p of l + 16); 1: (q of l - 16, q); 2, 3 likewise
  double v = p + q;
  v += dpp_row_shl<8>(v);
  v += dpp_row_shl<4>(v);
  v += dpp_row_shl<2>(v);
  v += dpp_row_shl<1>(v);
  return v;
}

// Block-wide sum of one value per thread; result valid in thread 0.
// `scratch` must hold blockDim.x/64 elements.  Fixed combine order.
template <typename T>
__device__ __forceinline__ T block_sum(T v, T* scratch) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) scratch[wid] = v;
  __syncthreads();
  T r = T(0);
  if (threadIdx.x == 0) {
    const int nw = (blockDim.x + 63) >> 6;
    for (int w = 0; w < nw; ++w) r += scratch[w];
  }
  return r;
}

// Element loaders for the supported image dtypes.
template <typename T> __device__ __forceinline__ float to_f(T v) { return (float)v; }

}  // namespace mw
