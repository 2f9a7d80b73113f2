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
