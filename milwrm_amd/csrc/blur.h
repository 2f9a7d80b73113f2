// Fused log-normalise + separable Gaussian blur (img.log_normalize +
// img.blurring('gaussian'), MxIF.py:416-455 / 375-394; scipy gaussian_filter
// mode='nearest', truncate=4, axis 0 then axis 1) — the fast path.
//
// One workgroup = a band of BW output columns x kBlurBH output rows, all C
// channels, one output element PAIR per thread (C even: a pair never straddles
// a pixel).  Rows stream top to bottom:
//   * each input row segment (r-pixel halo, edge-clamped) is fetched 2r rows
//     ahead into a register ring (2r+1 row slots, static slot = row mod 2r+1,
//     so no register moves wait on in-flight loads), log-normalised and
//     stored to a double-buffered LDS
//     row laid out [pixel][CP2 pairs] with CP2 = next power of two >= C/2 (a
//     compile-time pixel stride, so the 2r+1 horizontal taps are immediate
//     ds_read_b64 offsets from one base address);
//   * the horizontal pass reads all taps first, then a packed-FMA chain;
//   * the vertical pass keeps the last 2r+1 horizontally filtered rows in a
//     register ring (static indices: the row loop is unrolled by 2r+1).
// Output rows are contiguous HWC segments (coalesced 8-byte stores).
// Instantiated per input dtype in blur_u8.hip / blur_u16.hip / blur_f32.hip.
#pragma once

#include <stdlib.h>

#include "common.h"

namespace mw {

constexpr int kMaxRadius = 32;
struct BlurTaps { float w[2 * kMaxRadius + 1]; };
constexpr int kBlurBH = 256;
constexpr int kBlurMaxR = 12;    // fast path radius bound (register ring)
constexpr int kBlurMaxL = 2;     // input-row pair loads per thread per row (BW >= 2r)

typedef float bf2 __attribute__((ext_vector_type(2)));

// fused fast paths (matrix-core kernel, then the VALU kernel below), defined in
// blur_mfma.h and instantiated per dtype in blur_{u8,u16,f32}.hip
template <typename T>
int launch_blur_fast(const T* in, int H, int W, int C, const float* inv_mean, float p,
                     const struct BlurTaps& taps, int r, float* out, hipStream_t st);
constexpr int kEpiStore = 0, kEpiSample = 1, kEpiAssign = 2;
constexpr int kEpiKMax = 16;  // assign epilogue: centers per launch (distance tables in LDS)

struct BlurEpi {
  const int32_t* slots;    // kEpiSample: (n_pix + 128) x 2: the first two sample slots of p (-1: none)
  int64_t S;               //   rows of X
  float* X;                //   S x F
  int F;
  const int32_t* feat;     //   F channel indices (device)
  const uint8_t* mask;     // kEpiAssign: nonzero = tissue (readable 128 B past the end)
  int8_t* lab;             //   label per pixel (-1 outside the mask)
  float* conf;             //   confidence per pixel (NaN outside the mask)
  const float* a;          //   scaler per channel (features = all channels in order)
  const float* b;
  const float* centers;    //   k x C, scaled space
  int k;
  // row window (fused epilogues): the input array holds slide rows [row_off,
  // row_off + H); only array rows [r0, r1) are output (the rows around them
  // are read as the vertical halo), and the side data (slots, mask) and the
  // per-pixel outputs (lab, conf) are indexed by SLIDE pixel (row + row_off) *
  // W + x -- a slide streamed band by band gives the whole-slide results
  int64_t row_off;
  int r0, r1;
};

template <typename T>
int launch_blur_epi(const T* in, int H, int W, int C, const float* inv_mean, float p,
                    const struct BlurTaps& taps, int r, const BlurEpi& ep, int epi, hipStream_t st);

// 1/v to ~12% from the exponent/mantissa bits (one integer subtract): the
// factor of the rounding-error correction below, whose size is at most half
// an ulp of v — a 12% error there moves the result by < 2^-27 relative, and
// saves the quarter-rate v_rcp_f32 per element
__device__ __forceinline__ float rcp_coarse(float v) {
  return __builtin_bit_cast(float, 0x7EF311C3u - __builtin_bit_cast(uint32_t, v));
}

// accurate log10(t + p) for t >= 0 (log1p-style correction of the rounding
// of t + p, so small t keep full relative accuracy)
__device__ __forceinline__ float lognorm1(float x, float inv, float p) {
  const float t = x * inv;
  const float v = t + p;
  const float e = (v - p) - t;  // rounding error of t + p (exact)
  const float l2 = __builtin_amdgcn_logf(v);  // log2, 1 ulp
  return l2 * 0.30102999566398120f - (e * rcp_coarse(v)) * 0.43429448190325182f;
}

// log2(t + p) on an element pair, no rounding correction: the matrix-core
// kernel folds log10(2) into its horizontal taps.  The rounding of t + p moves
// the result by <= 2^-24 / ln 2 absolute (2.6e-8 after the log10 scale) —
// far inside the fp32 blur's own rounding for values of order 1, and 2
// instructions per pair instead of 9 on a VALU-issue-bound kernel.
__device__ __forceinline__ bf2 log2norm2(bf2 x, bf2 inv, float p) {
  const bf2 v = __builtin_elementwise_fma(x, inv, bf2{p, p});
  return bf2{__builtin_amdgcn_logf(v.x), __builtin_amdgcn_logf(v.y)};
}

// the same on an element pair with packed arithmetic (v_pk_*; the two
// transcendentals per element stay scalar)
__device__ __forceinline__ bf2 lognorm2(bf2 x, bf2 inv, float p) {
  const bf2 pp = bf2{p, p};
  const bf2 t = x * inv;
  const bf2 v = t + pp;
  const bf2 e = (v - pp) - t;
  const bf2 l2 = bf2{__builtin_amdgcn_logf(v.x), __builtin_amdgcn_logf(v.y)};
  const bf2 rv = bf2{rcp_coarse(v.x), rcp_coarse(v.y)};
  return __builtin_elementwise_fma(l2, bf2{0.30102999566398120f, 0.30102999566398120f},
                                   (e * rv) * bf2{-0.43429448190325182f, -0.43429448190325182f});
}

// ds_read_b64 with an immediate offset.  Written as inline asm because the
// compiler otherwise pairs the taps into ds_read2_b64, which runs at half the
// LDS rate of ds_read_b64 (8 vs 2 cycles per wave for the same bytes, §LDS of
// the MI355X guide).  The caller waits with lds_wait() before using results.
template <int OFF>
__device__ __forceinline__ bf2 lds_read_b64(uint32_t addr) {
  bf2 r;
  asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(r) : "v"(addr), "i"(OFF));
  return r;
}
template <int N>
__device__ __forceinline__ void lds_wait(bf2 (&v)[N]) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
  for (int j = 0; j < N; ++j) asm volatile("" : "+v"(v[j]));  // uses ordered after the wait
}
template <int CP2, int J, int NR>
__device__ __forceinline__ void read_taps(uint32_t addr, bf2 (&tap)[NR]) {
  if constexpr (J < NR) {
    tap[J] = lds_read_b64<J * CP2 * 8>(addr);
    read_taps<CP2, J + 1, NR>(addr, tap);
  }
}

// An element pair as one packed global load (u8: 16 bits, u16: 32 bits, f32:
// 64 bits), issued as inline asm: the row ring keeps 2r+1 rows of loads in
// flight, and the compiler's own wait insertion cannot follow loads consumed
// one unrolled loop trip later (it waits for everything, flattening the
// pipeline to one row), so the kernel places counted vmcnt waits itself.
template <typename T> struct Pair2;
template <> struct Pair2<uint8_t> {
  using type = uint32_t;
  static __device__ __forceinline__ type load(const uint8_t* p) {
    type r;
    asm volatile("global_load_ushort %0, %1, off" : "=v"(r) : "v"(p) : "memory");
    return r;
  }
  static __device__ __forceinline__ bf2 cvt(type v) { return bf2{(float)(v & 0xffu), (float)((v >> 8) & 0xffu)}; }
};
template <> struct Pair2<uint16_t> {
  using type = uint32_t;
  static __device__ __forceinline__ type load(const uint16_t* p) {
    type r;
    asm volatile("global_load_dword %0, %1, off" : "=v"(r) : "v"(p) : "memory");
    return r;
  }
  static __device__ __forceinline__ bf2 cvt(type v) { return bf2{(float)(v & 0xffffu), (float)(v >> 16)}; }
};
template <> struct Pair2<float> {
  using type = bf2;
  static __device__ __forceinline__ type load(const float* p) {
    type r;
    asm volatile("global_load_dwordx2 %0, %1, off" : "=v"(r) : "v"(p) : "memory");
    return r;
  }
  static __device__ __forceinline__ bf2 cvt(type v) { return v; }
};
// wait until at most N vector-memory operations are outstanding, then mark the
// registers as (re)defined so their uses stay below the wait
template <int N, typename V, int L>
__device__ __forceinline__ void vm_wait(V (&v)[L]) {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
#pragma unroll
  for (int k = 0; k < L; ++k) asm volatile("" : "+v"(v[k]));
}

// register budget: the in-flight row ring is (2r+1) x 2 pairs per thread
template <typename T, int R>
constexpr int blur_max_threads() { return (sizeof(T) == 4 || R > 8) ? 512 : 1024; }

template <typename T, int R, int CP2>
__global__ void __launch_bounds__((blur_max_threads<T, R>())) blur_kernel(const T* __restrict__ in, int H, int W, int C,
                                                    int BW, const float* __restrict__ inv_mean,
                                                    float pseudo, BlurTaps taps,
                                                    float* __restrict__ out) {
  using P2 = typename Pair2<T>::type;
  constexpr int NR = 2 * R + 1;
  extern __shared__ __attribute__((aligned(16))) bf2 s_row2[];  // 2 x (BW+2R)*CP2 pairs
  const int t = threadIdx.x;
  const int nt = blockDim.x;
  const int CP = C >> 1;
  const int x0 = blockIdx.x * BW;
  const int y0 = blockIdx.y * kBlurBH;
  const int y1 = min(H, y0 + kBlurBH);
  const int bw = min(BW, W - x0);
  const int seg2 = (bw + 2 * R) * CP2;  // halo'd row pair SLOTS (CP2 per pixel)
  const int rowcap = (BW + 2 * R) * CP2;
  const int nrows = (y1 - y0) + 2 * R;
  const bool logn = inv_mean != nullptr;

  // this thread's output pair: lanes map 1:1 onto the [pixel][CP2] slots, so
  // 32 consecutive lanes touch 32 consecutive slots (conflict-free b64 reads);
  // slots cp >= C/2 idle
  const int o_px = t / CP2, o_cp = t & (CP2 - 1);
  const bool e_ok = o_px < bw && o_cp < CP;
  const int lds_base = t;  // tap j at + j * CP2
  // LDS byte addresses of this thread's first tap in the two row buffers
  uint32_t lds_row[2];
#pragma unroll
  for (int b = 0; b < 2; ++b)
    lds_row[b] = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) bf2*)(s_row2 + b * rowcap + lds_base));
  float* out_base = out + (int64_t)(x0 + (e_ok ? o_px : 0)) * C + 2 * (e_ok ? o_cp : 0);
  const int64_t out_row = (int64_t)W * C;

  // input load slots (pairs), fixed for every row; unused slots load pair 0
  int l_src[kBlurMaxL], l_dst[kBlurMaxL];
  bool l_ok[kBlurMaxL];
  bf2 l_inv[kBlurMaxL];
#pragma unroll
  for (int k = 0; k < kBlurMaxL; ++k) {
    const int q = t + k * nt;
    const int px = q / CP2;
    const int cp = q & (CP2 - 1);
    l_ok[k] = q < seg2 && cp < CP;
    l_src[k] = 0;
    l_dst[k] = q;
    l_inv[k] = bf2{1.f, 1.f};
    if (l_ok[k]) {
      int gx = x0 - R + px;
      gx = gx < 0 ? 0 : (gx >= W ? W - 1 : gx);
      l_src[k] = gx * C + 2 * cp;
      if (logn) l_inv[k] = bf2{inv_mean[2 * cp], inv_mean[2 * cp + 1]};
    }
  }
  bf2 wv[NR];
#pragma unroll
  for (int j = 0; j < NR; ++j) wv[j] = bf2{taps.w[j], taps.w[j]};
  bf2 ring[NR];
#pragma unroll
  for (int j = 0; j < NR; ++j) ring[j] = bf2{0.f, 0.f};

  // raw input rows in flight: slot q % NR holds row q (static index inside the
  // NR-unrolled row loop)
  P2 pf[NR][kBlurMaxL];
  auto fetch_row = [&](int rr, P2 (&dst)[kBlurMaxL]) {
    int yy = y0 - R + rr;
    yy = yy < 0 ? 0 : (yy >= H ? H - 1 : yy);
    yy = rr < nrows ? yy : y0;  // past the end: harmless re-read
    const T* src = in + (int64_t)yy * W * C;
#pragma unroll
    for (int k = 0; k < kBlurMaxL; ++k) dst[k] = Pair2<T>::load(src + l_src[k]);
  };
  // the loads of row q are followed by those of rows q+1 .. q+NR-1 before
  // row q is consumed (and possibly by output stores, which only add to the
  // count): at most kBlurMaxL*(NR-1) younger operations may remain in flight
  constexpr int kVmWait = kBlurMaxL * (NR - 1);
  static_assert(kVmWait <= 63, "vmcnt field is 6 bits");
  auto store_row = [&](int buf, const P2 (&v)[kBlurMaxL]) {
    bf2* dst = s_row2 + buf * rowcap;
#pragma unroll
    for (int k = 0; k < kBlurMaxL; ++k) {
      if (l_ok[k]) {
        bf2 x = Pair2<T>::cvt(v[k]);
        if (logn) x = lognorm2(x, l_inv[k], pseudo);
        dst[l_dst[k]] = x;
      }
    }
  };

#pragma unroll
  for (int q = 0; q < NR; ++q) fetch_row(q, pf[q]);
  vm_wait<kVmWait>(pf[0]);
  store_row(0, pf[0]);
  fetch_row(NR, pf[0]);
  __syncthreads();
  for (int base = 0; base < nrows; base += NR) {
#pragma unroll
    for (int s = 0; s < NR; ++s) {
      const int rr = base + s;
      if (rr < nrows) {
        bf2 tap[NR];
        read_taps<CP2, 0, NR>(lds_row[rr & 1], tap);
        lds_wait(tap);
        // two interleaved FMA chains per pass (dependent v_pk_fma issue stalls)
        bf2 h0 = bf2{0.f, 0.f}, h1 = bf2{0.f, 0.f};
#pragma unroll
        for (int j = 0; j < NR; j += 2) h0 = __builtin_elementwise_fma(wv[j], tap[j], h0);
#pragma unroll
        for (int j = 1; j < NR; j += 2) h1 = __builtin_elementwise_fma(wv[j], tap[j], h1);
        ring[s] = h0 + h1;
        if (rr >= 2 * R) {
          bf2 v0 = bf2{0.f, 0.f}, v1 = bf2{0.f, 0.f};
#pragma unroll
          for (int j = 0; j < NR; j += 2) v0 = __builtin_elementwise_fma(wv[j], ring[(s + 1 + j) % NR], v0);
#pragma unroll
          for (int j = 1; j < NR; j += 2) v1 = __builtin_elementwise_fma(wv[j], ring[(s + 1 + j) % NR], v1);
          const bf2 v = v0 + v1;
          if (e_ok) *reinterpret_cast<bf2*>(out_base + (int64_t)(y0 + rr - 2 * R) * out_row) = v;
        }
        const int nx = (s + 1) % NR;  // slot of row rr+1 (loaded NR-1 rows ago)
        vm_wait<kVmWait>(pf[nx]);
        if (rr + 1 < nrows) store_row((rr + 1) & 1, pf[nx]);
        fetch_row(rr + 1 + NR, pf[nx]);
        __syncthreads();
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // drain the prefetches past the end
}

template <typename T, int R, int CP2>
static int launch_blur_rc(const T* in, int H, int W, int C, const float* inv_mean, float p,
                          const BlurTaps& taps, float* out, hipStream_t st) {
  // one output pair per thread: BW * C / 2 <= 1024 threads
  constexpr int kMaxT = blur_max_threads<T, R>();
  int BW = 128;
  while (BW > 1 && BW * CP2 > kMaxT) BW >>= 1;
  if (const char* e = getenv("MW_BLUR_BW")) {  // tuning override
    const int b = atoi(e);
    if (b >= 1 && b <= BW) BW = b;
  }
  const int nt = ((BW * CP2 + 63) / 64) * 64;
  const size_t lds = 2 * (size_t)(BW + 2 * R) * CP2 * sizeof(bf2);
  if (nt > kMaxT || lds > 160 * 1024 || (BW + 2 * R) * CP2 > kBlurMaxL * nt) {
    set_error("mw_blur: fast path cannot tile C=%d r=%d", C, R);
    return MW_EUNSUPPORTED;
  }
  dim3 grid((W + BW - 1) / BW, (H + kBlurBH - 1) / kBlurBH);
  hipLaunchKernelGGL((blur_kernel<T, R, CP2>), grid, dim3(nt), lds, st, in, H, W, C, BW, inv_mean,
                     p, taps, out);
  MW_LAUNCH_CHECK();
  return MW_OK;
}

template <typename T, int R>
static int launch_blur_r(const T* in, int H, int W, int C, const float* inv_mean, float p,
                         const BlurTaps& taps, float* out, hipStream_t st) {
  const int cp = C / 2;
  if (cp <= 4) return launch_blur_rc<T, R, 4>(in, H, W, C, inv_mean, p, taps, out, st);
  if (cp <= 8) return launch_blur_rc<T, R, 8>(in, H, W, C, inv_mean, p, taps, out, st);
  if (cp <= 16) return launch_blur_rc<T, R, 16>(in, H, W, C, inv_mean, p, taps, out, st);
  return launch_blur_rc<T, R, 32>(in, H, W, C, inv_mean, p, taps, out, st);
}

// Fast path for even C <= 64 and r <= kBlurMaxR; MW_EUNSUPPORTED otherwise
// (the caller then takes the two-pass fallback).
template <typename T>
int launch_blur_valu(const T* in, int H, int W, int C, const float* inv_mean, float p,
                     const BlurTaps& taps, int r, float* out, hipStream_t st) {
  if (C % 2 != 0 || C > 64 || r < 0 || r > kBlurMaxR) return MW_EUNSUPPORTED;
  switch (r) {
#define MW_R(N) case N: return launch_blur_r<T, N>(in, H, W, C, inv_mean, p, taps, out, st);
    MW_R(0) MW_R(1) MW_R(2) MW_R(3) MW_R(4) MW_R(5) MW_R(6) MW_R(7) MW_R(8) MW_R(9) MW_R(10)
    MW_R(11) MW_R(12)
#undef MW_R
    default: return MW_EUNSUPPORTED;
  }
}

}  // namespace mw
