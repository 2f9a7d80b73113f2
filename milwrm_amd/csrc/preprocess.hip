// Preprocessing kernels of the MILWRM MxIF hot path on MI355X (gfx950).
//
//   nz_stats   img.calculate_non_zero_mean   MxIF.py:519-541
//   lognorm    img.log_normalize             MxIF.py:416-455
//   blur       img.blurring('gaussian')      MxIF.py:375-394 (skimage → scipy
//              gaussian_filter(mode='nearest', truncate=4), axes 0 then 1)
//   block_mean img.downsample(f, np.mean)    MxIF.py:494-517 (block_reduce, cval 0)
//   mask_rank  mask != 0 row-major compaction MxIF.py:486-488
//   gather     tmp[np.ix_(idx, features)]    MxIF.py:490-491 + StandardScaler stats
//
// Data layout: images are HWC (pixel-interleaved channels, as the reference's
// img.img), element type u8/u16/f32 on input, fp32 after the first transform.
// All reductions are deterministic: fixed block decomposition per size and a
// fixed combine order (no floating-point atomics).
#include <stdarg.h>
#include <math.h>

#include "common.h"

namespace mw {

static thread_local char g_err[512];

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

constexpr int kTile = 256;       // rows (samples / pixels) per block tile
constexpr int kMaxBlocks = 1024; // streaming workgroups (4 per CU)

static inline int stream_blocks(int64_t n) {
  int64_t tiles = (n + kTile - 1) / kTile;
  if (tiles < 1) tiles = 1;
  return (int)(tiles < kMaxBlocks ? tiles : kMaxBlocks);
}
// rows per block: whole tiles, identical for a given n
static inline int64_t rows_per_block(int64_t n) {
  int64_t tiles = (n + kTile - 1) / kTile;
  int g = stream_blocks(n);
  return ((tiles + g - 1) / g) * kTile;
}

// accurate log10(t + p) for t >= 0 (log1p-style correction of the rounding
// of t + p, so small t keep full relative accuracy)
__device__ __forceinline__ float lognorm1(float x, float inv, float p) {
  const float t = x * inv;
  const float v = t + p;
  const float e = (v - p) - t;  // rounding error of t + p (exact)
  const float l2 = __builtin_amdgcn_logf(v);  // log2, 1 ulp
  return l2 * 0.30102999566398120f - (e / v) * 0.43429448190325182f;
}

template <typename T> struct VecOf;
template <> struct VecOf<uint8_t> { static constexpr int N = 16; };
template <> struct VecOf<uint16_t> { static constexpr int N = 8; };
template <> struct VecOf<float> { static constexpr int N = 4; };

template <typename T, int N>
struct alignas(16) Pack { T v[N]; };

// ------------------------------------------------------------------ nz_stats
// Block b owns elements [b*epb, (b+1)*epb) of the flat HWC array; epb is a
// multiple of V*Teff where Teff*V % C == 0, so each lane's V channels are
// fixed for the whole block.  Per-lane fp64 sums / int64 counts, combined in a
// fixed order into per-block partial records [C sums | C counts].
template <typename T>
__global__ void __launch_bounds__(256) nz_stats_kernel(const T* __restrict__ img, int64_t n_elem,
                                                       int C, int teff, int64_t epb,
                                                       double* __restrict__ part) {
  constexpr int V = VecOf<T>::N;
  __shared__ double s_sum[256 * 16];
  __shared__ long long s_cnt[256 * 16];
  const int t = threadIdx.x;
  const int64_t lo = (int64_t)blockIdx.x * epb;
  const int64_t hi = min(n_elem, lo + epb);
  double acc[V];
  long long cnt[V];
#pragma unroll
  for (int i = 0; i < V; ++i) { acc[i] = 0.0; cnt[i] = 0; }
  if (t < teff) {
    const int64_t stride = (int64_t)teff * V;
    int64_t e = lo + (int64_t)t * V;
    for (; e + V <= hi; e += stride) {
      Pack<T, V> p = *reinterpret_cast<const Pack<T, V>*>(img + e);
#pragma unroll
      for (int i = 0; i < V; ++i) {
        const float x = (float)p.v[i];
        const bool nz = p.v[i] != T(0);
        acc[i] += nz ? (double)x : 0.0;
        cnt[i] += nz ? 1 : 0;
      }
    }
    // tail (partial vector): same lane → same channel assignment
    if (e < hi) {
#pragma unroll
      for (int i = 0; i < V; ++i) {
        if (e + i < hi) {
          const T v = img[e + i];
          if (v != T(0)) { acc[i] += (double)(float)v; cnt[i] += 1; }
        }
      }
    }
  }
#pragma unroll
  for (int i = 0; i < V; ++i) { s_sum[t * V + i] = acc[i]; s_cnt[t * V + i] = cnt[i]; }
  __syncthreads();
  if (t < C) {
    double s = 0.0;
    long long n = 0;
    for (int q = 0; q < teff * V; ++q) {
      if (q % C == t) { s += s_sum[q]; n += s_cnt[q]; }
    }
    part[(size_t)blockIdx.x * 2 * C + t] = s;
    part[(size_t)blockIdx.x * 2 * C + C + t] = (double)n;
  }
}

__global__ void nz_stats_reduce(const double* __restrict__ part, int G, int C,
                                double* __restrict__ sum, int64_t* __restrict__ cnt) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  double s = 0.0, n = 0.0;
  for (int b = 0; b < G; ++b) {
    s += part[(size_t)b * 2 * C + c];
    n += part[(size_t)b * 2 * C + C + c];
  }
  sum[c] = s;
  cnt[c] = (int64_t)n;
}

static inline int gcd_i(int a, int b) { while (b) { int t = a % b; a = b; b = t; } return a; }

struct NzPlan { int teff; int64_t epb; int G; };
template <typename T>
static NzPlan nz_plan(int64_t n_pix, int C) {
  constexpr int V = VecOf<T>::N;
  const int unit = C / gcd_i(V, C);  // lanes per channel period
  NzPlan p;
  p.teff = (256 / unit) * unit;
  const int64_t n_elem = n_pix * C;
  const int64_t chunk = (int64_t)p.teff * V;  // multiple of C, of V
  int64_t chunks = (n_elem + chunk - 1) / chunk;
  int G = (int)(chunks < kMaxBlocks ? chunks : kMaxBlocks);
  if (G < 1) G = 1;
  p.epb = ((chunks + G - 1) / G) * chunk;
  p.G = (int)((n_elem + p.epb - 1) / p.epb);
  if (p.G < 1) p.G = 1;
  return p;
}

// ------------------------------------------------------------------ lognorm
template <typename T>
__global__ void lognorm_kernel(const T* __restrict__ img, int64_t n_elem, int C,
                               const float* __restrict__ inv_mean, float p,
                               float* __restrict__ out) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n_elem; e += stride) {
    const int c = (int)(e % C);
    out[e] = lognorm1((float)img[e], inv_mean[c], p);
  }
}

// --------------------------------------------------------------------- blur
// One workgroup = a band of BW output columns x BH output rows, all C
// channels.  Rows stream top to bottom: each input row segment (with r-pixel
// horizontal halo, edge-clamped) is log-normalised into a double-buffered LDS
// row, the horizontal 2r+1-tap pass reads it from LDS, and the vertical pass
// keeps the last 2r+1 horizontally filtered rows in a register ring per
// element (static indices: the row loop is unrolled by 2r+1).  Output rows are
// written as contiguous HWC segments (coalesced).
constexpr int kMaxRadius = 32;
struct BlurTaps { float w[2 * kMaxRadius + 1]; };

constexpr int kEPT = 4;     // output elements per thread per row
constexpr int kMaxL = 12;   // input-row loads per thread per row (static bound)
constexpr int kBlurBH = 128;

template <typename T, int R>
__global__ void __launch_bounds__(1024) blur_kernel(const T* __restrict__ in, int H, int W, int C, int BW,
                                                    const float* __restrict__ inv_mean, float pseudo,
                                                    BlurTaps taps, float* __restrict__ out) {
  constexpr int NR = 2 * R + 1;
  extern __shared__ __attribute__((aligned(16))) float s_row[];  // 2 x (BW+2R)*C
  const int t = threadIdx.x;
  const int nt = blockDim.x;
  const int x0 = blockIdx.x * BW;
  const int y0 = blockIdx.y * kBlurBH;
  const int y1 = min(H, y0 + kBlurBH);
  const int bw = min(BW, W - x0);
  const int seg = (bw + 2 * R) * C;  // halo'd row elements
  const int rowcap = (BW + 2 * R) * C;
  const int nrows = (y1 - y0) + 2 * R;
  const bool logn = inv_mean != nullptr;

  // this thread's output elements (fixed for every row)
  int e_pos[kEPT];
  bool e_ok[kEPT];
#pragma unroll
  for (int i = 0; i < kEPT; ++i) {
    const int e = t * kEPT + i;
    e_ok[i] = e < bw * C;
    e_pos[i] = e_ok[i] ? e : 0;
  }
  // this thread's input-row load slots (fixed for every row): source element
  // offset inside the row (edge-clamped column) and the channel's 1/mean
  int l_src[kMaxL];
  float l_inv[kMaxL];
#pragma unroll
  for (int k = 0; k < kMaxL; ++k) {
    const int q = t + k * nt;
    l_src[k] = -1;
    l_inv[k] = 1.f;
    if (q < seg) {
      const int px = q / C;
      const int c = q - px * C;
      int gx = x0 - R + px;
      gx = gx < 0 ? 0 : (gx >= W ? W - 1 : gx);
      l_src[k] = gx * C + c;
      if (inv_mean) l_inv[k] = inv_mean[c];
    }
  }
  float ring[kEPT][NR];
#pragma unroll
  for (int i = 0; i < kEPT; ++i)
#pragma unroll
    for (int j = 0; j < NR; ++j) ring[i][j] = 0.f;

  float pre[kMaxL];
  auto fetch_row = [&](int rr) {
    int yy = y0 - R + rr;
    yy = yy < 0 ? 0 : (yy >= H ? H - 1 : yy);
    const T* src = in + (int64_t)yy * W * C;
#pragma unroll
    for (int k = 0; k < kMaxL; ++k) pre[k] = l_src[k] >= 0 ? (float)src[l_src[k]] : 0.f;
  };
  auto store_row = [&](int buf) {
    float* dst = s_row + buf * rowcap;
#pragma unroll
    for (int k = 0; k < kMaxL; ++k)
      if (l_src[k] >= 0) dst[t + k * nt] = logn ? lognorm1(pre[k], l_inv[k], pseudo) : pre[k];
  };

  fetch_row(0);
  store_row(0);
  __syncthreads();
  for (int base = 0; base < nrows; base += NR) {
#pragma unroll
    for (int s = 0; s < NR; ++s) {
      const int rr = base + s;
      if (rr < nrows) {
        const bool more = rr + 1 < nrows;
        if (more) fetch_row(rr + 1);  // global loads in flight during the compute
        const float* row = s_row + (rr & 1) * rowcap;
#pragma unroll
        for (int i = 0; i < kEPT; ++i) {
          float h = 0.f;
#pragma unroll
          for (int j = 0; j < NR; ++j) h = fmaf(taps.w[j], row[e_pos[i] + j * C], h);
          ring[i][s] = h;
        }
        if (rr >= 2 * R) {
          const int y = y0 + rr - 2 * R;
          float* orow = out + ((int64_t)y * W + x0) * C;
#pragma unroll
          for (int i = 0; i < kEPT; ++i) {
            float v = 0.f;
#pragma unroll
            for (int j = 0; j < NR; ++j) v = fmaf(taps.w[j], ring[i][(s + 1 + j) % NR], v);
            if (e_ok[i]) orow[e_pos[i]] = v;
          }
        }
        if (more) store_row((rr + 1) & 1);
        __syncthreads();
      }
    }
  }
}

template <typename T, int R>
static int launch_blur_r(const T* in, int H, int W, int C, const float* inv_mean, float p,
                         const BlurTaps& taps, float* out, hipStream_t st) {
  int BW = 64;
  while (BW > 1 && (BW * C + kEPT - 1) / kEPT > 1024) BW >>= 1;
  MW_CHECK_ARG((BW * C + kEPT - 1) / kEPT <= 1024, "mw_blur: C=%d too large", C);
  int nt = (BW * C + kEPT - 1) / kEPT;
  nt = ((nt + 63) / 64) * 64;
  const size_t lds = 2 * (size_t)(BW + 2 * R) * C * sizeof(float);
  MW_CHECK_ARG(lds <= 160 * 1024, "mw_blur: LDS %zu too large (C=%d, r=%d)", lds, C, R);
  MW_CHECK_ARG((BW + 2 * R) * C <= kMaxL * nt, "mw_blur: row segment exceeds load slots (C=%d r=%d)", C, R);
  dim3 grid((W + BW - 1) / BW, (H + kBlurBH - 1) / kBlurBH);
  hipLaunchKernelGGL((blur_kernel<T, R>), grid, dim3(nt), lds, st, in, H, W, C, BW, inv_mean, p,
                     taps, out);
  MW_LAUNCH_CHECK();
  return MW_OK;
}

// Generic-radius fallback (r > kRingMax): two separable passes through an fp32
// HWC temporary.  Pass 1 (axis 0): tmp[y,x,c] = sum_j w_j f(in[clamp(y+j-r),x,c]);
// pass 2 (axis 1): out[y,x,c] = sum_j w_j tmp[y,clamp(x+j-r),c].
template <typename T>
__global__ void blur_axis0_kernel(const T* __restrict__ in, int H, int W, int C,
                                  const float* __restrict__ inv_mean, float pseudo, BlurTaps taps,
                                  int r, float* __restrict__ tmp) {
  const int64_t n = (int64_t)H * W * C;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += stride) {
    const int64_t rowlen = (int64_t)W * C;
    const int y = (int)(e / rowlen);
    const int64_t xc = e - (int64_t)y * rowlen;
    const int c = (int)(xc % C);
    float acc = 0.f;
    for (int j = 0; j <= 2 * r; ++j) {
      int yy = y + j - r;
      yy = yy < 0 ? 0 : (yy >= H ? H - 1 : yy);
      float v = (float)in[(int64_t)yy * rowlen + xc];
      if (inv_mean) v = lognorm1(v, inv_mean[c], pseudo);
      acc = fmaf(taps.w[j], v, acc);
    }
    tmp[e] = acc;
  }
}
__global__ void blur_axis1_kernel(const float* __restrict__ tmp, int H, int W, int C, BlurTaps taps,
                                  int r, float* __restrict__ out) {
  const int64_t n = (int64_t)H * W * C;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += stride) {
    const int64_t p = e / C;
    const int c = (int)(e - p * C);
    const int x = (int)(p % W);
    const int64_t rowbase = (p - x) * C;
    float acc = 0.f;
    for (int j = 0; j <= 2 * r; ++j) {
      int xx = x + j - r;
      xx = xx < 0 ? 0 : (xx >= W ? W - 1 : xx);
      acc = fmaf(taps.w[j], tmp[rowbase + (int64_t)xx * C + c], acc);
    }
    out[e] = acc;
  }
}

constexpr int kRingMax = 12;

template <typename T>
static int launch_blur(const T* in, int H, int W, int C, const float* inv_mean, float p,
                       const BlurTaps& taps, int r, float* out, float* tmp, hipStream_t st) {
  switch (r) {
#define MW_R(N) case N: return launch_blur_r<T, N>(in, H, W, C, inv_mean, p, taps, out, st);
    MW_R(0) MW_R(1) MW_R(2) MW_R(3) MW_R(4) MW_R(5) MW_R(6) MW_R(7) MW_R(8) MW_R(9) MW_R(10)
    MW_R(11) MW_R(12)
#undef MW_R
    default: {
      MW_CHECK_ARG(tmp != nullptr, "mw_blur: radius %d needs a workspace (mw_blur_ws_bytes)", r);
      const int64_t n = (int64_t)H * W * C;
      const int grid = (int)std::min<int64_t>((n + 255) / 256, 16384);
      hipLaunchKernelGGL(blur_axis0_kernel<T>, dim3(grid), dim3(256), 0, st, in, H, W, C, inv_mean,
                         p, taps, r, tmp);
      MW_LAUNCH_CHECK();
      hipLaunchKernelGGL(blur_axis1_kernel, dim3(grid), dim3(256), 0, st, tmp, H, W, C, taps, r, out);
      MW_LAUNCH_CHECK();
      return MW_OK;
    }
  }
}

// --------------------------------------------------------------- block_mean
template <typename T>
__global__ void block_mean_kernel(const T* __restrict__ in, int H, int W, int C, int f, int Ho,
                                  int Wo, float* __restrict__ out) {
  const int64_t n = (int64_t)Ho * Wo * C;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const double inv = 1.0 / ((double)f * f);
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += stride) {
    const int c = (int)(e % C);
    const int64_t p = e / C;
    const int ox = (int)(p % Wo), oy = (int)(p / Wo);
    double s = 0.0;
    for (int dy = 0; dy < f; ++dy) {
      const int y = oy * f + dy;
      if (y >= H) break;
      for (int dx = 0; dx < f; ++dx) {
        const int x = ox * f + dx;
        if (x >= W) break;
        s += (double)(float)in[((int64_t)y * W + x) * C + c];
      }
    }
    out[e] = (float)(s * inv);
  }
}

// ---------------------------------------------------------------- mask_rank
constexpr int kMaskChunk = 16384;  // pixels per block (4 iterations x 4096)

__global__ void __launch_bounds__(256) mask_count_kernel(const uint8_t* __restrict__ m, int64_t n,
                                                         uint32_t* __restrict__ cnt) {
  __shared__ uint32_t s_red[4];
  const int64_t lo = (int64_t)blockIdx.x * kMaskChunk;
  uint32_t c = 0;
  for (int it = 0; it < kMaskChunk / 4096; ++it) {
    const int64_t p = lo + (int64_t)it * 4096 + threadIdx.x * 16;
    if (p + 16 <= n) {
      uint4 v = *reinterpret_cast<const uint4*>(m + p);
      const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int b = 0; b < 4; ++b) c += ((w[k] >> (8 * b)) & 0xFF) ? 1u : 0u;
    } else {
      for (int64_t q = p; q < n && q < p + 16; ++q) c += m[q] ? 1u : 0u;
    }
  }
  const uint32_t tot = block_sum(c, s_red);
  if (threadIdx.x == 0) cnt[blockIdx.x] = tot;
}

// exclusive scan of the per-block counts (single workgroup), total → *count
__global__ void __launch_bounds__(1024) mask_scan_kernel(uint32_t* __restrict__ cnt, int nb,
                                                         int64_t* __restrict__ count) {
  __shared__ unsigned long long s[1024];
  const int t = threadIdx.x;
  const int per = (nb + 1023) / 1024;
  const int lo = t * per, hi = min(nb, lo + per);
  unsigned long long loc = 0;
  for (int i = lo; i < hi; ++i) loc += cnt[i];
  s[t] = loc;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {
    unsigned long long v = t >= o ? s[t - o] : 0ull;
    __syncthreads();
    s[t] += v;
    __syncthreads();
  }
  unsigned long long run = s[t] - loc;  // exclusive
  for (int i = lo; i < hi; ++i) {
    const uint32_t c = cnt[i];
    cnt[i] = (uint32_t)run;  // fits: < 2^32 pixels supported
    run += c;
  }
  if (t == 1023) *count = (int64_t)s[1023];
}

__global__ void __launch_bounds__(256) mask_scatter_kernel(const uint8_t* __restrict__ m, int64_t n,
                                                           const uint32_t* __restrict__ base,
                                                           uint32_t* __restrict__ r2p) {
  __shared__ uint32_t s_w[4];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  uint32_t run = base[blockIdx.x];
  const int64_t lo = (int64_t)blockIdx.x * kMaskChunk;
  for (int it = 0; it < kMaskChunk / 4096; ++it) {
    const int64_t p = lo + (int64_t)it * 4096 + threadIdx.x * 16;
    uint32_t bits = 0;  // 16 flags
    for (int q = 0; q < 16; ++q) {
      const int64_t pp = p + q;
      if (pp < n && m[pp]) bits |= 1u << q;
    }
    const uint32_t c = __popc(bits);
    // inclusive scan within the wave
    uint32_t incl = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t v = __shfl_up(incl, o, 64);
      if (lane >= o) incl += v;
    }
    if (lane == 63) s_w[wid] = incl;
    __syncthreads();
    uint32_t wbase = 0;
    for (int w = 0; w < wid; ++w) wbase += s_w[w];
    uint32_t pos = run + wbase + incl - c;
    while (bits) {
      const int q = __ffs(bits) - 1;
      bits &= bits - 1;
      r2p[pos++] = (uint32_t)(p + q);
    }
    const uint32_t tot = s_w[0] + s_w[1] + s_w[2] + s_w[3];
    __syncthreads();
    run += tot;
  }
}

// ------------------------------------------------------------------- gather
// Block b owns sample rows [b*R, (b+1)*R) in 256-row tiles.  Per tile: gather
// rows into LDS, write them coalesced, and fold per-column Chan statistics.
// Stats threads: f = t % F, part = t / F (nparts = 256 / F).  Record per block:
// [n, mean[F], M2[F]].
__device__ __forceinline__ void chan_merge(double& n_a, double& m_a, double& q_a, double n_b,
                                           double m_b, double q_b) {
  if (n_b == 0.0) return;
  if (n_a == 0.0) { n_a = n_b; m_a = m_b; q_a = q_b; return; }
  const double n = n_a + n_b;
  const double d = m_b - m_a;
  m_a += d * (n_b / n);
  q_a += q_b + d * d * (n_a * n_b / n);
  n_a = n;
}

__global__ void __launch_bounds__(256) gather_kernel(const float* __restrict__ img, int C,
                                                     const int32_t* __restrict__ feat, int F,
                                                     const int32_t* __restrict__ idx,
                                                     const uint32_t* __restrict__ r2p, int64_t S,
                                                     int64_t R, float* __restrict__ X,
                                                     double* __restrict__ rec) {
  extern __shared__ __attribute__((aligned(16))) float s_tile[];  // 256*F floats + stats scratch
  __shared__ int s_feat[256];
  const int t = threadIdx.x;
  for (int f = t; f < F; f += 256) s_feat[f] = feat[f];
  const int nparts = 256 / F;
  const bool st_on = t < nparts * F;
  const int sf = st_on ? t % F : 0, spart = st_on ? t / F : 0;
  double n_acc = 0.0, m_acc = 0.0, q_acc = 0.0;
  const int64_t lo = (int64_t)blockIdx.x * R;
  const int64_t hi = min(S, lo + R);
  __syncthreads();
  for (int64_t r0 = lo; r0 < hi; r0 += kTile) {
    const int nrow = (int)min((int64_t)kTile, hi - r0);
    if (t < nrow) {
      const int64_t j = r0 + t;
      const uint32_t p = r2p[idx[j]];
      const float* src = img + (int64_t)p * C;
      for (int f = 0; f < F; ++f) s_tile[t * F + f] = src[s_feat[f]];
    }
    __syncthreads();
    // coalesced write of the tile (rows contiguous in X)
    float* dst = X + r0 * F;
    const int ne = nrow * F;
    for (int q = t; q < ne; q += 256) dst[q] = s_tile[q];
    // column statistics of this tile part
    if (st_on) {
      double s = 0.0, cnt = 0.0;
      for (int r = spart; r < nrow; r += nparts) { s += (double)s_tile[r * F + sf]; cnt += 1.0; }
      if (cnt > 0.0) {
        const double m = s / cnt;
        double q = 0.0;
        for (int r = spart; r < nrow; r += nparts) {
          const double d = (double)s_tile[r * F + sf] - m;
          q += d * d;
        }
        chan_merge(n_acc, m_acc, q_acc, cnt, m, q);
      }
    }
    __syncthreads();
  }
  // merge parts in fixed order: stage (n, m, q) in LDS (reuse tile memory)
  double* s_st = reinterpret_cast<double*>(s_tile);
  if (st_on) {
    s_st[3 * t + 0] = n_acc;
    s_st[3 * t + 1] = m_acc;
    s_st[3 * t + 2] = q_acc;
  }
  __syncthreads();
  double* out = rec + (size_t)blockIdx.x * (1 + 2 * F);
  if (t < F) {
    double n = 0.0, m = 0.0, q = 0.0;
    for (int part = 0; part < nparts; ++part) {
      const int u = part * F + t;
      chan_merge(n, m, q, s_st[3 * u], s_st[3 * u + 1], s_st[3 * u + 2]);
    }
    if (t == 0) out[0] = n;
    out[1 + t] = m;
    out[1 + F + t] = q;
  }
}

__global__ void col_stats_kernel(const double* __restrict__ rec, int G, int F, double* __restrict__ st,
                                 int accumulate) {
  const int f = threadIdx.x;
  double n = 0.0, m = 0.0, q = 0.0;
  if (f < F) {
    if (accumulate) { n = st[0]; m = st[1 + f]; q = st[1 + F + f]; }
    for (int b = 0; b < G; ++b) {
      const double* r = rec + (size_t)b * (1 + 2 * F);
      chan_merge(n, m, q, r[0], r[1 + f], r[1 + F + f]);
    }
  }
  __syncthreads();  // every thread has read st[0] before it is rewritten
  if (f < F) {
    if (f == 0) st[0] = n;
    st[1 + f] = m;
    st[1 + F + f] = q;
  }
}

// ------------------------------------------------------------- synth slide
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}
__device__ __forceinline__ float u01(uint64_t h) { return ((h >> 40) + 0.5f) * (1.0f / 16777216.0f); }

__global__ void synth_kernel(int H, int W, int C, const float* __restrict__ syx, int ns,
                             const float* __restrict__ prof, int nd, int shape_k, int bg_rows,
                             uint64_t seed, uint16_t* __restrict__ img, uint8_t* __restrict__ mask) {
  const int64_t n = (int64_t)H * W;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n; p += stride) {
    const int y = (int)(p / W), x = (int)(p % W);
    float best = 3.4e38f;
    int dom = 0;
    for (int s = 0; s < ns; ++s) {
      const float dy = y - syx[2 * s], dx = x - syx[2 * s + 1];
      const float d = dy * dy + dx * dx;
      if (d < best) { best = d; dom = s % nd; }
    }
    const bool bg = y < bg_rows;
    mask[p] = bg ? 0 : 1;
    for (int c = 0; c < C; ++c) {
      // Gamma(shape_k, 1/shape_k) as a mean of shape_k unit exponentials
      float g = 0.f;
      for (int k = 0; k < shape_k; ++k) {
        const uint64_t h = splitmix64(seed ^ (((uint64_t)p * C + c) * 8 + k) * 0xD1B54A32D192ED03ull);
        g += -__logf(u01(h));
      }
      g /= (float)shape_k;
      float v = prof[dom * C + c] * g;
      if (bg) v *= 0.05f;
      v = rintf(v);
      v = v < 0.f ? 0.f : (v > 65535.f ? 65535.f : v);
      img[p * C + c] = (uint16_t)v;
    }
  }
}

}  // namespace mw

using namespace mw;

// ======================================================================= C ABI
extern "C" {

int mw_version(void) { return 10000; }
const char* mw_last_error(void) { return mw::g_err; }
int mw_stream_blocks(int64_t n) { return stream_blocks(n); }

size_t mw_nz_stats_ws_bytes(int64_t n_pix, int C) {
  // worst case over dtypes: the u8 plan has the most blocks
  return (size_t)kMaxBlocks * 2 * (size_t)C * sizeof(double) + 256;
}

int mw_nz_stats(const void* d_img, int dtype, int64_t n_pix, int C, double* d_sum, int64_t* d_cnt,
                void* d_ws, void* stream) {
  MW_CHECK_ARG(d_img && d_sum && d_cnt && d_ws, "mw_nz_stats: null pointer");
  MW_CHECK_ARG(n_pix > 0 && C > 0 && C <= 4096, "mw_nz_stats: bad shape n_pix=%lld C=%d",
               (long long)n_pix, C);
  MW_CHECK_ARG(((uintptr_t)d_img & 15) == 0, "mw_nz_stats: image must be 16-byte aligned");
  hipStream_t st = as_stream(stream);
  double* part = reinterpret_cast<double*>(d_ws);
  const int64_t n_elem = n_pix * C;
  NzPlan p;
  switch (dtype) {
    case MW_U8:
      p = nz_plan<uint8_t>(n_pix, C);
      hipLaunchKernelGGL(nz_stats_kernel<uint8_t>, dim3(p.G), dim3(256), 0, st,
                         (const uint8_t*)d_img, n_elem, C, p.teff, p.epb, part);
      break;
    case MW_U16:
      p = nz_plan<uint16_t>(n_pix, C);
      hipLaunchKernelGGL(nz_stats_kernel<uint16_t>, dim3(p.G), dim3(256), 0, st,
                         (const uint16_t*)d_img, n_elem, C, p.teff, p.epb, part);
      break;
    case MW_F32:
      p = nz_plan<float>(n_pix, C);
      hipLaunchKernelGGL(nz_stats_kernel<float>, dim3(p.G), dim3(256), 0, st,
                         (const float*)d_img, n_elem, C, p.teff, p.epb, part);
      break;
    default:
      set_error("mw_nz_stats: bad dtype %d", dtype);
      return MW_EINVAL;
  }
  MW_LAUNCH_CHECK();
  hipLaunchKernelGGL(nz_stats_reduce, dim3((C + 255) / 256), dim3(256), 0, st, part, p.G, C, d_sum,
                     d_cnt);
  MW_LAUNCH_CHECK();
  return MW_OK;
}

int mw_lognorm(const void* d_img, int dtype, int64_t n_pix, int C, const float* d_inv_mean,
               float pseudoval, float* d_out, void* stream) {
  MW_CHECK_ARG(d_img && d_inv_mean && d_out, "mw_lognorm: null pointer");
  MW_CHECK_ARG(n_pix > 0 && C > 0, "mw_lognorm: bad shape");
  hipStream_t st = as_stream(stream);
  const int64_t n = n_pix * C;
  const int grid = (int)std::min<int64_t>((n + 255) / 256, 8192);
  switch (dtype) {
    case MW_U8: hipLaunchKernelGGL(lognorm_kernel<uint8_t>, dim3(grid), dim3(256), 0, st, (const uint8_t*)d_img, n, C, d_inv_mean, pseudoval, d_out); break;
    case MW_U16: hipLaunchKernelGGL(lognorm_kernel<uint16_t>, dim3(grid), dim3(256), 0, st, (const uint16_t*)d_img, n, C, d_inv_mean, pseudoval, d_out); break;
    case MW_F32: hipLaunchKernelGGL(lognorm_kernel<float>, dim3(grid), dim3(256), 0, st, (const float*)d_img, n, C, d_inv_mean, pseudoval, d_out); break;
    default: set_error("mw_lognorm: bad dtype %d", dtype); return MW_EINVAL;
  }
  MW_LAUNCH_CHECK();
  return MW_OK;
}

size_t mw_blur_ws_bytes(int H, int W, int C, int radius) {
  return radius > kRingMax ? (size_t)H * W * C * sizeof(float) + 256 : 0;
}

int mw_blur(const void* d_img, int dtype, int H, int W, int C, const float* d_inv_mean,
            float pseudoval, const float* h_w, int radius, float* d_out, void* d_ws, void* stream) {
  MW_CHECK_ARG(d_img && d_out && h_w, "mw_blur: null pointer");
  MW_CHECK_ARG(H > 0 && W > 0 && C > 0, "mw_blur: bad shape %dx%dx%d", H, W, C);
  MW_CHECK_ARG(d_img != (const void*)d_out, "mw_blur: out must not alias in");
  MW_CHECK_ARG(radius >= 0, "mw_blur: bad radius");
  if (radius > kMaxRadius) {
    set_error("mw_blur: radius %d unsupported (max %d, i.e. sigma <= 7.9)", radius, kMaxRadius);
    return MW_EUNSUPPORTED;
  }
  BlurTaps taps;
  memset(&taps, 0, sizeof(taps));
  for (int j = 0; j <= 2 * radius; ++j) taps.w[j] = h_w[j];
  hipStream_t st = as_stream(stream);
  float* tmp = reinterpret_cast<float*>(d_ws);
  switch (dtype) {
    case MW_U8: return launch_blur<uint8_t>((const uint8_t*)d_img, H, W, C, d_inv_mean, pseudoval, taps, radius, d_out, tmp, st);
    case MW_U16: return launch_blur<uint16_t>((const uint16_t*)d_img, H, W, C, d_inv_mean, pseudoval, taps, radius, d_out, tmp, st);
    case MW_F32: return launch_blur<float>((const float*)d_img, H, W, C, d_inv_mean, pseudoval, taps, radius, d_out, tmp, st);
    default: set_error("mw_blur: bad dtype %d", dtype); return MW_EINVAL;
  }
}

int mw_block_mean(const void* d_img, int dtype, int H, int W, int C, int fact, float* d_out,
                  void* stream) {
  MW_CHECK_ARG(d_img && d_out, "mw_block_mean: null pointer");
  MW_CHECK_ARG(H > 0 && W > 0 && C > 0 && fact > 0, "mw_block_mean: bad shape");
  const int Ho = (H + fact - 1) / fact, Wo = (W + fact - 1) / fact;
  const int64_t n = (int64_t)Ho * Wo * C;
  const int grid = (int)std::min<int64_t>((n + 255) / 256, 8192);
  hipStream_t st = as_stream(stream);
  switch (dtype) {
    case MW_U8: hipLaunchKernelGGL(block_mean_kernel<uint8_t>, dim3(grid), dim3(256), 0, st, (const uint8_t*)d_img, H, W, C, fact, Ho, Wo, d_out); break;
    case MW_U16: hipLaunchKernelGGL(block_mean_kernel<uint16_t>, dim3(grid), dim3(256), 0, st, (const uint16_t*)d_img, H, W, C, fact, Ho, Wo, d_out); break;
    case MW_F32: hipLaunchKernelGGL(block_mean_kernel<float>, dim3(grid), dim3(256), 0, st, (const float*)d_img, H, W, C, fact, Ho, Wo, d_out); break;
    default: set_error("mw_block_mean: bad dtype %d", dtype); return MW_EINVAL;
  }
  MW_LAUNCH_CHECK();
  return MW_OK;
}

size_t mw_mask_rank_ws_bytes(int64_t n_pix) {
  const int64_t nb = (n_pix + kMaskChunk - 1) / kMaskChunk;
  return (size_t)nb * sizeof(uint32_t) + 256;
}

int mw_mask_rank(const uint8_t* d_mask, int64_t n_pix, uint32_t* d_rank2pix, int64_t* d_count,
                 void* d_ws, void* stream) {
  MW_CHECK_ARG(d_mask && d_rank2pix && d_count && d_ws, "mw_mask_rank: null pointer");
  MW_CHECK_ARG(n_pix > 0 && n_pix < (int64_t)4294967295LL, "mw_mask_rank: n_pix out of range");
  MW_CHECK_ARG(((uintptr_t)d_mask & 15) == 0, "mw_mask_rank: mask must be 16-byte aligned");
  hipStream_t st = as_stream(stream);
  const int nb = (int)((n_pix + kMaskChunk - 1) / kMaskChunk);
  uint32_t* cnt = reinterpret_cast<uint32_t*>(d_ws);
  hipLaunchKernelGGL(mask_count_kernel, dim3(nb), dim3(256), 0, st, d_mask, n_pix, cnt);
  MW_LAUNCH_CHECK();
  hipLaunchKernelGGL(mask_scan_kernel, dim3(1), dim3(1024), 0, st, cnt, nb, d_count);
  MW_LAUNCH_CHECK();
  hipLaunchKernelGGL(mask_scatter_kernel, dim3(nb), dim3(256), 0, st, d_mask, n_pix, cnt, d_rank2pix);
  MW_LAUNCH_CHECK();
  return MW_OK;
}

size_t mw_gather_ws_bytes(int64_t S, int F) {
  return (size_t)stream_blocks(S) * (1 + 2 * (size_t)F) * sizeof(double) + 256;
}

int mw_gather_rows(const float* d_img, int C, const int32_t* d_feat, int F, const int32_t* d_idx,
                   const uint32_t* d_rank2pix, int64_t S, float* d_X, void* d_ws, void* stream) {
  MW_CHECK_ARG(d_img && d_feat && d_idx && d_rank2pix && d_X && d_ws, "mw_gather_rows: null pointer");
  MW_CHECK_ARG(S > 0 && F > 0 && F <= 256 && C > 0, "mw_gather_rows: bad shape S=%lld F=%d",
               (long long)S, F);
  hipStream_t st = as_stream(stream);
  const int G = stream_blocks(S);
  const int64_t R = rows_per_block(S);
  size_t lds = (size_t)kTile * F * sizeof(float);
  if (lds < 3 * 256 * sizeof(double)) lds = 3 * 256 * sizeof(double);
  hipLaunchKernelGGL(gather_kernel, dim3(G), dim3(256), lds, st, d_img, C, d_feat, F, d_idx,
                     d_rank2pix, S, R, d_X, reinterpret_cast<double*>(d_ws));
  MW_LAUNCH_CHECK();
  return MW_OK;
}

int mw_col_stats_finalize(const void* d_ws, int64_t S, int F, double* d_stats, int accumulate,
                          void* stream) {
  MW_CHECK_ARG(d_ws && d_stats && F > 0 && F <= 1024, "mw_col_stats_finalize: bad args");
  hipLaunchKernelGGL(col_stats_kernel, dim3(1), dim3(1024), 0, as_stream(stream),
                     reinterpret_cast<const double*>(d_ws), stream_blocks(S), F, d_stats, accumulate);
  MW_LAUNCH_CHECK();
  return MW_OK;
}

int mw_synth_slide(int H, int W, int C, const float* d_seed_yx, int n_seeds, const float* d_profiles,
                   int n_domains, int shape_k, int bg_rows, uint64_t seed, uint16_t* d_img,
                   uint8_t* d_mask, void* stream) {
  MW_CHECK_ARG(d_seed_yx && d_profiles && d_img && d_mask, "mw_synth_slide: null pointer");
  MW_CHECK_ARG(H > 0 && W > 0 && C > 0 && n_seeds > 0 && n_domains > 0 && shape_k > 0,
               "mw_synth_slide: bad args");
  const int64_t n = (int64_t)H * W;
  const int grid = (int)std::min<int64_t>((n + 255) / 256, 65536);
  hipLaunchKernelGGL(synth_kernel, dim3(grid), dim3(256), 0, as_stream(stream), H, W, C, d_seed_yx,
                     n_seeds, d_profiles, n_domains, shape_k, bg_rows, seed, d_img, d_mask);
  MW_LAUNCH_CHECK();
  return MW_OK;
}

}  // extern "C"
