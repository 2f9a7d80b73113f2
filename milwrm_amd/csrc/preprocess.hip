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
#include "blur.h"

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
    // four independent 16-B loads in flight per iteration
    for (; e + 3 * stride + V <= hi; e += 4 * stride) {
      Pack<T, V> p[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) p[u] = *reinterpret_cast<const Pack<T, V>*>(img + e + u * stride);
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int i = 0; i < V; ++i) {
          const bool nz = p[u].v[i] != T(0);
          acc[i] += nz ? (double)(float)p[u].v[i] : 0.0;
          cnt[i] += nz ? 1 : 0;
        }
    }
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

// uint16 slides (the MxIF case): exact integer accumulation, two VALU
// operations per element instead of a fp64 add, an int64 add and conversions
// (the fp64 form made this pure read stream VALU-bound at 4.4 TB/s).  Per
// lane and 16-byte load (8 channels, 4 words of 2): the low and high halves
// of each word go into uint32 sums, and min(word, 0x00010001) -- 1 per
// non-zero half -- into packed uint16 counts (v_pk_min_u16 / v_pk_add_u16).
// The 32-bit sums and 16-bit counts are flushed to 64-bit totals every
// kNzFlush loads (65535 * kNzFlush < 2^32, kNzFlush < 2^16).  Block records
// as nz_stats_kernel: [C sums | C counts], integer-valued fp64.
typedef unsigned short nz_us2 __attribute__((ext_vector_type(2)));
constexpr int kNzFlush = 32768;
__global__ void __launch_bounds__(256) nz_stats_u16_kernel(const uint16_t* __restrict__ img,
                                                           int64_t n_elem, int C, int teff,
                                                           int64_t epb, double* __restrict__ part) {
  constexpr int V = 8;
  __shared__ unsigned long long s_sum[256 * V];
  __shared__ unsigned int s_cnt[256 * V];
  const int t = threadIdx.x;
  const int64_t lo = (int64_t)blockIdx.x * epb;
  const int64_t hi = min(n_elem, lo + epb);
  unsigned long long tot[V], totc[V];
#pragma unroll
  for (int i = 0; i < V; ++i) { tot[i] = 0ull; totc[i] = 0ull; }
  if (t < teff) {
    const int64_t stride = (int64_t)teff * V;
    int64_t e = lo + (int64_t)t * V;
    while (e < hi) {
      unsigned int sum[V];
      nz_us2 cnt[V / 2];
#pragma unroll
      for (int i = 0; i < V; ++i) sum[i] = 0u;
#pragma unroll
      for (int j = 0; j < V / 2; ++j) cnt[j] = nz_us2{0, 0};
      auto take = [&](const uint4& w4) {
        const unsigned int w[4] = {w4.x, w4.y, w4.z, w4.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          sum[2 * j] += w[j] & 0xffffu;
          sum[2 * j + 1] += w[j] >> 16;
          const nz_us2 h = __builtin_bit_cast(nz_us2, w[j]);
          cnt[j] += __builtin_elementwise_min(h, nz_us2{1, 1});
        }
      };
      // up to kNzFlush loads, four 16-B loads in flight
      int n = 0;
      for (; n + 4 <= kNzFlush && e + 3 * stride + V <= hi; n += 4, e += 4 * stride) {
        uint4 w[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) w[u] = *reinterpret_cast<const uint4*>(img + e + u * stride);
#pragma unroll
        for (int u = 0; u < 4; ++u) take(w[u]);
      }
      for (; n < kNzFlush && e + V <= hi; ++n, e += stride) take(*reinterpret_cast<const uint4*>(img + e));
      if (n < kNzFlush && e < hi) {  // tail (partial vector): same lane, same channels
        uint4 w4 = uint4{0u, 0u, 0u, 0u};
        unsigned int* wp = reinterpret_cast<unsigned int*>(&w4);
        for (int i = 0; i < V; ++i)
          if (e + i < hi) wp[i >> 1] |= (unsigned int)img[e + i] << (16 * (i & 1));
        take(w4);
        e = hi;
      }
#pragma unroll
      for (int j = 0; j < V / 2; ++j) {
        tot[2 * j] += sum[2 * j];
        tot[2 * j + 1] += sum[2 * j + 1];
        totc[2 * j] += cnt[j].x;
        totc[2 * j + 1] += cnt[j].y;
      }
    }
  }
#pragma unroll
  for (int i = 0; i < V; ++i) { s_sum[t * V + i] = tot[i]; s_cnt[t * V + i] = (unsigned int)totc[i]; }
  __syncthreads();
  if (t < C) {
    unsigned long long sm = 0ull, nn = 0ull;
    for (int q = t; q < teff * V; q += C) { sm += s_sum[q]; nn += s_cnt[q]; }
    part[(size_t)blockIdx.x * 2 * C + t] = (double)sm;
    part[(size_t)blockIdx.x * 2 * C + C + t] = (double)nn;
  }
}

// per channel (one workgroup each) the sum of the G block records: integer-
// valued fp64 below 2^53, so exact in any order
__global__ void __launch_bounds__(256) nz_stats_reduce(const double* __restrict__ part, int G, int C,
                                                       double* __restrict__ sum, int64_t* __restrict__ cnt) {
  __shared__ double s_s[256], s_n[256];
  const int c = blockIdx.x, t = threadIdx.x;
  double sm = 0.0, n = 0.0;
  for (int b = t; b < G; b += 256) {
    sm += part[(size_t)b * 2 * C + c];
    n += part[(size_t)b * 2 * C + C + c];
  }
  s_s[t] = sm;
  s_n[t] = n;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (t < o) { s_s[t] += s_s[t + o]; s_n[t] += s_n[t + o]; }
    __syncthreads();
  }
  if (t == 0) { sum[c] = s_s[0]; cnt[c] = (int64_t)s_n[0]; }
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
// Fast path: blur.h, instantiated per dtype in blur_{u8,u16,f32}.hip.
extern template int launch_blur_fast<uint8_t>(const uint8_t*, int, int, int, const float*, float,
                                              const BlurTaps&, int, float*, hipStream_t);
extern template int launch_blur_fast<uint16_t>(const uint16_t*, int, int, int, const float*, float,
                                               const BlurTaps&, int, float*, hipStream_t);
extern template int launch_blur_fast<float>(const float*, int, int, int, const float*, float,
                                            const BlurTaps&, int, float*, hipStream_t);

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

template <typename T>
static int launch_blur(const T* in, int H, int W, int C, const float* inv_mean, float p,
                       const BlurTaps& taps, int r, float* out, float* tmp, hipStream_t st) {
  const int rc = launch_blur_fast<T>(in, H, W, C, inv_mean, p, taps, r, out, st);
  if (rc != MW_EUNSUPPORTED) return rc;
  // two-pass fallback (odd C, C > 64 or r > kBlurMaxR)
  MW_CHECK_ARG(tmp != nullptr, "mw_blur: radius %d / C=%d needs a workspace (mw_blur_ws_bytes)", r, C);
  const int64_t n = (int64_t)H * W * C;
  const int grid = (int)std::min<int64_t>((n + 255) / 256, 16384);
  hipLaunchKernelGGL(blur_axis0_kernel<T>, dim3(grid), dim3(256), 0, st, in, H, W, C, inv_mean,
                     p, taps, r, tmp);
  MW_LAUNCH_CHECK();
  hipLaunchKernelGGL(blur_axis1_kernel, dim3(grid), dim3(256), 0, st, tmp, H, W, C, taps, r, out);
  MW_LAUNCH_CHECK();
  return MW_OK;
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

// ------------------------------------------------------------ rank index
// The mask rank as a compact index instead of a rank -> pixel table: per
// 64-pixel word its mask bits (u64) and the tissue pixels before it (u32
// prefix, one extra entry = M), and per 64 ranks the word holding the first
// of them.  A lookup (rank_pixel) reads blk, one or two prefix entries and
// one bit word, then selects the bit: ~1/6 byte of index per pixel (24 MB at
// 10k^2 instead of a 340 MB table), so the random lookups of the subsample
// hit the on-die caches instead of HBM lines.
struct RankIndexPtrs {
  const uint64_t* bits;
  const uint32_t* pre;
  const uint32_t* blk;
};
__host__ __device__ inline int64_t rank_words(int64_t n) { return (n + 63) / 64; }
__host__ __device__ inline size_t rank_al(size_t x) { return (x + 255) & ~(size_t)255; }
__host__ __device__ inline size_t rank_pre_off(int64_t n) { return rank_al((size_t)rank_words(n) * 8); }
__host__ __device__ inline size_t rank_blk_off(int64_t n) {
  return rank_pre_off(n) + rank_al((size_t)(rank_words(n) + 1) * 4);
}
__host__ __device__ inline size_t rank_index_bytes(int64_t n) {
  return rank_blk_off(n) + rank_al((size_t)(rank_words(n) + 1) * 4);
}
__host__ __device__ inline RankIndexPtrs rank_ptrs(const void* base, int64_t n) {
  const char* b = reinterpret_cast<const char*>(base);
  return RankIndexPtrs{reinterpret_cast<const uint64_t*>(b), reinterpret_cast<const uint32_t*>(b + rank_pre_off(n)),
                       reinterpret_cast<const uint32_t*>(b + rank_blk_off(n))};
}
// position of the r-th (0-based) set bit of m (r < popcount(m))
__device__ __forceinline__ uint32_t select64(uint64_t m, uint32_t r) {
  uint32_t pos = 0;
  uint32_t x = (uint32_t)m;
  uint32_t c = __popc(x);
  if (r >= c) { r -= c; pos = 32; x = (uint32_t)(m >> 32); }
  c = __popc(x & 0xFFFFu);
  if (r >= c) { r -= c; pos += 16; x >>= 16; }
  c = __popc(x & 0xFFu);
  if (r >= c) { r -= c; pos += 8; x >>= 8; }
  c = __popc(x & 0xFu);
  if (r >= c) { r -= c; pos += 4; x >>= 4; }
  c = __popc(x & 0x3u);
  if (r >= c) { r -= c; pos += 2; x >>= 2; }
  c = x & 1u;
  if (r >= c) pos += 1;
  return pos;
}
// pixel of tissue rank rho (rho < M)
__device__ __forceinline__ uint32_t rank_pixel(const RankIndexPtrs& ix, uint32_t rho) {
  uint32_t w = ix.blk[rho >> 6];
  uint32_t p0 = ix.pre[w], p1 = ix.pre[w + 1];
  while (p1 <= rho) {
    ++w;
    p0 = p1;
    p1 = ix.pre[w + 1];
  }
  return w * 64u + select64(ix.bits[w], rho - p0);
}

// per 64-pixel word: bits, prefix (block base from mask_scan_kernel + the
// block's own scan), and blk[] for the ranks 64b that fall in the word
__global__ void __launch_bounds__(256) rank_words_kernel(const uint8_t* __restrict__ m, int64_t n,
                                                         const uint32_t* __restrict__ base,
                                                         const int64_t* __restrict__ count,
                                                         uint64_t* __restrict__ bits, uint32_t* __restrict__ pre,
                                                         uint32_t* __restrict__ blk) {
  __shared__ uint32_t s_w[4];
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  const int64_t NW = rank_words(n);
  const int64_t w = (int64_t)blockIdx.x * (kMaskChunk / 64) + t;  // 256 words per block
  const int64_t p = w * 64;
  uint64_t b = 0;
  if (p + 64 <= n) {
    const uint4* v4 = reinterpret_cast<const uint4*>(m + p);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint4 v = v4[j];
      const uint32_t ww[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int q = 0; q < 4; ++q)
          b |= ((ww[k] >> (8 * q)) & 0xFFu) ? 1ull << (16 * j + 4 * k + q) : 0ull;
    }
  } else if (p < n) {
    for (int q = 0; q < 64 && p + q < n; ++q) b |= m[p + q] ? 1ull << q : 0ull;
  }
  const uint32_t c = __popcll(b);
  uint32_t incl = c;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t v = __shfl_up(incl, o, 64);
    if (lane >= o) incl += v;
  }
  if (lane == 63) s_w[wid] = incl;
  __syncthreads();
  uint32_t wbase = base[blockIdx.x];
  for (int j = 0; j < wid; ++j) wbase += s_w[j];
  const uint32_t lo = wbase + incl - c;
  if (w < NW) {
    bits[w] = b;
    pre[w] = lo;
    for (uint32_t r = (lo + 63) & ~63u; r < lo + c; r += 64) blk[r >> 6] = (uint32_t)w;
  }
  if (w == NW - 1) {
    pre[NW] = (uint32_t)*count;
    if (((uint32_t)*count & 63u) == 0) blk[(uint32_t)*count >> 6] = (uint32_t)NW;  // sentinel (never read for rho < M)
  }
}

__global__ void __launch_bounds__(256) mask_scatter_kernel(const uint8_t* __restrict__ m, int64_t n,
                                                           const uint32_t* __restrict__ base,
                                                           uint32_t* __restrict__ r2p) {
  // per 4096-pixel step: 16 mask bytes per lane in one 16-byte load, a block
  // scan of the per-lane counts, the step's pixel indices staged in LDS at
  // their ranks, then written as one contiguous coalesced run
  __shared__ uint32_t s_w[4];
  __shared__ uint32_t s_pix[4096];
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  uint32_t run = base[blockIdx.x];
  const int64_t lo = (int64_t)blockIdx.x * kMaskChunk;
  for (int it = 0; it < kMaskChunk / 4096; ++it) {
    const int64_t p = lo + (int64_t)it * 4096 + t * 16;
    uint32_t bits = 0;  // 16 flags
    if (p + 16 <= n) {
      const uint4 v = *reinterpret_cast<const uint4*>(m + p);
      const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int q = 0; q < 4; ++q) bits |= ((w[k] >> (8 * q)) & 0xFFu) ? 1u << (4 * k + q) : 0u;
    } else {
      for (int q = 0; q < 16; ++q)
        if (p + q < n && m[p + q]) bits |= 1u << q;
    }
    const uint32_t c = __popc(bits);
    uint32_t incl = c;  // inclusive scan within the wave
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t v = __shfl_up(incl, o, 64);
      if (lane >= o) incl += v;
    }
    if (lane == 63) s_w[wid] = incl;
    __syncthreads();
    uint32_t wbase = 0;
    for (int w = 0; w < wid; ++w) wbase += s_w[w];
    uint32_t loc = wbase + incl - c;
    while (bits) {
      const int q = __ffs(bits) - 1;
      bits &= bits - 1;
      s_pix[loc++] = (uint32_t)(p + q);
    }
    const uint32_t tot = s_w[0] + s_w[1] + s_w[2] + s_w[3];
    __syncthreads();
    for (uint32_t i = t; i < tot; i += 256) r2p[run + i] = s_pix[i];
    run += tot;
    __syncthreads();  // s_pix / s_w reused by the next step
  }
}

// ------------------------------------------------------------------- gather
// Block b owns sample rows [b*R, (b+1)*R) in 256-row tiles.  Per tile: gather
// rows into LDS, write them coalesced, and fold per-column Chan statistics.
// Stats threads: f = t % F, part = t / F (nparts = 256 / F).  Record per block:
// [n, mean[F], M2[F], max|x|[F]] (the column maxima feed the fixed-point
// exponents of the Lloyd M-step: no separate pass over the rows).
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

// GATHER false: the rows are already in X (written by the fused blur sample
// epilogue) and only the statistics are taken, over the same block/tile
// partition and in the same order, so both give identical records.
// RI: the sample -> pixel lookups through the rank index (rank_pixel, + pix_off)
// instead of the rank -> pixel table r2p
// PX: idx already holds pixels (mw_rank_to_pixel_ri ran on the draws)
template <bool GATHER, bool RI = false, bool PX = false>
__global__ void __launch_bounds__(256) gather_kernel(const float* __restrict__ img, int C,
                                                     const int32_t* __restrict__ feat, int F,
                                                     const int32_t* __restrict__ idx,
                                                     const uint32_t* __restrict__ r2p, int64_t S,
                                                     int64_t R, float* __restrict__ X,
                                                     double* __restrict__ rec, RankIndexPtrs ix = {},
                                                     int64_t pix_off = 0) {
  auto pix_of = [&](int32_t rho) -> uint32_t {
    if constexpr (PX) return (uint32_t)rho;
    else if constexpr (RI) return rank_pixel(ix, (uint32_t)rho) + (uint32_t)pix_off;
    else return r2p[rho];
  };
  extern __shared__ __attribute__((aligned(16))) float s_tile[];  // 256*F floats + stats scratch
  __shared__ int s_feat[64];
  __shared__ uint32_t s_pix[2][256];  // pixel of each row of this tile / the next one
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  for (int f = t; f < 64; f += 256) s_feat[f] = (GATHER && f < F) ? feat[f] : 0;
  const int nparts = 256 / F;
  const bool st_on = t < nparts * F;
  const int sf = st_on ? t % F : 0, spart = st_on ? t / F : 0;
  double n_acc = 0.0, m_acc = 0.0, q_acc = 0.0;
  float a_acc = 0.0f;
  // cooperative row loads: a wave instruction covers RPI rows x FP features
  const int FP = F <= 32 ? 32 : 64;
  const int RPI = 64 / FP;
  const int lf = lane % FP, lr = lane / FP;
  const int64_t lo = (int64_t)blockIdx.x * R;
  const int64_t hi = min(S, lo + R);
  __syncthreads();
  const int fcol = lf < F ? (GATHER ? s_feat[lf] : lf) : 0;
  // the sample -> pixel lookups (idx, then r2p: two dependent random reads)
  // of tile i+1 are issued before tile i's row loads and stored after them
  if (GATHER && lo < hi && t < (int)min((int64_t)kTile, hi - lo)) s_pix[0][t] = pix_of(idx[lo + t]);
  int buf = 0;
  for (int64_t r0 = lo; r0 < hi; r0 += kTile, buf ^= 1) {
    const int nrow = (int)min((int64_t)kTile, hi - r0);
    __syncthreads();
    const uint32_t* pix = s_pix[buf];
    const int64_t r1 = r0 + kTile;
    const bool nxt = GATHER && r1 < hi && t < (int)min((int64_t)kTile, hi - r1);
    const int32_t nidx = nxt ? idx[r1 + t] : 0;
    // wave wid loads rows [wid*64, wid*64+64) of the tile, RPI rows per instruction
    constexpr int kBatch = 16;
    uint32_t npix = 0;
    bool npix_issued = false;
    for (int i0 = 0; i0 < 64 / RPI; i0 += kBatch) {
      if (i0 == kBatch && nxt) {  // nidx has landed with the first batch of rows
        npix = pix_of(nidx);
        npix_issued = true;
      }
      float v[kBatch];
#pragma unroll
      for (int i = 0; i < kBatch; ++i) {
        const int row = min(wid * 64 + (i0 + i) * RPI + lr, nrow - 1);  // clamped: always valid
        v[i] = GATHER ? ld_stream(img + (int64_t)pix[row] * C + fcol) : X[(r0 + row) * F + fcol];
      }
#pragma unroll
      for (int i = 0; i < kBatch; ++i) {
        const int row = wid * 64 + (i0 + i) * RPI + lr;
        if (i0 + i < 64 / RPI && row < nrow && lf < F) s_tile[row * F + lf] = v[i];
      }
    }
    if (nxt) s_pix[buf ^ 1][t] = npix_issued ? npix : pix_of(nidx);
    __syncthreads();
    // coalesced write of the tile (rows contiguous in X)
    if (GATHER) {
      float* dst = X + r0 * F;
      const int ne = nrow * F;
      for (int q = t; q < ne; q += 256) dst[q] = s_tile[q];
    }
    // column statistics of this tile part
    if (st_on) {
      double s = 0.0, cnt = 0.0;
      for (int r = spart; r < nrow; r += nparts) {
        s += (double)s_tile[r * F + sf];
        cnt += 1.0;
        a_acc = fmaxf(a_acc, fabsf(s_tile[r * F + sf]));
      }
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
    s_st[4 * t + 0] = n_acc;
    s_st[4 * t + 1] = m_acc;
    s_st[4 * t + 2] = q_acc;
    s_st[4 * t + 3] = (double)a_acc;
  }
  __syncthreads();
  double* out = rec + (size_t)blockIdx.x * (1 + 3 * F);
  if (t < F) {
    double n = 0.0, m = 0.0, q = 0.0, a = 0.0;
    for (int part = 0; part < nparts; ++part) {
      const int u = part * F + t;
      chan_merge(n, m, q, s_st[4 * u], s_st[4 * u + 1], s_st[4 * u + 2]);
      a = fmax(a, s_st[4 * u + 3]);
    }
    if (t == 0) out[0] = n;
    out[1 + t] = m;
    out[1 + F + t] = q;
    out[1 + 2 * F + t] = a;
  }
}

// mw_col_stats_rows: gather_kernel's statistics over rows already in X (the
// fused blur sample epilogue wrote them) with the same block / tile / part
// partition and the same operation order, so the records are identical, but
// read straight from global memory into registers instead of through an
// LDS tile: at each of a part thread's rows the block's threads read nparts
// consecutive rows (nparts * F floats, coalesced), and both passes read the
// registers.  Without the 256 x F tile 4 blocks fit a CU at any F (the tile
// allowed 2 at F = 50).
__global__ void __launch_bounds__(256, 4) col_stats_rows_kernel(const float* __restrict__ X, int F,
                                                             int64_t S, int64_t R,
                                                             double* __restrict__ rec) {
  __shared__ double s_st[4 * 256];
  const int t = threadIdx.x;
  const int nparts = 256 / F;
  const bool st_on = t < nparts * F;
  const int sf = st_on ? t % F : 0, spart = st_on ? t / F : 0;
  double n_acc = 0.0, m_acc = 0.0, q_acc = 0.0;
  float a_acc = 0.0f;
  const int64_t lo = (int64_t)blockIdx.x * R, hi = min(S, lo + R);
  // a part thread's rows of one tile (spart, spart + nparts, ...: at most
  // 64 for F <= 64) are loaded together into registers, then both passes
  // run from them: one memory round trip per tile instead of one per batch
  constexpr int kRows = 64;
  if (st_on) {
    for (int64_t r0 = lo; r0 < hi; r0 += kTile) {
      const int nrow = (int)min((int64_t)kTile, hi - r0);
      // buffer loads: per-lane offset of the thread's first row, the row
      // steps as scalar offsets (no 64-bit address per load); past the
      // array's end they return 0 (unused: the passes skip rows >= nrow)
      const uint64_t nb = (uint64_t)(S - r0) * F * 4;
      const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
          const_cast<float*>(X + r0 * F), (short)0, (int)(uint32_t)(nb < 0xFFFFFFFFull ? nb : 0xFFFFFFFFull),
          0x00020000);
      const int voff = (spart * F + sf) * 4, step4 = nparts * F * 4;
      float v[kRows];
#pragma unroll
      for (int i = 0; i < kRows; ++i)
        v[i] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rx, voff, i * step4, 0));
      // this thread's rows in the tile (rows spart + i * nparts < nrow)
      int nmine = nrow > spart ? (nrow - spart + nparts - 1) / nparts : 0;
      double s = 0.0, cnt = 0.0;
#pragma unroll
      for (int i = 0; i < kRows; ++i)
        if (i < nmine) {
          s += (double)v[i];
          cnt += 1.0;
          a_acc = fmaxf(a_acc, fabsf(v[i]));
        }
      // (opaque to the compiler: pass 2 converts again instead of keeping 64
      // fp64 copies live across the division)
#pragma unroll
      for (int i = 0; i < kRows; ++i) asm volatile("" : "+v"(v[i]));
      asm volatile("" : "+v"(nmine));
      if (cnt > 0.0) {
        const double m = s / cnt;
        double q = 0.0;
#pragma unroll
        for (int i = 0; i < kRows; ++i)
          if (i < nmine) {
            const double d = (double)v[i] - m;
            q += d * d;
          }
        chan_merge(n_acc, m_acc, q_acc, cnt, m, q);
      }
    }
    s_st[4 * t + 0] = n_acc;
    s_st[4 * t + 1] = m_acc;
    s_st[4 * t + 2] = q_acc;
    s_st[4 * t + 3] = (double)a_acc;
  }
  __syncthreads();
  double* out = rec + (size_t)blockIdx.x * (1 + 3 * F);
  if (t < F) {
    double n = 0.0, m = 0.0, q = 0.0, a = 0.0;
    for (int part = 0; part < nparts; ++part) {
      const int u = part * F + t;
      chan_merge(n, m, q, s_st[4 * u], s_st[4 * u + 1], s_st[4 * u + 2]);
      a = fmax(a, s_st[4 * u + 3]);
    }
    if (t == 0) out[0] = n;
    out[1 + t] = m;
    out[1 + F + t] = q;
    out[1 + 2 * F + t] = a;
  }
}

// Merge per-block (n, mean, M2) records: n = sum n_b, mean = sum n_b m_b / n,
// M2 = sum [M2_b + n_b (m_b - mean)^2]  (fixed order; optional prior record).
// Fixed-order fold of the G per-block Chan records: 16 parts x 64 features
// (part p takes records p, p+16, ...), two passes (mean, then M2 about it),
// the 16 partials combined in part order — deterministic, and G/16 dependent
// adds per thread instead of G/4.
constexpr int kColParts = 16;
__global__ void __launch_bounds__(64 * kColParts) col_stats_kernel(const double* __restrict__ rec, int G,
                                                                   int F, double* __restrict__ st,
                                                                   int accumulate) {
  __shared__ double s_n[kColParts][64], s_s[kColParts][64], s_mean[64];
  const int f = threadIdx.x & 63, part = threadIdx.x >> 6;
  const int rl = 1 + 3 * F;
  double n = 0.0, sm = 0.0, q = 0.0;
  double n0 = 0.0, m0 = 0.0, q0 = 0.0;
  if (accumulate && f < F) { n0 = st[0]; m0 = st[1 + f]; q0 = st[1 + F + f]; }
  if (f < F)
    for (int b = part; b < G; b += kColParts) {
      const double nb = rec[(size_t)b * rl];
      n += nb;
      sm += nb * rec[(size_t)b * rl + 1 + f];
    }
  s_n[part][f] = n;
  s_s[part][f] = sm;
  __syncthreads();
  if (part == 0 && f < F) {
    double N = n0, SM = n0 * m0;
    for (int p2 = 0; p2 < kColParts; ++p2) { N += s_n[p2][f]; SM += s_s[p2][f]; }
    s_mean[f] = N > 0 ? SM / N : 0.0;
    s_n[0][f] = N;
  }
  __syncthreads();
  if (f < F) {
    const double mean = s_mean[f];
    for (int b = part; b < G; b += kColParts) {
      const double nb = rec[(size_t)b * rl];
      const double d = rec[(size_t)b * rl + 1 + f] - mean;
      q += rec[(size_t)b * rl + 1 + F + f] + nb * d * d;
    }
  }
  __syncthreads();
  s_s[part][f] = q;
  __syncthreads();
  if (part == 0 && f < F) {
    const double mean = s_mean[f];
    double Q = n0 > 0 ? q0 + n0 * (m0 - mean) * (m0 - mean) : 0.0;
    for (int p2 = 0; p2 < kColParts; ++p2) Q += s_s[p2][f];
    if (f == 0) st[0] = s_n[0][0];
    st[1 + f] = mean;
    st[1 + F + f] = Q;
  }
}

// column max |x| over the block records (record field 1 + 2F + f), maxed
// into out[f] when accumulating (a max: any order gives the same value)
__global__ void __launch_bounds__(64 * kColParts) col_absmax_rec_kernel(const double* __restrict__ rec, int G,
                                                                        int F, float* __restrict__ out,
                                                                        int accumulate) {
  __shared__ double s_a[kColParts][64];
  const int f = threadIdx.x & 63, part = threadIdx.x >> 6;
  const int rl = 1 + 3 * F;
  double a = 0.0;
  if (f < F)
    for (int b = part; b < G; b += kColParts) a = fmax(a, rec[(size_t)b * rl + 1 + 2 * F + f]);
  s_a[part][f] = a;
  __syncthreads();
  if (part == 0 && f < F) {
    for (int p2 = 1; p2 < kColParts; ++p2) a = fmax(a, s_a[p2][f]);
    const float v = (float)a;  // a max of floats: exact
    out[f] = accumulate ? fmaxf(out[f], v) : v;
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

// Rows [y_beg, y_end) of the slide: every value is a function of its slide
// pixel index alone (counter-based hash), so a band generated on its own is
// bit for bit the same rows of the whole slide (streamed synthetic slides,
// milwrm_amd.stream.SynthSource).  A block makes 256 consecutive pixels: the
// values go through LDS and leave as one contiguous HWC run.
constexpr int kSynthPx = 256;
__global__ void __launch_bounds__(kSynthPx) synth_kernel(int W, int C, int y_beg, int y_end,
                                                         const float* __restrict__ syx, int ns,
                                                         const float* __restrict__ prof, int nd, int shape_k,
                                                         int bg_rows, uint64_t seed, uint16_t* __restrict__ img,
                                                         uint8_t* __restrict__ mask) {
  extern __shared__ uint16_t s_px[];  // kSynthPx x C
  const int64_t n = (int64_t)(y_end - y_beg) * W;
  const int64_t p_base = (int64_t)y_beg * W;
  for (int64_t base = (int64_t)blockIdx.x * kSynthPx; base < n; base += (int64_t)gridDim.x * kSynthPx) {
    const int64_t pl = base + threadIdx.x;
    if (pl < n) {
      const int64_t p = p_base + pl;  // slide pixel
      const int y = (int)(p / W), x = (int)(p % W);
      float best = 3.4e38f;
      int dom = 0;
      for (int s = 0; s < ns; ++s) {
        const float dy = y - syx[2 * s], dx = x - syx[2 * s + 1];
        const float d = dy * dy + dx * dx;
        if (d < best) { best = d; dom = s % nd; }
      }
      const bool bg = y < bg_rows;
      if (mask) mask[pl] = bg ? 0 : 1;
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
        s_px[threadIdx.x * C + c] = (uint16_t)v;
      }
    }
    __syncthreads();
    const int nel = (int)(n - base < kSynthPx ? n - base : (int64_t)kSynthPx) * C;
    uint16_t* dst = img + base * C;
    for (int e = threadIdx.x; e < nel; e += kSynthPx) dst[e] = s_px[e];
    __syncthreads();
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
      hipLaunchKernelGGL(nz_stats_u16_kernel, dim3(p.G), dim3(256), 0, st,
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
  hipLaunchKernelGGL(nz_stats_reduce, dim3(C), dim3(256), 0, st, part, p.G, C, d_sum,
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
  return (radius > kBlurMaxR || C % 2 || C > 64) ? (size_t)H * W * C * sizeof(float) + 256 : 0;
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

size_t mw_rank_index_bytes(int64_t n_pix) { return rank_index_bytes(n_pix); }

int mw_mask_rank_index(const uint8_t* d_mask, int64_t n_pix, void* d_index, int64_t* d_count, void* d_ws,
                       void* stream) {
  MW_CHECK_ARG(d_mask && d_index && d_count && d_ws, "mw_mask_rank_index: null pointer");
  MW_CHECK_ARG(n_pix > 0 && n_pix < (int64_t)4294967295LL - 64, "mw_mask_rank_index: n_pix out of range");
  MW_CHECK_ARG(((uintptr_t)d_mask & 15) == 0, "mw_mask_rank_index: mask must be 16-byte aligned");
  hipStream_t st = as_stream(stream);
  const int nb = (int)((n_pix + kMaskChunk - 1) / kMaskChunk);
  uint32_t* cnt = reinterpret_cast<uint32_t*>(d_ws);
  hipLaunchKernelGGL(mask_count_kernel, dim3(nb), dim3(256), 0, st, d_mask, n_pix, cnt);
  MW_LAUNCH_CHECK();
  hipLaunchKernelGGL(mask_scan_kernel, dim3(1), dim3(1024), 0, st, cnt, nb, d_count);
  MW_LAUNCH_CHECK();
  char* b = reinterpret_cast<char*>(d_index);
  hipLaunchKernelGGL(rank_words_kernel, dim3(nb), dim3(256), 0, st, d_mask, n_pix, cnt, d_count,
                     reinterpret_cast<uint64_t*>(b), reinterpret_cast<uint32_t*>(b + rank_pre_off(n_pix)),
                     reinterpret_cast<uint32_t*>(b + rank_blk_off(n_pix)));
  MW_LAUNCH_CHECK();
  return MW_OK;
}

int mw_gather_rows_ri(const float* d_img, int C, const int32_t* d_feat, int F, const int32_t* d_idx,
                      const void* d_index, int64_t n_pix, int64_t pix_off, int64_t S, float* d_X, void* d_ws,
                      void* stream) {
  MW_CHECK_ARG(d_img && d_feat && d_idx && d_index && d_X && d_ws, "mw_gather_rows_ri: null pointer");
  MW_CHECK_ARG(S > 0 && F > 0 && F <= 64 && C > 0 && n_pix > 0 && pix_off >= 0,
               "mw_gather_rows_ri: bad shape S=%lld F=%d", (long long)S, F);
  hipStream_t st = as_stream(stream);
  const int G = stream_blocks(S);
  const int64_t R = rows_per_block(S);
  size_t lds = (size_t)kTile * F * sizeof(float);
  if (lds < 4 * 256 * sizeof(double)) lds = 4 * 256 * sizeof(double);
  hipLaunchKernelGGL((gather_kernel<true, true>), dim3(G), dim3(256), lds, st, d_img, C, d_feat, F, d_idx,
                     nullptr, S, R, d_X, reinterpret_cast<double*>(d_ws), rank_ptrs(d_index, n_pix), pix_off);
  MW_LAUNCH_CHECK();
  return MW_OK;
}

// draws -> pixels in place through the rank index (several independent
// lookups per lane in flight: the index sits in the on-die caches, so the
// pass is latency-bound, not HBM-bound)
__global__ void __launch_bounds__(256) rank_to_pixel_kernel(int32_t* __restrict__ idx, int64_t S,
                                                            RankIndexPtrs ix, int64_t pix_off) {
  constexpr int U = 4;
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t j0 = (int64_t)blockIdx.x * 256 + threadIdx.x; j0 < S; j0 += U * stride) {
    int32_t r[U];
#pragma unroll
    for (int u = 0; u < U; ++u) r[u] = j0 + u * stride < S ? idx[j0 + u * stride] : 0;
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (j0 + u * stride < S) idx[j0 + u * stride] = (int32_t)(rank_pixel(ix, (uint32_t)r[u]) + (uint32_t)pix_off);
  }
}

int mw_rank_to_pixel_ri(int32_t* d_idx, int64_t S, const void* d_index, int64_t n_pix, int64_t pix_off,
                        void* stream) {
  MW_CHECK_ARG(d_idx && d_index, "mw_rank_to_pixel_ri: null pointer");
  MW_CHECK_ARG(S >= 0 && n_pix > 0 && pix_off >= 0 && n_pix + pix_off <= 0x7fffffffll,
               "mw_rank_to_pixel_ri: bad sizes S=%lld n_pix=%lld", (long long)S, (long long)n_pix);
  if (S == 0) return MW_OK;
  const int grid = (int)std::min<int64_t>((S + 1023) / 1024, 8192);
  hipLaunchKernelGGL(rank_to_pixel_kernel, dim3(grid), dim3(256), 0, as_stream(stream), d_idx, S,
                     rank_ptrs(d_index, n_pix), pix_off);
  MW_LAUNCH_CHECK();
  return MW_OK;
}

int mw_gather_rows_px(const float* d_img, int C, const int32_t* d_feat, int F, const int32_t* d_pix, int64_t S,
                      float* d_X, void* d_ws, void* stream) {
  MW_CHECK_ARG(d_img && d_feat && d_pix && d_X && d_ws, "mw_gather_rows_px: null pointer");
  MW_CHECK_ARG(S > 0 && F > 0 && F <= 64 && C > 0, "mw_gather_rows_px: bad shape S=%lld F=%d",
               (long long)S, F);
  hipStream_t st = as_stream(stream);
  const int G = stream_blocks(S);
  const int64_t R = rows_per_block(S);
  size_t lds = (size_t)kTile * F * sizeof(float);
  if (lds < 4 * 256 * sizeof(double)) lds = 4 * 256 * sizeof(double);
  hipLaunchKernelGGL((gather_kernel<true, false, true>), dim3(G), dim3(256), lds, st, d_img, C, d_feat, F, d_pix,
                     nullptr, S, R, d_X, reinterpret_cast<double*>(d_ws), RankIndexPtrs{}, (int64_t)0);
  MW_LAUNCH_CHECK();
  return MW_OK;
}

size_t mw_gather_ws_bytes(int64_t S, int F) {
  return (size_t)stream_blocks(S) * (1 + 3 * (size_t)F) * sizeof(double) + 256;
}

int mw_gather_rows(const float* d_img, int C, const int32_t* d_feat, int F, const int32_t* d_idx,
                   const uint32_t* d_rank2pix, int64_t S, float* d_X, void* d_ws, void* stream) {
  MW_CHECK_ARG(d_img && d_feat && d_idx && d_rank2pix && d_X && d_ws, "mw_gather_rows: null pointer");
  MW_CHECK_ARG(S > 0 && F > 0 && F <= 64 && C > 0, "mw_gather_rows: bad shape S=%lld F=%d",
               (long long)S, F);
  hipStream_t st = as_stream(stream);
  const int G = stream_blocks(S);
  const int64_t R = rows_per_block(S);
  size_t lds = (size_t)kTile * F * sizeof(float);
  if (lds < 4 * 256 * sizeof(double)) lds = 4 * 256 * sizeof(double);
  hipLaunchKernelGGL((gather_kernel<true, false>), dim3(G), dim3(256), lds, st, d_img, C, d_feat, F, d_idx,
                     d_rank2pix, S, R, d_X, reinterpret_cast<double*>(d_ws), RankIndexPtrs{}, (int64_t)0);
  MW_LAUNCH_CHECK();
  return MW_OK;
}

int mw_col_stats_rows(const float* d_X, int64_t S, int F, void* d_ws, void* stream) {
  MW_CHECK_ARG(d_X && d_ws, "mw_col_stats_rows: null pointer");
  MW_CHECK_ARG(S > 0 && F > 0 && F <= 64, "mw_col_stats_rows: bad shape S=%lld F=%d", (long long)S, F);
  hipStream_t st = as_stream(stream);
  hipLaunchKernelGGL(col_stats_rows_kernel, dim3(stream_blocks(S)), dim3(256), 0, st, d_X, F, S,
                     rows_per_block(S), reinterpret_cast<double*>(d_ws));
  MW_LAUNCH_CHECK();
  return MW_OK;
}

// ------------------------------------------------- fused blur + subsample
// Per sampled pixel p its first two sample slots (idx draws with replacement):
// slots[p] = (j0, j1), -1 where absent; a third or later draw of p goes to the
// overflow list ovf[1 + i] (ovf[0] = count; Poisson(0.2): ~0.6 % of the
// sampled pixels).  The blur's sample epilogue writes rows j0 and j1 of X
// (both read from the side data, no dependent load); mw_sample_overflow then
// copies row j0 to the overflow slots.  Which draw lands in which place
// depends on the atomic order, the rows written do not.
extern "C++" {
template <bool RI = false>
__global__ void __launch_bounds__(256) sample_map_kernel(const int32_t* __restrict__ idx,
                                                         const uint32_t* __restrict__ r2p, int64_t S,
                                                         int32_t* __restrict__ slots,
                                                         int32_t* __restrict__ ovf, RankIndexPtrs ix = {},
                                                         int64_t pix_off = 0) {
  for (int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x; j < S; j += (int64_t)gridDim.x * 256) {
    uint32_t p;
    if constexpr (RI) p = rank_pixel(ix, (uint32_t)idx[j]) + (uint32_t)pix_off;
    else p = r2p[idx[j]];
    if (atomicCAS(slots + 2 * (int64_t)p, -1, (int32_t)j) == -1) continue;
    if (atomicCAS(slots + 2 * (int64_t)p + 1, -1, (int32_t)j) == -1) continue;
    ovf[1 + atomicAdd(ovf, 1)] = (int32_t)j;
  }
}
template <bool RI = false>
__global__ void __launch_bounds__(256) sample_overflow_kernel(const int32_t* __restrict__ idx,
                                                              const uint32_t* __restrict__ r2p,
                                                              const int32_t* __restrict__ slots,
                                                              const int32_t* __restrict__ ovf, int F,
                                                              float* __restrict__ X, RankIndexPtrs ix = {},
                                                              int64_t pix_off = 0) {
  const int n = ovf[0];
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    const int32_t j = ovf[1 + i];
    uint32_t p;
    if constexpr (RI) p = rank_pixel(ix, (uint32_t)idx[j]) + (uint32_t)pix_off;
    else p = r2p[idx[j]];
    const int32_t h = slots[2 * (int64_t)p];
    const float* src = X + (int64_t)h * F;
    float* dst = X + (int64_t)j * F;
    for (int f = 0; f < F; ++f) dst[f] = src[f];
  }
}

}  // extern "C++"

// The sample epilogue as a pass of its own over a materialised fp32 band of
// n pixels (slide pixels pix_off ..): X[j] = band[p - pix_off, feat] for both
// table slots j of every sampled pixel p.  The streamed subsample of a slide
// whose shape the fused kernel does not take (odd C, C > 64, radius > 8).
__global__ void __launch_bounds__(256) slot_gather_kernel(const float* __restrict__ band, int C, int64_t n,
                                                          int64_t pix_off, const int32_t* __restrict__ slots,
                                                          int64_t S, const int32_t* __restrict__ feat, int F,
                                                          float* __restrict__ X) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int2 sl = reinterpret_cast<const int2*>(slots)[pix_off + i];
    if ((uint64_t)(uint32_t)sl.x >= (uint64_t)S) continue;
    const bool two = (uint64_t)(uint32_t)sl.y < (uint64_t)S;
    const float* src = band + i * C;
    float* d0 = X + (int64_t)sl.x * F;
    float* d1 = X + (int64_t)(two ? sl.y : sl.x) * F;
    for (int f = 0; f < F; ++f) {
      const float v = src[feat[f]];
      d0[f] = v;
      d1[f] = v;
    }
  }
}

size_t mw_sample_slot_elems(int64_t n_pix) { return 2 * ((size_t)n_pix + 128); }

int mw_slot_gather(const float* d_band, int C, int64_t n_pix, int64_t pix_off, const int32_t* d_slots,
                   int64_t S, const int32_t* d_feat, int F, float* d_X, void* stream) {
  MW_CHECK_ARG(d_band && d_slots && d_feat && d_X, "mw_slot_gather: null pointer");
  MW_CHECK_ARG(C > 0 && F > 0 && n_pix >= 0 && pix_off >= 0 && S > 0 && S < 0x7fffffffll,
               "mw_slot_gather: bad args");
  if (n_pix == 0) return MW_OK;
  const int grid = (int)std::min<int64_t>((n_pix + 255) / 256, 16384);
  hipLaunchKernelGGL(slot_gather_kernel, dim3(grid), dim3(256), 0, as_stream(stream), d_band, C, n_pix, pix_off,
                     d_slots, S, d_feat, F, d_X);
  MW_LAUNCH_CHECK();
  return MW_OK;
}

int mw_sample_map(const int32_t* d_idx, const uint32_t* d_rank2pix, int64_t S, int64_t n_pix,
                  int32_t* d_slots, int32_t* d_ovf, void* stream) {
  MW_CHECK_ARG(d_idx && d_rank2pix && d_slots && d_ovf, "mw_sample_map: null pointer");
  MW_CHECK_ARG(S > 0 && S < 0x7fffffffll && n_pix > 0, "mw_sample_map: bad sizes S=%lld n_pix=%lld",
               (long long)S, (long long)n_pix);
  hipStream_t st = as_stream(stream);
  MW_HIP(hipMemsetAsync(d_slots, 0xff, mw_sample_slot_elems(n_pix) * sizeof(int32_t), st));
  MW_HIP(hipMemsetAsync(d_ovf, 0, sizeof(int32_t), st));
  const int grid = (int)std::min<int64_t>((S + 255) / 256, 8192);
  hipLaunchKernelGGL(sample_map_kernel<false>, dim3(grid), dim3(256), 0, st, d_idx, d_rank2pix, S, d_slots, d_ovf,
                     RankIndexPtrs{}, (int64_t)0);
  MW_LAUNCH_CHECK();
  return MW_OK;
}

int mw_sample_map_ri(const int32_t* d_idx, const void* d_index, int64_t n_index, int64_t pix_off, int64_t S,
                     int64_t n_pix, int32_t* d_slots, int32_t* d_ovf, void* stream) {
  MW_CHECK_ARG(d_idx && d_index && d_slots && d_ovf, "mw_sample_map_ri: null pointer");
  MW_CHECK_ARG(S > 0 && S < 0x7fffffffll && n_pix > 0 && n_index > 0 && pix_off >= 0,
               "mw_sample_map_ri: bad sizes S=%lld n_pix=%lld", (long long)S, (long long)n_pix);
  hipStream_t st = as_stream(stream);
  MW_HIP(hipMemsetAsync(d_slots, 0xff, mw_sample_slot_elems(n_pix) * sizeof(int32_t), st));
  MW_HIP(hipMemsetAsync(d_ovf, 0, sizeof(int32_t), st));
  const int grid = (int)std::min<int64_t>((S + 255) / 256, 8192);
  hipLaunchKernelGGL(sample_map_kernel<true>, dim3(grid), dim3(256), 0, st, d_idx, nullptr, S, d_slots, d_ovf,
                     rank_ptrs(d_index, n_index), pix_off);
  MW_LAUNCH_CHECK();
  return MW_OK;
}

int mw_sample_overflow_ri(const int32_t* d_idx, const void* d_index, int64_t n_index, int64_t pix_off,
                          const int32_t* d_slots, const int32_t* d_ovf, int64_t S, int F, float* d_X,
                          void* stream) {
  MW_CHECK_ARG(d_idx && d_index && d_slots && d_ovf && d_X && S > 0 && F > 0 && n_index > 0,
               "mw_sample_overflow_ri: bad args");
  hipStream_t st = as_stream(stream);
  const int grid = (int)std::min<int64_t>((S / 64 + 255) / 256 + 1, 1024);
  hipLaunchKernelGGL(sample_overflow_kernel<true>, dim3(grid), dim3(256), 0, st, d_idx, nullptr, d_slots, d_ovf,
                     F, d_X, rank_ptrs(d_index, n_index), pix_off);
  MW_LAUNCH_CHECK();
  return MW_OK;
}

int mw_sample_overflow(const int32_t* d_idx, const uint32_t* d_rank2pix, const int32_t* d_slots,
                       const int32_t* d_ovf, int64_t S, int F, float* d_X, void* stream) {
  MW_CHECK_ARG(d_idx && d_rank2pix && d_slots && d_ovf && d_X && S > 0 && F > 0,
               "mw_sample_overflow: bad args");
  hipStream_t st = as_stream(stream);
  const int grid = (int)std::min<int64_t>((S / 64 + 255) / 256 + 1, 1024);
  hipLaunchKernelGGL(sample_overflow_kernel<false>, dim3(grid), dim3(256), 0, st, d_idx, d_rank2pix, d_slots,
                     d_ovf, F, d_X, RankIndexPtrs{}, (int64_t)0);
  MW_LAUNCH_CHECK();
  return MW_OK;
}

static int blur_taps_from_host(const float* h_w, int radius, BlurTaps& taps) {
  if (radius < 0 || radius > kMaxRadius) return MW_EUNSUPPORTED;
  memset(&taps, 0, sizeof(taps));
  for (int j = 0; j <= 2 * radius; ++j) taps.w[j] = h_w[j];
  return MW_OK;
}

static int blur_epi_dispatch(const void* d_img, int dtype, int H, int W, int C, const float* d_inv_mean,
                             float pseudoval, const float* h_w, int radius, const BlurEpi& ep, int epi,
                             void* stream, const char* who) {
  BlurTaps taps;
  if (blur_taps_from_host(h_w, radius, taps) != MW_OK) {
    set_error("%s: radius %d unsupported", who, radius);
    return MW_EUNSUPPORTED;
  }
  hipStream_t st = as_stream(stream);
  int rc;
  switch (dtype) {
    case MW_U8: rc = launch_blur_epi<uint8_t>((const uint8_t*)d_img, H, W, C, d_inv_mean, pseudoval, taps, radius, ep, epi, st); break;
    case MW_U16: rc = launch_blur_epi<uint16_t>((const uint16_t*)d_img, H, W, C, d_inv_mean, pseudoval, taps, radius, ep, epi, st); break;
    case MW_F32: rc = launch_blur_epi<float>((const float*)d_img, H, W, C, d_inv_mean, pseudoval, taps, radius, ep, epi, st); break;
    default: set_error("%s: bad dtype %d", who, dtype); return MW_EINVAL;
  }
  if (rc == MW_EUNSUPPORTED)
    set_error("%s: no fused kernel for dtype %d C=%d W=%d radius %d (materialise the blur instead)", who,
              dtype, C, W, radius);
  return rc;
}

int mw_blur_sample_rows(const void* d_img, int dtype, int H, int W, int C, int64_t row_off, int r0, int r1,
                        const float* d_inv_mean, float pseudoval, const float* h_w, int radius,
                        const int32_t* d_slots, int64_t S, const int32_t* d_feat, int F, float* d_X,
                        void* stream) {
  MW_CHECK_ARG(d_img && d_inv_mean && h_w && d_slots && d_feat && d_X, "mw_blur_sample: null pointer");
  MW_CHECK_ARG(H > 0 && W > 0 && C > 0 && F > 0 && S > 0 && S < 0x7fffffffll,
               "mw_blur_sample: bad shape");
  MW_CHECK_ARG(0 <= r0 && r0 <= r1 && r1 <= H && row_off >= 0, "mw_blur_sample: bad row window [%d, %d) of %d rows",
               r0, r1, H);
  BlurEpi ep{};
  ep.slots = d_slots;
  ep.S = S;
  ep.X = d_X;
  ep.F = F;
  ep.feat = d_feat;
  ep.row_off = row_off;
  ep.r0 = r0;
  ep.r1 = r1;
  return blur_epi_dispatch(d_img, dtype, H, W, C, d_inv_mean, pseudoval, h_w, radius, ep, kEpiSample,
                           stream, "mw_blur_sample");
}

int mw_blur_sample(const void* d_img, int dtype, int H, int W, int C, const float* d_inv_mean,
                   float pseudoval, const float* h_w, int radius, const int32_t* d_slots, int64_t S,
                   const int32_t* d_feat, int F, float* d_X, void* stream) {
  return mw_blur_sample_rows(d_img, dtype, H, W, C, 0, 0, H, d_inv_mean, pseudoval, h_w, radius, d_slots, S,
                             d_feat, F, d_X, stream);
}

int mw_blur_assign_rows(const void* d_img, int dtype, int H, int W, int C, int64_t row_off, int r0, int r1,
                        const float* d_inv_mean, float pseudoval, const float* h_w, int radius,
                        const float* d_a, const float* d_b, const float* d_centers, int k,
                        const uint8_t* d_mask, int8_t* d_label, float* d_conf, void* stream) {
  MW_CHECK_ARG(d_img && d_inv_mean && h_w && d_a && d_b && d_centers && d_mask && d_label && d_conf,
               "mw_blur_assign_conf: null pointer");
  MW_CHECK_ARG(H > 0 && W > 0 && C > 0 && k >= 1, "mw_blur_assign_conf: bad shape");
  MW_CHECK_ARG(0 <= r0 && r0 <= r1 && r1 <= H && row_off >= 0,
               "mw_blur_assign_conf: bad row window [%d, %d) of %d rows", r0, r1, H);
  BlurEpi ep{};
  ep.mask = d_mask;
  ep.lab = d_label;
  ep.conf = d_conf;
  ep.a = d_a;
  ep.b = d_b;
  ep.centers = d_centers;
  ep.k = k;
  ep.row_off = row_off;
  ep.r0 = r0;
  ep.r1 = r1;
  return blur_epi_dispatch(d_img, dtype, H, W, C, d_inv_mean, pseudoval, h_w, radius, ep, kEpiAssign,
                           stream, "mw_blur_assign_conf");
}

int mw_blur_assign_conf(const void* d_img, int dtype, int H, int W, int C, const float* d_inv_mean,
                        float pseudoval, const float* h_w, int radius, const float* d_a,
                        const float* d_b, const float* d_centers, int k, const uint8_t* d_mask,
                        int8_t* d_label, float* d_conf, void* stream) {
  return mw_blur_assign_rows(d_img, dtype, H, W, C, 0, 0, H, d_inv_mean, pseudoval, h_w, radius, d_a, d_b,
                             d_centers, k, d_mask, d_label, d_conf, stream);
}

int mw_col_stats_finalize(const void* d_ws, int64_t S, int F, double* d_stats, int accumulate,
                          void* stream) {
  MW_CHECK_ARG(d_ws && d_stats && F > 0 && F <= 64, "mw_col_stats_finalize: bad args (F <= 64)");
  hipLaunchKernelGGL(col_stats_kernel, dim3(1), dim3(64 * kColParts), 0, as_stream(stream),
                     reinterpret_cast<const double*>(d_ws), stream_blocks(S), F, d_stats, accumulate);
  MW_LAUNCH_CHECK();
  return MW_OK;
}

int mw_col_stats_absmax(const void* d_ws, int64_t S, int F, float* d_out, int accumulate, void* stream) {
  MW_CHECK_ARG(d_ws && d_out && S > 0 && F > 0 && F <= 64, "mw_col_stats_absmax: bad args (F <= 64)");
  hipLaunchKernelGGL(col_absmax_rec_kernel, dim3(1), dim3(64 * kColParts), 0, as_stream(stream),
                     reinterpret_cast<const double*>(d_ws), stream_blocks(S), F, d_out, accumulate);
  MW_LAUNCH_CHECK();
  return MW_OK;
}

int mw_synth_rows(int H, int W, int C, int y0, int y1, const float* d_seed_yx, int n_seeds,
                  const float* d_profiles, int n_domains, int shape_k, int bg_rows, uint64_t seed,
                  uint16_t* d_img, uint8_t* d_mask, void* stream) {
  MW_CHECK_ARG(d_seed_yx && d_profiles && d_img, "mw_synth_rows: null pointer");
  MW_CHECK_ARG(H > 0 && W > 0 && C > 0 && C <= 128 && n_seeds > 0 && n_domains > 0 && shape_k > 0,
               "mw_synth_rows: bad args (C <= 128)");
  MW_CHECK_ARG(0 <= y0 && y0 <= y1 && y1 <= H, "mw_synth_rows: rows [%d, %d) of %d", y0, y1, H);
  const int64_t n = (int64_t)(y1 - y0) * W;
  if (n == 0) return MW_OK;
  const int grid = (int)std::min<int64_t>((n + kSynthPx - 1) / kSynthPx, 65536);
  hipLaunchKernelGGL(synth_kernel, dim3(grid), dim3(kSynthPx), (size_t)kSynthPx * C * sizeof(uint16_t),
                     as_stream(stream), W, C, y0, y1, d_seed_yx, n_seeds, d_profiles, n_domains, shape_k,
                     bg_rows, seed, d_img, d_mask);
  MW_LAUNCH_CHECK();
  return MW_OK;
}

int mw_synth_slide(int H, int W, int C, const float* d_seed_yx, int n_seeds, const float* d_profiles,
                   int n_domains, int shape_k, int bg_rows, uint64_t seed, uint16_t* d_img,
                   uint8_t* d_mask, void* stream) {
  MW_CHECK_ARG(d_mask, "mw_synth_slide: null pointer");
  return mw_synth_rows(H, W, C, 0, H, d_seed_yx, n_seeds, d_profiles, n_domains, shape_k, bg_rows, seed,
                       d_img, d_mask, stream);
}

}  // extern "C"
