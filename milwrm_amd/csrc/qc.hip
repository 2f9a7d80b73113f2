// Clustering QC statistics: per-domain squared error against the centroids and
// the whole-slide scaled sums, in one streaming pass over an HWC fp32 slide.
//
// Serves `estimate_percentage_variance_mxif` (MILWRM.py:280-333) and
// `estimate_mse_mxif` (MILWRM.py:453-515): both scale the feature channels
// with the StandardScaler (x' = x*a + b, a = 1/scale, b = -mean/scale), then
//   dc   = sum over pixels with tissue_ID == d of (x'_f - c_df)^2   (per d, f)
//   dm   = sum over ALL pixels of (x'_f - mean_f(x'))^2             (per f)
// dm is recovered on the host from the per-feature sums of y = x' - p and y^2
// about a pivot p_f (the shifted-data variance: with p near the mean, e.g. a
// pixel's own value, a near-constant feature loses no digits to cancellation).
// Masked-out pixels (tissue_ID NaN → label -1 here) add to dm only, as in the
// reference (`tissue_ID == i` is false for NaN).  Domains d0 .. d0+k-1 per
// launch (label l counts as domain l - d0): more domains take more launches.
//
// Exact sums: every fp64 term (the squared error, y, y^2) is rounded to a
// per-feature two-level fixed point, q = rint(v * 2^e) with |q| <= 2^38 (the
// host derives e from the column max |x| of the slide, its scaler and the
// centers) plus the residual's own 38 bits, r = rint((v * 2^e - q) * 2^38), and
// both are summed as int64: a term far below the column bound (the squared
// error of a domain packed around its center) keeps ~2^-76 of the bound, not
// 2^-38 — fp64-grade relative accuracy.  Integer sums do not depend on order, so the
// statistics are the same bits for any split of the pixels: a slide blurred
// band by band into a reused buffer (the deferred-blur mode, no full fp32
// copy) gives exactly the materialised slide's numbers, and so would pixels
// sharded over GPUs.  Per-block results leave as pairs of integer-valued fp64
// limbs (hi = floor(v / 2^32), lo = v - hi * 2^32) that the fixed-order fold
// and any number of band launches add exactly.
//
// Layout: a block of 256 threads is split into floor(256/F) groups of F lanes;
// lane f of a group owns feature f, so a wave reads whole pixels (F contiguous
// floats for identity features) and every lane keeps its own per-domain
// column of int64 accumulators in LDS (no atomics, no bank conflicts);
// sixteen pixels' loads are issued before their updates (kQcUnroll = 16: 8 ->
// 16 took a 40k^2 x 50 slide's QC sums from 202 to 171 ms, 32 measured the
// same).  Per-block partials go to a workspace and a second kernel folds them
// in a fixed order.  Algorithmic bytes n_pix * (C*4 + 1); it runs at ~2 TB/s,
// bound by the three fixed-point conversions and the LDS read-modify-write of
// every element, not by HBM.
#include "common.h"

namespace mw {

constexpr int kQcThreads = 256;
constexpr int kQcMaxK = 20;  // LDS <= 2*20*256*8 + 4*256*8 + 20*256*4 (F = 1) = 108 KiB
constexpr int kQcMaxBlocks = 2048;
constexpr int kQcUnroll = 16;

// rint(s) as a double and as an int64 for |s| < 2^51: s + 1.5 2^52 lands in
// [2^52, 2^53), where the ulp is 1, so the add rounds s to the nearest
// integer (ties to even, as rint) and the low mantissa bits are that integer
// (offset by the constant's): two VALU ops instead of rint plus the
// multi-instruction fp64 -> int64 conversion, and the same values
__device__ __forceinline__ long long qc_rint64(double s, double& h) {
  constexpr double kMagic = 6755399441055744.0;  // 1.5 * 2^52
  const double t = s + kMagic;
  h = t - kMagic;
  return __double_as_longlong(t) - __double_as_longlong(kMagic);
}

// two-level fixed point of v at exponent e: hi += rint(v 2^e), lo += rint(residual 2^38)
__device__ __forceinline__ void qc_fix2(double v, int e, long long& hi, long long& lo) {
  const double s = ldexp(v, e);
  double h, r;
  hi += qc_rint64(s, h);
  lo += qc_rint64(ldexp(s - h, 38), r);  // s - h exact (|s| < 2^39), |(s - h) 2^38| <= 2^37
}

__device__ __forceinline__ void qc_limbs(long long v, double& hi, double& lo) {
  const long long h = v >> 32;  // arithmetic shift: floor
  hi = (double)h;
  lo = (double)(v - h * (1LL << 32));
}

template <typename TI>
__global__ __launch_bounds__(kQcThreads) void domain_sse_kernel(
    const TI* __restrict__ img, int C, const int32_t* __restrict__ feat, int F,
    const double* __restrict__ a, const double* __restrict__ b, const double* __restrict__ pivot,
    const double* __restrict__ centers, const int32_t* __restrict__ qe, int k, int d0,
    const int8_t* __restrict__ label, int64_t n_pix, int M, double* __restrict__ part) {
  extern __shared__ long long lds[];
  long long* sse = lds;                                        // [2][k][256] (hi, lo)
  long long* sacc = sse + 2 * (size_t)k * kQcThreads;          // [4][256]: s1 hi, lo, s2 hi, lo
  uint32_t* cnt = reinterpret_cast<uint32_t*>(sacc + 4 * kQcThreads);  // [k][groups]
  const size_t KL = (size_t)k * kQcThreads;                    // lo offset
  const int t = threadIdx.x;
  const int groups = kQcThreads / F;
  const int g = t / F, f = t - g * F;
  for (int d = 0; d < 2 * k; ++d) sse[d * kQcThreads + t] = 0;
  for (int i = t; i < k * groups; i += kQcThreads) cnt[i] = 0u;
  __syncthreads();
  long long s1 = 0, s1l = 0, s2 = 0, s2l = 0;
  if (g < groups) {
    const int ch = feat[f];
    const double af = a[f], bf = b[f], pf = pivot[f];
    const int es = qe[f], e1 = qe[F + f], e2 = qe[2 * F + f];
    const int64_t step = (int64_t)gridDim.x * groups;
    auto add = [&](TI v, int l) {
      const double x = (double)v * af + bf;
      const double y = x - pf;
      qc_fix2(y, e1, s1, s1l);
      qc_fix2(y * y, e2, s2, s2l);
      l -= d0;
      if (l >= 0 && l < k) {
        const double dd = x - centers[l * F + f];
        long long h = 0, lo = 0;
        qc_fix2(dd * dd, es, h, lo);
        sse[l * kQcThreads + t] += h;
        sse[KL + l * kQcThreads + t] += lo;
        if (f == 0) cnt[l * groups + g] += 1u;
      }
    };
    int64_t p = (int64_t)blockIdx.x * groups + g;
    // kQcUnroll pixels' loads in flight before their (LDS read-modify-write) updates
    for (; p + (kQcUnroll - 1) * step < n_pix; p += kQcUnroll * step) {
      TI v[kQcUnroll];
      int l[kQcUnroll];
#pragma unroll
      for (int u = 0; u < kQcUnroll; ++u) {
        v[u] = img[(p + u * step) * C + ch];
        l[u] = label[p + u * step];
      }
#pragma unroll
      for (int u = 0; u < kQcUnroll; ++u) add(v[u], l[u]);
    }
    for (; p < n_pix; p += step) add(img[p * C + ch], label[p]);
  }
  sacc[t] = s1;
  sacc[kQcThreads + t] = s1l;
  sacc[2 * kQcThreads + t] = s2;
  sacc[3 * kQcThreads + t] = s2l;
  __syncthreads();
  // fold the groups (int64, exact) and emit limbs: quantities
  // [sse k*F | sum F | sumsq F], each level (hi sums, then lo sums) as
  // (upper, lower) 32-bit limbs, then count k:
  //   [L0 upper NQ | L0 lower NQ | L1 upper NQ | L1 lower NQ | count k]
  const int NQ = k * F + 2 * F;
  for (int e = t; e < 2 * NQ + k; e += kQcThreads) {
    if (e < 2 * NQ) {
      const int lv = e >= NQ, qi = e - lv * NQ;
      long long r = 0;
      if (qi < k * F) {
        const int d = qi / F, ff = qi - d * F;
        for (int gg = 0; gg < groups; ++gg) r += sse[lv * KL + d * kQcThreads + gg * F + ff];
      } else {
        const int which = qi < k * F + F ? 0 : 1, ff = qi - k * F - which * F;
        const long long* sa = sacc + (2 * which + lv) * kQcThreads;
        for (int gg = 0; gg < groups; ++gg) r += sa[gg * F + ff];
      }
      double hi, lo;
      qc_limbs(r, hi, lo);
      part[(size_t)blockIdx.x * M + 2 * lv * NQ + qi] = hi;
      part[(size_t)blockIdx.x * M + (2 * lv + 1) * NQ + qi] = lo;
    } else {
      const int d = e - 2 * NQ;
      double r = 0.0;
      for (int gg = 0; gg < groups; ++gg) r += (double)cnt[d * groups + gg];
      part[(size_t)blockIdx.x * M + 4 * NQ + d] = r;
    }
  }
}

// One workgroup per output element: lane i sums blocks i, i+256, ... in order,
// then a fixed-order block tree (integer-valued limbs below 2^53: exact).
// accumulate: add to out (band after band) instead of overwriting it.
__global__ __launch_bounds__(256) void domain_sse_reduce(const double* __restrict__ part, int G,
                                                         int M, int accumulate, double* __restrict__ out) {
  __shared__ double scratch[256 / kWave];
  const int e = blockIdx.x;
  double r = 0.0;
  for (int i = threadIdx.x; i < G; i += 256) r += part[(size_t)i * M + e];
  r = block_sum(r, scratch);
  if (threadIdx.x == 0) out[e] = accumulate ? out[e] + r : r;
}

static int qc_blocks(int64_t n_pix, int F) {
  const int groups = kQcThreads / F;
  const int64_t want = (n_pix + (int64_t)groups * 64 - 1) / ((int64_t)groups * 64);
  return (int)std::max<int64_t>(1, std::min<int64_t>(want, kQcMaxBlocks));
}

}  // namespace mw

using namespace mw;

extern "C" {

int mw_domain_sse_out_len(int k, int F) { return 4 * (k * F + 2 * F) + k; }

size_t mw_domain_sse_ws_bytes(int64_t n_pix, int k, int F) {
  if (n_pix <= 0 || k <= 0 || F <= 0 || F > kQcThreads) return 0;
  return (size_t)qc_blocks(n_pix, F) * mw_domain_sse_out_len(k, F) * sizeof(double);
}

// the int64 sums are exact while a block's terms (each <= 2^38) stay below 2^62
static int64_t qc_pixels_per_block(int64_t n_pix, int F) {
  const int64_t G = qc_blocks(n_pix, F);
  return (n_pix + G - 1) / G;
}

}  // extern "C"

template <typename TI>
static int domain_sse_launch(const TI* d_img, int C, const int32_t* d_feat, int F, const double* d_a,
                             const double* d_b, const double* d_pivot, const double* d_centers,
                             const int32_t* d_qexp, int k, int d0, const int8_t* d_label, int64_t n_pix,
                             double* d_out, int accumulate, void* d_ws, void* stream) {
  MW_CHECK_ARG(d_img && d_feat && d_a && d_b && d_pivot && d_centers && d_qexp && d_label && d_out && d_ws,
               "mw_domain_sse: null pointer");
  MW_CHECK_ARG(n_pix > 0 && C > 0 && F > 0 && F <= kQcThreads && k >= 1 && k <= kQcMaxK && d0 >= 0,
               "mw_domain_sse: bad shape n_pix=%lld C=%d F=%d k=%d d0=%d (F <= 256, k <= 20 per launch)",
               (long long)n_pix, C, F, k, d0);
  MW_CHECK_ARG(qc_pixels_per_block(n_pix, F) <= (1LL << 24),
               "mw_domain_sse: %lld pixels per launch exceed the exact int64 sums (split the slide)",
               (long long)n_pix);
  hipStream_t st = as_stream(stream);
  const int G = qc_blocks(n_pix, F);
  const int M = mw_domain_sse_out_len(k, F);
  const size_t lds = 2 * (size_t)k * kQcThreads * sizeof(long long) + 4 * kQcThreads * sizeof(long long) +
                     (size_t)k * (kQcThreads / F) * sizeof(uint32_t);
  double* part = reinterpret_cast<double*>(d_ws);
  hipLaunchKernelGGL(domain_sse_kernel<TI>, dim3(G), dim3(kQcThreads), lds, st, d_img, C, d_feat, F,
                     d_a, d_b, d_pivot, d_centers, d_qexp, k, d0, d_label, n_pix, M, part);
  MW_LAUNCH_CHECK();
  hipLaunchKernelGGL(domain_sse_reduce, dim3(M), dim3(256), 0, st, part, G, M, accumulate, d_out);
  MW_LAUNCH_CHECK();
  return MW_OK;
}

extern "C" {

int mw_domain_sse(const float* d_img, int C, const int32_t* d_feat, int F, const double* d_a,
                  const double* d_b, const double* d_pivot, const double* d_centers,
                  const int32_t* d_qexp, int k, int d0, const int8_t* d_label, int64_t n_pix,
                  double* d_out, int accumulate, void* d_ws, void* stream) {
  return domain_sse_launch<float>(d_img, C, d_feat, F, d_a, d_b, d_pivot, d_centers, d_qexp, k, d0, d_label,
                                  n_pix, d_out, accumulate, d_ws, stream);
}

int mw_domain_sse_f64(const double* d_rows, int C, const int32_t* d_feat, int F, const double* d_a,
                      const double* d_b, const double* d_pivot, const double* d_centers,
                      const int32_t* d_qexp, int k, int d0, const int8_t* d_label, int64_t n_pix,
                      double* d_out, int accumulate, void* d_ws, void* stream) {
  return domain_sse_launch<double>(d_rows, C, d_feat, F, d_a, d_b, d_pivot, d_centers, d_qexp, k, d0, d_label,
                                   n_pix, d_out, accumulate, d_ws, stream);
}

}  // extern "C"

// ---- ST feature blur: neighbour mean over a CSR spatial graph ----------------
// blur_features_st (ST.py:25-77): for spot i the pandas mean (NaN skipped) of
// its features over [nonzero columns of row i] + [i], summed in that order.
// One thread per (spot, feature); spots ~1e3-1e5, degree ~6: launch-bound.
namespace mw {
__global__ __launch_bounds__(256) void neighbor_mean_kernel(const int64_t* __restrict__ indptr,
                                                            const int32_t* __restrict__ indices,
                                                            int64_t n, const double* __restrict__ X,
                                                            int F, double* __restrict__ out) {
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= n * F) return;
  const int64_t i = q / F;
  const int f = (int)(q - i * F);
  double s = 0.0;
  int64_t c = 0;
  for (int64_t e = indptr[i]; e < indptr[i + 1]; ++e) {
    const double v = X[(int64_t)indices[e] * F + f];
    if (v == v) { s += v; ++c; }
  }
  const double v = X[i * F + f];
  if (v == v) { s += v; ++c; }
  out[q] = c > 0 ? s / (double)c : __builtin_nan("");
}
}  // namespace mw

extern "C" int mw_neighbor_mean(const int64_t* d_indptr, const int32_t* d_indices, int64_t n,
                                const double* d_X, int F, double* d_out, void* stream) {
  MW_CHECK_ARG(d_indptr && d_indices && d_X && d_out && n > 0 && F > 0, "mw_neighbor_mean: bad arguments");
  const int64_t total = n * (int64_t)F;
  hipLaunchKernelGGL(mw::neighbor_mean_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                     mw::as_stream(stream), d_indptr, d_indices, n, d_X, F, d_out);
  MW_LAUNCH_CHECK();
  return MW_OK;
}
