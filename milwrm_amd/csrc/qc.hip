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
// Layout: a block of 256 threads is split into floor(256/F) groups of F lanes;
// lane f of a group owns feature f, so a wave reads whole pixels (F contiguous
// floats for identity features) and every lane keeps its own per-domain
// column of fp64 accumulators in LDS (no atomics, no bank conflicts); eight
// pixels' loads are issued before their updates (kQcUnroll = 8).  Per-block partials go to a
// workspace and a second kernel folds them in a fixed order (deterministic).  HBM-bound: n_pix * (C*4 + 1) bytes.
#include "common.h"

namespace mw {

constexpr int kQcThreads = 256;
constexpr int kQcMaxK = 20;  // LDS <= 20*256*8 + 2*256*8 + 20*256*4 (F = 1) = 64 KiB, the default limit
constexpr int kQcMaxBlocks = 2048;
constexpr int kQcUnroll = 8;

__global__ __launch_bounds__(kQcThreads) void domain_sse_kernel(
    const float* __restrict__ img, int C, const int32_t* __restrict__ feat, int F,
    const double* __restrict__ a, const double* __restrict__ b, const double* __restrict__ pivot,
    const double* __restrict__ centers, int k, int d0, const int8_t* __restrict__ label, int64_t n_pix,
    int M, double* __restrict__ part) {
  extern __shared__ double lds[];
  double* sse = lds;                                           // [k][256]
  double* s1s = sse + (size_t)k * kQcThreads;                  // [256]
  double* s2s = s1s + kQcThreads;                              // [256]
  uint32_t* cnt = reinterpret_cast<uint32_t*>(s2s + kQcThreads);  // [k][groups]
  const int t = threadIdx.x;
  const int groups = kQcThreads / F;
  const int g = t / F, f = t - g * F;
  for (int d = 0; d < k; ++d) sse[d * kQcThreads + t] = 0.0;
  for (int i = t; i < k * groups; i += kQcThreads) cnt[i] = 0u;
  __syncthreads();
  double s1 = 0.0, s2 = 0.0;
  if (g < groups) {
    const int ch = feat[f];
    const double af = a[f], bf = b[f], pf = pivot[f];
    const int64_t step = (int64_t)gridDim.x * groups;
    auto add = [&](float v, int l) {
      const double x = (double)v * af + bf;
      const double y = x - pf;
      s1 += y;
      s2 += y * y;
      l -= d0;
      if (l >= 0 && l < k) {
        const double dd = x - centers[l * F + f];
        sse[l * kQcThreads + t] += dd * dd;
        if (f == 0) cnt[l * groups + g] += 1u;
      }
    };
    int64_t p = (int64_t)blockIdx.x * groups + g;
    // kQcUnroll pixels' loads in flight before their (LDS read-modify-write) updates
    for (; p + (kQcUnroll - 1) * step < n_pix; p += kQcUnroll * step) {
      float v[kQcUnroll];
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
  s1s[t] = s1;
  s2s[t] = s2;
  __syncthreads();
  // fold the groups: output [sse k*F | sum F | sumsq F | count k]
  for (int e = t; e < M; e += kQcThreads) {
    double r = 0.0;
    if (e < k * F) {
      const int d = e / F, ff = e - d * F;
      for (int gg = 0; gg < groups; ++gg) r += sse[d * kQcThreads + gg * F + ff];
    } else if (e < k * F + F) {
      const int ff = e - k * F;
      for (int gg = 0; gg < groups; ++gg) r += s1s[gg * F + ff];
    } else if (e < k * F + 2 * F) {
      const int ff = e - k * F - F;
      for (int gg = 0; gg < groups; ++gg) r += s2s[gg * F + ff];
    } else {
      const int d = e - k * F - 2 * F;
      for (int gg = 0; gg < groups; ++gg) r += (double)cnt[d * groups + gg];
    }
    part[(size_t)blockIdx.x * M + e] = r;
  }
}

// One workgroup per output element: lane i sums blocks i, i+256, ... in order,
// then a fixed-order block tree (deterministic).
__global__ __launch_bounds__(256) void domain_sse_reduce(const double* __restrict__ part, int G,
                                                         int M, double* __restrict__ out) {
  __shared__ double scratch[256 / kWave];
  const int e = blockIdx.x;
  double r = 0.0;
  for (int i = threadIdx.x; i < G; i += 256) r += part[(size_t)i * M + e];
  r = block_sum(r, scratch);
  if (threadIdx.x == 0) out[e] = r;
}

static int qc_blocks(int64_t n_pix, int F) {
  const int groups = kQcThreads / F;
  const int64_t want = (n_pix + (int64_t)groups * 64 - 1) / ((int64_t)groups * 64);
  return (int)std::max<int64_t>(1, std::min<int64_t>(want, kQcMaxBlocks));
}

}  // namespace mw

using namespace mw;

extern "C" {

size_t mw_domain_sse_ws_bytes(int64_t n_pix, int k, int F) {
  if (n_pix <= 0 || k <= 0 || F <= 0 || F > kQcThreads) return 0;
  const int M = k * F + 2 * F + k;
  return (size_t)qc_blocks(n_pix, F) * M * sizeof(double);
}

int mw_domain_sse(const float* d_img, int C, const int32_t* d_feat, int F, const double* d_a,
                  const double* d_b, const double* d_pivot, const double* d_centers, int k, int d0,
                  const int8_t* d_label, int64_t n_pix, double* d_out, void* d_ws, void* stream) {
  MW_CHECK_ARG(d_img && d_feat && d_a && d_b && d_pivot && d_centers && d_label && d_out && d_ws,
               "mw_domain_sse: null pointer");
  MW_CHECK_ARG(n_pix > 0 && C > 0 && F > 0 && F <= kQcThreads && k >= 1 && k <= kQcMaxK && d0 >= 0,
               "mw_domain_sse: bad shape n_pix=%lld C=%d F=%d k=%d d0=%d (F <= 256, k <= 20 per launch)",
               (long long)n_pix, C, F, k, d0);
  hipStream_t st = as_stream(stream);
  const int G = qc_blocks(n_pix, F);
  const int M = k * F + 2 * F + k;
  const size_t lds = (size_t)k * kQcThreads * sizeof(double) + 2 * kQcThreads * sizeof(double) +
                     (size_t)k * (kQcThreads / F) * sizeof(uint32_t);
  double* part = reinterpret_cast<double*>(d_ws);
  hipLaunchKernelGGL(domain_sse_kernel, dim3(G), dim3(kQcThreads), lds, st, d_img, C, d_feat, F,
                     d_a, d_b, d_pivot, d_centers, k, d0, d_label, n_pix, M, part);
  MW_LAUNCH_CHECK();
  hipLaunchKernelGGL(domain_sse_reduce, dim3(M), dim3(256), 0, st, part, G, M, d_out);
  MW_LAUNCH_CHECK();
  return MW_OK;
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
