// k-means kernels of the MILWRM hot path on MI355X (gfx950, wave64).
//
//   (k-means++ is kpp.hip, the Lloyd iteration lloyd.hip)
//   farthest     _relocate_empty_clusters_dense      _k_means_common.pyx:181-226
//   assign_conf  KMeans.predict + estimate_confidence_score_mxif
//                                                    MILWRM.py:237-277, 389-450
//
// Rows are fp32 feature vectors (sample rows S x F, or HWC pixels with a
// feature subset) scaled on the fly by the folded StandardScaler affine.
// Every reduction is deterministic: fixed row→block map per size, per-block
// fp64 records, fixed-order combine.  Labels: lowest index wins ties (strict
// '<'), as the reference's argmin.
#include <math.h>
#include <stdlib.h>

#include "kmeans_common.h"

namespace mw {

constexpr int kAssignWPS = 1;  // label pass: minimum workgroups per CU (launch bound)

static inline size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }

__global__ void __launch_bounds__(256) rec_reduce_kernel(const double* __restrict__ rec, int G,
                                                           int rl, double* __restrict__ out) {
  rec_reduce_body(rec, G, rl, out);
}

// ============================================================== farthest
// pass 1: fp64 distance of each row to its assigned center
__global__ void __launch_bounds__(256) dist_assigned_kernel(const float* __restrict__ X, int64_t S,
                                                            int F, const float* __restrict__ ga,
                                                            const float* __restrict__ gb,
                                                            const double* __restrict__ C,
                                                            const uint8_t* __restrict__ labels,
                                                            double* __restrict__ dist) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < S; s += stride) {
    const int l = labels[s];
    double d = 0.0;
    for (int f = 0; f < F; ++f) {
      const double x = (double)fmaf(X[s * F + f], ga[f], gb[f]);
      const double v = x - C[l * F + f];
      d = fma(v, v, d);
    }
    dist[s] = d;
  }
}
// pass 2 (repeated n times): block argmax (value desc, index asc) → partials
__global__ void __launch_bounds__(256) argmax_kernel(const double* __restrict__ dist, int64_t S,
                                                     double* __restrict__ pv, int64_t* __restrict__ pi) {
  __shared__ double sv[256];
  __shared__ int64_t si[256];
  double bv = -1.0;
  int64_t bi = S;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < S; s += stride) {
    const double v = dist[s];
    if (v > bv || (v == bv && s < bi)) { bv = v; bi = s; }
  }
  sv[threadIdx.x] = bv;
  si[threadIdx.x] = bi;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) {
      const double v = sv[threadIdx.x + o];
      const int64_t i = si[threadIdx.x + o];
      if (v > sv[threadIdx.x] || (v == sv[threadIdx.x] && i < si[threadIdx.x])) {
        sv[threadIdx.x] = v;
        si[threadIdx.x] = i;
      }
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) { pv[blockIdx.x] = sv[0]; pi[blockIdx.x] = si[0]; }
}
__global__ void argmax_final_kernel(const double* __restrict__ pv, const int64_t* __restrict__ pi,
                                    int nb, double* __restrict__ dist, int which,
                                    int64_t* __restrict__ top_idx, double* __restrict__ top_val) {
  if (threadIdx.x != 0) return;
  double bv = -1.0;
  int64_t bi = -1;
  for (int b = 0; b < nb; ++b) {
    if (pi[b] < 0) continue;
    if (pv[b] > bv || (pv[b] == bv && pi[b] < bi)) { bv = pv[b]; bi = pi[b]; }
  }
  top_idx[which] = bi;
  top_val[which] = bv;
  if (bi >= 0) dist[bi] = -2.0;  // exclude from the next round
}

// ============================================================ assign_conf
__host__ __device__ inline size_t assign_wave_bytes(int k, int CMAX) {
  return (size_t)(k + 1) * 64 * 12 + (size_t)64 * CMAX * 4;
}
// XL: the wave's tile (64 x C floats, CMAX floats of readable pad: the last
// row's pair reads past C), reused for the per-lane sums at the end
constexpr int kAssignXLK = 8;  // XL keeps the per-label sums in registers: k <= 8
__host__ __device__ inline size_t assign_wave_bytes_xl(int k, int C, int CMAX) {
  const size_t tile = (size_t)64 * C * 4 + (size_t)CMAX * 4, sums = (size_t)(k + 1) * 64 * 12;
  return ((tile > sums ? tile : sums) + 15) & ~(size_t)15;
}
// Per-domain confidence sums in fixed point: each confidence (fp32 in [0, 1],
// or NaN) as the integer rint(conf * 2^32) held in an fp64 (exact), so a
// lane's sum is an exact integer (< 2^53 while a lane takes < 2^21 pixels), a
// block's sum an exact uint64, and the records two 32-bit limbs: the domain
// sums are the same bits however the pixels are split into launches, bands
// or ranks (np.mean's fp64 sum of the reference, MILWRM.py:447-449, to
// 2^-33 per pixel).
constexpr int kDomRec = 3;  // per-block record: [conf hi k | conf lo k | count k]
__device__ __forceinline__ double conf_fixed(float c) { return (double)rintf(c * 4294967296.f); }

// The per-block record from the waves' lane-private slots (per wave at
// `slots` + w * wslot: fp64 conf sums [k+1][64] | u32 counts [k+1][64]).
// A NaN confidence makes its domain's limbs NaN (the reference's mean is NaN).
__device__ void domain_block_record(const char* slots, size_t wslot, int nw, int k, double* out) {
  for (int q = threadIdx.x; q < 2 * k; q += blockDim.x) {
    const int j = q < k ? q : q - k;
    unsigned long long s = 0;
    bool nan = false;
    for (int w = 0; w < nw; ++w) {
      const double* cs = reinterpret_cast<const double*>(slots + (size_t)w * wslot);
      const unsigned* cc = reinterpret_cast<const unsigned*>(cs + (k + 1) * 64);
      for (int l = 0; l < 64; ++l) {
        if (q < k) {
          const double v = cs[j * 64 + l];
          nan |= v != v;
          s += nan ? 0ull : (unsigned long long)v;
        } else {
          s += cc[j * 64 + l];
        }
      }
    }
    if (q < k) {
      out[q] = nan ? __builtin_nan("") : (double)(s >> 32);
      out[k + q] = nan ? __builtin_nan("") : (double)(s & 0xffffffffull);
    } else {
      out[k + q] = (double)s;
    }
  }
}

// canonical limbs of the reduced domain records: lo in [0, 2^32) (NaN stays NaN)
__global__ void dom_carry_kernel(double* __restrict__ dom, int k) {
  for (int j = threadIdx.x; j < k; j += blockDim.x) {
    const double c = floor(dom[k + j] * (1.0 / 4294967296.0));  // exact: power-of-two scale
    dom[j] += c;
    dom[k + j] -= c * 4294967296.0;
  }
}

// KMeans.predict + estimate_confidence_score_mxif (MILWRM.py:237-277,
// 389-450) over every pixel of an HWC image: label of the nearest center
// (strict argmin, same packed-FMA distance as the Lloyd E-step), confidence
// (d2 - d1) / d2 from the two smallest distances, -1 / NaN outside the mask.
// Per-block record: [conf hi k | conf lo k | count k] (exact fp64 limbs,
// domain_block_record).
// Waves stream 64-pixel tiles (64*C floats) with the next tile in flight.
template <int CMAX, int KS, bool SC, bool XL = false>
__global__ void __launch_bounds__(256, kAssignWPS) assign_kernel(const float* __restrict__ img, int C,
                                                     const int32_t* __restrict__ feat, int F,
                                                     const float* __restrict__ ga,
                                                     const float* __restrict__ gb,
                                                     const float* __restrict__ gc,
                                                     const f2v* __restrict__ gT, int k,
                                                     const uint8_t* __restrict__ mask, int64_t n,
                                                     int64_t R, int8_t* __restrict__ lab_out,
                                                     float* __restrict__ conf_out,
                                                     double* __restrict__ rec, int il = 0) {
  constexpr int NV = CMAX / 4;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __shared__ __attribute__((aligned(16))) float s_a[CMAX], s_b[CMAX];
  __shared__ int s_feat[CMAX];
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6, nw = blockDim.x >> 6;
  // SC: centers by scalar loads from gT (no LDS traffic; the pair loads are
  // serialised, so only for small k); else a pair-major LDS image
  f2v* s_cT = reinterpret_cast<f2v*>(smem);
  const size_t cent_bytes = SC ? 0 : cent_t_bytes(KS, CMAX);
  __shared__ int s_ident;
  // per wave: conf sums fp64 [k+1][64] | counts u32 [k+1][64] | tile [64*CMAX]
  // (XL: the tile, then the sums written over it from registers at the end)
  const size_t wslot = XL ? assign_wave_bytes_xl(k, C, CMAX) : assign_wave_bytes(k, CMAX);
  char* wb = smem + cent_bytes + (size_t)wid * wslot;
  double* w_csum = reinterpret_cast<double*>(wb);
  unsigned* w_ccnt = reinterpret_cast<unsigned*>(w_csum + (k + 1) * 64);
  float* s_tile = XL ? reinterpret_cast<float*>(wb) : reinterpret_cast<float*>(w_ccnt + (k + 1) * 64);
  double r_cs[XL ? kAssignXLK + 1 : 1];
  unsigned r_cc[XL ? kAssignXLK + 1 : 1];
#pragma unroll
  for (int j = 0; j < (XL ? kAssignXLK + 1 : 1); ++j) {
    r_cs[j] = 0.0;
    r_cc[j] = 0u;
  }
  if (!SC) load_centers_T<CMAX, KS>(gc, k, F, s_cT);
  if (t == 0) s_ident = F == C;
  __syncthreads();
  for (int f = t; f < CMAX; f += blockDim.x) {
    s_feat[f] = f < F ? feat[f] : 0;
    s_a[f] = f < F ? ga[f] : 0.f;
    s_b[f] = f < F ? gb[f] : 0.f;
    if (f < F && feat[f] != f) s_ident = 0;  // features = all channels in order
  }
  if (!XL)
    for (int q = lane; q < (k + 1) * 64; q += 64) {
      w_csum[q] = 0.0;
      w_ccnt[q] = 0u;
    }
  else  // the pad past the tile: the last row's pair reads beyond C land here (finite: 0)
    for (int q = 64 * C + lane; q < 64 * C + CMAX; q += 64) s_tile[q] = 0.f;
  __syncthreads();

  // tiles: il = 0, the block's row range [lo, hi) (tile wid, wid + nw, ...);
  // il = 1, the whole image interleaved over every wave of the grid (wave w
  // of block b takes tiles b nw + w + j G nw): all waves move through the
  // image together (HBM row locality).  The records are exact integer sums,
  // the same totals for any partition
  const int64_t lo = il ? 0 : (int64_t)blockIdx.x * R, hi = il ? n : min(n, lo + R);
  const int ntile = hi > lo ? (int)((hi - lo + 63) / 64) : 0;
  const int tstep = il ? (int)gridDim.x * nw : nw;
  const int tc0 = il ? (int)blockIdx.x * nw + wid : wid;
  const int64_t total = n * (int64_t)C, n4 = total >> 2;
  const f4v* X4 = reinterpret_cast<const f4v*>(img);
  const bool ident = s_ident != 0;

  // two tiles in flight per wave (register ring): the LDS footprint allows
  // 2 waves per SIMD, and one 7.7-KB tile per wave in flight left the pass
  // latency-bound (~4.2 TB/s)
  auto fetch = [&](f4v (&vv)[NV], int& mm, int tt) {
    tt = tt < ntile ? tt : ntile - 1;
    const int64_t r = lo + (int64_t)tt * 64;
    mm = ld_stream(mask + min(r + lane, hi - 1));  // nt: read-once streams
    const int64_t q0 = (r * C) >> 2;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      int64_t q = q0 + lane + i * 64;
      q = q < n4 ? q : n4 - 1;
      vv[i] = ld_stream(X4 + q);
    }
  };
  auto body = [&](f4v (&vv)[NV], int& mm, int tc) {
    const int64_t p0 = lo + (int64_t)tc * 64;
    const int np = (int)min((int64_t)64, hi - p0);
    {
      f4v* s4 = reinterpret_cast<f4v*>(s_tile);
#pragma unroll
      for (int i = 0; i < NV; ++i)  // XL: the slot holds 64 * C floats (+ pad), not 64 * CMAX
        if (!XL || (lane + i * 64) * 4 < 64 * C) s4[lane + i * 64] = vv[i];
    }
    wt_tail(np * C, p0 * C, n4, img, total, s_tile, lane);
    const int mk = mm;
    fetch(vv, mm, tc + (XL ? 1 : 2) * tstep);  // XL: one tile in flight per wave (more waves)
    float m1, m2;
    int lab;
    if constexpr (XL) {  // the scaled row stays in LDS (SC centers): CMAX VGPRs fewer
      int z = 0;
      asm volatile("" : "+s"(z));
      nearest_centers_ls<CMAX, KS, true>(s_tile + lane * C, C, ident, s_feat + z,
                                          reinterpret_cast<const f2v*>(s_a) + z,
                                          reinterpret_cast<const f2v*>(s_b) + z, gT, k, lab, m1, m2);
    } else {
    f2v x2[CMAX / 2];
    if (ident) {
      load_scaled_row<CMAX>(s_tile, lane, C, s_a, s_b, x2);
    } else {
      int z = 0;
      asm volatile("" : "+s"(z));
      const f2v* sa = reinterpret_cast<const f2v*>(s_a) + z;
      const f2v* sb = reinterpret_cast<const f2v*>(s_b) + z;
      const int* sf = s_feat + z;
      const float* xs = s_tile + lane * C;
#pragma unroll
      for (int p = 0; p < CMAX / 2; ++p)
        x2[p] = __builtin_elementwise_fma(f2v{xs[sf[2 * p]], xs[sf[2 * p + 1]]}, sa[p], sb[p]);
    }
    if (SC)
      nearest_centers_s<CMAX, KS, true>(x2, gT, k, lab, m1, m2);
    else
      nearest_centers<CMAX, KS, true>(x2, s_cT, k, lab, m1, m2);
    }
    const bool valid = lane < np;
    const bool in_mask = valid && mk != 0;
    const float conf = in_mask ? (m2 - m1) / m2 : __builtin_nanf("");
    if (!in_mask) lab = -1;
    if (valid) {
      lab_out[p0 + lane] = (int8_t)lab;
      conf_out[p0 + lane] = conf;
    }
    // per-label sum of confidences and counts: lane-private slots in a fixed
    // order (pixels outside the mask/tile go to the sink slot k); the
    // confidences as the integers conf_q (conf_fixed), so every sum is exact
    if constexpr (XL) {  // the same per-slot add sequence, in registers (x + 0.0 == x)
      const int sl = lab < 0 ? k : lab;
      const double cv = in_mask ? conf_fixed(conf) : 0.0;
#pragma unroll
      for (int j = 0; j <= kAssignXLK; ++j) {
        r_cs[j] += sl == j ? cv : 0.0;
        r_cc[j] += sl == j ? 1u : 0u;
      }
    } else {
      const int slot = (lab < 0 ? k : lab) * 64 + lane;
      atomicAdd(&w_csum[slot], in_mask ? conf_fixed(conf) : 0.0);
      atomicAdd(&w_ccnt[slot], 1u);
    }
  };
  int tc = tc0;
  if constexpr (XL) {
    f4v va[NV];
    int ma = 0;
    if (tc < ntile) fetch(va, ma, tc);
    for (; tc < ntile; tc += tstep) body(va, ma, tc);
  } else {
    f4v va[NV], vb[NV];
    int ma = 0, mb = 0;
    if (tc < ntile) {
      fetch(va, ma, tc);
      fetch(vb, mb, tc + tstep);
    }
    for (; tc < ntile; tc += 2 * tstep) {
      body(va, ma, tc);
      if (tc + tstep < ntile) body(vb, mb, tc + tstep);
    }
  }
  if constexpr (XL) {  // lane-private slots, as the LDS-sum form leaves them
#pragma unroll
    for (int j = 0; j <= kAssignXLK; ++j)
      if (j <= k) {
        w_csum[j * 64 + lane] = r_cs[j];
        w_ccnt[j * 64 + lane] = r_cc[j];
      }
  }
  __syncthreads();
  domain_block_record(smem + cent_bytes, wslot, nw, k, rec + (size_t)blockIdx.x * kDomRec * k);
}

// Per-block domain records [sum conf k | count k] from label/confidence maps
// (the fused blur assign epilogue writes only the maps): the assign kernel's
// block partition, wave/tile order and lane-private fp64 slots, so the
// records, and the domain means, are the same numbers it produces.
__global__ void __launch_bounds__(256) domain_records_kernel(const int8_t* __restrict__ lab,
                                                             const float* __restrict__ conf, int k,
                                                             int64_t n, int64_t R,
                                                             double* __restrict__ rec) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6, nw = blockDim.x >> 6;
  const size_t wslot = (size_t)(k + 1) * 64 * 12;
  char* wb = smem + (size_t)wid * wslot;
  double* w_csum = reinterpret_cast<double*>(wb);
  unsigned* w_ccnt = reinterpret_cast<unsigned*>(w_csum + (k + 1) * 64);
  for (int q = lane; q < (k + 1) * 64; q += 64) {
    w_csum[q] = 0.0;
    w_ccnt[q] = 0u;
  }
  const int64_t lo = (int64_t)blockIdx.x * R, hi = min(n, lo + R);
  const int ntile = hi > lo ? (int)((hi - lo + 63) / 64) : 0;
  for (int tc = wid; tc < ntile; tc += nw) {
    const int64_t p = lo + (int64_t)tc * 64 + lane;
    const bool valid = p < hi;
    const int lb = valid ? (int)lab[p] : -1;
    const float c = valid ? conf[p] : 0.f;
    const int slot = (lb < 0 ? k : lb) * 64 + lane;
    w_csum[slot] += lb >= 0 ? conf_fixed(c) : 0.0;
    w_ccnt[slot] += 1u;
  }
  __syncthreads();
  domain_block_record(smem, wslot, nw, k, rec + (size_t)blockIdx.x * kDomRec * k);
}

// waves per assign block (LDS-bound for large k and C): shared with the
// domain-records kernel so both partition the image the same way
static int assign_waves(int k, int C) {
  const int CM = C <= 8 ? 8 : C <= 16 ? 16 : C <= 32 ? 32 : 64;
  const size_t cent = cent_t_bytes(k <= 64 ? 64 : 128, CM);
  int nw = 4;
  while (nw > 1 && cent + nw * assign_wave_bytes(k, CM) > 160 * 1024) --nw;
  return nw;
}

}  // namespace mw

using namespace mw;

extern "C" {

size_t mw_farthest_ws_bytes(int64_t S) {
  return al256((size_t)S * sizeof(double)) + 1024 * (sizeof(double) + sizeof(int64_t)) + 256;
}

int mw_farthest(const float* d_X, int64_t S, int F, const float* d_a, const float* d_b,
                const double* d_centers, int k, const uint8_t* d_labels, int n, int64_t* d_top_idx,
                double* d_top_val, void* d_ws, void* stream) {
  MW_CHECK_ARG(d_X && d_a && d_b && d_centers && d_labels && d_top_idx && d_top_val && d_ws,
               "mw_farthest: null pointer");
  MW_CHECK_ARG(n >= 1 && n <= 64 && S > 0 && F > 0 && k >= 1, "mw_farthest: bad args");
  hipStream_t s = as_stream(stream);
  char* base = reinterpret_cast<char*>(d_ws);
  double* dist = reinterpret_cast<double*>(base);
  double* pv = reinterpret_cast<double*>(base + al256((size_t)S * sizeof(double)));
  int64_t* pi = reinterpret_cast<int64_t*>(pv + 1024);
  const int nb = (int)std::min<int64_t>((S + 255) / 256, 1024);
  hipLaunchKernelGGL(dist_assigned_kernel, dim3(nb), dim3(256), 0, s, d_X, S, F, d_a, d_b,
                     d_centers, d_labels, dist);
  MW_LAUNCH_CHECK();
  for (int i = 0; i < n; ++i) {
    hipLaunchKernelGGL(argmax_kernel, dim3(nb), dim3(256), 0, s, dist, S, pv, pi);
    hipLaunchKernelGGL(argmax_final_kernel, dim3(1), dim3(64), 0, s, pv, pi, nb, dist, i, d_top_idx,
                       d_top_val);
  }
  MW_LAUNCH_CHECK();
  return MW_OK;
}

// workspace: per-block records [G][3k] fp64 | pair-major centers image
static size_t assign_rec_bytes(int64_t n_pix, int k) {
  return ((size_t)kblocks(n_pix) * kDomRec * k * sizeof(double) + 255) & ~(size_t)255;
}
size_t mw_assign_ws_bytes(int64_t n_pix, int k) {
  return assign_rec_bytes(n_pix, k) + cent_t_bytes(k <= 64 ? 64 : 128, 64) + 256;
}

int mw_assign_conf(const float* d_img, int C, const int32_t* d_feat, int F, const float* d_a,
                   const float* d_b, const float* d_centers, int k, const uint8_t* d_mask,
                   int64_t n_pix, int8_t* d_label, float* d_conf, void* d_ws, void* stream) {
  MW_CHECK_ARG(d_img && d_feat && d_a && d_b && d_centers && d_mask && d_label && d_conf && d_ws,
               "mw_assign_conf: null pointer");
  MW_CHECK_ARG(n_pix > 0 && C > 0 && F > 0 && k >= 1, "mw_assign_conf: bad shape");
  if (k > 127 || F > C || C > 64) {
    set_error("mw_assign_conf: k=%d C=%d F=%d unsupported (k <= 127, F <= C <= 64)", k, C, F);
    return MW_EUNSUPPORTED;
  }
  hipStream_t s = as_stream(stream);
  const int G = kblocks(n_pix);
  const int64_t R = krows(n_pix);
  double* rec = reinterpret_cast<double*>(d_ws);
  f2v* gT = reinterpret_cast<f2v*>(static_cast<char*>(d_ws) + assign_rec_bytes(n_pix, k));
  static const int sc_k = [] {  // largest k for the scalar-load E-step (tuning: MW_ASSIGN_SC_K)
    const char* e = getenv("MW_ASSIGN_SC_K");
    return e ? atoi(e) : 8;
  }();
  const bool sc = k <= sc_k;
  static const bool xl = [] {  // scaled row re-read from LDS (MW_ASSIGN_XL=0: held in registers)
    const char* e = getenv("MW_ASSIGN_XL");
    return !(e && e[0] == '0');
  }();
  // tiles interleaved over the grid (config 2: 2.78 -> 2.73 ms, the same
  // labels, confidences and domain sums; MW_ASSIGN_IL=0: block row ranges)
  const int il = [] {
    const char* e = getenv("MW_ASSIGN_IL");
    return (e && e[0] == '0') ? 0 : 1;
  }();
#define MW_AS2(CM, KSV, SCV)                                                                    \
  {                                                                                             \
    const size_t cent = SCV ? 0 : cent_t_bytes(KSV, CM);                                        \
    const bool xlv = SCV && CM >= 32 && xl && k <= kAssignXLK;                                  \
    const int nw = xlv ? 4 : assign_waves(k, C);                                                \
    const size_t lds = cent + nw * (xlv ? assign_wave_bytes_xl(k, C, CM) : assign_wave_bytes(k, CM)); \
    if (lds > 160 * 1024) {                                                                     \
      set_error("mw_assign_conf: LDS %zu too large (C=%d k=%d)", lds, C, k);                    \
      return MW_EUNSUPPORTED;                                                                   \
    }                                                                                           \
    if (xlv)                                                                                    \
      hipLaunchKernelGGL((assign_kernel<CM, KSV, SCV, SCV && (CM >= 32)>), dim3(G), dim3(64 * nw), lds, s, \
                         d_img, C, d_feat, F, d_a, d_b, d_centers, gT, k, d_mask, n_pix, R, d_label, \
                         d_conf, rec, il);                                                      \
    else                                                                                        \
      hipLaunchKernelGGL((assign_kernel<CM, KSV, SCV>), dim3(G), dim3(64 * nw), lds, s, d_img, C, \
                         d_feat, F, d_a, d_b, d_centers, gT, k, d_mask, n_pix, R, d_label, d_conf, rec, il); \
  }
#define MW_AS(CM, KSV)                                                                          \
  {                                                                                             \
    if (sc) {                                                                                   \
      hipLaunchKernelGGL((centers_T_kernel<CM, KSV>), dim3(1), dim3(256), 0, s, d_centers, k, F, gT); \
      MW_AS2(CM, KSV, true)                                                                     \
    } else MW_AS2(CM, KSV, false)                                                               \
  }
#define MW_ASK(CM)             \
  if (k <= 64) MW_AS(CM, 64)   \
  else MW_AS(CM, 128)
  if (C <= 8) { MW_ASK(8) }
  else if (C <= 16) { MW_ASK(16) }
  else if (C <= 32) { MW_ASK(32) }
  else if (C <= 52 && sc && xl && k <= kAssignXLK) { MW_AS(52, 64) }  // XL: 26 feature pairs, not 32
  else { MW_ASK(64) }
#undef MW_ASK
#undef MW_AS
#undef MW_AS2
  MW_LAUNCH_CHECK();
  return MW_OK;
}

int mw_domain_records(const int8_t* d_label, const float* d_conf, int64_t n_pix, int C, int k,
                      void* d_ws, void* stream) {
  MW_CHECK_ARG(d_label && d_conf && d_ws && n_pix > 0 && C > 0 && k >= 1 && k <= 127,
               "mw_domain_records: bad args");
  const int nw = assign_waves(k, C);
  const size_t lds = (size_t)nw * (k + 1) * 64 * 12;
  if (lds > 160 * 1024) {
    set_error("mw_domain_records: k=%d too large", k);
    return MW_EUNSUPPORTED;
  }
  hipLaunchKernelGGL(domain_records_kernel, dim3(kblocks(n_pix)), dim3(64 * nw), lds, as_stream(stream),
                     d_label, d_conf, k, n_pix, krows(n_pix), reinterpret_cast<double*>(d_ws));
  MW_LAUNCH_CHECK();
  return MW_OK;
}

int mw_assign_reduce(const void* d_ws, int64_t n_pix, int k, double* d_dom, void* stream) {
  MW_CHECK_ARG(d_ws && d_dom && k >= 1, "mw_assign_reduce: bad args");
  // integer-valued limbs below 2^32 over <= 1024 blocks: the fp64 sums are exact;
  // then the lo limbs' carries into the hi limbs (one canonical form: lo < 2^32)
  hipLaunchKernelGGL(rec_reduce_kernel, dim3((kDomRec * k + 31) / 32), dim3(256), 0, as_stream(stream),
                     reinterpret_cast<const double*>(d_ws), kblocks(n_pix), kDomRec * k, d_dom);
  hipLaunchKernelGGL(dom_carry_kernel, dim3(1), dim3(128), 0, as_stream(stream), d_dom, k);
  MW_LAUNCH_CHECK();
  return MW_OK;
}

}  // extern "C"
