// k-means kernels of the MILWRM hot path on MI355X (gfx950, wave64).
//
//   kpp_*        sklearn _kmeans_plusplus            _kmeans.py:174-272
//   (the Lloyd iteration itself is lloyd.hip)
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

#ifndef MW_ASSIGN_WPS
#define MW_ASSIGN_WPS 1
#endif
#ifndef MW_KPP_WPS
#define MW_KPP_WPS 1
#endif

constexpr int kKppTab = 64 * 9;  // doubles: k-means++ candidate table inv[64] | b[64][8]

// ===================================================================== kpp
// Workspace layout (bytes, 256-aligned sections):
//   bank[2][T][S] fp64  candidate-min distance arrays (ping-pong per step)
//   bsum[2][T][G] fp64  their per-block sums
//   st: cand[T] i64, chosen[256] i64, best i32
struct KppLayout {
  size_t bank, bsum, st, tab, total;
  int G;
};
static inline size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }
static KppLayout kpp_layout(int64_t S, int T) {
  KppLayout L;
  L.G = kblocks(S);
  L.bank = 0;
  L.bsum = al256(L.bank + 2 * (size_t)T * S * sizeof(double));
  L.st = al256(L.bsum + 2 * (size_t)T * L.G * sizeof(double));
  L.tab = al256(L.st + (size_t)(T + 256) * sizeof(int64_t) + 64);
  L.total = al256(L.tab + (size_t)kKppTab * sizeof(double));
  return L;
}
struct KppState {
  int64_t* cand;
  int64_t* chosen;
  int* best;
};
__device__ __host__ inline KppState kpp_state(char* base, const KppLayout& L, int T) {
  KppState s;
  s.cand = reinterpret_cast<int64_t*>(base + L.st);
  s.chosen = s.cand + T;
  s.best = reinterpret_cast<int*>(s.chosen + 256);
  return s;
}

// inclusive scan of G block sums in LDS (fixed order; shared by search and
// select so the potential used for the targets equals the selected one)
__device__ __forceinline__ void scan_blocks(const double* __restrict__ bs, int G, double* s) {
  const int t = threadIdx.x;  // blockDim = 1024 >= G
  s[t] = t < G ? bs[t] : 0.0;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {
    const double v = t >= o ? s[t - o] : 0.0;
    __syncthreads();
    s[t] += v;
    __syncthreads();
  }
}

// local potentials of the n_cur arrays (same scan order as the search)
__global__ void __launch_bounds__(1024) kpp_pots_kernel(const double* __restrict__ bsum_cur,
                                                        int n_cur, int G, double* __restrict__ pots) {
  __shared__ double s[1024];
  for (int i = 0; i < n_cur; ++i) {
    scan_blocks(bsum_cur + (size_t)i * G, G, s);
    if (threadIdx.x == 0) pots[i] = s[G - 1];
    __syncthreads();
  }
}

// select best candidate of the finished step (argmin of potentials, first
// wins), then draw the next step's candidates: targets u_t * pot, located by
// the block prefix then a chunked scan inside the block.
// cur_bank: bank holding the step's candidate arrays; G blocks of R rows.
__global__ void __launch_bounds__(1024) kpp_search_kernel(const double* __restrict__ bank_cur,
                                                          const double* __restrict__ bsum_cur,
                                                          int n_cur, int64_t S, int G, int64_t R,
                                                          int c_done, double u0, double u1,
                                                          double u2, double u3, double u4,
                                                          double u5, double u6, double u7, int T,
                                                          int64_t* __restrict__ cand,
                                                          int64_t* __restrict__ chosen,
                                                          int* __restrict__ best_out,
                                                          int best_given,
                                                          const double* __restrict__ rv_given) {
  __shared__ double s[1024];
  __shared__ double s_pot[8];
  __shared__ int s_best;
  __shared__ double s_chunk[1024];
  __shared__ int s_found;
  const int t = threadIdx.x;
  if (best_given >= 0) {
    // sharded mode: the host chose the global best
    if (t == 0) { s_best = best_given; *best_out = best_given; }
    __syncthreads();
  } else {
    // 1) potentials of the n_cur arrays of the finished step → best
    for (int i = 0; i < n_cur; ++i) {
      scan_blocks(bsum_cur + (size_t)i * G, G, s);
      if (t == 0) s_pot[i] = s[G - 1];
      __syncthreads();
    }
    if (t == 0) {
      int b = 0;
      for (int i = 1; i < n_cur; ++i)
        if (s_pot[i] < s_pot[b]) b = i;
      s_best = b;
      *best_out = b;
      if (c_done > 0) chosen[c_done] = cand[b];
    }
    __syncthreads();
  }
  const int b = s_best;
  if (T == 0) return;  // final selection only
  const double* d = bank_cur + (size_t)b * S;
  scan_blocks(bsum_cur + (size_t)b * G, G, s);
  const double pot = s[G - 1];
  const double us[8] = {u0, u1, u2, u3, u4, u5, u6, u7};
  for (int k = 0; k < T; ++k) {
    const double rv = rv_given ? rv_given[k] : us[k] * pot;
    if (rv < 0.0) {  // target not on this shard
      if (t == 0) cand[k] = -1;
      continue;      // uniform: every thread reads the same rv
    }
    // first block whose inclusive prefix reaches rv (else the last block)
    if (t == 0) s_found = G - 1;
    __syncthreads();
    if (t < G) {
      const double prev = t > 0 ? s[t - 1] : 0.0;
      if (s[t] >= rv && (t == 0 || prev < rv)) s_found = t;
    }
    __syncthreads();
    const int blk = s_found;
    const double base = blk > 0 ? s[blk - 1] : 0.0;
    const int64_t lo = (int64_t)blk * R, hi = min(S, lo + R);
    const int64_t len = hi - lo;
    const int64_t per = (len + 1023) / 1024;
    const int64_t c_lo = lo + t * per, c_hi = min(hi, c_lo + per);
    double part = 0.0;
    for (int64_t i = c_lo; i < c_hi; ++i) part += d[i];
    // inclusive scan of the chunk sums (fixed order), base-offset
    s_chunk[t] = part;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {
      const double v = t >= o ? s_chunk[t - o] : 0.0;
      __syncthreads();
      s_chunk[t] += v;
      __syncthreads();
    }
    if (t == 0) s_found = -1;
    __syncthreads();
    {
      const double incl = base + s_chunk[t];
      const double excl = base + (t > 0 ? s_chunk[t - 1] : 0.0);
      if (c_lo < c_hi && incl >= rv && (t == 0 || excl < rv)) s_found = t;
    }
    __syncthreads();
    if (t == 0) {
      int64_t idx = hi - 1;  // rounding fallback: clip to the block's end
      const int q = s_found;
      if (q >= 0) {
        const int64_t ql = lo + q * per, qh = min(hi, ql + per);
        double r2 = base + (q > 0 ? s_chunk[q - 1] : 0.0);
        idx = qh - 1;
        for (int64_t i = ql; i < qh; ++i) {
          r2 += d[i];
          if (r2 >= rv) { idx = i; break; }
        }
      }
      if (idx > S - 1) idx = S - 1;
      if (idx < 0) idx = 0;
      cand[k] = idx;
    }
    __syncthreads();
  }
}

// k-means++ candidate table (one per distance pass): w_tf = x_f * inv_f - b_tf
// with b_tf = mu_f * inv_f + c_tf, c_t the scaled candidate rows (from `rows`,
// T x F floats, or X[cand[t]]); padded features get inv = b = 0.  Stored
// feature-major [f][8] so the distance pass reads it with uniform (scalar)
// loads.
__global__ void __launch_bounds__(512) kpp_prep_kernel(const float* __restrict__ X, int F,
                                                       const double* __restrict__ mu,
                                                       const double* __restrict__ inv,
                                                       const int64_t* __restrict__ cand,
                                                       const float* __restrict__ rows, int T,
                                                       double* __restrict__ tab,
                                                       int64_t* __restrict__ chosen_reset) {
  const int q = threadIdx.x;  // 512 = 64 features x 8 candidates
  const int f = q >> 3, c = q & 7;
  double bv = 0.0;
  if (f < F && c < T) {
    const float xv = rows ? rows[c * F + f] : X[cand[c] * F + f];
    const double cs = ((double)xv - mu[f]) * inv[f];
    bv = fma(mu[f], inv[f], cs);
  }
  tab[64 + f * 8 + c] = bv;
  if (c == 0) tab[f] = f < F ? inv[f] : 0.0;
  if (chosen_reset && q == 0) chosen_reset[0] = -1;
}

// Distance pass of k-means++ (sklearn _kmeans_plusplus, _kmeans.py:225-260):
// fp64 squared distances of every row to T candidate rows, w = fma(x, inv,
// -b) per feature (the scaler folded in, one rounding) and T independent FMA
// chains (features in order), elementwise min with the current closest
// distances cur = bank_prev[best] (init: no min), written to bank_new[t],
// plus per-block sums.  Waves stream 64-row tiles (buffer loads, next tile in
// flight); the candidate table comes through scalar loads.
template <int FMAX, int T>
__global__ void __launch_bounds__(256, MW_KPP_WPS) kpp_dist_kernel(
    const float* __restrict__ X, int64_t S, int F, const double* __restrict__ tab,
    const double* __restrict__ bank_prev, const int* __restrict__ best, int best_val, int64_t R,
    double* __restrict__ bank_new, double* __restrict__ bsum_new) {
  constexpr int NV = FMAX / 4;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __shared__ double s_red[4];
  const int t = threadIdx.x, lane = t & 63, nw = blockDim.x >> 6;
  const int wid = __builtin_amdgcn_readfirstlane(t >> 6);
  float* s_tile = reinterpret_cast<float*>(smem) + (size_t)wid * 64 * FMAX;
  const bool has_cur = bank_prev != nullptr;
  const double* cur = has_cur ? bank_prev + (size_t)(best ? *best : best_val) * S : nullptr;

  const int64_t lo = (int64_t)blockIdx.x * R, hi = min(S, lo + R);
  const int ntile = hi > lo ? (int)((hi - lo + 63) / 64) : 0;
  const int64_t total = S * (int64_t)F, n4 = total >> 2;
  const __amdgpu_buffer_rsrc_t rx = make_rsrc(X + lo * F, (S - lo) * F * 4);
  const __amdgpu_buffer_rsrc_t rc =
      make_rsrc(has_cur ? static_cast<const void*>(cur + lo) : static_cast<const void*>(X),
                has_cur ? (hi - lo) * 8 : 0);
  const int tile_bytes = 64 * F * 4;
  double acc[T];
#pragma unroll
  for (int c = 0; c < T; ++c) acc[c] = 0.0;

  f4v v[NV];
  double cur_next = 0.0;
  auto fetch = [&](int tt) {
    tt = tt < ntile ? tt : ntile - 1;
    if (has_cur)
      cur_next = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rc, lane * 8, tt * 512, 0));
    tile_load<NV>(rx, tt * tile_bytes, lane, v);
  };
  int tc = wid;
  if (tc < ntile) fetch(tc);
  for (; tc < ntile; tc += nw) {
    const int64_t r0 = lo + (int64_t)tc * 64;
    const int nrow = (int)min((int64_t)64, hi - r0);
    {
      f4v* s4 = reinterpret_cast<f4v*>(s_tile);
#pragma unroll
      for (int i = 0; i < NV; ++i) s4[lane + i * 64] = v[i];
    }
    wt_tail(nrow * F, r0 * F, n4, X, total, s_tile, lane);
    const double cd = cur_next;
    fetch(tc + nw);
    const float* xr = s_tile + lane * F;
    const double* tb = tab;  // uniform: hipcc keeps the table in SGPRs/VGPRs
    double d[T];
#pragma unroll
    for (int c = 0; c < T; ++c) d[c] = 0.0;
#pragma unroll
    for (int f = 0; f < FMAX; ++f) {
      const double xd = (double)xr[f];  // features past F: inv = b = 0 (rows finite)
      const double iv = tb[f];
#pragma unroll
      for (int c = 0; c < T; ++c) {
        const double w = fma(xd, iv, -tb[64 + f * 8 + c]);
        d[c] = fma(w, w, d[c]);
      }
    }
    const bool valid = lane < nrow;
    const int64_t row = r0 + lane;
#pragma unroll
    for (int c = 0; c < T; ++c) {
      const double m = (has_cur && cd < d[c]) ? cd : d[c];
      if (valid) {
        bank_new[(size_t)c * S + row] = m;
        acc[c] += m;
      }
    }
  }
#pragma unroll
  for (int c = 0; c < T; ++c) {
    const double tot = block_sum(acc[c], s_red);
    if (t == 0) bsum_new[(size_t)c * gridDim.x + blockIdx.x] = tot;
  }
}

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
// KMeans.predict + estimate_confidence_score_mxif (MILWRM.py:237-277,
// 389-450) over every pixel of an HWC image: label of the nearest center
// (strict argmin, same packed-FMA distance as the Lloyd E-step), confidence
// (d2 - d1) / d2 from the two smallest distances, -1 / NaN outside the mask.
// Per-block record: [sum conf k | count k] (fp64, fixed combine order).
// Waves stream 64-pixel tiles (64*C floats) with the next tile in flight.
template <int CMAX, int KS>
__global__ void __launch_bounds__(256, MW_ASSIGN_WPS) assign_kernel(const float* __restrict__ img, int C,
                                                     const int32_t* __restrict__ feat, int F,
                                                     const float* __restrict__ ga,
                                                     const float* __restrict__ gb,
                                                     const float* __restrict__ gc, int k,
                                                     const uint8_t* __restrict__ mask, int64_t n,
                                                     int64_t R, int8_t* __restrict__ lab_out,
                                                     float* __restrict__ conf_out,
                                                     double* __restrict__ rec) {
  constexpr int NV = CMAX / 4;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __shared__ __attribute__((aligned(16))) float s_a[CMAX], s_b[CMAX];
  __shared__ int s_feat[CMAX];
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6, nw = blockDim.x >> 6;
  f2v* s_cT = reinterpret_cast<f2v*>(smem);  // pair-major centers
  const size_t cent_bytes = cent_t_bytes(KS, CMAX);
  __shared__ int s_ident;
  // per wave: conf sums fp64 [k+1][64] | counts u32 [k+1][64] | tile [64*CMAX]
  const size_t wslot = assign_wave_bytes(k, CMAX);
  char* wb = smem + cent_bytes + (size_t)wid * wslot;
  double* w_csum = reinterpret_cast<double*>(wb);
  unsigned* w_ccnt = reinterpret_cast<unsigned*>(w_csum + (k + 1) * 64);
  float* s_tile = reinterpret_cast<float*>(w_ccnt + (k + 1) * 64);
  load_centers_T<CMAX, KS>(gc, k, F, s_cT);
  if (t == 0) s_ident = F == C;
  __syncthreads();
  for (int f = t; f < CMAX; f += blockDim.x) {
    s_feat[f] = f < F ? feat[f] : 0;
    s_a[f] = f < F ? ga[f] : 0.f;
    s_b[f] = f < F ? gb[f] : 0.f;
    if (f < F && feat[f] != f) s_ident = 0;  // features = all channels in order
  }
  for (int q = lane; q < (k + 1) * 64; q += 64) {
    w_csum[q] = 0.0;
    w_ccnt[q] = 0u;
  }
  __syncthreads();

  const int64_t lo = (int64_t)blockIdx.x * R, hi = min(n, lo + R);
  const int ntile = hi > lo ? (int)((hi - lo + 63) / 64) : 0;
  const int64_t total = n * (int64_t)C, n4 = total >> 2;
  const f4v* X4 = reinterpret_cast<const f4v*>(img);
  const bool ident = s_ident != 0;

  f4v v[NV];
  int mask_next = 0;
  auto fetch = [&](int tt) {
    tt = tt < ntile ? tt : ntile - 1;
    const int64_t r = lo + (int64_t)tt * 64;
    mask_next = mask[min(r + lane, hi - 1)];
    const int64_t q0 = (r * C) >> 2;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      int64_t q = q0 + lane + i * 64;
      q = q < n4 ? q : n4 - 1;
      v[i] = X4[q];
    }
  };
  int tc = wid;
  if (tc < ntile) fetch(tc);
  for (; tc < ntile; tc += nw) {
    const int64_t p0 = lo + (int64_t)tc * 64;
    const int np = (int)min((int64_t)64, hi - p0);
    {
      f4v* s4 = reinterpret_cast<f4v*>(s_tile);
#pragma unroll
      for (int i = 0; i < NV; ++i) s4[lane + i * 64] = v[i];
    }
    wt_tail(np * C, p0 * C, n4, img, total, s_tile, lane);
    const int mk = mask_next;
    fetch(tc + nw);
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
    float m1, m2;
    int lab;
    nearest_centers<CMAX, KS, true>(x2, s_cT, k, lab, m1, m2);
    const bool valid = lane < np;
    const bool in_mask = valid && mk != 0;
    const float conf = in_mask ? (m2 - m1) / m2 : __builtin_nanf("");
    if (!in_mask) lab = -1;
    if (valid) {
      lab_out[p0 + lane] = (int8_t)lab;
      conf_out[p0 + lane] = conf;
    }
    // per-label sum of confidences and counts: lane-private LDS slots in a
    // fixed order (pixels outside the mask/tile go to the sink slot k)
    {
      const int slot = (lab < 0 ? k : lab) * 64 + lane;
      atomicAdd(&w_csum[slot], in_mask ? (double)conf : 0.0);
      atomicAdd(&w_ccnt[slot], 1u);
    }
  }
  __syncthreads();
  double* out = rec + (size_t)blockIdx.x * 2 * k;
  for (int q = t; q < 2 * k; q += blockDim.x) {
    const int j = q < k ? q : q - k;
    double sacc = 0.0;
    for (int w = 0; w < nw; ++w) {
      const double* cs = reinterpret_cast<const double*>(smem + cent_bytes + (size_t)w * wslot);
      const unsigned* cc = reinterpret_cast<const unsigned*>(cs + (k + 1) * 64);
      if (q < k) {
        for (int l = 0; l < 64; ++l) sacc += cs[j * 64 + l];
      } else {
        unsigned long long c = 0;
        for (int l = 0; l < 64; ++l) c += cc[j * 64 + l];
        sacc += (double)c;
      }
    }
    out[q] = sacc;
  }
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
    w_csum[slot] += lb >= 0 ? (double)c : 0.0;
    w_ccnt[slot] += 1u;
  }
  __syncthreads();
  double* out = rec + (size_t)blockIdx.x * 2 * k;
  for (int q = t; q < 2 * k; q += blockDim.x) {
    const int j = q < k ? q : q - k;
    double sacc = 0.0;
    for (int w = 0; w < nw; ++w) {
      const double* cs = reinterpret_cast<const double*>(smem + (size_t)w * wslot);
      const unsigned* cc = reinterpret_cast<const unsigned*>(cs + (k + 1) * 64);
      if (q < k) {
        for (int l = 0; l < 64; ++l) sacc += cs[j * 64 + l];
      } else {
        unsigned long long cn = 0;
        for (int l = 0; l < 64; ++l) cn += cc[j * 64 + l];
        sacc += (double)cn;
      }
    }
    out[q] = sacc;
  }
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

size_t mw_kpp_ws_bytes(int64_t S, int T) { return kpp_layout(S, T).total; }

struct KppPtrs {
  KppLayout L;
  KppState st;
  double *bank, *bsum;
  double* bank_of(int c, int T, int64_t S) const { return bank + (size_t)(c & 1) * T * S; }
  double* bsum_of(int c, int T) const { return bsum + (size_t)(c & 1) * T * L.G; }
};
static KppPtrs kpp_ptrs(const void* d_ws, int64_t S, int T) {
  KppPtrs p;
  p.L = kpp_layout(S, T);
  char* base = reinterpret_cast<char*>(const_cast<void*>(d_ws));
  p.st = kpp_state(base, p.L, T);
  p.bank = reinterpret_cast<double*>(base + p.L.bank);
  p.bsum = reinterpret_cast<double*>(base + p.L.bsum);
  return p;
}

// candidate table, then the distance pass with the (FMAX, T) instance
static int kpp_dist_launch(const float* X, int64_t S, int F, const double* mu, const double* inv,
                           const double* bank_prev, const int* best, int best_val,
                           const int64_t* cand, const float* rows, int T, const KppLayout& L,
                           char* ws, double* bank_new, double* bsum_new, int64_t* chosen_reset,
                           hipStream_t s) {
  double* tab = reinterpret_cast<double*>(ws + L.tab);
  hipLaunchKernelGGL(kpp_prep_kernel, dim3(1), dim3(512), 0, s, X, F, mu, inv, cand, rows, T, tab,
                     chosen_reset);
  MW_LAUNCH_CHECK();
  const int FM = F <= 8 ? 8 : F <= 16 ? 16 : F <= 32 ? 32 : 64;
  const size_t lds = (size_t)4 * 64 * FM * sizeof(float);
#define MW_KD(FMV, TV)                                                                          \
  hipLaunchKernelGGL((kpp_dist_kernel<FMV, TV>), dim3(L.G), dim3(256), lds, s, X, S, F, tab,   \
                     bank_prev, best, best_val, krows(S), bank_new, bsum_new)
#define MW_KDT(FMV)                                                                  \
  switch (T) {                                                                       \
    case 1: MW_KD(FMV, 1); break; case 2: MW_KD(FMV, 2); break;                      \
    case 3: MW_KD(FMV, 3); break; case 4: MW_KD(FMV, 4); break;                      \
    case 5: MW_KD(FMV, 5); break; case 6: MW_KD(FMV, 6); break;                      \
    case 7: MW_KD(FMV, 7); break; default: MW_KD(FMV, 8); break;                     \
  }
  if (FM == 8) { MW_KDT(8) }
  else if (FM == 16) { MW_KDT(16) }
  else if (FM == 32) { MW_KDT(32) }
  else { MW_KDT(64) }
#undef MW_KDT
#undef MW_KD
  MW_LAUNCH_CHECK();
  return MW_OK;
}

int mw_kpp_init(const float* d_X, int64_t S, int F, const double* d_mu, const double* d_inv,
                const float* d_center_row, int T, void* d_ws, void* stream) {
  MW_CHECK_ARG(d_X && d_mu && d_inv && d_ws && d_center_row, "mw_kpp_init: null pointer");
  MW_CHECK_ARG(S > 0 && F > 0 && F <= 64, "mw_kpp_init: bad shape (F <= 64)");
  MW_CHECK_ARG(T >= 1 && T <= 8, "mw_kpp_init: n_local_trials must be in [1, 8]");
  const KppPtrs p = kpp_ptrs(d_ws, S, T);
  return kpp_dist_launch(d_X, S, F, d_mu, d_inv, nullptr, nullptr, 0, nullptr, d_center_row, 1,
                         p.L, static_cast<char*>(d_ws), p.bank_of(0, T, S), p.bsum_of(0, T),
                         p.st.chosen, as_stream(stream));
}

int mw_kpp_step(const float* d_X, int64_t S, int F, const double* d_mu, const double* d_inv, int c,
                const double* h_u, int T, void* d_ws, void* stream) {
  MW_CHECK_ARG(d_X && d_mu && d_inv && d_ws && h_u, "mw_kpp_step: null pointer");
  MW_CHECK_ARG(c >= 1 && c < 256, "mw_kpp_step: center index %d out of range", c);
  MW_CHECK_ARG(T >= 1 && T <= 8 && F <= 64, "mw_kpp_step: T in [1,8], F <= 64 required");
  const KppPtrs p = kpp_ptrs(d_ws, S, T);
  const int n_cur = c == 1 ? 1 : T;
  double u[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int i = 0; i < T; ++i) u[i] = h_u[i];
  hipStream_t s = as_stream(stream);
  // select the previous step's best (c >= 2), then locate this step's candidates
  hipLaunchKernelGGL(kpp_search_kernel, dim3(1), dim3(1024), 0, s, p.bank_of(c - 1, T, S),
                     p.bsum_of(c - 1, T), n_cur, S, p.L.G, krows(S), c - 1, u[0], u[1], u[2], u[3],
                     u[4], u[5], u[6], u[7], T, p.st.cand, p.st.chosen, p.st.best, -1,
                     (const double*)nullptr);
  MW_LAUNCH_CHECK();
  return kpp_dist_launch(d_X, S, F, d_mu, d_inv, p.bank_of(c - 1, T, S), p.st.best, 0, p.st.cand,
                         nullptr, T, p.L, static_cast<char*>(d_ws), p.bank_of(c, T, S),
                         p.bsum_of(c, T), nullptr, s);
}

int mw_kpp_indices(const void* d_ws, int64_t S, int T, int k, int64_t* d_idx_out, void* stream) {
  MW_CHECK_ARG(d_ws && d_idx_out && k >= 1 && k <= 256, "mw_kpp_indices: bad args");
  const KppPtrs p = kpp_ptrs(d_ws, S, T);
  hipStream_t s = as_stream(stream);
  if (k >= 2) {
    // final selection among the last step's T candidates
    hipLaunchKernelGGL(kpp_search_kernel, dim3(1), dim3(1024), 0, s, p.bank_of(k - 1, T, S),
                       p.bsum_of(k - 1, T), T, S, p.L.G, krows(S), k - 1, 0.0, 0.0, 0.0, 0.0, 0.0,
                       0.0, 0.0, 0.0, 0, p.st.cand, p.st.chosen, p.st.best, -1,
                       (const double*)nullptr);
    MW_LAUNCH_CHECK();
  }
  MW_HIP(hipMemcpyAsync(d_idx_out, p.st.chosen, sizeof(int64_t) * k, hipMemcpyDeviceToDevice, s));
  return MW_OK;
}

int mw_kpp_pots(const void* d_ws, int64_t S, int T, int c, double* d_pots, void* stream) {
  MW_CHECK_ARG(d_ws && d_pots && c >= 1 && T >= 1 && T <= 8, "mw_kpp_pots: bad args");
  const KppPtrs p = kpp_ptrs(d_ws, S, T);
  hipLaunchKernelGGL(kpp_pots_kernel, dim3(1), dim3(1024), 0, as_stream(stream),
                     p.bsum_of(c - 1, T), c == 1 ? 1 : T, p.L.G, d_pots);
  MW_LAUNCH_CHECK();
  return MW_OK;
}

int mw_kpp_search(void* d_ws, int64_t S, int T, int c, int best, const double* d_rv,
                  int64_t* d_local_idx, void* stream) {
  MW_CHECK_ARG(d_ws && d_rv && d_local_idx, "mw_kpp_search: null pointer");
  MW_CHECK_ARG(c >= 1 && T >= 1 && T <= 8 && best >= 0 && best < (c == 1 ? 1 : T),
               "mw_kpp_search: bad args (c=%d best=%d)", c, best);
  const KppPtrs p = kpp_ptrs(d_ws, S, T);
  hipStream_t s = as_stream(stream);
  hipLaunchKernelGGL(kpp_search_kernel, dim3(1), dim3(1024), 0, s, p.bank_of(c - 1, T, S),
                     p.bsum_of(c - 1, T), c == 1 ? 1 : T, S, p.L.G, krows(S), 0, 0.0, 0.0, 0.0,
                     0.0, 0.0, 0.0, 0.0, 0.0, T, p.st.cand, p.st.chosen, p.st.best, best, d_rv);
  MW_LAUNCH_CHECK();
  MW_HIP(hipMemcpyAsync(d_local_idx, p.st.cand, sizeof(int64_t) * T, hipMemcpyDeviceToDevice, s));
  return MW_OK;
}

int mw_kpp_trial(const float* d_X, int64_t S, int F, const double* d_mu, const double* d_inv, int c,
                 int best, const float* d_rows, int T, void* d_ws, void* stream) {
  MW_CHECK_ARG(d_X && d_mu && d_inv && d_rows && d_ws, "mw_kpp_trial: null pointer");
  MW_CHECK_ARG(c >= 1 && T >= 1 && T <= 8 && F <= 64 && best >= 0 && best < (c == 1 ? 1 : T),
               "mw_kpp_trial: bad args");
  const KppPtrs p = kpp_ptrs(d_ws, S, T);
  return kpp_dist_launch(d_X, S, F, d_mu, d_inv, p.bank_of(c - 1, T, S), nullptr, best, nullptr,
                         d_rows, T, p.L, static_cast<char*>(d_ws), p.bank_of(c, T, S),
                         p.bsum_of(c, T), nullptr, as_stream(stream));
}

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

size_t mw_assign_ws_bytes(int64_t n_pix, int k) {
  return (size_t)kblocks(n_pix) * 2 * k * sizeof(double) + 256;
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
#define MW_AS(CM, KSV)                                                                          \
  {                                                                                             \
    const size_t cent = cent_t_bytes(KSV, CM);                                                  \
    const int nw = assign_waves(k, C);                                                          \
    const size_t lds = cent + nw * assign_wave_bytes(k, CM);                                    \
    if (lds > 160 * 1024) {                                                                     \
      set_error("mw_assign_conf: LDS %zu too large (C=%d k=%d)", lds, C, k);                    \
      return MW_EUNSUPPORTED;                                                                   \
    }                                                                                           \
    hipLaunchKernelGGL((assign_kernel<CM, KSV>), dim3(G), dim3(64 * nw), lds, s, d_img, C,      \
                       d_feat, F, d_a, d_b, d_centers, k, d_mask, n_pix, R, d_label, d_conf, rec); \
  }
#define MW_ASK(CM)             \
  if (k <= 64) MW_AS(CM, 64)   \
  else MW_AS(CM, 128)
  if (C <= 8) { MW_ASK(8) }
  else if (C <= 16) { MW_ASK(16) }
  else if (C <= 32) { MW_ASK(32) }
  else { MW_ASK(64) }
#undef MW_ASK
#undef MW_AS
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
  hipLaunchKernelGGL(rec_reduce_kernel, dim3((2 * k + 31) / 32), dim3(256), 0, as_stream(stream),
                     reinterpret_cast<const double*>(d_ws), kblocks(n_pix), 2 * k, d_dom);
  MW_LAUNCH_CHECK();
  return MW_OK;
}

}  // extern "C"
