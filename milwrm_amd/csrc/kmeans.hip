// k-means kernels of the MILWRM hot path on MI355X (gfx950, wave64).
//
//   kpp_*        sklearn _kmeans_plusplus            _kmeans.py:174-272
//   lloyd_step   lloyd_iter_chunked_dense            _k_means_lloyd.pyx:23-218
//                (+ _inertia_dense, _k_means_common.pyx:94-124)
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

#include "common.h"

namespace mw {

constexpr int kT = 256;          // rows per tile = threads per block
constexpr int kMaxG = 1024;

static inline int kblocks(int64_t n) {
  int64_t tiles = (n + kT - 1) / kT;
  if (tiles < 1) tiles = 1;
  return (int)(tiles < kMaxG ? tiles : kMaxG);
}
static inline int64_t krows(int64_t n) {
  int64_t tiles = (n + kT - 1) / kT;
  int g = kblocks(n);
  return ((tiles + g - 1) / g) * kT;
}

// coalesced copy of `n` consecutive floats into LDS: 16-B vectors issued in
// batches of 8 per thread (all loads in flight before the first LDS store),
// then the tail.
__device__ __forceinline__ void stage(const float* __restrict__ src, int n, float* dst) {
  const int n4 = n >> 2;
  const float4* s4 = reinterpret_cast<const float4*>(src);
  float4* d4 = reinterpret_cast<float4*>(dst);
  const int nt = blockDim.x;
  for (int q0 = threadIdx.x; q0 < n4; q0 += 8 * nt) {
    float4 r[8];
    // unconditional loads from clamped (valid) addresses: a guarded load makes
    // hipcc branch around it and wait vmcnt(0) per element
#pragma unroll
    for (int i = 0; i < 8; ++i) r[i] = s4[min(q0 + i * nt, n4 - 1)];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int q = q0 + i * nt;
      if (q < n4) d4[q] = r[i];
    }
  }
  for (int q = (n4 << 2) + threadIdx.x; q < n; q += nt) dst[q] = src[q];
}

// ===================================================================== kpp
// Workspace layout (bytes, 256-aligned sections):
//   bank[2][T][S] fp64  candidate-min distance arrays (ping-pong per step)
//   bsum[2][T][G] fp64  their per-block sums
//   st: cand[T] i64, chosen[256] i64, best i32
struct KppLayout {
  size_t bank, bsum, st, total;
  int G;
};
static inline size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }
static KppLayout kpp_layout(int64_t S, int T) {
  KppLayout L;
  L.G = kblocks(S);
  L.bank = 0;
  L.bsum = al256(L.bank + 2 * (size_t)T * S * sizeof(double));
  L.st = al256(L.bsum + 2 * (size_t)T * L.G * sizeof(double));
  L.total = al256(L.st + (size_t)(T + 256) * sizeof(int64_t) + 64);
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

// distance of every row to one center row (fp64), block sums.  Writes
// bank[0][0][:] and bsum[0][0][:].
__global__ void __launch_bounds__(256) kpp_init_kernel(const float* __restrict__ X, int64_t S, int F,
                                                       const double* __restrict__ mu,
                                                       const double* __restrict__ inv,
                                                       const float* __restrict__ crow,
                                                       int64_t R, double* __restrict__ out,
                                                       double* __restrict__ bsum,
                                                       int64_t* __restrict__ chosen) {
  extern __shared__ __attribute__((aligned(16))) float s_tile[];
  __shared__ double s_c[256];
  __shared__ double s_red[4];
  const int t = threadIdx.x;
  for (int f = t; f < F; f += 256) s_c[f] = ((double)crow[f] - mu[f]) * inv[f];
  if (blockIdx.x == 0 && t == 0) chosen[0] = -1;  // the caller knows the first index
  const int64_t lo = (int64_t)blockIdx.x * R, hi = min(S, lo + R);
  double acc = 0.0;
  __syncthreads();
  for (int64_t r0 = lo; r0 < hi; r0 += kT) {
    const int nrow = (int)min((int64_t)kT, hi - r0);
    stage(X + r0 * F, nrow * F, s_tile);
    __syncthreads();
    if (t < nrow) {
      double d = 0.0;
      for (int f = 0; f < F; ++f) {
        const double v = ((double)s_tile[t * F + f] - mu[f]) * inv[f] - s_c[f];
        d = fma(v, v, d);
      }
      out[r0 + t] = d;
      acc += d;
    }
    __syncthreads();
  }
  const double tot = block_sum(acc, s_red);
  if (t == 0) bsum[blockIdx.x] = tot;
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

// trial pass: distances to the T candidates, elementwise min with the current
// closest distances, per-block sums.  cur = bank_prev + best*S.
__global__ void __launch_bounds__(256) kpp_trial_kernel(const float* __restrict__ X, int64_t S, int F,
                                                        const double* __restrict__ mu,
                                                        const double* __restrict__ inv,
                                                        const double* __restrict__ bank_prev,
                                                        const int* __restrict__ best, int best_val,
                                                        const int64_t* __restrict__ cand,
                                                        const float* __restrict__ cand_rows, int T,
                                                        int64_t R, double* __restrict__ bank_new,
                                                        double* __restrict__ bsum_new) {
  extern __shared__ __attribute__((aligned(16))) float s_tile[];
  __shared__ double s_c[8 * 64];
  __shared__ double s_red[4];
  const int t = threadIdx.x;
  for (int q = t; q < T * F; q += 256) {
    const int k = q / F, f = q - k * F;
    const float xv = cand_rows ? cand_rows[k * F + f] : X[cand[k] * F + f];
    s_c[k * 64 + f] = ((double)xv - mu[f]) * inv[f];
  }
  const double* cur = bank_prev + (size_t)(best ? *best : best_val) * S;
  const int64_t lo = (int64_t)blockIdx.x * R, hi = min(S, lo + R);
  double acc[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) acc[k] = 0.0;
  __syncthreads();
  for (int64_t r0 = lo; r0 < hi; r0 += kT) {
    const int nrow = (int)min((int64_t)kT, hi - r0);
    stage(X + r0 * F, nrow * F, s_tile);
    __syncthreads();
    if (t < nrow) {
      const int64_t s = r0 + t;
      const double cd = cur[s];
      double d[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) d[k] = 0.0;
      for (int f = 0; f < F; ++f) {
        const double x = ((double)s_tile[t * F + f] - mu[f]) * inv[f];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          if (k < T) {
            const double v = x - s_c[k * 64 + f];
            d[k] = fma(v, v, d[k]);
          }
        }
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        if (k < T) {
          const double m = d[k] < cd ? d[k] : cd;
          bank_new[(size_t)k * S + s] = m;
          acc[k] += m;
        }
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    if (k < T) {
      const double tot = block_sum(acc[k], s_red);
      if (t == 0) bsum_new[(size_t)k * gridDim.x + blockIdx.x] = tot;
    }
  }
}

// ================================================================== Lloyd
// Per-block record: [sums k*F | counts k | changed | inertia] (fp64).
__host__ __device__ inline int lloyd_rec(int k, int F) { return k * F + k + 2; }

template <int FMAX>
__global__ void __launch_bounds__(256) lloyd_kernel(const float* __restrict__ X, int64_t S, int F,
                                                    const float* __restrict__ ga,
                                                    const float* __restrict__ gb,
                                                    const float* __restrict__ gc, int k,
                                                    uint8_t* __restrict__ labels, int mode,
                                                    int64_t R, double* __restrict__ rec) {
  // LDS carve (16-B aligned sections): tile[256*F] f32 | cent[k*FMAX] f32 |
  // seg[256*k] f32 | acc64[k*F] f64 | sorted[256] i32 | lab[256] i32 |
  // wcnt[4*k] i32 | base[k] i32 | cnt[k] i32
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* s_tile = reinterpret_cast<float*>(smem);
  float* s_cent = s_tile + kT * F + ((4 - (kT * F) % 4) % 4);
  float* s_seg = s_cent + k * FMAX;
  double* s_acc = reinterpret_cast<double*>(s_seg + kT * k + ((kT * k) % 2));
  int* s_sorted = reinterpret_cast<int*>(s_acc + k * F);
  int* s_lab = s_sorted + kT;
  int* s_wcnt = s_lab + kT;
  int* s_base = s_wcnt + 4 * k;
  int* s_cnt = s_base + k;
  __shared__ double s_red[4];
  __shared__ float s_a[FMAX], s_b[FMAX];

  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  for (int q = t; q < k * FMAX; q += kT) {
    const int j = q / FMAX, f = q - j * FMAX;
    s_cent[q] = f < F ? gc[j * F + f] : 0.f;
  }
  for (int f = t; f < FMAX; f += kT) {
    s_a[f] = f < F ? ga[f] : 0.f;
    s_b[f] = f < F ? gb[f] : 0.f;
  }
  for (int q = t; q < k * F; q += kT) s_acc[q] = 0.0;
  const int nseg = kT / F;           // segments for the M-step walk
  const int sf = t % F, sg = t / F;  // walk thread → (feature, segment)
  const int64_t lo = (int64_t)blockIdx.x * R, hi = min(S, lo + R);
  double inert = 0.0;
  long long changed = 0;
  long long cnt_tot = 0;
  __syncthreads();
  for (int64_t r0 = lo; r0 < hi; r0 += kT) {
    const int nrow = (int)min((int64_t)kT, hi - r0);
    stage(X + r0 * F, nrow * F, s_tile);
    __syncthreads();
    int lab = -1;
    if (t < nrow) {
      float xr[FMAX];
#pragma unroll
      for (int f = 0; f < FMAX; ++f)
        xr[f] = f < F ? fmaf(s_tile[t * F + f], s_a[f], s_b[f]) : 0.f;
      const int old = labels[r0 + t];
      if (mode == 2) {
        lab = old;
        float d = 0.f;
#pragma unroll
        for (int f = 0; f < FMAX; ++f) {
          const float v = xr[f] - s_cent[lab * FMAX + f];
          d = fmaf(v, v, d);
        }
        inert += (double)d;
      } else {
        float best = 0.f;
        for (int j = 0; j < k; ++j) {
          float d = 0.f;
#pragma unroll
          for (int f = 0; f < FMAX; ++f) {
            const float v = xr[f] - s_cent[j * FMAX + f];
            d = fmaf(v, v, d);
          }
          if (j == 0 || d < best) { best = d; lab = j; }
        }
        changed += (lab != old) ? 1 : 0;
        labels[r0 + t] = (uint8_t)lab;
        if (mode == 1) inert += (double)best;
        if (mode == 0) {
#pragma unroll
          for (int f = 0; f < FMAX; ++f)
            if (f < F) s_tile[t * F + f] = xr[f];  // scaled row for the M-step
        }
      }
    }
    if (mode == 0) {
      // ---- counting sort of the tile's rows by label (wave ballots) ----
      s_lab[t] = lab;
      int my_rank = 0;
      for (int j = 0; j < k; ++j) {
        const unsigned long long m = __ballot(lab == j);
        if (lab == j) my_rank = __popcll(m & ((1ull << lane) - 1ull));
        if (lane == 0) s_wcnt[j * 4 + wid] = __popcll(m);
      }
      __syncthreads();
      if (wid == 0) {
        // lanes j < k (k <= 64): totals, exclusive scan over labels
        int tot = 0;
        if (lane < k) tot = s_wcnt[lane * 4] + s_wcnt[lane * 4 + 1] + s_wcnt[lane * 4 + 2] + s_wcnt[lane * 4 + 3];
        int incl = tot;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
          const int v = __shfl_up(incl, o, 64);
          if (lane >= o) incl += v;
        }
        if (lane < k) {
          s_base[lane] = incl - tot;
          s_cnt[lane] = tot;
        }
      }
      __syncthreads();
      if (lab >= 0) {
        int pos = s_base[lab] + my_rank;
        for (int w = 0; w < wid; ++w) pos += s_wcnt[lab * 4 + w];
        s_sorted[pos] = t;
      }
      __syncthreads();
      // ---- segmented walk: thread (sf, sg) sums feature sf over sorted
      //      positions [sg*L, (sg+1)*L), one store per label run ----
      const int L = (nrow + nseg - 1) / nseg;
      if (sg < nseg) {
        const int p_lo = sg * L, p_hi = min(nrow, p_lo + L);
        if (p_lo < p_hi) {
          int cur = s_lab[s_sorted[p_lo]];
          float acc = 0.f;
          for (int p = p_lo; p < p_hi; ++p) {
            const int row = s_sorted[p];
            const int l = s_lab[row];
            if (l != cur) {
              s_seg[(sg * k + cur) * F + sf] = acc;
              acc = 0.f;
              cur = l;
            }
            acc += s_tile[row * F + sf];
          }
          s_seg[(sg * k + cur) * F + sf] = acc;
        }
      }
      __syncthreads();
      // ---- fold segment partials into the fp64 block accumulators ----
      for (int q = t; q < k * F; q += kT) {
        const int j = q / F, f = q - j * F;
        const int c = s_cnt[j];
        if (c > 0) {
          const int b0 = s_base[j];
          const int g0 = b0 / L, g1 = (b0 + c - 1) / L;
          double sd = 0.0;
          for (int g = g0; g <= g1; ++g) sd += (double)s_seg[(g * k + j) * F + f];
          s_acc[q] += sd;
        }
      }
      __syncthreads();
      // accumulate per-label counts into the record tail (held in registers of
      // threads t < k across tiles)
      if (t < k) cnt_tot += s_cnt[t];
      __syncthreads();
    } else {
      __syncthreads();
    }
  }
  // ---- block record ----
  const int rl = lloyd_rec(k, F);
  double* out = rec + (size_t)blockIdx.x * rl;
  const double ch = block_sum((double)changed, s_red);
  const double in = block_sum(inert, s_red);
  if (mode == 0) {
    for (int q = t; q < k * F; q += kT) out[q] = s_acc[q];
    if (t < k) out[k * F + t] = (double)cnt_tot;
  } else {
    for (int q = t; q < k * F + k; q += kT) out[q] = 0.0;
  }
  if (t == 0) {
    out[k * F + k] = ch;
    out[k * F + k + 1] = in;
  }
}

// fixed-order sum of G per-block records: thread (q, part) sums blocks
// b = part, part+8, ... with 8 independent partial sums, then parts combine
// in order.
__global__ void __launch_bounds__(256) lloyd_reduce_kernel(const double* __restrict__ rec, int G,
                                                           int rl, double* __restrict__ out) {
  __shared__ double s[8][33];
  const int lane = threadIdx.x & 31, part = threadIdx.x >> 5;  // 32 columns x 8 parts
  const int q = blockIdx.x * 32 + lane;
  double acc[4] = {0.0, 0.0, 0.0, 0.0};
  if (q < rl) {
    int b = part;
    for (; b + 24 < G; b += 32) {
#pragma unroll
      for (int u = 0; u < 4; ++u) acc[u] += rec[(size_t)(b + 8 * u) * rl + q];
    }
    for (; b < G; b += 8) acc[0] += rec[(size_t)b * rl + q];
  }
  s[part][lane] = (acc[0] + acc[1]) + (acc[2] + acc[3]);
  __syncthreads();
  if (part == 0 && q < rl) {
    double t = 0.0;
#pragma unroll
    for (int p2 = 0; p2 < 8; ++p2) t += s[p2][lane];
    out[q] = t;
  }
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
// Per-block record: [sum conf k | count k] (fp64).
template <int FMAX>
__global__ void __launch_bounds__(256) assign_kernel(const float* __restrict__ img, int C,
                                                     const int32_t* __restrict__ feat, int F,
                                                     const float* __restrict__ ga,
                                                     const float* __restrict__ gb,
                                                     const float* __restrict__ gc, int k,
                                                     const uint8_t* __restrict__ mask, int64_t n,
                                                     int64_t R, int8_t* __restrict__ lab_out,
                                                     float* __restrict__ conf_out,
                                                     double* __restrict__ rec) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* s_tile = reinterpret_cast<float*>(smem);                       // 256*C
  float* s_cent = s_tile + kT * C + ((4 - (kT * C) % 4) % 4);           // k*FMAX
  double* s_wacc = reinterpret_cast<double*>(s_cent + k * FMAX + ((k * FMAX) % 2));  // 4 waves x 2k
  __shared__ int s_feat[FMAX];
  __shared__ float s_a[FMAX], s_b[FMAX];
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  for (int q = t; q < k * FMAX; q += kT) {
    const int j = q / FMAX, f = q - j * FMAX;
    s_cent[q] = f < F ? gc[j * F + f] : 0.f;
  }
  for (int f = t; f < FMAX; f += kT) {
    s_feat[f] = f < F ? feat[f] : 0;
    s_a[f] = f < F ? ga[f] : 0.f;
    s_b[f] = f < F ? gb[f] : 0.f;
  }
  for (int q = t; q < 8 * k; q += kT) s_wacc[q] = 0.0;
  const int64_t lo = (int64_t)blockIdx.x * R, hi = min(n, lo + R);
  __syncthreads();
  for (int64_t p0 = lo; p0 < hi; p0 += kT) {
    const int np = (int)min((int64_t)kT, hi - p0);
    stage(img + p0 * C, np * C, s_tile);
    __syncthreads();
    int lab = -1;
    float conf = __builtin_nanf("");
    if (t < np) {
      const int64_t p = p0 + t;
      if (mask[p] != 0) {
        float xr[FMAX];
#pragma unroll
        for (int f = 0; f < FMAX; ++f)
          xr[f] = f < F ? fmaf(s_tile[t * C + s_feat[f]], s_a[f], s_b[f]) : 0.f;
        float m1 = 0.f, m2 = __builtin_inff();
        for (int j = 0; j < k; ++j) {
          float d = 0.f;
#pragma unroll
          for (int f = 0; f < FMAX; ++f) {
            const float v = xr[f] - s_cent[j * FMAX + f];
            d = fmaf(v, v, d);
          }
          if (j == 0) { m1 = d; lab = 0; }
          else if (d < m1) { m2 = m1; m1 = d; lab = j; }
          else if (d < m2) { m2 = d; }
        }
        conf = (m2 - m1) / m2;
      }
      lab_out[p] = (int8_t)lab;
      conf_out[p] = conf;
    }
    // per-label sum of confidences and counts (wave-private fp64 slots)
    for (int j = 0; j < k; ++j) {
      const bool mine = lab == j;
      const float v = wave_sum(mine ? conf : 0.f);
      const unsigned long long m = __ballot(mine);
      if (lane == 0 && m) {
        s_wacc[(wid * 2 + 0) * k + j] += (double)v;
        s_wacc[(wid * 2 + 1) * k + j] += (double)__popcll(m);
      }
    }
    __syncthreads();
  }
  double* out = rec + (size_t)blockIdx.x * 2 * k;
  for (int q = t; q < 2 * k; q += kT) {
    const int which = q / k, j = q - which * k;
    double s = 0.0;
    for (int w = 0; w < 4; ++w) s += s_wacc[(w * 2 + which) * k + j];
    out[q] = s;
  }
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

int mw_kpp_init(const float* d_X, int64_t S, int F, const double* d_mu, const double* d_inv,
                const float* d_center_row, int T, void* d_ws, void* stream) {
  MW_CHECK_ARG(d_X && d_mu && d_inv && d_ws && d_center_row, "mw_kpp_init: null pointer");
  MW_CHECK_ARG(S > 0 && F > 0 && F <= 256, "mw_kpp_init: bad shape");
  MW_CHECK_ARG(T >= 1 && T <= 8, "mw_kpp_init: n_local_trials must be in [1, 8]");
  const KppPtrs p = kpp_ptrs(d_ws, S, T);
  hipLaunchKernelGGL(kpp_init_kernel, dim3(p.L.G), dim3(256), (size_t)kT * F * sizeof(float),
                     as_stream(stream), d_X, S, F, d_mu, d_inv, d_center_row, krows(S),
                     p.bank_of(0, T, S), p.bsum_of(0, T), p.st.chosen);
  MW_LAUNCH_CHECK();
  return MW_OK;
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
  hipLaunchKernelGGL(kpp_trial_kernel, dim3(p.L.G), dim3(256), (size_t)kT * F * sizeof(float), s,
                     d_X, S, F, d_mu, d_inv, p.bank_of(c - 1, T, S), p.st.best, 0, p.st.cand,
                     (const float*)nullptr, T, krows(S), p.bank_of(c, T, S), p.bsum_of(c, T));
  MW_LAUNCH_CHECK();
  return MW_OK;
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
  hipLaunchKernelGGL(kpp_trial_kernel, dim3(p.L.G), dim3(256), (size_t)kT * F * sizeof(float),
                     as_stream(stream), d_X, S, F, d_mu, d_inv, p.bank_of(c - 1, T, S),
                     (const int*)nullptr, best, (const int64_t*)nullptr, d_rows, T, krows(S),
                     p.bank_of(c, T, S), p.bsum_of(c, T));
  MW_LAUNCH_CHECK();
  return MW_OK;
}

size_t mw_lloyd_ws_bytes(int64_t S, int k, int F) {
  return (size_t)kblocks(S) * lloyd_rec(k, F) * sizeof(double) + 256;
}

static size_t lloyd_lds(int k, int F, int FMAX) {
  size_t b = 0;
  b += ((size_t)kT * F + 4) * 4;   // tile
  b += (size_t)k * FMAX * 4;       // centers
  b += ((size_t)kT * k + 2) * 4;   // segment partials
  b += (size_t)k * F * 8;          // fp64 accumulators
  b += (size_t)(2 * kT + 6 * k) * 4 + 64;
  return (b + 15) & ~(size_t)15;
}

int mw_lloyd_step(const float* d_X, int64_t S, int F, const float* d_a, const float* d_b,
                  const float* d_centers, int k, uint8_t* d_labels, int mode, void* d_ws,
                  void* stream) {
  MW_CHECK_ARG(d_X && d_a && d_b && d_centers && d_labels && d_ws, "mw_lloyd_step: null pointer");
  MW_CHECK_ARG(S > 0 && F > 0 && k >= 1, "mw_lloyd_step: bad shape");
  MW_CHECK_ARG(mode >= 0 && mode <= 2, "mw_lloyd_step: bad mode");
  if (k > 64 || F > 64 || (mode == 0 && F > kT)) {
    set_error("mw_lloyd_step: k=%d F=%d unsupported (k <= 64, F <= 64)", k, F);
    return MW_EUNSUPPORTED;
  }
  hipStream_t s = as_stream(stream);
  const int G = kblocks(S);
  const int64_t R = krows(S);
  double* rec = reinterpret_cast<double*>(d_ws);
#define MW_LL(FM)                                                                               \
  {                                                                                             \
    const size_t lds = lloyd_lds(k, F, FM);                                                     \
    if (lds > 160 * 1024) {                                                                     \
      set_error("mw_lloyd_step: LDS %zu too large (k=%d F=%d)", lds, k, F);                     \
      return MW_EUNSUPPORTED;                                                                   \
    }                                                                                           \
    hipLaunchKernelGGL(lloyd_kernel<FM>, dim3(G), dim3(kT), lds, s, d_X, S, F, d_a, d_b,        \
                       d_centers, k, d_labels, mode, R, rec);                                   \
  }
  if (F <= 4) MW_LL(4)
  else if (F <= 8) MW_LL(8)
  else if (F <= 16) MW_LL(16)
  else if (F <= 32) MW_LL(32)
  else MW_LL(64)
#undef MW_LL
  MW_LAUNCH_CHECK();
  return MW_OK;
}

int mw_lloyd_reduce(const void* d_ws, int64_t S, int k, int F, double* d_out, void* stream) {
  MW_CHECK_ARG(d_ws && d_out, "mw_lloyd_reduce: null pointer");
  const int rl = lloyd_rec(k, F);
  hipLaunchKernelGGL(lloyd_reduce_kernel, dim3((rl + 31) / 32), dim3(256), 0, as_stream(stream),
                     reinterpret_cast<const double*>(d_ws), kblocks(S), rl, d_out);
  MW_LAUNCH_CHECK();
  return MW_OK;
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
  if (k > 127 || F > 64) {
    set_error("mw_assign_conf: k=%d F=%d unsupported (k <= 127, F <= 64)", k, F);
    return MW_EUNSUPPORTED;
  }
  hipStream_t s = as_stream(stream);
  const int G = kblocks(n_pix);
  const int64_t R = krows(n_pix);
  double* rec = reinterpret_cast<double*>(d_ws);
#define MW_AS(FM)                                                                               \
  {                                                                                             \
    size_t lds = ((size_t)kT * C + 4) * 4 + ((size_t)k * FM + 2) * 4 + (size_t)8 * k * 8 + 16;  \
    lds = (lds + 15) & ~(size_t)15;                                                             \
    if (lds > 160 * 1024) {                                                                     \
      set_error("mw_assign_conf: LDS %zu too large (C=%d k=%d)", lds, C, k);                    \
      return MW_EUNSUPPORTED;                                                                   \
    }                                                                                           \
    hipLaunchKernelGGL(assign_kernel<FM>, dim3(G), dim3(kT), lds, s, d_img, C, d_feat, F, d_a,  \
                       d_b, d_centers, k, d_mask, n_pix, R, d_label, d_conf, rec);              \
  }
  if (F <= 4) MW_AS(4)
  else if (F <= 8) MW_AS(8)
  else if (F <= 16) MW_AS(16)
  else if (F <= 32) MW_AS(32)
  else MW_AS(64)
#undef MW_AS
  MW_LAUNCH_CHECK();
  return MW_OK;
}

int mw_assign_reduce(const void* d_ws, int64_t n_pix, int k, double* d_dom, void* stream) {
  MW_CHECK_ARG(d_ws && d_dom && k >= 1, "mw_assign_reduce: bad args");
  hipLaunchKernelGGL(lloyd_reduce_kernel, dim3((2 * k + 31) / 32), dim3(256), 0, as_stream(stream),
                     reinterpret_cast<const double*>(d_ws), kblocks(n_pix), 2 * k, d_dom);
  MW_LAUNCH_CHECK();
  return MW_OK;
}

}  // extern "C"
