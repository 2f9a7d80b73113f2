// k-means++ seeding (sklearn _kmeans_plusplus, _kmeans.py:174-272) on MI355X.
//
// Per step c = 1..k-1 sklearn draws T = n_local_trials targets u_t * pot,
// locates each in the cumulative sum of the closest squared distances, takes
// the T rows found as candidates, and keeps the one whose trial array
// min(closest, d(x, cand_t)) has the smallest sum.  Here:
//   * one streaming pass per step over the S x F fp32 rows (the scaler folded
//     in, fp64 distances): it first folds the center chosen at the previous
//     step into `cur` (the closest distance of every row, one fp64 array,
//     read and rewritten), then forms the T trial values min(cur, d_t) and
//     keeps only their sums, per 64-row tile and per block.  The trial arrays
//     themselves are never stored: 136 bytes of HBM traffic per row and step
//     (row + cur in, cur out) instead of 160 with T = 4 stored arrays;
//   * the search for step c's targets walks the block sums, then the tile
//     sums of the located block, and recomputes the 64 values of the located
//     tile (same fp64 expression as the pass, so the same bits);
//   * block sums are the potentials; their fixed-order scan gives the
//     selection (argmin, first wins) and the target positions, as before.
// Single device: mw_kpp_init, then per step mw_kpp_step (selection + search
// kernel, candidate table, pass), mw_kpp_indices; no host round trip.
// Row-sharded (milwrm_amd/dist.py DistComm.kpp): mw_kpp_pots, host argmin and
// target ownership, mw_kpp_search, host all-reduce of the candidate rows,
// mw_kpp_trial.  The block grid (kblocks/krows) and every summation order are
// fixed functions of S.
#include <math.h>
#include <stdlib.h>

#include "kmeans_common.h"

namespace mw {

// table (doubles): inv[64] | b[64][8] (feature-major) | mi[64] | cc[8]
constexpr int kKppTab = 64 + 64 * 8 + 64 + 8;
constexpr int kKppTabBytes = kKppTab * 8;

static inline size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }

// Workspace (256-aligned sections):
//   cur   [S] fp64                 closest distance of every row
//   bsum  [2][T][G] fp64           per-block trial sums (ping-pong by step parity)
//   tsum  [2][T][NTL] fp64         per-64-row-tile trial sums (same)
//   tab   [2][kKppTab] fp64        candidate tables (same)
//   st    cand[T] i64, chosen[256] i64, best i32
struct KppLayout {
  size_t cur, bsum, tsum, tab, st, total;
  int G;
  int64_t NTL;
};
static KppLayout kpp_layout(int64_t S, int T) {
  KppLayout L;
  L.G = kblocks(S);
  L.NTL = (S + 63) / 64;
  L.cur = 0;
  L.bsum = al256((size_t)S * sizeof(double));
  L.tsum = al256(L.bsum + 2 * (size_t)T * L.G * sizeof(double));
  L.tab = al256(L.tsum + 2 * (size_t)T * L.NTL * sizeof(double));
  L.st = al256(L.tab + 2 * (size_t)kKppTabBytes);
  L.total = al256(L.st + (size_t)(T + 256) * sizeof(int64_t) + 64);
  return L;
}

struct KppPtrs {
  KppLayout L;
  double *cur, *bsum, *tsum, *tab;
  int64_t *cand, *chosen;
  int* best;
  double* bsum_of(int c, int T) const { return bsum + (size_t)(c & 1) * T * L.G; }
  double* tsum_of(int c, int T) const { return tsum + (size_t)(c & 1) * T * L.NTL; }
  double* tab_of(int c) const { return tab + (size_t)(c & 1) * kKppTab; }
};
static KppPtrs kpp_ptrs(const void* d_ws, int64_t S, int T) {
  KppPtrs p;
  p.L = kpp_layout(S, T);
  char* base = reinterpret_cast<char*>(const_cast<void*>(d_ws));
  p.cur = reinterpret_cast<double*>(base + p.L.cur);
  p.bsum = reinterpret_cast<double*>(base + p.L.bsum);
  p.tsum = reinterpret_cast<double*>(base + p.L.tsum);
  p.tab = reinterpret_cast<double*>(base + p.L.tab);
  p.cand = reinterpret_cast<int64_t*>(base + p.L.st);
  p.chosen = p.cand + T;
  p.best = reinterpret_cast<int*>(p.chosen + 256);
  return p;
}

// Candidate table for the GEMM form of the squared distance, as sklearn's
// _euclidean_distances (|x|^2 - 2 x.c + |c|^2, clipped at 0; pairwise.py):
// per feature inv_f and mi_f = mu_f * inv_f (x'_f = x_f * inv_f - mi_f, one
// rounding), the scaled candidate rows c_t (from `rows`, T x F floats, or
// X[cand[t]]) and cc_t = |c_t|^2; padded features and candidates are 0.  Three
// fp64 FMAs per feature and candidate fewer than (x' - c)^2 chains: the pass
// is partly FMA-bound (the fp64 VALU issues a wave FMA every 4 cycles).
__global__ void __launch_bounds__(512) kpp_prep_kernel(const float* __restrict__ X, int F,
                                                       const double* __restrict__ mu,
                                                       const double* __restrict__ inv,
                                                       const int64_t* __restrict__ cand,
                                                       const float* __restrict__ rows, int T,
                                                       double* __restrict__ tab,
                                                       int64_t* __restrict__ chosen_reset) {
  const int q = threadIdx.x;  // 512 = 64 features x 8 candidates
  const int f = q >> 3, c = q & 7;
  // GEMM form (sklearn's _euclidean_distances): b = the scaled candidate,
  // mi = mu * inv, cc = |c|^2 (features in order)
  double cs = 0.0;
  if (f < F && c < T) {
    const float xv = rows ? rows[c * F + f] : X[cand[c] * F + f];
    cs = ((double)xv - mu[f]) * inv[f];
  }
  tab[64 + f * 8 + c] = cs;
  if (c == 0) {
    tab[f] = f < F ? inv[f] : 0.0;
    tab[576 + f] = f < F ? mu[f] * inv[f] : 0.0;
  }
  __syncthreads();
  if (q < 8) {
    double cc = 0.0;
    for (int g = 0; g < 64; ++g) cc = fma(tab[64 + g * 8 + q], tab[64 + g * 8 + q], cc);
    tab[640 + q] = cc;
  }
  if (chosen_reset && q == 0) chosen_reset[0] = -1;
}

// the fp64 squared distance of one row (features in order) to table column
// col; identical bits to the pass below (which adds exact zeros past F)
__device__ __forceinline__ double kpp_dist_row(const float* __restrict__ x, int F,
                                               const double* __restrict__ tab, int col) {
  double xx = 0.0, dot = 0.0;
  for (int f = 0; f < F; ++f) {
    const double xs = fma((double)x[f], tab[f], -tab[576 + f]);
    xx = fma(xs, xs, xx);
    dot = fma(xs, tab[64 + f * 8 + col], dot);
  }
  const double d = fma(-2.0, dot, xx) + tab[640 + col];
  return d > 0.0 ? d : 0.0;
}

// The pass.  MODE 0 (init, T = 1): cur = d(x, c0).  MODE 1 (step 1): cur as
// is.  MODE 2 (steps >= 2): cur = min(cur, d(x, pending)), the pending
// center being column `best` of the previous step's table.  Then the trial
// values m_t = min(cur, d(x, cand_t)): their sums per tile (wave sum) and per
// block (lanes over their tiles, then the block sum).  Waves stream 64-row
// tiles (buffer loads, next tile and its cur in flight) transposed through
// LDS; the table comes through scalar loads, so registers hold only the
// stream and the T + 2 chains: <= 128 VGPRs, 4 waves per SIMD (FMAX = 64:
// the 16-KB tiles allow 2 waves per SIMD, so the registers may grow instead
// of spilling).  All LDS is dynamic (16-B aligned).
template <int FMAX, int T, int MODE>
__global__ void __launch_bounds__(256, FMAX == 64 ? 2 : 4) kpp_pass_kernel(
    const float* __restrict__ X, int64_t S, int F, const double* __restrict__ tab,
    const double* __restrict__ tab_prev, const int* __restrict__ best, int best_val,
    double* __restrict__ cur, int64_t R, int64_t NTL, double* __restrict__ bsum_new,
    double* __restrict__ tsum_new) {
  constexpr int NV = FMAX / 4;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  double* s_red = reinterpret_cast<double*>(smem);  // [4] block-sum scratch
  const int t = threadIdx.x, lane = t & 63, nw = blockDim.x >> 6;
  const int wid = __builtin_amdgcn_readfirstlane(t >> 6);
  // per-wave tile of 64 rows x FMAX floats; FMAX = 64 (FS): 64 rows x F
  // floats (+4: the pair read past an odd-F tile's last row, kept finite) and
  // the feature loop stops at F, so at F = 50 three blocks fit a CU instead
  // of two (at F <= 32 the fixed-trip loop is faster: config 2 +0.4 ms)
  constexpr bool FS = FMAX == 64;
  const int tstride = FS ? 64 * F + 4 : 64 * FMAX;
  const int fend = FS ? F : FMAX;
  float* s_tile = reinterpret_cast<float*>(smem + 64) + (size_t)wid * tstride;
  if (FS && lane < 4) s_tile[64 * F + lane] = 0.f;

  const int64_t lo = (int64_t)blockIdx.x * R, hi = min(S, lo + R);
  const int ntile = hi > lo ? (int)((hi - lo + 63) / 64) : 0;
  const int64_t total = S * (int64_t)F, n4 = total >> 2;
  const __amdgpu_buffer_rsrc_t rx = make_rsrc(X + lo * F, (S - lo) * F * 4);
  const __amdgpu_buffer_rsrc_t rc = make_rsrc(cur + lo, MODE == 0 ? 0 : (hi - lo) * 8);
  const int tile_bytes = 64 * F * 4;
  double acc[T];
#pragma unroll
  for (int c = 0; c < T; ++c) acc[c] = 0.0;
  __syncthreads();

  // candidate table: scalar loads from global memory inside the feature loop
  // (uniform addresses; the loop is not fully unrolled, so hipcc cannot hoist
  // the whole table into registers).  Broadcast LDS reads of it cost ~15%:
  // the LDS pipe is shared by the CU's four SIMDs and also carries the tile.
  const double* tb = tab;
  const int pb = MODE == 2 ? (best ? *best : best_val) : 0;
  const double* tp = tab_prev + 64 + pb;
  const double tcc = MODE == 2 ? tab_prev[640 + pb] : 0.0;
  f4v v[NV];
  double cur_next = 0.0;
  auto fetch = [&](int tt) {
    tt = tt < ntile ? tt : ntile - 1;
    if (MODE != 0)
      cur_next = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rc, lane * 8, tt * 512, 0));
#pragma unroll
    for (int i = 0; i < NV; ++i)  // only the vectors that hold the tile's 64 x F floats
      if (!FS || i * 1024 < tile_bytes)
        v[i] = __builtin_bit_cast(f4v, __builtin_amdgcn_raw_buffer_load_b128(rx, lane * 16 + i * 1024, tt * tile_bytes, 0));
  };
  int tc = wid;
  if (tc < ntile) fetch(tc);
  for (; tc < ntile; tc += nw) {
    const int64_t r0 = lo + (int64_t)tc * 64;
    const int nrow = (int)min((int64_t)64, hi - r0);
    {
      f4v* s4 = reinterpret_cast<f4v*>(s_tile);
#pragma unroll
      for (int i = 0; i < NV; ++i)
        if (!FS || (lane + i * 64) * 16 < tile_bytes) s4[lane + i * 64] = v[i];
    }
    wt_tail(nrow * F, r0 * F, n4, X, total, s_tile, lane);
    double cd = cur_next;
    fetch(tc + nw);
    const float* xr = s_tile + lane * F;
    double d[T], dp = 0.0;
#pragma unroll
    for (int c = 0; c < T; ++c) d[c] = 0.0;
    double xx = 0.0, dot[T], dotp = 0.0;
#pragma unroll
    for (int c = 0; c < T; ++c) dot[c] = 0.0;
    auto feat = [&](double xv, int f) {  // past F: inv = mi = c = 0, exact zeros
      const double xs = fma(xv, tb[f], -tb[576 + f]);
      xx = fma(xs, xs, xx);
      if (MODE == 2) dotp = fma(xs, tp[f * 8], dotp);
#pragma unroll
      for (int c = 0; c < T; ++c) dot[c] = fma(xs, tb[64 + f * 8 + c], dot[c]);
    };
    if ((F & 1) == 0) {
      // feature pairs as 8-byte LDS reads (conflict-free for 16 lanes; the
      // 4-byte reads of rows F floats apart conflict 2-way for even F)
      // the table entries of the next feature pair are loaded (scalar loads)
      // while this pair computes: the scalar-cache latency is not exposed
      // once per pair (same operations in the same order: same bits; 535 ->
      // 520 us per step pass at config 2, tools/gpu/kvariants.sh)
      struct TabF { double inv, mi, c[T], pend; };
      auto ld = [&](int f) {
        TabF r;
        const int g = f < 64 ? f : 63;
        r.inv = tb[g];
        r.mi = tb[576 + g];
#pragma unroll
        for (int c = 0; c < T; ++c) r.c[c] = tb[64 + g * 8 + c];
        r.pend = MODE == 2 ? tp[g * 8] : 0.0;
        return r;
      };
      auto featt = [&](double xv, const TabF& q) {
        const double xs = fma(xv, q.inv, -q.mi);
        xx = fma(xs, xs, xx);
        if (MODE == 2) dotp = fma(xs, q.pend, dotp);
#pragma unroll
        for (int c = 0; c < T; ++c) dot[c] = fma(xs, q.c[c], dot[c]);
      };
      if constexpr (FMAX >= 64) {  // (FMAX = 64: the pipelined form below)
        // the row's feature pairs into registers first (one LDS wait), then
        // per pair: wait for the table loads issued one pair earlier (nothing
        // else is outstanding on the shared LDS/scalar counter), issue the next
        // pair's table loads, compute from registers only, so the scalar loads
        // land under the FMAs instead of being waited for with each LDS read
        f2v xrow[FMAX / 2];
#pragma unroll
        for (int p = 0; p < FMAX / 2; ++p)
          xrow[p] = 2 * p < fend ? *reinterpret_cast<const f2v*>(xr + 2 * p) : f2v{0.f, 0.f};
        TabF t0 = ld(0), t1 = ld(1);
#pragma unroll
        for (int p = 0; p < FMAX / 2; ++p) {
          if (2 * p >= fend) break;  // features past F add exact zeros
          __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): t0, t1 (and the row reads) landed
          const TabF n0 = ld(2 * p + 2), n1 = ld(2 * p + 3);
          featt((double)xrow[p].x, t0);
          featt((double)xrow[p].y, t1);
          t0 = n0;
          t1 = n1;
        }
        // (config-5 slice, F = 50: k-means++ 4 ms faster per slide at 2 waves
        // per SIMD; at F <= 32 it measured neutral, the form below stays)
      } else {
        TabF t0 = ld(0), t1 = ld(1);
        for (int f = 0; f < fend; f += 2) {  // features past F add exact zeros
          const TabF n0 = ld(f + 2), n1 = ld(f + 3);
          const f2v x2 = *reinterpret_cast<const f2v*>(xr + f);
          featt((double)x2.x, t0);
          featt((double)x2.y, t1);
          t0 = n0;
          t1 = n1;
        }
      }
    } else {
#pragma unroll 4
      for (int f = 0; f < fend; ++f) feat((double)xr[f], f);
    }
#pragma unroll
    for (int c = 0; c < T; ++c) {
      const double e = fma(-2.0, dot[c], xx) + tb[640 + c];
      d[c] = e > 0.0 ? e : 0.0;
    }
    if (MODE == 2) {
      const double e = fma(-2.0, dotp, xx) + tcc;
      dp = e > 0.0 ? e : 0.0;
    }
    const bool valid = lane < nrow;
    const int64_t row = r0 + lane;
    if (MODE == 0) cd = d[0];
    if (MODE == 2) cd = cd < dp ? cd : dp;
    if (MODE != 1 && valid) cur[row] = cd;
#pragma unroll
    for (int c = 0; c < T; ++c) {
      const double m = MODE == 0 ? d[0] : (cd < d[c] ? cd : d[c]);
      const double mv = valid ? m : 0.0;
      acc[c] += mv;
      const double ts = wave_sum_lane0(mv);  // lane 0 stores it
      if (lane == 0) tsum_new[(size_t)c * NTL + (r0 >> 6)] = ts;
    }
  }
#pragma unroll
  for (int c = 0; c < T; ++c) {
    const double tot = block_sum(acc[c], s_red);
    if (t == 0) bsum_new[(size_t)c * gridDim.x + blockIdx.x] = tot;
  }
}

// inclusive scan of G block sums in LDS (fixed order; shared by selection,
// search and mw_kpp_pots so that the potential used for the targets equals
// the selected one)
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

// the same scan of n <= 4 arrays (array i at bs + i * G) at once: each
// array gets the additions scan_blocks gives it, in the same order, under
// one barrier pair per step for all of them (the search kernel's selection
// scanned its T arrays one after another: 20 barriers each)
__device__ __forceinline__ void scan_blocks4(const double* __restrict__ bs, int n, int G, double (*s)[1024]) {
  const int t = threadIdx.x;  // blockDim = 1024 >= G
#pragma unroll
  for (int i = 0; i < 4; ++i) s[i][t] = (i < n && t < G) ? bs[(size_t)i * G + t] : 0.0;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {
    double v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = (i < n && t >= o) ? s[i][t - o] : 0.0;
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (i < n) s[i][t] += v[i];
    __syncthreads();
  }
}

__global__ void __launch_bounds__(1024) kpp_pots_kernel(const double* __restrict__ bsum_cur,
                                                        int n_cur, int G, double* __restrict__ pots) {
  __shared__ double s[1024];
  for (int i = 0; i < n_cur; ++i) {
    scan_blocks(bsum_cur + (size_t)i * G, G, s);
    if (threadIdx.x == 0) pots[i] = s[G - 1];
    __syncthreads();
  }
}

// Selection of the finished step's best array (argmin of the potentials,
// first wins; skipped when the host gives it), then the search for this
// step's T targets (u_t * pot, or the host's local targets, < 0 = not on this
// shard), one wave per target: block by the block prefix, tile by a chunked
// scan of the block's tile sums, row by the recomputed values of the tile.
// The array searched is min(cur, d(x, pending)) (pending: column `best` of
// tab_prev; none at step 1, where it is cur).
__global__ void __launch_bounds__(1024) kpp_search_kernel(
    const float* __restrict__ X, int F, const double* __restrict__ cur,
    const double* __restrict__ tab_prev, int has_pend, const double* __restrict__ bsum_cur,
    const double* __restrict__ tsum_cur, int n_cur, int64_t S, int G, int64_t R, int64_t NTL,
    int c_done, double u0, double u1, double u2, double u3, double u4, double u5, double u6,
    double u7, int T, int64_t* __restrict__ cand, int64_t* __restrict__ chosen,
    int* __restrict__ best_out, int best_given, const double* __restrict__ rv_given) {
  __shared__ double s4[4][1024];
  __shared__ double s_pot[8];
  __shared__ double s_row[8][64];
  __shared__ int s_best;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  int g_last = -1;  // first array of the group whose scans s4 holds
  if (best_given >= 0) {
    if (t == 0) { s_best = best_given; *best_out = best_given; }
    __syncthreads();
  } else {
    for (int g0 = 0; g0 < n_cur; g0 += 4) {
      scan_blocks4(bsum_cur + (size_t)g0 * G, min(4, n_cur - g0), G, s4);
      if (t < 4 && g0 + t < n_cur) s_pot[g0 + t] = s4[t][G - 1];
      __syncthreads();
      g_last = g0;
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
  // the best array's scan: still in s4 when its group was the last scanned
  const double* s;
  if (g_last >= 0 && b >= g_last && b < g_last + 4) {
    s = s4[b - g_last];
  } else {
    scan_blocks4(bsum_cur + (size_t)b * G, 1, G, s4);
    s = s4[0];
  }
  if (w >= T) return;  // one wave per target from here on (no more barriers)
  const double pot = s[G - 1];
  const double us[8] = {u0, u1, u2, u3, u4, u5, u6, u7};
  const double rv = rv_given ? rv_given[w] : us[w] * pot;
  if (rv < 0.0) {  // target not on this shard
    if (lane == 0) cand[w] = -1;
    return;
  }
  // 1) first block whose inclusive prefix reaches rv (else the last block)
  int blk = G - 1;
  for (int i = lane; i < G; i += 64) {
    const double prev = i > 0 ? s[i - 1] : 0.0;
    if (s[i] >= rv && (i == 0 || prev < rv)) blk = min(blk, i);
  }
  for (int o = 32; o > 0; o >>= 1) blk = min(blk, __shfl_xor(blk, o, 64));
  const double base = blk > 0 ? s[blk - 1] : 0.0;
  const int64_t lo = (int64_t)blk * R, hi = min(S, lo + R);
  int64_t idx = hi - 1;  // rounding fallback: the block's last row
  // 2) chunked scan of the block's tile sums: lane l owns tiles [t0 + l*per, ...)
  const int64_t t0 = lo >> 6, t1 = (hi + 63) >> 6, ntl = t1 - t0;
  const int64_t per = (ntl + 63) / 64;
  const int64_t c_lo = t0 + lane * per, c_hi = min(t1, c_lo + per);
  const double* ts = tsum_cur + (size_t)b * NTL;
  double part = 0.0;
  for (int64_t i = c_lo; i < c_hi; ++i) part += ts[i];
  double incl = part;
  for (int o = 1; o < 64; o <<= 1) {
    const double v = __shfl_up(incl, o, 64);
    if (lane >= o) incl += v;
  }
  double excl = __shfl_up(incl, 1, 64);
  if (lane == 0) excl = 0.0;
  const bool hit = c_lo < c_hi && base + incl >= rv && (lane == 0 || base + excl < rv);
  const uint64_t mask = __ballot(hit);
  if (mask) {
    const int q = __builtin_ctzll(mask);
    // 3) the tile inside chunk q (sequential over its tiles)
    const int64_t q_lo = t0 + q * per, q_hi = min(t1, q_lo + per);
    double r2 = base + __shfl(excl, q, 64);
    int64_t tile = q_hi - 1;
    for (int64_t i = q_lo; i < q_hi; ++i) {
      if (r2 + ts[i] >= rv) { tile = i; break; }
      r2 += ts[i];
    }
    // r2 = prefix before `tile` (or before the chunk's last tile on fallback)
    if (tile == q_hi - 1) {
      r2 = base + __shfl(excl, q, 64);
      for (int64_t i = q_lo; i < tile; ++i) r2 += ts[i];
    }
    // 4) the tile's values, recomputed, then the first row reaching rv
    const int64_t row = tile * 64 + lane;
    double a = 0.0;
    if (row < hi) {
      a = cur[row];
      if (has_pend) {
        const double dp = kpp_dist_row(X + row * F, F, tab_prev, b);
        a = a < dp ? a : dp;
      }
    }
    s_row[w][lane] = a;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    if (lane == 0) {
      const int nrow = (int)min((int64_t)64, hi - tile * 64);
      idx = tile * 64 + nrow - 1;
      double r = r2;
      for (int i = 0; i < nrow; ++i) {
        r += s_row[w][i];
        if (r >= rv) { idx = tile * 64 + i; break; }
      }
    }
  }
  if (lane == 0) {
    if (idx > S - 1) idx = S - 1;
    if (idx < 0) idx = 0;
    cand[w] = idx;
  }
}

// candidate table, then the pass with the (FMAX, T, MODE) instance
static int kpp_pass_launch(const float* X, int64_t S, int F, const double* mu, const double* inv,
                           const KppPtrs& p, int c, const int* best, int best_val,
                           const int64_t* cand, const float* rows, int T, int64_t* chosen_reset,
                           hipStream_t s) {
  double* tab = p.tab_of(c);
  hipLaunchKernelGGL(kpp_prep_kernel, dim3(1), dim3(512), 0, s, X, F, mu, inv, cand, rows, T, tab,
                     chosen_reset);
  MW_LAUNCH_CHECK();
  const int FM = F <= 8 ? 8 : F <= 16 ? 16 : F <= 32 ? 32 : 64;
  const size_t lds = 64 + (size_t)4 * (FM == 64 ? 64 * F + 4 : 64 * FM) * sizeof(float);  // the pass's tiles
  const int mode = c == 0 ? 0 : c == 1 ? 1 : 2;
  const double* tab_prev = c >= 1 ? p.tab_of(c - 1) : nullptr;
  double* bs = p.bsum_of(c, T);
  double* tsm = p.tsum_of(c, T);
  const int64_t R = krows(S);
#define MW_KP(FMV, TV, MV)                                                                      \
  hipLaunchKernelGGL((kpp_pass_kernel<FMV, TV, MV>), dim3(p.L.G), dim3(256), lds, s, X, S, F, tab, \
                     tab_prev, best, best_val, p.cur, R, p.L.NTL, bs, tsm)
#define MW_KPM(FMV, TV) \
  if (mode == 1) MW_KP(FMV, TV, 1); else MW_KP(FMV, TV, 2);
#define MW_KPT(FMV)                                                                        \
  if (mode == 0) { MW_KP(FMV, 1, 0); }                                                     \
  else switch (T) {                                                                        \
    case 1: MW_KPM(FMV, 1) break; case 2: MW_KPM(FMV, 2) break;                            \
    case 3: MW_KPM(FMV, 3) break; case 4: MW_KPM(FMV, 4) break;                            \
    case 5: MW_KPM(FMV, 5) break; case 6: MW_KPM(FMV, 6) break;                            \
    case 7: MW_KPM(FMV, 7) break; default: MW_KPM(FMV, 8) break;                           \
  }
  if (FM == 8) { MW_KPT(8) }
  else if (FM == 16) { MW_KPT(16) }
  else if (FM == 32) { MW_KPT(32) }
  else { MW_KPT(64) }
#undef MW_KPT
#undef MW_KPM
#undef MW_KP
  MW_LAUNCH_CHECK();
  return MW_OK;
}

// T: the workspace's n_local_trials; n_tgt: targets to search (0 = selection only)
static int kpp_search_launch(const float* X, int64_t S, int F, const KppPtrs& p, int c, int n_cur,
                             const double* u, int T, int n_tgt, int best_given,
                             const double* rv_given, hipStream_t s) {
  hipLaunchKernelGGL(kpp_search_kernel, dim3(1), dim3(1024), 0, s, X, F, p.cur, p.tab_of(c - 1),
                     c >= 2 ? 1 : 0, p.bsum_of(c - 1, T), p.tsum_of(c - 1, T), n_cur, S, p.L.G,
                     krows(S), p.L.NTL, best_given >= 0 ? 0 : c - 1, u[0], u[1], u[2], u[3], u[4],
                     u[5], u[6], u[7], n_tgt, p.cand, p.chosen, p.best, best_given, rv_given);
  MW_LAUNCH_CHECK();
  return MW_OK;
}

}  // namespace mw

using namespace mw;

extern "C" {

size_t mw_kpp_ws_bytes(int64_t S, int T) { return kpp_layout(S, T).total; }

int mw_kpp_init(const float* d_X, int64_t S, int F, const double* d_mu, const double* d_inv,
                const float* d_center_row, int T, void* d_ws, void* stream) {
  MW_CHECK_ARG(d_X && d_mu && d_inv && d_ws && d_center_row, "mw_kpp_init: null pointer");
  MW_CHECK_ARG(S > 0 && F > 0 && F <= 64, "mw_kpp_init: bad shape (F <= 64)");
  MW_CHECK_ARG(T >= 1 && T <= 8, "mw_kpp_init: n_local_trials must be in [1, 8]");
  const KppPtrs p = kpp_ptrs(d_ws, S, T);
  return kpp_pass_launch(d_X, S, F, d_mu, d_inv, p, 0, nullptr, 0, nullptr, d_center_row, 1,
                         p.chosen, as_stream(stream));
}

int mw_kpp_step(const float* d_X, int64_t S, int F, const double* d_mu, const double* d_inv, int c,
                const double* h_u, int T, void* d_ws, void* stream) {
  MW_CHECK_ARG(d_X && d_mu && d_inv && d_ws && h_u, "mw_kpp_step: null pointer");
  MW_CHECK_ARG(c >= 1 && c < 256, "mw_kpp_step: center index %d out of range", c);
  MW_CHECK_ARG(T >= 1 && T <= 8 && F > 0 && F <= 64, "mw_kpp_step: T in [1,8], F <= 64 required");
  const KppPtrs p = kpp_ptrs(d_ws, S, T);
  double u[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int i = 0; i < T; ++i) u[i] = h_u[i];
  hipStream_t s = as_stream(stream);
  // select the previous step's best (c >= 2), then locate this step's candidates
  const int rc = kpp_search_launch(d_X, S, F, p, c, c == 1 ? 1 : T, u, T, T, -1, nullptr, s);
  if (rc != MW_OK) return rc;
  return kpp_pass_launch(d_X, S, F, d_mu, d_inv, p, c, p.best, 0, p.cand, nullptr, T, nullptr, s);
}

int mw_kpp_indices(const void* d_ws, int64_t S, int T, int k, int64_t* d_idx_out, void* stream) {
  MW_CHECK_ARG(d_ws && d_idx_out && k >= 1 && k <= 256, "mw_kpp_indices: bad args");
  const KppPtrs p = kpp_ptrs(d_ws, S, T);
  hipStream_t s = as_stream(stream);
  if (k >= 2) {  // final selection among the last step's T candidates
    const double u[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const int rc = kpp_search_launch(nullptr, S, 0, p, k, T, u, T, 0, -1, nullptr, s);
    if (rc != MW_OK) return rc;
  }
  MW_HIP(hipMemcpyAsync(d_idx_out, p.chosen, sizeof(int64_t) * k, hipMemcpyDeviceToDevice, s));
  return MW_OK;
}

int mw_kpp_pots(const void* d_ws, int64_t S, int T, int c, double* d_pots, void* stream) {
  MW_CHECK_ARG(d_ws && d_pots && c >= 1 && T >= 1 && T <= 8, "mw_kpp_pots: bad args");
  const KppPtrs p = kpp_ptrs(d_ws, S, T);
  hipLaunchKernelGGL(kpp_pots_kernel, dim3(1), dim3(1024), 0, as_stream(stream), p.bsum_of(c - 1, T),
                     c == 1 ? 1 : T, p.L.G, d_pots);
  MW_LAUNCH_CHECK();
  return MW_OK;
}

int mw_kpp_search(const float* d_X, int64_t S, int F, void* d_ws, int T, int c, int best,
                  const double* d_rv, int64_t* d_local_idx, void* stream) {
  MW_CHECK_ARG(d_X && d_ws && d_rv && d_local_idx, "mw_kpp_search: null pointer");
  MW_CHECK_ARG(c >= 1 && T >= 1 && T <= 8 && F > 0 && F <= 64 && best >= 0 && best < (c == 1 ? 1 : T),
               "mw_kpp_search: bad args (c=%d best=%d)", c, best);
  const KppPtrs p = kpp_ptrs(d_ws, S, T);
  hipStream_t s = as_stream(stream);
  const double u[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const int rc = kpp_search_launch(d_X, S, F, p, c, c == 1 ? 1 : T, u, T, T, best, d_rv, s);
  if (rc != MW_OK) return rc;
  MW_HIP(hipMemcpyAsync(d_local_idx, p.cand, sizeof(int64_t) * T, hipMemcpyDeviceToDevice, s));
  return MW_OK;
}

int mw_kpp_trial(const float* d_X, int64_t S, int F, const double* d_mu, const double* d_inv, int c,
                 int best, const float* d_rows, int T, void* d_ws, void* stream) {
  MW_CHECK_ARG(d_X && d_mu && d_inv && d_rows && d_ws, "mw_kpp_trial: null pointer");
  MW_CHECK_ARG(c >= 1 && T >= 1 && T <= 8 && F > 0 && F <= 64 && best >= 0 && best < (c == 1 ? 1 : T),
               "mw_kpp_trial: bad args");
  const KppPtrs p = kpp_ptrs(d_ws, S, T);
  return kpp_pass_launch(d_X, S, F, d_mu, d_inv, p, c, nullptr, best, nullptr, d_rows, T, nullptr,
                         as_stream(stream));
}

}  // extern "C"
