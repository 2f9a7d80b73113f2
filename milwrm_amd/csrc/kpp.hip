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

// The tile sums of a pass's T trial values (lane = row of the 64-row tile):
// trial c's at ts[c * NTL] (wave_sum_lane0's bits; four trials at a time by
// register exchanges instead of LDS-permute chains, wave_sum4_rows)
template <int T>
__device__ __forceinline__ void kpp_tile_sums(const double (&mv)[T], int lane, double* __restrict__ ts,
                                              int64_t NTL) {
  if constexpr (T == 1) {
    const double v = wave_sum_lane0(mv[0]);  // lane 0 stores it
    if (lane == 0) ts[0] = v;
  } else {
#pragma unroll
    for (int g = 0; g < T; g += 4) {
      const double v = wave_sum4_rows(mv[g], g + 1 < T ? mv[g + 1] : 0.0, g + 2 < T ? mv[g + 2] : 0.0,
                                      g + 3 < T ? mv[g + 3] : 0.0);
      const int c = g + (lane >> 4);
      if ((lane & 15) == 0 && c < T) ts[(size_t)c * NTL] = v;
    }
  }
}

// The squared distances (GEMM form, fp64) of the lane's row xr (F floats in
// LDS, features past F read as the next row's values times exact-zero table
// entries) to the T candidates of table tb and (MODE 2) to the pending
// center (column tp, |c|^2 tcc), features 0..fend-1 in order: the FMAX <= 32
// form of the pass (kpp_dist_row's expression per column)
template <int T, int MODE>
__device__ __forceinline__ void kpp_row_dists(const float* __restrict__ xr, int F, int fend,
                                              const double* __restrict__ tb, const double* __restrict__ tp,
                                              double tcc, double (&d)[T], double& dp) {
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
    // 4-byte reads of rows F floats apart conflict 2-way for even F); the
    // table entries of the next feature pair are loaded (scalar loads) while
    // this pair computes: the scalar-cache latency is not exposed once per
    // pair (same operations in the same order: same bits; 535 -> 520 us per
    // step pass at config 2, tools/gpu/kvariants.sh)
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
    TabF t0 = ld(0), t1 = ld(1);
    for (int f = 0; f < fend; f += 2) {  // features past F add exact zeros
      const TabF n0 = ld(f + 2), n1 = ld(f + 3);
      const f2v x2 = *reinterpret_cast<const f2v*>(xr + f);
      featt((double)x2.x, t0);
      featt((double)x2.y, t1);
      t0 = n0;
      t1 = n1;
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
      cur_next = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rc, lane * 8, tt * 512, kStreamAux));
#pragma unroll
    for (int i = 0; i < NV; ++i)  // only the vectors that hold the tile's 64 x F floats
      if (!FS || i * 1024 < tile_bytes)
        v[i] = __builtin_bit_cast(f4v, __builtin_amdgcn_raw_buffer_load_b128(rx, lane * 16 + i * 1024, tt * tile_bytes, kStreamAux));
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
    if constexpr (FMAX < 64) {
      kpp_row_dists<T, MODE>(xr, F, fend, tb, tp, tcc, d, dp);
    } else {
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
      {  // FMAX = 64: the pipelined form
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
        // per SIMD; at F <= 32 it measured neutral: kpp_row_dists' form)
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
    }
    const bool valid = lane < nrow;
    const int64_t row = r0 + lane;
    if (MODE == 0) cd = d[0];
    if (MODE == 2) cd = cd < dp ? cd : dp;
    if (MODE != 1 && valid) cur[row] = cd;
    double mv[T];
#pragma unroll
    for (int c = 0; c < T; ++c) {
      const double m = MODE == 0 ? d[0] : (cd < d[c] ? cd : d[c]);
      mv[c] = valid ? m : 0.0;
      acc[c] += mv[c];
    }
    kpp_tile_sums<T>(mv, lane, tsum_new + (r0 >> 6), NTL);
  }
#pragma unroll
  for (int c = 0; c < T; ++c) {
    const double tot = block_sum(acc[c], s_red);
    if (t == 0) bsum_new[(size_t)c * gridDim.x + blockIdx.x] = tot;
  }
}

// ---- the last step's pass with the first Lloyd E-step folded in ----------
// (single device, F <= 32, T <= 4; fit.cpp calls it through mw_kpp_step_fold
// for the last k-means++ step of a seeded fit).  Besides the step's trial
// sums (the pass above, bit for bit: the same four waves take the same tiles
// in the same order), every row gets lloyd_pass kFirst's E-step against the
// k - 1 centers chosen so far (its fp32 chains: nearest_centers) and its
// distances e_t to the T candidates: the base label, ub = sqrt(m1), lb =
// sqrt(min(m2, min_t e_t)) (a lower bound of the second-closest distance
// whichever candidate wins), the bits e_t < m1 (the row moves to the new
// center k - 1 if candidate t wins; ties keep the lower index) and the base
// cluster sums (kFirst's one-hot fp64 MFMA form, exact fixed point) in Lloyd
// block records.  After the final selection the winner's moved rows are
// listed (mw_lloyd_list_moved) and a Lloyd list pass over the k final
// centers moves them: labels, sums and counts are those of the kFirst pass
// over the final centers, bit for bit (integer sums; the listed rows are
// recomputed with the same chains; the bounds only steer which rows are
// read).  cur is not written (no later step reads it).
//
// 512 threads: waves 0-3 are the k-means++ pass's four waves (tiles w, w + 4,
// ... of the block, prefetched one ahead in registers), waves 4-7 run the
// E-step of the tile their partner w - 4 staged, from a double-buffered LDS
// tile: one LDS barrier per round, two blocks (16 waves) per CU.
struct KppFoldArg {
  const float* a32;   // fp32 scaler (x' = x a + b), as the Lloyd passes
  const float* b32;
  const int* qexp;    // fixed-point exponents of the M-step
  const f2v* gT;      // pair-major centers [16 pairs][kFoldKS slots]: base 0..k-2, candidates kFoldSlot..
  int kb;             // k - 1 base centers
  uint8_t* labels;
  float* ub;
  float* lb;
  uint8_t* moved;     // per row: bit t = moves to the new center if candidate t wins
  double* rec;        // Lloyd block records [G][lloyd_rec(k, F)] (k = kb + 1)
};
constexpr int kFoldSlot = 16;  // center-image slot of candidate 0
constexpr int kFoldKS = 32;    // center-image slots per feature pair
// per-wave row tile: 64 x F floats and the pairs the scaled row reads past
// them (lane 63 reads up to 63 F + 31), zeroed
__host__ __device__ inline int kpp_fold_tstride(int F) { return ((63 * F + 36) + 3) & ~3; }
// LDS: block-sum scratch | 2 x 4 tiles | center image | scaler, exponents,
// counts, per-wave labels | int64 base sums (16-byte sections)
__host__ __device__ inline size_t kpp_fold_lds(int k, int F) {
  return 64 + (size_t)8 * kpp_fold_tstride(F) * 4 + 16 * kFoldKS * 8 + 32 * 4 * 3 + 64 * 4 + 4 * 64 * 4 +
         (((size_t)k * F * 8 + 15) & ~(size_t)15);
}
constexpr size_t kFoldLdsMax = 80 * 1024;  // two blocks per CU

__device__ __forceinline__ void fold_lds_barrier() {  // LDS hand-off only (no vmcnt drain of the prefetch)
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

template <int T>
__global__ void __launch_bounds__(512, 4) kpp_fold_kernel(
    const float* __restrict__ X, int64_t S, int F, const double* __restrict__ tab,
    const double* __restrict__ tab_prev, const int* __restrict__ best, const double* __restrict__ cur,
    int64_t R, int64_t NTL, double* __restrict__ bsum_new, double* __restrict__ tsum_new, KppFoldArg fa) {
  static_assert(T >= 1 && T <= 4, "fold: T <= 4");
  constexpr int NV = 8;  // 1-KB pieces of a 64 x 32-float tile load
  extern __shared__ __attribute__((aligned(16))) char smem[];
  double* s_red = reinterpret_cast<double*>(smem);  // [8] block-sum scratch
  const int t = threadIdx.x, lane = t & 63;
  const int wid = __builtin_amdgcn_readfirstlane(t >> 6);
  const int w4 = wid & 3;
  const int tstride = kpp_fold_tstride(F);
  float* s_tiles = reinterpret_cast<float*>(smem + 64);  // [round parity][wave][tstride]
  char* fx = smem + 64 + (size_t)8 * tstride * 4;
  f2v* s_cT = reinterpret_cast<f2v*>(fx);
  fx += 16 * kFoldKS * 8;
  float* s_a = reinterpret_cast<float*>(fx);
  float* s_b = s_a + 32;
  int* s_e = reinterpret_cast<int*>(s_b + 32);
  int* s_cnt = s_e + 32;
  int* s_lab = s_cnt + 64 + w4 * 64;
  unsigned long long* s_acc = reinterpret_cast<unsigned long long*>(s_cnt + 64 + 4 * 64);
  const int kf = fa.kb + 1;
  for (int q = t; q < 8 * tstride; q += blockDim.x)
    if (q % tstride >= 64 * F) s_tiles[q] = 0.f;  // the pairs read past a tile's rows: finite zeros
  if (t < 32) {
    s_a[t] = t < F ? fa.a32[t] : 0.f;  // padded features scale to exactly 0
    s_b[t] = t < F ? fa.b32[t] : 0.f;
    s_e[t] = t < F ? fa.qexp[t] : 0;
  }
  if (t < 64) s_cnt[t] = 0;
  for (int q = t; q < kf * F; q += blockDim.x) s_acc[q] = 0ull;
  for (int q = t; q < 16 * kFoldKS; q += blockDim.x) s_cT[q] = fa.gT[q];
  __syncthreads();

  const int64_t lo = (int64_t)blockIdx.x * R, hi = min(S, lo + R);
  const int ntile = hi > lo ? (int)((hi - lo + 63) / 64) : 0;
  const int nround = (ntile + 3) / 4;
  double acc[T];
#pragma unroll
  for (int c = 0; c < T; ++c) acc[c] = 0.0;
  if (wid < 4) {
    // ===== k-means++ waves: kpp_pass_kernel<32, T, 2>'s tile loop =====
    const int64_t total = S * (int64_t)F, n4 = total >> 2;
    const __amdgpu_buffer_rsrc_t rx = make_rsrc(X + lo * F, (S - lo) * F * 4);
    const __amdgpu_buffer_rsrc_t rc = make_rsrc(cur + lo, (hi - lo) * 8);
    const int tile_bytes = 64 * F * 4;
    const double* tb = tab;
    const int pb = *best;
    const double* tp = tab_prev + 64 + pb;
    const double tcc = tab_prev[640 + pb];
    f4v v[NV];
    double cur_next = 0.0;
    auto fetch = [&](int tt) {
      tt = tt < ntile ? tt : ntile - 1;
      cur_next = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rc, lane * 8, tt * 512, kStreamAux));
#pragma unroll
      for (int i = 0; i < NV; ++i)
        v[i] = __builtin_bit_cast(f4v, __builtin_amdgcn_raw_buffer_load_b128(rx, lane * 16 + i * 1024, tt * tile_bytes, kStreamAux));
    };
    if (w4 < ntile) fetch(w4);
    for (int it = 0; it < nround; ++it) {
      const int tc = w4 + 4 * it;
      float* s_tile = s_tiles + (size_t)((it & 1) * 4 + w4) * tstride;
      const bool has = tc < ntile;
      const int64_t r0 = lo + (int64_t)tc * 64;
      const int nrow = has ? (int)min((int64_t)64, hi - r0) : 0;
      double cd = 0.0;
      if (has) {
        f4v* s4 = reinterpret_cast<f4v*>(s_tile);
#pragma unroll
        for (int i = 0; i < NV; ++i)
          if ((lane + i * 64) * 16 < tile_bytes) s4[lane + i * 64] = v[i];
        wt_tail(nrow * F, r0 * F, n4, X, total, s_tile, lane);
        cd = cur_next;
        fetch(tc + 4);
      }
      fold_lds_barrier();  // the tile is staged for the partner E-step wave
      if (!has) continue;
      double d[T], dp = 0.0;
      kpp_row_dists<T, 2>(s_tile + lane * F, F, 32, tb, tp, tcc, d, dp);
      cd = cd < dp ? cd : dp;
      const bool valid = lane < nrow;
      double mv[T];
#pragma unroll
      for (int c = 0; c < T; ++c) {
        const double m = cd < d[c] ? cd : d[c];
        mv[c] = valid ? m : 0.0;
        acc[c] += mv[c];
      }
      kpp_tile_sums<T>(mv, lane, tsum_new + (r0 >> 6), NTL);
    }
  } else {
    // ===== E-step waves: lloyd_pass kFirst on the partner's tile =====
    typedef double d4f __attribute__((ext_vector_type(4)));
    // one-hot sums, features 0-15 / 16-31, two chains each (even / odd
    // k-steps: integer sums, added exactly at the flush)
    d4f am[4] = {d4f{0.0, 0.0, 0.0, 0.0}, d4f{0.0, 0.0, 0.0, 0.0}, d4f{0.0, 0.0, 0.0, 0.0},
                 d4f{0.0, 0.0, 0.0, 0.0}};
    const int kk = lane >> 4, mm = lane & 15;  // MFMA operand lane map
    auto flush = [&]() {  // the fp64 MFMA sums (exact integers) into the int64 LDS sums
#pragma unroll
      for (int nbk = 0; nbk < 2; ++nbk) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int lab_i = kk + 4 * r, f = 16 * nbk + mm;  // f64 D map: row (l>>4)+4r, col l&15
          const double v = am[nbk][r] + am[2 + nbk][r];  // integers below 2^52 each
          if (lab_i < kf && f < F && v != 0.0)
            atomicAdd(&s_acc[lab_i * F + f], (unsigned long long)(long long)v);
        }
        am[nbk] = d4f{0.0, 0.0, 0.0, 0.0};
        am[2 + nbk] = d4f{0.0, 0.0, 0.0, 0.0};
      }
    };
    int since_flush = 0;
    for (int it = 0; it < nround; ++it) {
      const int tc = w4 + 4 * it;
      const float* s_tile = s_tiles + (size_t)((it & 1) * 4 + w4) * tstride;
      fold_lds_barrier();
      if (tc >= ntile) continue;
      const int64_t r0 = lo + (int64_t)tc * 64;
      const int nrow = (int)min((int64_t)64, hi - r0);
      const bool valid = lane < nrow;
      const int64_t row = r0 + lane;
      f2v x2[16];
      load_scaled_row<32>(s_tile, lane, F, s_a, s_b, x2);
      int lab;
      float m1, m2;
      nearest_centers<32, kFoldKS, true>(x2, s_cT, fa.kb, lab, m1, m2);
      f2v ac[4] = {f2v{0.f, 0.f}, f2v{0.f, 0.f}, f2v{0.f, 0.f}, f2v{0.f, 0.f}};
#pragma unroll
      for (int p = 0; p < 16; ++p) {
        const f2v* cp = s_cT + p * kFoldKS + kFoldSlot;  // broadcast reads
        const f2v c4[4] = {cp[0], cp[1], cp[2], cp[3]};
        dist4(x2[p], c4, ac);
      }
      float lbm = m2;
      unsigned bits = 0u;
#pragma unroll
      for (int q = 0; q < T; ++q) {
        const float e = ac[q].x + ac[q].y;
        bits |= e < m1 ? 1u << q : 0u;
        lbm = fminf(lbm, e);
      }
      if (valid) {
        fa.labels[row] = (uint8_t)lab;
        fa.ub[row] = sqrtf(m1);
        fa.lb[row] = sqrtf(lbm);
        fa.moved[row] = (uint8_t)bits;
        atomicAdd(&s_cnt[lab], 1);
      }
      // base sums: one-hot A[label][row] x B[row][f] = q(x_f), as kFirst
      s_lab[lane] = valid ? lab : -1;
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int st = 0; st < 16; ++st) {
        const int rr = 4 * st + kk;
        const int lr = s_lab[rr];
        const double a = lr == mm ? 1.0 : 0.0;
#pragma unroll
        for (int nbk = 0; nbk < 2; ++nbk) {
          const int f = 16 * nbk + mm;
          const double bq = f < F ? fixq64(s_tile[rr * F + f], s_e[f]) : 0.0;
          am[2 * (st & 1) + nbk] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, bq, am[2 * (st & 1) + nbk], 0, 0, 0);
        }
      }
      if (++since_flush == 32) {  // sums stay below 32 * 64 * 2^41 = 2^52: exact
        flush();
        since_flush = 0;
      }
    }
    flush();
  }
  // k-means++ block sums (the E-step waves add exact zeros after the pass's
  // four wave sums: the same bits), then the Lloyd block record
#pragma unroll
  for (int c = 0; c < T; ++c) {
    const double tot = block_sum(acc[c], s_red);
    if (t == 0) bsum_new[(size_t)c * gridDim.x + blockIdx.x] = tot;
  }
  __syncthreads();
  const int rlen = lloyd_rec(kf, F);
  double* out = fa.rec + (size_t)blockIdx.x * rlen;
  for (int q = t; q < kf * F; q += blockDim.x) {
    double h, l;
    limbs((long long)s_acc[q], h, l);
    out[q] = h;
    out[kf * F + q] = l;
  }
  for (int j = t; j < kf; j += blockDim.x) out[2 * kf * F + j] = (double)s_cnt[j];
  if (t == 0) {  // every row changed from unlabelled, was computed and read
    const double nv = (double)(hi > lo ? hi - lo : 0);
    out[2 * kf * F + kf] = nv;
    out[2 * kf * F + kf + 1] = nv;
    out[2 * kf * F + kf + 2] = 0.0;
    out[2 * kf * F + kf + 3] = nv;
  }
}

// The fold pass's center image: pair-major fp32 scaled rows (x - mu) * inv of
// the k - 1 centers chosen so far (first, then chosen[1..k-2]) at slots
// 0..k-2 and of the T candidates at kFoldSlot..: the fp32 centers the Lloyd
// passes get (fit.cpp: upload of the fp64 scaled rows), zero elsewhere
__global__ void __launch_bounds__(256) kpp_fold_centers_kernel(const float* __restrict__ X, int F,
                                                               const double* __restrict__ mu,
                                                               const double* __restrict__ inv,
                                                               const int64_t* __restrict__ chosen, int64_t first,
                                                               int kb, const int64_t* __restrict__ cand, int T,
                                                               f2v* __restrict__ gT) {
  for (int q = threadIdx.x; q < 16 * kFoldKS; q += blockDim.x) {
    const int p = q / kFoldKS, j = q % kFoldKS;
    int64_t r = -1;
    if (j < kb) r = j == 0 ? first : chosen[j];
    else if (j >= kFoldSlot && j < kFoldSlot + T) r = cand[j - kFoldSlot];
    float v[2] = {0.f, 0.f};
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int f = 2 * p + u;
      if (r >= 0 && f < F) v[u] = (float)(((double)X[r * F + f] - mu[f]) * inv[f]);
    }
    gT[q] = f2v{v[0], v[1]};
  }
}

// fixed-order fold of the fold pass's G block records (kmeans_common.h)
__global__ void __launch_bounds__(256) kpp_fold_reduce_kernel(const double* __restrict__ rec, int G, int rl,
                                                              double* __restrict__ out) {
  if ((int)blockIdx.x * 32 >= rl) return;
  rec_reduce_body(rec, G, rl, out);
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

int mw_kpp_fold_supported(int k, int F, int T) {
  return k >= 3 && k <= 16 && T >= 1 && T <= 4 && F >= 1 && F <= 32 && kpp_fold_lds(k, F) <= kFoldLdsMax;
}

size_t mw_kpp_fold_rec_bytes(int64_t S, int k, int F) {
  return (size_t)kblocks(S) * lloyd_rec(k, F) * sizeof(double);
}

const int* mw_kpp_best_ptr(const void* d_ws, int64_t S, int T) { return kpp_ptrs(d_ws, S, T).best; }

int mw_kpp_step_fold(const float* d_X, int64_t S, int F, const double* d_mu, const double* d_inv, int c,
                     const double* h_u, int T, void* d_ws, int64_t first, const float* d_a32,
                     const float* d_b32, const int32_t* d_qexp, uint8_t* d_labels, float* d_ub, float* d_lb,
                     uint8_t* d_moved, void* d_centers_img, double* d_rec, double* d_rec_out, void* stream) {
  MW_CHECK_ARG(d_X && d_mu && d_inv && d_ws && h_u && d_a32 && d_b32 && d_qexp && d_labels && d_ub && d_lb &&
                   d_moved && d_centers_img && d_rec && d_rec_out,
               "mw_kpp_step_fold: null pointer");
  MW_CHECK_ARG(c >= 2 && mw_kpp_fold_supported(c + 1, F, T) && first >= 0 && first < S,
               "mw_kpp_step_fold: unsupported (k=%d F=%d T=%d: mw_kpp_fold_supported)", c + 1, F, T);
  const KppPtrs p = kpp_ptrs(d_ws, S, T);
  double u[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int i = 0; i < T; ++i) u[i] = h_u[i];
  hipStream_t s = as_stream(stream);
  // the previous step's selection and this step's candidates, as mw_kpp_step
  const int rc = kpp_search_launch(d_X, S, F, p, c, T, u, T, T, -1, nullptr, s);
  if (rc != MW_OK) return rc;
  double* tab = p.tab_of(c);
  hipLaunchKernelGGL(kpp_prep_kernel, dim3(1), dim3(512), 0, s, d_X, F, d_mu, d_inv, p.cand, nullptr, T, tab,
                     nullptr);
  f2v* gT = reinterpret_cast<f2v*>(d_centers_img);
  hipLaunchKernelGGL(kpp_fold_centers_kernel, dim3(1), dim3(256), 0, s, d_X, F, d_mu, d_inv, p.chosen, first, c,
                     p.cand, T, gT);
  MW_LAUNCH_CHECK();
  KppFoldArg fa{};
  fa.a32 = d_a32;
  fa.b32 = d_b32;
  fa.qexp = d_qexp;
  fa.gT = gT;
  fa.kb = c;
  fa.labels = d_labels;
  fa.ub = d_ub;
  fa.lb = d_lb;
  fa.moved = d_moved;
  fa.rec = d_rec;
  const size_t lds = kpp_fold_lds(c + 1, F);
  const int64_t R = krows(S);
  const double* tab_prev = p.tab_of(c - 1);
  double* bs = p.bsum_of(c, T);
  double* tsm = p.tsum_of(c, T);
#define MW_KF(TV)                                                                                  \
  hipLaunchKernelGGL((kpp_fold_kernel<TV>), dim3(p.L.G), dim3(512), lds, s, d_X, S, F, tab, tab_prev, \
                     p.best, p.cur, R, p.L.NTL, bs, tsm, fa)
  switch (T) {
    case 1: MW_KF(1); break;
    case 2: MW_KF(2); break;
    case 3: MW_KF(3); break;
    default: MW_KF(4); break;
  }
#undef MW_KF
  MW_LAUNCH_CHECK();
  const int rl = lloyd_rec(c + 1, F);
  hipLaunchKernelGGL(kpp_fold_reduce_kernel, dim3((rl + 31) / 32), dim3(256), 0, s, d_rec, p.L.G, rl, d_rec_out);
  MW_LAUNCH_CHECK();
  return MW_OK;
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
