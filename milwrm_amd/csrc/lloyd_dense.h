// The batched sweep's dense Lloyd pass (find_optimal_k's k = 2..20 fits,
// MILWRM.py:29-90 / 659-704): one launch computes, for every row, the
// distances to the centers of every fit in the launch as a GEMM x . C^T on the
// matrix cores -- the dense contraction the k sweep is (sum of k = 209 centers
// x F features per row) -- instead of one bounded E-step per fit.
//
// Per block: a row block of the rows and a GROUP of fits (at most 64 centers
// together: four 16-center MFMA tiles; the groups of one row block are
// dispatched together, so their row reads after the first come from the
// on-die caches).  Per wave: 64-row tiles, 16 rows at a time:
//   * A = the group's centers (16 per tile x 32 features), B = 16 scaled rows
//     (32 features x 16 rows), both split into f16 hi + lo (v = hi + lo to
//     2^-22); x . c = hi.hi + lo.hi + hi.lo on v_mfma_f32_16x16x32_f16 (the
//     lo.lo term, ~2^-22 relative, dropped);
//   * approximate squared distance d~ = |x|^2 + |c|^2 - 2 x.c, staged in LDS
//     [row][center], scanned per (row, fit) for the two smallest;
//   * the label is exactly the one the fp32 direct-difference E-step of
//     lloyd_pass_kernel gives: it is taken from d~ only when the top-2 gap
//     exceeds a bound on |d~ - d| + the fp32 rounding of d (bscale x (|x|^2 +
//     max|c|^2), see lloyd_dense_bound); otherwise the row is recomputed with
//     dist_one (the same fp32 chain as nearest_centers, strict '<').  So the
//     labels, and with them the exact fixed-point M-step, n_iter, centers and
//     inertia, are bit for bit those of every other pass kind
//     (tests/test_gpu_lloyd_kinds.py);
//   * changed rows move their q between the fit's cluster sums (LDS int64
//     atomics, lane = feature), as kTile's move_rows;
//   * no distance bounds are kept (the next bounded pass of a fit is a kTile
//     pass with infinite drift, which recomputes every row and writes them);
//     a fit flagged in `bounds` gets ub = sqrt(d~1 + B), lb = sqrt(d~2 - B)
//     instead (valid bounds: the bound covers the approximation).
// Records per fit and row block: the lloyd_pass_kernel layout, reduced by
// lloyd_reduce_fits_kernel.
#pragma once

namespace mw {

constexpr int kDense = 5;
constexpr int kDenseMaxK = 64;    // centers per fit group (4 MFMA tiles of 16)
constexpr int kDenseMaxFits = 8;  // fits per group
constexpr int kDenseSD = 68;      // LDS pitch of a row's approximate distances (floats)
constexpr int kDenseMaxFitK = 20; // centers per fit in the dense pass (the k = 2..20 sweep)

struct DenseGroup {
  int g0, n;                     // fits [g0, g0 + n) of the launch
  int off[kDenseMaxFits + 1];    // center offsets of the fits in the group
};
struct DenseArg {
  DenseGroup grp[kMaxFits];
  int ngroups;
  int G;                         // row blocks
  int bounds;                    // bit g: write ub / lb of fit g
  float bscale;                  // decision bound = bscale * (|x|^2 + max |c|^2)
};

typedef _Float16 h8d __attribute__((ext_vector_type(8)));
typedef float f4d __attribute__((ext_vector_type(4)));

// Bound on |d~ - d_fp32| for the f16-split product: the dropped lo.lo term and
// the f16 rounding of lo (<= 3 * 2^-22 |x_f||c_f| per feature, + f16
// subnormal spacing), the fp32 accumulation of 96 exact products inside the
// MFMA (<= 96 * 2^-24 sum |x_f c_f|), |x|^2 in fp32 and the final sums,
// against |x||c| <= (|x|^2 + |c|^2) / 2; plus the fp32 rounding of the direct
// chain (F * 2^-24 d, d <= 2 (|x|^2 + |c|^2)).  About 1.5e-5 (|x|^2 + |c|^2)
// for both sides of a comparison; the default bscale 1e-4 leaves margin.
constexpr float kDenseBScale = 1e-4f;

__host__ __device__ inline size_t dense_lds_bytes(int FMAX, int F) {
  size_t b = 3 * 64 * 4;                                 // scaler a, b, qexp
  b += (size_t)(FMAX / 2) * kDenseMaxK * 8;              // pair-major centers (exact recheck)
  b += kDenseMaxK * 4 + kDenseMaxFits * 4 * 4;           // |c|^2, per fit: max |c|^2, changed, recomputed, pad
  b += ((size_t)kDenseMaxK * F * 8 + 15) & ~(size_t)15;  // cluster sums (int64)
  b += kDenseMaxK * 4;                                   // size deltas
  b += 4 * ((size_t)64 * FMAX * 4 + 16 * kDenseSD * 4 + kDenseMaxFits * 64);  // per wave: tile, d~, labels
  return b;
}

template <int FMAX>
__global__ void __launch_bounds__(256, FMAX == 64 ? 1 : 2) lloyd_dense_kernel(const float* __restrict__ X, int64_t S, int F,
                                                            const float* __restrict__ ga,
                                                            const float* __restrict__ gb,
                                                            const int* __restrict__ qexp, const LloydFitsArg fits,
                                                            const DenseArg da, int64_t R) {
  constexpr int KB = FMAX / 32;  // 32-feature MFMA k-blocks
  static_assert(FMAX == 32 || FMAX == 64, "dense pass: FMAX 32 or 64");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // block id -> (row block, group): the groups of one row block run on one
  // XCD (block ids 8 apart share an XCD), dispatched close together, so the
  // rows come from HBM once and from that XCD's L2 for the other groups
  const int xcd = blockIdx.x & 7, jj = blockIdx.x >> 3;
  const int grp = jj % da.ngroups, blk = (jj / da.ngroups) * 8 + xcd;
  if (blk >= da.G) return;  // the grid is padded to whole XCD rounds (block-uniform)
  const DenseGroup& dg = da.grp[grp];
  const int nf = dg.n, kt = dg.off[nf];
  const int t = threadIdx.x, lane = t & 63;
  const int wid = __builtin_amdgcn_readfirstlane(t >> 6);
  char* sp = smem;
  float* s_a = reinterpret_cast<float*>(sp);
  float* s_b = s_a + 64;
  int* s_e = reinterpret_cast<int*>(s_b + 64);
  sp += 3 * 64 * 4;
  f2v* s_cT = reinterpret_cast<f2v*>(sp);  // [FMAX/2][64] pairs
  sp += (size_t)(FMAX / 2) * kDenseMaxK * 8;
  float* s_cc = reinterpret_cast<float*>(sp);
  float* s_cmax = s_cc + kDenseMaxK;
  int* s_chg = reinterpret_cast<int*>(s_cmax + kDenseMaxFits);
  int* s_rec = s_chg + kDenseMaxFits;
  sp += kDenseMaxK * 4 + kDenseMaxFits * 4 * 4;
  unsigned long long* s_acc = reinterpret_cast<unsigned long long*>(sp);
  sp += ((size_t)kDenseMaxK * F * 8 + 15) & ~(size_t)15;
  int* s_cnt = reinterpret_cast<int*>(sp);
  sp += kDenseMaxK * 4;
  const size_t wave_bytes = (size_t)64 * FMAX * 4 + 16 * kDenseSD * 4 + kDenseMaxFits * 64;
  char* wp = sp + wid * wave_bytes;
  float* s_tile = reinterpret_cast<float*>(wp);                    // 64 rows x F (row stride F)
  float* s_d = reinterpret_cast<float*>(wp + (size_t)64 * FMAX * 4);  // [16][kDenseSD]
  uint8_t* s_lab = reinterpret_cast<uint8_t*>(s_d + 16 * kDenseSD);  // [nf][64]

  for (int f = t; f < 64; f += blockDim.x) {
    s_a[f] = f < F ? ga[f] : 0.f;
    s_b[f] = f < F ? gb[f] : 0.f;
    s_e[f] = f < F ? qexp[f] : 0;
  }
  // the group's centers: pair-major image (exact recheck), |c|^2, and the
  // per-fit maxima of |c|^2 (the decision bound)
  for (int q = t; q < (FMAX / 2) * kDenseMaxK; q += blockDim.x) {
    const int p = q / kDenseMaxK, c = q - p * kDenseMaxK;
    f2v v = f2v{0.f, 0.f};
    if (c < kt) {
      int gi = 0;
      while (c >= dg.off[gi + 1]) ++gi;
      const int lc = c - dg.off[gi];  // the slots past a fit's k (alignment pad) stay 0
      if (lc < fits.f[dg.g0 + gi].k) {
        const float* cr = fits.f[dg.g0 + gi].centers + (size_t)lc * F;
        v = f2v{2 * p < F ? cr[2 * p] : 0.f, 2 * p + 1 < F ? cr[2 * p + 1] : 0.f};
      }
    }
    s_cT[q] = v;
  }
  for (int q = t; q < kDenseMaxK * F; q += blockDim.x) s_acc[q] = 0ull;
  for (int q = t; q < kDenseMaxK; q += blockDim.x) s_cnt[q] = 0;
  if (t < kDenseMaxFits) s_chg[t] = s_rec[t] = 0;
  __syncthreads();
  for (int c = t; c < kDenseMaxK; c += blockDim.x) {
    double s = 0.0;
    for (int p = 0; p < FMAX / 2; ++p) {
      const f2v v = s_cT[p * kDenseMaxK + c];
      s += (double)v.x * v.x + (double)v.y * v.y;
    }
    s_cc[c] = c < kt ? (float)s : 0.f;
  }
  __syncthreads();
  if (t < nf) {
    float m = 0.f;
    for (int c = dg.off[t]; c < dg.off[t + 1]; ++c) m = fmaxf(m, s_cc[c]);
    s_cmax[t] = m;
  }
  // A operands: center 16 tt + (lane & 15), features 32 kb + 8 (lane >> 4) + i
  h8d a_hi[4][KB], a_lo[4][KB];
  const int am = lane & 15, aq = lane >> 4;
#pragma unroll
  for (int tt = 0; tt < 4; ++tt)
#pragma unroll
    for (int kb = 0; kb < KB; ++kb)
#pragma unroll
      for (int i = 0; i < 8; i += 2) {
        const int f = 32 * kb + 8 * aq + i;  // even
        const f2v v = s_cT[(f / 2) * kDenseMaxK + 16 * tt + am];
        const _Float16 h0 = (_Float16)v.x, h1 = (_Float16)v.y;
        a_hi[tt][kb][i] = h0;
        a_hi[tt][kb][i + 1] = h1;
        a_lo[tt][kb][i] = (_Float16)(v.x - (float)h0);
        a_lo[tt][kb][i + 1] = (_Float16)(v.y - (float)h1);
      }
  const int ntt = (kt + 15) >> 4;
  __syncthreads();

  const int64_t lo = (int64_t)blk * R, hi = min(S, lo + R);
  const int ntile = hi > lo ? (int)((hi - lo + 63) / 64) : 0;
  const int nl = lane & 15, ql = lane >> 4;  // (row in the 16-row chunk, quarter)
  const float bscale = da.bscale;
  int chg[2] = {0, 0}, rec[2] = {0, 0};
  for (int tc = wid; tc < ntile; tc += 4) {
    const int64_t r0 = lo + (int64_t)tc * 64;
    const int nrow = (int)min((int64_t)64, hi - r0);
    // the tile's rows (row stride F; 16-byte loads, all issued before the
    // first store) and every fit's labels of them
    {
      constexpr int NV = FMAX / 4;  // float4 per lane for 64 x FMAX floats
      const int n4 = (nrow * F) >> 2;
      const f4v* src = reinterpret_cast<const f4v*>(X + r0 * F);  // 16-byte aligned: r0 % 64 == 0
      f4v v[NV];
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const int q = lane + 64 * i;
        if (q < n4) v[i] = src[q];
      }
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const int q = lane + 64 * i;
        if (q < n4) reinterpret_cast<f4v*>(s_tile)[q] = v[i];
      }
      for (int q = 4 * n4 + lane; q < nrow * F; q += 64) s_tile[q] = X[r0 * F + q];
    }
    {
      uint8_t lb[kDenseMaxFits];
#pragma unroll
      for (int gi = 0; gi < kDenseMaxFits; ++gi)
        lb[gi] = (gi < nf && lane < nrow) ? fits.f[dg.g0 + gi].labels[r0 + lane] : (uint8_t)0;
#pragma unroll
      for (int gi = 0; gi < kDenseMaxFits; ++gi) s_lab[gi * 64 + lane] = lb[gi];
    }
    __builtin_amdgcn_wave_barrier();
#pragma unroll 1
    for (int ch = 0; ch < 4; ++ch) {
      if (16 * ch >= nrow) break;  // wave-uniform
      // ---- B operands: row 16 ch + nl, features 32 kb + 8 ql + i (scaled, split) ----
      const int brow = min(16 * ch + nl, nrow - 1);
      h8d b_hi[KB], b_lo[KB];
      float xx = 0.f;
#pragma unroll
      for (int kb = 0; kb < KB; ++kb)
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int f = 32 * kb + 8 * ql + i;
          const float x = f < F ? __builtin_fmaf(s_tile[brow * F + f], s_a[f], s_b[f]) : 0.f;
          const _Float16 h = (_Float16)x;
          b_hi[kb][i] = h;
          b_lo[kb][i] = (_Float16)(x - (float)h);
          xx = __builtin_fmaf(x, x, xx);
        }
      xx += __shfl_xor(xx, 16, 64);
      xx += __shfl_xor(xx, 32, 64);
      // ---- x . c on the matrix cores; d~ into LDS [row][center] ----
#pragma unroll
      for (int tt = 0; tt < 4; ++tt) {
        if (tt >= ntt) break;  // wave-uniform
        f4d acc = f4d{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kb = 0; kb < KB; ++kb) {
          acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a_hi[tt][kb], b_hi[kb], acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a_lo[tt][kb], b_hi[kb], acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a_hi[tt][kb], b_lo[kb], acc, 0, 0, 0);
        }
        // lane: row nl, centers 16 tt + 4 ql + r
        const int c0 = 16 * tt + 4 * ql;
        f4d d;
#pragma unroll
        for (int r = 0; r < 4; ++r) d[r] = xx + s_cc[c0 + r] - 2.f * acc[r];
        *reinterpret_cast<f4d*>(s_d + nl * kDenseSD + c0) = d;
      }
      __builtin_amdgcn_wave_barrier();
      // ---- per (row nl, fit gi = ql + 4 s): top two of d~, exact recheck near ties ----
      const int row = 16 * ch + nl;
      const bool valid = row < nrow;
#pragma unroll
      for (int sl = 0; sl < 2; ++sl) {
        const int gi = ql + 4 * sl;
        bool ch_ = false;
        int lab = 0, lab_old = 0, k = 1;
        if (gi < nf) {
          const int o = dg.off[gi];
          k = fits.f[dg.g0 + gi].k;
          // the fit's (<= 20, 4-aligned) distances in one batch of 16-byte reads
          // (branch-free: slots past k read as +inf, which changes nothing)
          const f4d* dr = reinterpret_cast<const f4d*>(s_d + nl * kDenseSD + o);
          const int ulast = (k - 1) >> 2;
          f4d dv[kDenseMaxFitK / 4];
#pragma unroll
          for (int u = 0; u < kDenseMaxFitK / 4; ++u) dv[u] = dr[u < ulast ? u : ulast];
          float m1 = dv[0][0], m2 = __builtin_inff();
          lab = 0;
#pragma unroll
          for (int j = 1; j < kDenseMaxFitK; ++j) {
            const float v = j < k ? dv[j >> 2][j & 3] : __builtin_inff();
            const bool lt1 = v < m1, lt2 = v < m2;
            m2 = lt1 ? m1 : (lt2 ? v : m2);
            m1 = lt1 ? v : m1;
            lab = lt1 ? j : lab;
          }
          const float B = bscale * (xx + s_cmax[gi]);
          if (valid && k > 1 && !(m2 - m1 > B)) {
            // near tie: the fp32 direct-difference chain (nearest_centers' bits)
            f2v x2[FMAX / 2];
#pragma unroll
            for (int p = 0; p < FMAX / 2; ++p) {
              const int f0 = 2 * p;
              x2[p] = f2v{f0 < F ? s_tile[row * F + f0] : 0.f, f0 + 1 < F ? s_tile[row * F + f0 + 1] : 0.f};
              x2[p] = __builtin_elementwise_fma(x2[p], f2v{s_a[f0], s_a[f0 + 1]}, f2v{s_b[f0], s_b[f0 + 1]});
            }
            float e1 = 0.f, e2 = __builtin_inff();
            int el = 0;
            for (int j = 0; j < k; ++j) {
              f2v acc2 = f2v{0.f, 0.f};
#pragma unroll
              for (int p = 0; p < FMAX / 2; ++p) {
                const f2v dd = x2[p] - s_cT[p * kDenseMaxK + o + j];
                acc2 = __builtin_elementwise_fma(dd, dd, acc2);
              }
              const float v = acc2.x + acc2.y;
              if (j == 0) { e1 = v; el = 0; }
              else if (v < e1) { e2 = e1; e1 = v; el = j; }
              else if (v < e2) { e2 = v; }
            }
            lab = el;
            m1 = e1;
            m2 = e2;
            rec[sl] += 1;
          }
          lab_old = s_lab[gi * 64 + row];
          ch_ = valid && lab != lab_old;
          const mw_lloyd_fit& fit = fits.f[dg.g0 + gi];
          if (ch_) fit.labels[r0 + row] = (uint8_t)lab;
          if (valid && ((da.bounds >> (dg.g0 + gi)) & 1)) {
            fit.ub[r0 + row] = sqrtf(m1 + B) * (1.f + 1e-6f);
            fit.lb[r0 + row] = k > 1 ? sqrtf(fmaxf(m2 - B, 0.f)) * (1.f - 1e-6f) : __builtin_inff();
          }
        }
        chg[sl] += ch_ ? 1 : 0;
        // ---- M-step of the changed (row, fit) pairs, lane = feature ----
        unsigned long long cm = __ballot(ch_);
        while (cm != 0ull) {  // wave-uniform
          const int j = __builtin_ctzll(cm);
          cm &= cm - 1ull;
          const int jg = __shfl(gi, j, 64), jl = __shfl(lab, j, 64), jo = __shfl(lab_old, j, 64);
          const int jr = __shfl(row, j, 64), jk = __shfl(k, j, 64);
          const int o = dg.off[jg];
          for (int f = lane; f < F; f += 64) {
            const long long q = fixq(s_tile[jr * F + f], s_e[f]);
            atomicAdd(&s_acc[(o + jl) * F + f], (unsigned long long)q);
            if (jo < jk) atomicAdd(&s_acc[(o + jo) * F + f], (unsigned long long)(-q));
          }
          if (lane == 0) {
            atomicAdd(&s_cnt[o + jl], 1);
            if (jo < jk) atomicAdd(&s_cnt[o + jo], -1);
          }
        }
      }
      __builtin_amdgcn_wave_barrier();  // s_d is rewritten by the next chunk
    }
    __builtin_amdgcn_wave_barrier();  // s_tile / s_lab are rewritten by the next tile
  }
  // per-fit counters: lanes of quarter ql hold fits ql and ql + 4
#pragma unroll
  for (int sl = 0; sl < 2; ++sl) {
    int c = chg[sl], r = rec[sl];
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) {
      c += __shfl_xor(c, o, 64);
      r += __shfl_xor(r, o, 64);
    }
    const int gi = ql + 4 * sl;
    if (nl == 0 && gi < nf) {
      atomicAdd(&s_chg[gi], c);
      atomicAdd(&s_rec[gi], r);
    }
  }
  __syncthreads();
  // records: per fit [dQ_hi kF | dQ_lo kF | dcount k | changed | recomputed | 0 | 0]
  for (int gi = 0; gi < nf; ++gi) {
    const mw_lloyd_fit& fit = fits.f[dg.g0 + gi];
    const int k = fit.k, o = dg.off[gi];
    const int rlen = lloyd_rec(k, F);
    double* out = reinterpret_cast<double*>(fit.ws) + (size_t)blk * rlen;
    for (int q = t; q < k * F; q += blockDim.x) {
      double h, l;
      limbs((long long)s_acc[o * F + q], h, l);
      out[q] = h;
      out[k * F + q] = l;
    }
    for (int j = t; j < k; j += blockDim.x) out[2 * k * F + j] = (double)s_cnt[o + j];
    if (t == 0) {
      out[2 * k * F + k] = (double)s_chg[gi];
      out[2 * k * F + k + 1] = (double)s_rec[gi];
      out[2 * k * F + k + 2] = 0.0;
      out[2 * k * F + k + 3] = 0.0;
    }
  }
}

// Fits [0, n) in groups of consecutive fits, each fit's centers at a
// 4-aligned offset, at most 64 center slots and 8 fits per group; false when
// a fit has more than kDenseMaxFitK centers.
static inline bool dense_groups(const mw_lloyd_fit* h, int n, DenseArg& da) {
  da.ngroups = 0;
  int g = 0;
  while (g < n) {
    if (h[g].k > kDenseMaxFitK) return false;
    DenseGroup& dg = da.grp[da.ngroups++];
    dg.g0 = g;
    dg.n = 0;
    dg.off[0] = 0;
    while (g < n && dg.n < kDenseMaxFits && dg.off[dg.n] + h[g].k <= kDenseMaxK) {
      dg.off[dg.n + 1] = dg.off[dg.n] + ((h[g].k + 3) & ~3);
      ++dg.n;
      ++g;
    }
  }
  return true;
}

}  // namespace mw
