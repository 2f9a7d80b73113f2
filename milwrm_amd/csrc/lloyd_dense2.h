// The batched sweep's dense Lloyd pass, second form (find_optimal_k's k =
// 2..20 fits, MILWRM.py:29-90 / 659-704; sklearn lloyd_iter_chunked_dense,
// _k_means_lloyd.pyx:23-218): ONE block per row block computes, for every row,
// x . C^T against the centers of EVERY fit of the launch on the matrix cores,
// and keeps per (row, fit) only the running top two.
//
// Layout (F <= 32 features; every fit's centers at an 8-aligned slot offset,
// at most kD2Slots slots = kD2Tiles MFMA tiles of 32 centers):
//   * A = 32 center slots x 16 features (f16 hi + lo, from LDS: ds_read_b128
//     per lane), B = 16 features x 32 rows (f16 hi + lo, the scaled rows x' =
//     x a + b from global memory), v_mfma_f32_32x32x16_f16, two k-steps and
//     three split products per tile: lane
//     (r = l & 31, h = l >> 5) holds row r and the 16 slots (reg & 3) +
//     8 (reg >> 2) + 4 h of the tile;
//   * d' = |c|^2 - 2 x.c (the row's |x|^2 is common to all its centers and
//     cancels in every comparison); per 8-slot group (one fit: both lane
//     halves see the same fit sequence) a branch-free top-two update
//     (strict '<' keeps the lowest index, v_med3 the second smallest), the
//     halves merged at the fit's end by one cross-half exchange;
//   * the label is the one the fp32 direct-difference E-step
//     (nearest_centers: even features in .x, odd in .y, then .x + .y) gives:
//     it is taken from d' only when the top-two gap exceeds a bound on the
//     error of the f16 products against that chain (kD2BScale x (|x|^2 +
//     max |c|^2)); other (row, fit) pairs go to a per-wave queue and are
//     recomputed with that chain, 64 at a time (one pair per lane), so the
//     labels -- and the exact fixed-point M-step, n_iter, centers, inertia --
//     are bit for bit those of every other pass kind;
//   * changed (row, fit) pairs go to a second queue: their q moves between the
//     fit's cluster sums (LDS int64 atomics, lane = feature).
// Records per fit and row block: the lloyd_pass_kernel layout over a grid of
// its own (kD2Blocks row blocks), reduced by lloyd_reduce_fits_kernel.
#pragma once

namespace mw {

constexpr int kD2Tiles = 10;                // MFMA tiles of 32 center slots
constexpr int kD2Slots = 32 * kD2Tiles;     // 8-aligned center slots of all fits
constexpr int kD2Groups = kD2Slots / 8;     // 8-slot groups (one fit each)
constexpr int kD2Waves = 12;                // waves per block at most (one block per CU:
                                            // 3 per SIMD; 8 when the LDS of the launch needs it)
constexpr int kD2MaxBlocks = 512;           // row blocks (records per fit)
// x' and c are split into f16 hi + lo (v = hi + lo to 2^-22); x . c =
// hi.hi + lo.hi + hi.lo on the matrix cores (lo.lo, ~2^-22, dropped).
// Bound on |d'_mfma - d'_chain| for BOTH values of a comparison, relative to
// |x|^2 + max |c|^2: the split (3 x 2^-22 per product), the fp32
// accumulation of 96 products (<= 96 x 2^-24 of sum |x_f c_f| <= (|x|^2 +
// |c|^2) / 2), the fp32 rounding of d' and of the direct chain (32 x 2^-24 d,
// d <= 2 (|x|^2 + |c|^2)): about 2 x 1e-5; the constant keeps a 2x margin
constexpr float kD2BScale = 8e-5f;
constexpr float kD2BAbs = 3e-5f;            // f16 subnormal spacing of the lo parts (x the norm scale)
// the norms ride in the two spare features (F <= 30): A[30] = -|c|^2 / 256
// against B[30] = 128, A[31] = 128 against B[31] = (-|x|^2 / 2 - delta) / 128,
// so one accumulator is acc = x.c - |c|^2 / 2 - |x|^2 / 2 - delta = -d / 2 -
// delta < 0.  An empty slot has A[30] = -65504 (f16 max): acc <= -8.38e6
// loses to every center while |x|^2, |c|^2 <= kD2NormMax (else the row, or
// the launch, goes to the exact chain)
constexpr float kD2NormMax = 5.5e6f;
constexpr int kD2MaxK = 32;                 // a fit spans at most two tiles
// keys: acc's bits with the low 6 replaced by (tile parity, slot in tile):
// the negative floats order as signed ints in reverse, so the smallest key is
// the largest acc -- the nearest center, the lowest slot on equal bits
constexpr unsigned kD2KeyMask = 0xFFFFFFC0u;

struct Dense2Arg {
  int nf;                  // fits in the launch
  int ntile;               // MFMA tiles in use
  int off8[kMaxFits + 1];  // slot offset of each fit (8-aligned); off8[nf] = slots used
  int coff[kMaxFits + 1];  // compact offset (cluster sums: sum of k)
  int bounds;              // bit g: write ub / lb of fit g
  int G;                   // row blocks of this launch
  int64_t R;               // rows per row block (multiple of 32)
};

__host__ __device__ inline size_t d2_acc_off(int ntile) {
  return 3 * 32 * 4 + kD2Groups * 4 + 4 * (kMaxFits + 1) * 4 + 4 * kMaxFits * 8 + kD2Slots * 4 +
         (size_t)ntile * 4 * 1024;
}
__host__ __device__ inline size_t d2_wave_bytes() { return kMaxFits * 32 + 2 * 64 * 4 + 128 * 4 + 16; }
__host__ __device__ inline size_t dense2_lds_bytes(int ksum, int F, int ntile, int waves) {
  size_t b = d2_acc_off(ntile);                                 // scaler, tables, |c|^2, A operands
  b += ((size_t)ksum * F * 8 + 15) & ~(size_t)15;               // cluster sums (int64)
  b += ((size_t)ksum * 4 + 2 * kMaxFits * 4 + 15) & ~(size_t)15;  // size deltas, changed, recomputed
  b += (size_t)waves * d2_wave_bytes();                         // per wave: labels, queues
  return b;
}

typedef _Float16 h8x __attribute__((ext_vector_type(8)));
typedef float f16x __attribute__((ext_vector_type(16)));
typedef unsigned u4d __attribute__((ext_vector_type(4)));

// the value of lane l ^ 32 (v_permlane32_swap: the halves exchanged in
// registers, no LDS round trip)
__device__ __forceinline__ unsigned d2_partner_u(unsigned x) {
  const auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
  return (threadIdx.x & 32) ? r[0] : r[1];
}
__device__ __forceinline__ float d2_partner(float x) {
  return __builtin_bit_cast(float, d2_partner_u(__builtin_bit_cast(unsigned, x)));
}

// top-two merge of the two lane halves' partial results for one fit (labels
// are fit-local center indices; the lower index wins a tie of the minimum)
__device__ __forceinline__ void d2_merge_halves(float& m1, int& lab, float& m2) {
  const float pm1 = d2_partner(m1), pm2 = d2_partner(m2);
  const int plab = (int)d2_partner_u((unsigned)lab);
  const bool take = pm1 < m1 || (pm1 == m1 && plab < lab);
  const float hi1 = take ? m1 : pm1;  // the larger of the two minima
  m2 = fminf(fminf(m2, pm2), hi1);
  m1 = take ? pm1 : m1;
  lab = take ? plab : lab;
}

__global__ void __launch_bounds__(64 * kD2Waves) lloyd_dense2_kernel(const float* __restrict__ X, int64_t S,
                                                                     int F, const float* __restrict__ ga,
                                                                     const float* __restrict__ gb,
                                                                     const int* __restrict__ qexp,
                                                                     const LloydFitsArg fits, const Dense2Arg da) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int t = threadIdx.x, lane = t & 63;
  const int wid = __builtin_amdgcn_readfirstlane(t >> 6);
  const int nw = __builtin_amdgcn_readfirstlane((int)(blockDim.x >> 6));  // waves of the block
  const int blk = blockIdx.x;
  const int nf = da.nf, ntile = da.ntile, ksum = da.coff[nf];
  char* sp = smem;
  float* s_a = reinterpret_cast<float*>(sp);
  float* s_b = s_a + 32;
  int* s_e = reinterpret_cast<int*>(s_b + 32);
  sp += 3 * 32 * 4;
  int* s_fit8 = reinterpret_cast<int*>(sp);  // fit of each 8-slot group (-1: none)
  sp += kD2Groups * 4;
  int* s_k = reinterpret_cast<int*>(sp);         // [kMaxFits + 1]
  float* s_cmax = reinterpret_cast<float*>(s_k + kMaxFits + 1);
  int* s_off8 = reinterpret_cast<int*>(s_cmax + kMaxFits + 1);
  int* s_coff = s_off8 + kMaxFits + 1;
  sp += 4 * (kMaxFits + 1) * 4;
  // per-fit pointers (lane-varying fit indices read them from LDS)
  uint8_t** s_labp = reinterpret_cast<uint8_t**>(sp);
  float** s_ubp = reinterpret_cast<float**>(s_labp + kMaxFits);
  float** s_lbp = s_ubp + kMaxFits;
  const float** s_cenp = const_cast<const float**>(s_lbp + kMaxFits);
  sp += 4 * kMaxFits * 8;
  float* s_cc = reinterpret_cast<float*>(sp);  // |c|^2 per slot (+inf: no center)
  sp += kD2Slots * 4;
  char* s_A = sp;  // [tile][kstep][hi, lo][lane][8 halves]
  sp += (size_t)ntile * 4 * 1024;
  unsigned long long* s_acc = reinterpret_cast<unsigned long long*>(sp);
  sp += ((size_t)ksum * F * 8 + 15) & ~(size_t)15;
  int* s_cnt = reinterpret_cast<int*>(sp);
  int* s_chg = s_cnt + ksum;
  int* s_rec = s_chg + kMaxFits;
  sp += ((size_t)ksum * 4 + 2 * kMaxFits * 4 + 15) & ~(size_t)15;
  char* wp = sp + (size_t)wid * d2_wave_bytes();
  uint8_t* w_lab = reinterpret_cast<uint8_t*>(wp);            // [fit][32 rows] old labels
  int* w_rq = reinterpret_cast<int*>(wp + kMaxFits * 32);      // recheck queue: row | fit << 8
  int* w_mq = w_rq + 2 * 64;                                   // M-step queue: row | fit << 8 | lab << 16 | old << 24

  // ---- block setup: scaler, fit tables, |c|^2, A operands, zeroed sums ----
  for (int f = t; f < 32; f += blockDim.x) {
    s_a[f] = f < F ? ga[f] : 0.f;
    s_b[f] = f < F ? gb[f] : 0.f;
    s_e[f] = f < F ? qexp[f] : 0;
  }
  for (int g = t; g < kD2Groups; g += blockDim.x) {
    int fi = -1;
    for (int i = 0; i < nf; ++i)
      if (8 * g >= da.off8[i] && 8 * g < da.off8[i + 1]) fi = i;
    s_fit8[g] = fi;
  }
  if (t < nf) {
    s_labp[t] = fits.f[t].labels;
    s_ubp[t] = fits.f[t].ub;
    s_lbp[t] = fits.f[t].lb;
    s_cenp[t] = fits.f[t].centers;
  }
  if (t <= kMaxFits) {
    s_k[t] = t < nf ? fits.f[t].k : 0;
    s_off8[t] = da.off8[t <= nf ? t : nf];
    s_coff[t] = da.coff[t <= nf ? t : nf];
  }
  __syncthreads();  // tables above
  // slot -> (fit, local center) for the tables below
  auto slot_center = [&](int m, const float*& cr) {
    cr = nullptr;
    const int fi = s_fit8[m >> 3];
    if (fi < 0) return;
    const int lc = m - s_off8[fi];
    if (lc < s_k[fi]) cr = s_cenp[fi] + (size_t)lc * F;
  };
  for (int m = t; m < kD2Slots; m += blockDim.x) {
    const float* cr;
    slot_center(m, cr);
    float s = __builtin_inff();
    if (cr) {
      s = 0.f;
      for (int f = 0; f < F; ++f) s = __builtin_fmaf(cr[f], cr[f], s);
    }
    s_cc[m] = s;
  }
  __syncthreads();  // s_cc (the A operands' norms)
  // A operands of tile tt, k-step ks, lane l: slot 32 tt + (l & 31),
  // features 16 ks + 8 (l >> 5) + j, as f16 hi (at [tt][ks][0]) and lo ([tt][ks][1])
  for (int q = t; q < ntile * 2 * 64; q += blockDim.x) {
    const int l = q & 63, ks = (q >> 6) & 1, tt = q >> 7;
    const float* cr;
    slot_center(32 * tt + (l & 31), cr);
    h8x vh, vl;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int f = 16 * ks + 8 * (l >> 5) + j;
      float c = (cr && f < F) ? cr[f] : 0.f;
      if (f == 30) c = cr ? -0.00390625f * s_cc[32 * tt + (l & 31)] : -65504.f;  // -|c|^2 / 256
      if (f == 31) c = 128.f;
      vh[j] = (_Float16)c;
      vl[j] = (_Float16)(c - (float)vh[j]);
    }
    char* dst = s_A + ((size_t)(tt * 2 + ks) * 2 * 64 + l) * 16;
    *reinterpret_cast<h8x*>(dst) = vh;
    *reinterpret_cast<h8x*>(dst + 64 * 16) = vl;
  }
  for (int q = t; q < ksum * F; q += blockDim.x) s_acc[q] = 0ull;
  for (int q = t; q < ksum; q += blockDim.x) s_cnt[q] = 0;
  if (t < kMaxFits) s_chg[t] = s_rec[t] = 0;
  __syncthreads();
  if (t <= kMaxFits) {  // per fit: max |c|^2 (the decision bound); 0 past the fits
    float m = 0.f;
    if (t < nf)
      for (int s = s_off8[t]; s < s_off8[t] + s_k[t]; ++s) m = fmaxf(m, s_cc[s]);
    s_cmax[t] = m;
  }
  __syncthreads();
  // the largest |c|^2 of the launch: the keys' offset delta, and past
  // kD2NormMax every pair goes to the exact chain
  float cmax_all = 0.f;
  for (int i = 0; i < nf; ++i) cmax_all = fmaxf(cmax_all, s_cmax[i]);
  const bool big = !(cmax_all <= kD2NormMax);

  // lane-indexed fit of each 8-slot group (read with v_readlane: wave-uniform)
  const int v_fit8 = lane < kD2Groups ? s_fit8[lane] : -1;
  const int64_t lo = (int64_t)blk * da.R, hi = min(S, lo + da.R);
  const int nchunk = hi > lo ? (int)((hi - lo + 31) / 32) : 0;
  const int r = lane & 31, h = lane >> 5;

  // ---- queues (rows of the current chunk, re-read from X: L2 hits); the
  // queue lengths are wave-uniform and live in scalar registers ----
  int nq_r = 0, nq_m = 0;
  // M-step of the queued changed (row, fit) pairs: two pairs per wave round,
  // lane = feature; four rounds' reads issued before their atomics
  auto flush_m = [&](int64_t r0) {
    const int f = r;  // feature
    for (int e0 = 0; e0 < nq_m; e0 += 8) {
      int v[4];
      float x[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int e = e0 + 2 * u + h;
        v[u] = e < nq_m ? w_mq[e] : -1;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) x[u] = (v[u] != -1 && f < F) ? X[(r0 + (v[u] & 0xFF)) * F + f] : 0.f;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (v[u] == -1 || f >= F) continue;
        const int fi = (v[u] >> 8) & 0xFF, lab = (v[u] >> 16) & 0xFF, old = (v[u] >> 24) & 0xFF;
        const long long q = fixq(x[u], s_e[f]);
        const int o = s_coff[fi], k = s_k[fi];
        atomicAdd(&s_acc[(o + lab) * F + f], (unsigned long long)q);
        if (old < k) atomicAdd(&s_acc[(o + old) * F + f], (unsigned long long)(-q));
        if (f == 0) {
          atomicAdd(&s_cnt[o + lab], 1);
          if (old < k) atomicAdd(&s_cnt[o + old], -1);
        }
      }
    }
    nq_m = 0;
    __builtin_amdgcn_wave_barrier();
  };
  // the queued near-tie (row, fit) pairs, two per wave round: lane (j = r,
  // half h) computes the exact fp32 chain of pair e0 + h to center j (the
  // nearest_centers bits: even features in .x, odd in .y, then .x + .y), and
  // the half's 32 lanes reduce to the top two (lowest index on ties)
  auto flush_r = [&](int64_t r0) {
    for (int e0 = 0; e0 < nq_r; e0 += 2) {
      const int e = e0 + h;
      const bool ev = e < nq_r;
      const int v = ev ? w_rq[e] : 0;
      const int row = v & 0xFF, fi = (v >> 8) & 0xFF;
      const int k = ev ? s_k[fi] : 0;
      const int j = r;
      float dd = __builtin_inff();
      if (j < k) {
        const float* xr = X + (r0 + row) * F;
        const float* cr = s_cenp[fi] + (size_t)j * F;
        f2v acc = f2v{0.f, 0.f};
        const int np = (F + 1) >> 1;  // pairs past F add exact zeros
#pragma unroll 2
        for (int p = 0; p < np; ++p) {
          const int f0 = 2 * p;
          const f2v xv = f2v{xr[f0], f0 + 1 < F ? xr[f0 + 1] : 0.f};
          const f2v x2 = __builtin_elementwise_fma(xv, f2v{s_a[f0], s_a[f0 + 1]}, f2v{s_b[f0], s_b[f0 + 1]});
          const f2v c = f2v{cr[f0], f0 + 1 < F ? cr[f0 + 1] : 0.f};
          const f2v d = x2 - c;
          acc = __builtin_elementwise_fma(d, d, acc);
        }
        dd = acc.x + acc.y;
      }
      // top two over the half (sequential-scan semantics: m1 the minimum at
      // the lowest index, m2 the second smallest value, duplicates counted)
      float m1 = dd, m2 = __builtin_inff();
      int lab = j;
#pragma unroll
      for (int o = 1; o < 32; o <<= 1) {
        const float pm1 = __shfl_xor(m1, o, 64), pm2 = __shfl_xor(m2, o, 64);
        const int plab = __shfl_xor(lab, o, 64);
        const bool take = pm1 < m1 || (pm1 == m1 && plab < lab);
        const float hi1 = take ? m1 : pm1;
        m2 = fminf(fminf(m2, pm2), hi1);
        m1 = take ? pm1 : m1;
        lab = take ? plab : lab;
      }
      const bool on = ev && j == 0;
      if (nq_m > 96) flush_m(r0);
      const int old = on ? (int)w_lab[fi * 32 + row] : 0;
      const bool ch = on && lab != old;
      if (ch) s_labp[fi][r0 + row] = (uint8_t)lab;
      if (on && ((da.bounds >> fi) & 1)) {  // exact distances: the bounded passes' bounds
        s_ubp[fi][r0 + row] = sqrtf(m1);
        s_lbp[fi][r0 + row] = k > 1 ? sqrtf(m2) : __builtin_inff();
      }
      const unsigned long long cm = __ballot(ch);
      if (ch) w_mq[nq_m + __popcll(cm & ((1ull << lane) - 1ull))] = row | (fi << 8) | (lab << 16) | (old << 24);
      nq_m = __builtin_amdgcn_readfirstlane(nq_m + (int)__popcll(cm));
      if (on) atomicAdd(&s_rec[fi], 1);
      if (ch) atomicAdd(&s_chg[fi], 1);
    }
    nq_r = 0;
    __builtin_amdgcn_wave_barrier();
  };

  // ---- chunk loads, one chunk ahead: lane (r, h) takes row r's features
  // 16 ks + 8 h + j (the B operand's); lane l < 2 nf the 16 labels of fit
  // l >> 1 at rows 16 (l & 1) .. + 15 (one buffer load: out of range reads 0)
  const __amdgpu_buffer_rsrc_t xrs = make_rsrc(X + lo * F, (hi > lo ? hi - lo : 0) * F * 4);  // this block's rows
  float xq[16];
  u4d lq = u4d{0u, 0u, 0u, 0u};
  const bool lq_on = lane < 2 * nf;
  uint8_t* const lq_base = lq_on ? s_labp[lane >> 1] : nullptr;
  auto load_chunk = [&](int ci) {
    const int64_t r0 = lo + (int64_t)ci * 32;
    const int nrow = (int)min((int64_t)32, hi - r0);
    const int64_t rr = r0 + (r < nrow ? r : nrow - 1);
    // buffer loads over the block's rows (out of range reads 0: no exec-mask
    // branch per load, one address); features past F are zeroed in the B build
    const int vo = (int)((rr - lo) * F) * 4;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int j = 0; j < 8; ++j)
        xq[8 * ks + j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(xrs, vo + (16 * ks + 8 * h + j) * 4, 0, 0));
    if (lq_on) {
      if (nrow == 32) {
        lq = *reinterpret_cast<const u4d*>(lq_base + r0 + (lane & 1) * 16);  // r0 % 32 == 0: aligned
      } else {  // the range's last, partial chunk: bytes (a 16-byte load would read past the rows)
        uint8_t b[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int row = (lane & 1) * 16 + i;
          b[i] = row < nrow ? lq_base[r0 + row] : (uint8_t)0;
        }
        lq = __builtin_bit_cast(u4d, b);
      }
    }
  };

  int ci = wid;
  if (ci < nchunk) load_chunk(ci);
  for (; ci < nchunk; ci += nw) {
    const int64_t r0 = lo + (int64_t)ci * 32;
    const int nrow = (int)min((int64_t)32, hi - r0);
    const bool valid = r < nrow;
    // this chunk's loads into LDS (rows for the queues, labels) and the B operands
    h8x bop[2], bol[2];
    float xx = 0.f;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int f = 16 * ks + 8 * h + j;
        const float x = f < F ? __builtin_fmaf(xq[8 * ks + j], s_a[f], s_b[f]) : 0.f;
        bop[ks][j] = (_Float16)x;
        bol[ks][j] = (_Float16)(x - (float)bop[ks][j]);
        xx = __builtin_fmaf(x, x, xx);
      }
    if (lq_on) *reinterpret_cast<u4d*>(w_lab + (lane >> 1) * 32 + (lane & 1) * 16) = lq;
    xx += d2_partner(xx);
    // the norm features 30 / 31 (lanes h = 1, k-step 1, j = 6 / 7)
    const float delta = kD2BScale * (xx + cmax_all) + kD2BAbs;
    const bool far = big || !(xx <= kD2NormMax);  // the exact chain decides every fit of this row
    {
      const float b31 = far ? 0.f : (-0.5f * xx - delta) * 0.0078125f;
      const _Float16 b31h = (_Float16)b31;
      const _Float16 b31l = (_Float16)(b31 - (float)b31h);
      bop[1][6] = h ? (_Float16)128.f : bop[1][6];
      bol[1][6] = h ? (_Float16)0.f : bol[1][6];
      bop[1][7] = h ? b31h : bop[1][7];
      bol[1][7] = h ? b31l : bol[1][7];
    }
    if (ci + nw < nchunk) load_chunk(ci + nw);  // the next chunk's loads fly during this one
    __builtin_amdgcn_wave_barrier();  // w_lab written
    // the old labels of the fits this lane decides (fi = h, h + 2, ...), packed
    // 4 per register (out of LDS once per chunk, not per close)
    constexpr int NLB = (kMaxFits + 1) / 2;
    unsigned olds[3] = {0u, 0u, 0u};
#pragma unroll
    for (int u = 0; u < NLB; ++u) {
      const int fi = 2 * u + h;
      const unsigned b = fi < nf ? (unsigned)w_lab[fi * 32 + r] : 0u;
      olds[u >> 2] |= b << (8 * (u & 3));
    }
    // fits close in pairs (fA = 2u, fA + 1): one exchange gives the lower
    // half fA's merged top two and the upper half fA + 1's, so every lane
    // decides one (row, fit) pair per close
    auto close2 = [&](int a1, int a2, int b1, int b2, int fA) {
      const int hb = h << 2;  // this half's slot bit
      const auto x1 = __builtin_amdgcn_permlane32_swap((unsigned)(a1 | hb), (unsigned)(b1 | hb), false, false);
      const auto x2 = __builtin_amdgcn_permlane32_swap((unsigned)(a2 | hb), (unsigned)(b2 | hb), false, false);
      const int p = (int)x1[0], q = (int)x1[1];
      const int k1 = min(p, q);
      const int k2 = min(max(p, q), min((int)x2[0], (int)x2[1]));
      const int fB = fA + 1;
      const int fi = fA + h;
      // this lane's fit constants from LDS (two addresses per wave: broadcast reads)
      const int kf = s_k[fi], o8 = s_off8[fi];
      const float cmx = s_cmax[fi];
      const int t0 = o8 >> 5;
      const int tile = (((k1 >> 5) ^ t0) & 1) ? t0 + 1 : t0;
      const int lab = 32 * tile + (k1 & 31) - o8;
      const float acc1 = __builtin_bit_cast(float, (unsigned)k1 & kD2KeyMask);
      const float acc2 = __builtin_bit_cast(float, (unsigned)k2 & kD2KeyMask);
      // (the row's delta rides in every accumulator: its rounding counts too)
      const float eb = kD2BScale * (xx + cmx + delta) + kD2BAbs;
      const bool act = valid && fi < nf;
      const bool tie = act && (far || (kf > 1 && !(acc1 - acc2 > 0.5f * eb)));
      const unsigned long long tm = __ballot(tie);
      if (tm) {
        if (nq_r + (int)__popcll(tm) > 64) flush_r(r0);
        if (tie) w_rq[nq_r + __popcll(tm & ((1ull << lane) - 1ull))] = r | (fi << 8);
        nq_r = __builtin_amdgcn_readfirstlane(nq_r + (int)__popcll(tm));
      }
      if (nq_m > 64) flush_m(r0);
      const int u = fA >> 1;
      const unsigned w = (u >> 2) == 0 ? olds[0] : ((u >> 2) == 1 ? olds[1] : olds[2]);
      const int old = (int)((w >> (8 * (u & 3))) & 0xFFu);
      const bool on = act && !tie;
      const bool ch = on && lab != old;
      if (ch) s_labp[fi][r0 + r] = (uint8_t)lab;  // (the pointer only where a label changed)
      if (da.bounds) {  // (kind 6 only): d = -2 (acc + delta)
        if (on && ((da.bounds >> fi) & 1)) {
          const float d1 = -2.f * (acc1 + delta), d2 = -2.f * (acc2 + delta);
          s_ubp[fi][r0 + r] = sqrtf(fmaxf(d1 + eb, 0.f)) * (1.f + 1e-6f);
          s_lbp[fi][r0 + r] = kf > 1 ? sqrtf(fmaxf(d2 - eb, 0.f)) * (1.f - 1e-6f) : __builtin_inff();
        }
      }
      const unsigned long long cm = __ballot(ch);
      if (cm) {
        if (ch) w_mq[nq_m + __popcll(cm & ((1ull << lane) - 1ull))] = r | (fi << 8) | (lab << 16) | (old << 24);
        nq_m = __builtin_amdgcn_readfirstlane(nq_m + (int)__popcll(cm));
        if (lane == 0) atomicAdd(&s_chg[fA], __popcll(cm & 0xFFFFFFFFull));
        if (lane == 32 && fB < nf) atomicAdd(&s_chg[fB], __popcll(cm >> 32));
      }
    };
    // running keys of the current fit; the finished even fit's; the pairs
    // closed after the tile's values are consumed (no accumulator live across
    // a close)
    constexpr int KMAX = 0x7FFFFFFF;
    int vmask;
    asm volatile("v_mov_b32 %0, 0xffffffc0" : "=v"(vmask));
    int cur = -1;
    int m1 = KMAX, m2 = KMAX, s1 = KMAX, s2 = KMAX;
    int pa1[3], pa2[3], pb1[3], pb2[3], pf[3];
    int npend = 0;
    auto push = [&](int b1, int b2, int fA) {
#pragma unroll
      for (int q = 0; q < 3; ++q)
        if (q == npend) {
          pa1[q] = s1;
          pa2[q] = s2;
          pb1[q] = b1;
          pb2[q] = b2;
          pf[q] = fA;
        }
      ++npend;
    };
    auto finish = [&]() {  // cur's slots ended
      if ((cur & 1) == 0) {
        s1 = m1;
        s2 = m2;
        if (cur == nf - 1) push(KMAX, KMAX, cur);
      } else {
        push(m1, m2, cur - 1);
      }
    };
    for (int tt = 0; tt < ntile; ++tt) {
      const char* ap = s_A + ((size_t)(4 * tt) * 64 + lane) * 16;
      const h8x a0h = *reinterpret_cast<const h8x*>(ap);
      const h8x a0l = *reinterpret_cast<const h8x*>(ap + 1024);
      const h8x a1h = *reinterpret_cast<const h8x*>(ap + 2048);
      const h8x a1l = *reinterpret_cast<const h8x*>(ap + 3072);
      f16x acc = {};
      acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0h, bop[0], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1h, bop[1], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0l, bop[0], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1l, bop[1], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0h, bol[0], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1h, bol[1], acc, 0, 0, 0);
      npend = 0;
      const int par = (tt & 1) << 5;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int g = 4 * tt + j;
        const int fi = __builtin_amdgcn_readlane(v_fit8, g);
        if (fi != cur) {  // wave-uniform
          if (cur >= 0) finish();
          cur = fi;
          m1 = m2 = KMAX;
        }
        if (fi < 0) continue;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float v = acc[4 * j + i];  // (a bit_cast of the vector element itself reads element 0)
          int sidx;  // opaque, or the compiler splits the and-or around the constant
          asm("s_or_b32 %0, %1, %2" : "=s"(sidx) : "s"(par), "i"(8 * j + i));
          // (bits & mask) | slot code: one v_and_or_b32 (the mask in a VGPR, the
          // code in an SGPR); compiled code, so the MFMA-result wait states hold
          const int key = (int)((__builtin_bit_cast(unsigned, v) & (unsigned)vmask) | (unsigned)sidx);
          int m2n;
          asm("v_med3_i32 %0, %1, %2, %3" : "=v"(m2n) : "v"(m1), "v"(key), "v"(m2));
          m2 = m2n;
          m1 = min(m1, key);
        }
      }
      if (tt == ntile - 1 && cur >= 0) {  // the last fit ends with the last tile
        finish();
        cur = -1;
      }
#pragma unroll 1
      for (int q = 0; q < npend; ++q) {
        const int c1 = q == 0 ? pa1[0] : q == 1 ? pa1[1] : pa1[2];
        const int c2 = q == 0 ? pa2[0] : q == 1 ? pa2[1] : pa2[2];
        const int d1 = q == 0 ? pb1[0] : q == 1 ? pb1[1] : pb1[2];
        const int d2 = q == 0 ? pb2[0] : q == 1 ? pb2[1] : pb2[2];
        const int fq = __builtin_amdgcn_readfirstlane(q == 0 ? pf[0] : q == 1 ? pf[1] : pf[2]);
        close2(c1, c2, d1, d2, fq);
      }
    }
    flush_r(r0);
    flush_m(r0);
  }
  __syncthreads();
  // ---- records: per fit [dQ_hi kF | dQ_lo kF | dcount k | changed | recomputed | 0 | 0] ----
  for (int fi = 0; fi < nf; ++fi) {
    const mw_lloyd_fit& fit = fits.f[fi];
    const int k = fit.k, o = s_coff[fi];
    const int rlen = lloyd_rec(k, F);
    double* out = reinterpret_cast<double*>(fit.ws) + (size_t)blk * rlen;
    for (int q = t; q < k * F; q += blockDim.x) {
      double hq, lq;
      limbs((long long)s_acc[o * F + q], hq, lq);
      out[q] = hq;
      out[k * F + q] = lq;
    }
    for (int j = t; j < k; j += blockDim.x) out[2 * k * F + j] = (double)s_cnt[o + j];
    if (t == 0) {
      out[2 * k * F + k] = (double)s_chg[fi];
      out[2 * k * F + k + 1] = (double)s_rec[fi];
      out[2 * k * F + k + 2] = 0.0;
      out[2 * k * F + k + 3] = 0.0;
    }
  }
}

// Fits [0, n) at 8-aligned slot offsets; false when they need more than
// kD2Slots slots or a fit has more than 64 centers
static inline bool dense2_plan(const mw_lloyd_fit* h, int n, int64_t S, int F, Dense2Arg& da) {
  if (F > 30 || n > kMaxFits) return false;  // features 30, 31 carry the norms
  da.nf = n;
  da.off8[0] = 0;
  da.coff[0] = 0;
  for (int g = 0; g < n; ++g) {
    if (h[g].k > kD2MaxK || h[g].k < 1) return false;
    da.off8[g + 1] = da.off8[g] + ((h[g].k + 7) & ~7);
    da.coff[g + 1] = da.coff[g] + h[g].k;
  }
  if (da.off8[n] > kD2Slots) return false;
  for (int g = n + 1; g <= kMaxFits; ++g) da.off8[g] = da.off8[n], da.coff[g] = da.coff[n];
  da.ntile = (da.off8[n] + 31) / 32;
  int G = lloyd_blocks(S, F);  // never more records than the fits' workspaces hold
  if (G > kD2MaxBlocks) G = kD2MaxBlocks;
  int64_t R = (S + G - 1) / G;
  R = (R + 31) & ~(int64_t)31;
  da.G = (int)((S + R - 1) / R);
  da.R = R;
  return true;
}

}  // namespace mw
