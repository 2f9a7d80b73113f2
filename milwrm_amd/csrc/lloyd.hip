// The Lloyd iteration of sklearn's KMeans (lloyd_iter_chunked_dense,
// _k_means_lloyd.pyx:23-218; _inertia_dense, _k_means_common.pyx:94-124) for
// one or several fits over the same rows (the k sweep of find_optimal_k,
// MILWRM.py:29-90), on MI355X (gfx950, wave64).
//
// E-step with distance bounds (Hamerly): per row the pass keeps ub >= the
// distance to its own center and lb <= the distance to the second closest.
// Between passes the centers move by drift_j, so ub += drift_label and lb -=
// max_j drift_j; a row whose ub is below max(lb, half the separation of its
// center from the nearest other center) by a relative margin kEps keeps its
// label without reading its features.  The margin (1e-4) is far above the
// fp32 rounding of the distances (F * 2^-24), so a skipped row always gets
// the label the full computation would give it: labels are exactly those of
// the plain argmin (strict '<', lowest index on ties).  Rows that fail the
// test are read, their own-center distance tightens ub (second test), and
// rows still undecided get all k distances.
//
// M-step, incremental and exact: every raw feature value is rounded once to a
// per-feature fixed point, q = rint(x * 2^e_f) with |q| < 2^41 (e_f from the
// column's max |x|), and a row whose label changes moves its q from the old
// label's sums to the new one's as int64 adds.  Integer sums do not depend on
// order, so the per-cluster sums equal the full recomputation, bit for bit,
// whatever the partition of rows into blocks, tiles or ranks: results are
// identical across 1 / 2 / 4 / 8 GPUs.  Per-block records carry each int64
// as two integer-valued fp64 limbs (hi = floor(v / 2^32), lo = v - hi*2^32),
// which the fixed-order fp64 fold and an RCCL fp64 all-reduce add exactly.
// The host keeps the running sums (kmeans.py).
//
// Inertia (modes 1 and 2) in the same fixed point: per row rint(D * 2^e_d).
#include <math.h>
#include <stdlib.h>

#include "kmeans_common.h"

namespace mw {
// Row blocks of the Lloyd passes.  At F <= 32 the tile, first, final and list
// passes hold three blocks per CU, so 1024 blocks ran in 1.33 rounds (a
// second round on a third of the chip); 3 x 256 CUs run in one: config-2 fit
// 7.36 -> 7.20 ms (MW_KBLOCKS A/B, profiles/r05/grid/).  The passes' sums are
// exact integers, so labels, centers and inertia do not depend on the grid
// (k-means++ keeps kblocks: its fp64 potentials are summed per block).
constexpr int kLloydBlocksF32 = 3 * 256;
static inline int lloyd_blocks(int64_t S, int F) {
  const int g = kblocks(S);
  return (F <= 32 && g > kLloydBlocksF32) ? kLloydBlocksF32 : g;
}
static inline int64_t lloyd_rows(int64_t S, int F) {
  int64_t tiles = (S + kT - 1) / kT;
  if (tiles < 1) tiles = 1;
  const int g = lloyd_blocks(S, F);
  return ((tiles + g - 1) / g) * kT;
}
}  // namespace mw

namespace mw {

constexpr int kMaxFits = 24;
constexpr float kEps = 1e-4f;  // bound-test margin (relative)

struct LloydFitsArg {
  mw_lloyd_fit f[kMaxFits];
};

__host__ __device__ inline size_t lloyd_al256(size_t x) { return (x + 255) & ~(size_t)255; }
// kList workspace after the G block records: per-block list lengths [G]
// int32, then per-block lists of undecided row indices [G][R] int32
__host__ __device__ inline size_t lloyd_list_off(int G, int k, int F) {
  return lloyd_al256((size_t)G * lloyd_rec(k, F) * sizeof(double));
}

// squared distance of the scaled row to one center (the same fp32 chain as
// nearest_centers: even features in .x, odd in .y, then .x + .y)
template <int FMAX>
__device__ __forceinline__ float dist_one(const f2v (&x2)[FMAX / 2], const f2v* cT, int j) {
  f2v acc = f2v{0.f, 0.f};
#pragma unroll
  for (int p = 0; p < FMAX / 2; ++p) {
    const f2v d = x2[p] - cT[p * 64 + j];
    acc = __builtin_elementwise_fma(d, d, acc);
  }
  return acc.x + acc.y;
}

// bytes of one wave's row tile: 64 rows x FMAX floats; FMAX = 64: 64 rows x
// F floats and FMAX - F floats more (zeroed: the padded pairs load_scaled_row
// reads past the last row), so at F = 50 two blocks fit a CU instead of one
// (at F <= 32 the full tile loads measured faster)
__host__ __device__ inline size_t lloyd_tile_bytes(int FMAX, int F) {
  if (FMAX != 64) return (size_t)64 * FMAX * 4;
  return (((size_t)64 * F + (FMAX - F) + 3) & ~(size_t)3) * 4;
}

// rows per bound-test chunk (kQueue passes): queue of u16 offsets (4096: 2
// blocks per CU for the LDS, the sweep's queue passes 15 % slower)
constexpr int kChunk = 2048;
static_assert(kChunk % 1024 == 0, "chunk = whole 4-wave x 256-row groups");

// small per-block LDS state (size a multiple of 16 bytes)
struct alignas(16) LloydSmall {
  float a[64], b[64];
  int e[64];
  float drift[64], half[64];
  int cnt[64];
  double red[4];
  long long red64[4];
  int qn, pad[3];
};

// LDS of one block: LloydSmall | pair-major centers | cluster sums k x F (int64, mode 0) |
// per-wave row tiles | per-wave labels (64 int) | chunk queue (sparse mode 0)
__host__ __device__ inline size_t lloyd_lds_bytes(int FMAX, int k, int F, int mode, int kind) {
  size_t b = sizeof(LloydSmall) + cent_t_bytes(64, FMAX);
  if (mode == 0) b += ((size_t)k * F * 8 + 15) & ~(size_t)15;
  b += 4 * (lloyd_tile_bytes(FMAX, F) + 64 * 4);
  if (mode == 0 && kind == 2) b += (size_t)kChunk * 2;  // kQueue
  return b;
}

// Kinds of mode-0 pass (mw_lloyd_pass `kind`):
constexpr int kFirst = 0;  // every row unlabelled: full E-step, sums of all rows
constexpr int kTile = 1;   // stream every tile's rows; bounds skip the E-step per lane
constexpr int kQueue = 2;  // stream only the row state; read the undecided rows
constexpr int kFirstAtomic = 3;  // kFirst with the sums by LDS atomics (A/B)
constexpr int kList = 4;  // kQueue as two launches: lloyd_mark_kernel lists, this kernel reads
constexpr int kFirstSum = 7;  // kFirst with per-feature fp64 sums of label-sorted rows (internal, k <= 16)
constexpr int kListGiven = 8;  // kList over lists already written (mw_lloyd_list_moved)

// One pass of fit g = blockIdx.x % n over row block blockIdx.x / n (the n
// blocks that read one row block are dispatched together: rows that several
// fits read come from the on-die caches).
//   MODE 0, kFirst: full E-step over streamed 64-row tiles; the cluster sums
//     of each tile's rows as a one-hot GEMM on the fp64 matrix cores
//     (A[label][row] = 1, B[row][f] = q(x_f): integer products and sums below
//     2^53 are exact), flushed to int64 every 32 tiles.
//   MODE 0, kTile: streamed tiles with the row state; the bound test per row,
//     the own-center distance for undecided rows, all k distances where still
//     undecided; changed rows move their q between cluster sums (LDS int64
//     atomics, lane = feature).  For passes where most rows are undecided.
//   MODE 0, kQueue: per chunk of kChunk rows the bound test streams only the
//     row state (4 rows per lane) and queues the rows it cannot decide; waves
//     gather the queued rows 64 at a time and finish them as kTile does.  For
//     passes where few rows are undecided.
//   MODE 0, kList: lloyd_mark_kernel (launched first) ran the bound test over
//     the block's whole range and listed its undecided rows; waves take the
//     list 64 rows at a time (state loads issued with the list entries, then
//     the gather) and finish them as kQueue does, with no block barrier.
//   MODE 1: full E-step (labels updated) + inertia of the new labels
//   MODE 2: inertia of the current labels
template <int FMAX, int MODE, int KIND, int MBT>
__device__ __forceinline__ void lloyd_pass_body(const float* __restrict__ X, int64_t S, int F,
                                                const float* __restrict__ ga, const float* __restrict__ gb,
                                                const int* __restrict__ qexp, const LloydFitsArg& fits, int n,
                                                int64_t R) {
  constexpr int NV = FMAX / 4;
  constexpr int RP = 64 / FMAX;  // changed rows folded per M-step round (lane = row slot x feature)
  constexpr int NB = FMAX <= 16 ? 1 : FMAX / 16;  // 16-feature MFMA column blocks
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int g = blockIdx.x % n, blk = blockIdx.x / n;
  const mw_lloyd_fit& fit = fits.f[g];
  const int k = fit.k;
  const int iexp = fit.inertia_exp;
  const int t = threadIdx.x, lane = t & 63, nw = blockDim.x >> 6;
  const int wid = __builtin_amdgcn_readfirstlane(t >> 6);
  // every LDS variable lives in the dynamic region at 16-byte aligned offsets
  // (static __shared__ would shift the dynamic base off 16 bytes:
  // misaligned 8-byte accesses replay, misaligned 64-bit atomics are unsafe)
  char* sp = smem;
  LloydSmall* sm = reinterpret_cast<LloydSmall*>(sp);
  sp += sizeof(LloydSmall);
  float* s_a = sm->a;
  float* s_b = sm->b;
  int* s_e = sm->e;
  float* s_drift = sm->drift;
  float* s_half = sm->half;
  int* s_cnt = sm->cnt;
  int& s_qn = sm->qn;
  double* s_red = sm->red;
  long long* s_red64 = sm->red64;
  f2v* s_cT = reinterpret_cast<f2v*>(sp);
  sp += cent_t_bytes(64, FMAX);
  unsigned long long* s_acc = reinterpret_cast<unsigned long long*>(sp);
  if (MODE == 0) sp += ((size_t)k * F * 8 + 15) & ~(size_t)15;
  const int tile_fl = (int)(lloyd_tile_bytes(FMAX, F) / 4);
  float* s_tile = reinterpret_cast<float*>(sp + (size_t)wid * tile_fl * 4);
  sp += 4 * (size_t)tile_fl * 4;
  int* s_lab = reinterpret_cast<int*>(sp) + wid * 64;
  sp += 4 * 64 * 4;
  uint16_t* s_q = reinterpret_cast<uint16_t*>(sp);
  // tiles and gathers write only the 64 x F floats of a tile; the scaled-row
  // read of the last row runs past them (padded features, times a zero
  // scaler), so the rest of the wave's tile buffer must hold finite values,
  // never stale LDS bits (NaN * 0 = NaN: nondeterministic labels)
  for (int q = 64 * F + lane; q < tile_fl; q += 64) s_tile[q] = 0.f;

  load_centers_T<FMAX, 64>(fit.centers, k, F, s_cT);
  for (int f = t; f < 64; f += blockDim.x) {
    s_a[f] = f < F ? ga[f] : 0.f;  // padded features scale to exactly 0
    s_b[f] = f < F ? gb[f] : 0.f;
    s_e[f] = f < F ? qexp[f] : 0;
  }
  constexpr bool BOUNDS = MODE == 0 && (KIND == kTile || KIND == kQueue || KIND == kList);
  for (int j = t; j < 64; j += blockDim.x) {
    s_drift[j] = (BOUNDS && j < k) ? fit.drift[j] : 0.f;
    s_half[j] = (BOUNDS && j < k) ? fit.half_sep[j] : 0.f;
    s_cnt[j] = 0;
  }
  if (t == 0) s_qn = 0;
  if (MODE == 0)
    for (int q = t; q < k * F; q += blockDim.x) s_acc[q] = 0ull;
  __syncthreads();
  const float dmax = fit.drift_max;

  const int64_t lo = (int64_t)blk * R, hi = min(S, lo + R);
  const int64_t total = S * (int64_t)F, n4 = total >> 2;
  const int64_t nb = hi > lo ? hi - lo : 0;
  uint8_t* __restrict__ labels = fit.labels;
  float* __restrict__ ubuf = fit.ub;
  float* __restrict__ lbuf = fit.lb;
  long long changed = 0, recomputed = 0, inert = 0;

  // ---- M-step of the changed rows of the wave's tile (lane = row slot x feature) ----
  auto move_rows = [&](unsigned long long cm, int lab, int lab_old) {
    const int sub = lane / FMAX, f = lane - sub * FMAX;
    while (cm != 0ull) {  // wave-uniform
      int jsel = -1;
#pragma unroll
      for (int r = 0; r < RP; ++r) {
        if (cm != 0ull) {
          const int j = __builtin_ctzll(cm);
          cm &= cm - 1ull;
          if (sub == r) jsel = j;
        }
      }
      const int jj = jsel < 0 ? 0 : jsel;
      const int ln = __shfl(lab, jj, 64), lo_ = __shfl(lab_old, jj, 64);
      if (jsel >= 0 && f < F) {
        const long long q = fixq(s_tile[jj * F + f], s_e[f]);
        atomicAdd(&s_acc[ln * F + f], (unsigned long long)q);
        if (lo_ < k) atomicAdd(&s_acc[lo_ * F + f], (unsigned long long)(-q));
        if (f == 0) {
          atomicAdd(&s_cnt[ln], 1);
          if (lo_ < k) atomicAdd(&s_cnt[lo_], -1);
        }
      }
    }
  };
  // ---- the undecided rows of a staged tile: tighten, full E-step, state, sums ----
  // (lane = row of the tile; `need`: the drifted bounds did not decide the row)
  auto finish_rows = [&](bool valid, bool need, int lab_old, float ub, float lbv, float thr,
                         auto&& store) {
    const bool has_old = lab_old < k;
    const int la = has_old ? lab_old : 0;
    f2v x2[FMAX / 2];
    load_scaled_row<FMAX>(s_tile, lane, F, s_a, s_b, x2);
    const float da = dist_one<FMAX>(x2, s_cT, la);
    bool need2 = need;
    if (need && has_old) {
      ub = sqrtf(da);
      need2 = !(ub * (1.f + kEps) < thr);
    }
    int lab = lab_old;
    if (__ballot(need2) != 0ull) {
      int ln;
      float m1, m2;
      nearest_centers<FMAX, 64, true>(x2, s_cT, k, ln, m1, m2);
      if (need2) {
        lab = ln;
        ub = sqrtf(m1);
        lbv = k > 1 ? sqrtf(m2) : __builtin_inff();
        recomputed += 1;
      }
    }
    const bool ch = valid && lab != lab_old;
    changed += ch ? 1 : 0;
    store(valid, ch, lab, ub, lbv);
    move_rows(__ballot(ch), lab, lab_old);
  };

  // the rows s_idx[0 .. cnt_b) into the wave tile (row j at s_tile + j*F)
  auto gather = [&](const int* s_idx, int cnt_b) {
    if ((F & 1) == 0) {
      const int P2 = F >> 1;
      int j = lane / P2, c = lane - (lane / P2) * P2;  // piece (j, c) = p, stepped by 64
      const int dj = 64 / P2, dc = 64 - dj * P2;
      constexpr int kGB = 8;
      for (int i0 = 0; i0 < P2; i0 += kGB) {
        f2v v[kGB];
        int dst[kGB];
#pragma unroll
        for (int i = 0; i < kGB; ++i) {
          const bool ok = i0 + i < P2;
          const int64_t rj = s_idx[j < cnt_b ? j : 0];
          v[i] = ok ? *reinterpret_cast<const f2v*>(X + rj * F + 2 * c) : f2v{0.f, 0.f};
          dst[i] = ok ? j * F + 2 * c : -1;
          j += dj;
          c += dc;
          if (c >= P2) { c -= P2; ++j; }
        }
#pragma unroll
        for (int i = 0; i < kGB; ++i)
          if (dst[i] >= 0) *reinterpret_cast<f2v*>(s_tile + dst[i]) = v[i];
      }
    } else {
      for (int p = lane; p < 64 * F; p += 64) {
        const int j = p / F, c = p - j * F;
        const int64_t rj = s_idx[j < cnt_b ? j : 0];
        s_tile[j * F + c] = X[rj * F + c];
      }
    }
  };

  if constexpr (MODE == 0 && KIND == kQueue) {
    // =========================== queue pass ===========================
    for (int64_t c0 = lo; c0 < hi; c0 += kChunk) {
      const int clen = (int)min((int64_t)kChunk, hi - c0);
      // ---- phase 1: bound test, 4 consecutive rows per lane, queue the undecided ----
      // (the wave's whole share of the chunk, kChunk / (4 waves * 256 rows) =
      // 4 row groups, is loaded before any of it is used: 12 loads in flight)
      constexpr int NI = kChunk / (4 * 256);
      uint32_t lab4[NI];
      f4v ub4[NI], lb4[NI];
#pragma unroll
      for (int it = 0; it < NI; ++it) {
        const int off0 = (wid + it * nw) * 256 + 4 * lane;
        const int64_t r0 = c0 + off0;
        if (off0 + 3 < clen) {  // r0 % 4 == 0: lo, c0 and off0 are multiples of 4
          lab4[it] = *reinterpret_cast<const uint32_t*>(labels + r0);
          ub4[it] = *reinterpret_cast<const f4v*>(ubuf + r0);
          lb4[it] = *reinterpret_cast<const f4v*>(lbuf + r0);
        } else {
          lab4[it] = 0xFFFFFFFFu;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            if (off0 + i < clen) {
              lab4[it] = (lab4[it] & ~(0xFFu << (8 * i))) | ((uint32_t)labels[r0 + i] << (8 * i));
              ub4[it][i] = ubuf[r0 + i];
              lb4[it][i] = lbuf[r0 + i];
            }
          }
        }
      }
#pragma unroll
      for (int it = 0; it < NI; ++it) {
        const int off0 = (wid + it * nw) * 256 + 4 * lane;
        if ((wid + it * nw) * 256 >= clen) break;  // wave-uniform
        const int64_t r0 = c0 + off0;
        bool skip[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int lab_old = (lab4[it] >> (8 * i)) & 0xFF;
          const int la = lab_old < k ? lab_old : 0;
          const float ub = ub4[it][i] + s_drift[la];
          const float lbv = lb4[it][i] - dmax;
          const float thr = fmaxf(lbv, s_half[la]);
          const bool valid = off0 + i < clen;
          const bool need = valid && (lab_old >= k || !(ub * (1.f + kEps) < thr));
          skip[i] = valid && !need;
          ub4[it][i] = ub;
          lb4[it][i] = lbv;
          const unsigned long long m = __ballot(need);
          if (m != 0ull) {
            int qb = 0;
            if (lane == 0) qb = atomicAdd(&s_qn, __popcll(m));
            qb = __shfl(qb, 0, 64);
            if (need) s_q[qb + __popcll(m & ((1ull << lane) - 1ull))] = (uint16_t)(off0 + i);
          }
        }
        if (skip[0] && skip[1] && skip[2] && skip[3]) {
          *reinterpret_cast<f4v*>(ubuf + r0) = ub4[it];
          *reinterpret_cast<f4v*>(lbuf + r0) = lb4[it];
        } else {
#pragma unroll
          for (int i = 0; i < 4; ++i)
            if (skip[i]) {
              ubuf[r0 + i] = ub4[it][i];
              lbuf[r0 + i] = lb4[it][i];
            }
        }
      }
      __syncthreads();
      const int nq = s_qn;
      if (t == 0) inert += nq;  // mode 0: the record's inertia slots count the rows read
      // ---- phase 2: the queued rows, 64 per wave batch ----
      for (int e0 = wid * 64; e0 < nq; e0 += nw * 64) {
        const int cnt_b = min(64, nq - e0);
        const bool valid = lane < cnt_b;
        const int64_t r = c0 + s_q[e0 + (valid ? lane : 0)];
        // gather the batch's rows into the wave tile (row j at s_tile + j*F)
        if ((F & 1) == 0) {
          // pieces (row j, pair c) = lane + 64 i, in batches of kGB loads in
          // flight (one load -> store round trip per piece made this phase
          // latency-bound)
          const int P2 = F >> 1;
          int j = lane / P2, c = lane - (lane / P2) * P2;  // piece (j, c) = p, stepped by 64
          const int dj = 64 / P2, dc = 64 - dj * P2;
          constexpr int kGB = 8;
          for (int i0 = 0; i0 < P2; i0 += kGB) {
            f2v v[kGB];
            int dst[kGB];
#pragma unroll
            for (int i = 0; i < kGB; ++i) {
              const bool ok = i0 + i < P2;
              const int64_t rj = c0 + s_q[e0 + (j < cnt_b ? j : 0)];
              v[i] = ok ? *reinterpret_cast<const f2v*>(X + rj * F + 2 * c) : f2v{0.f, 0.f};
              dst[i] = ok ? j * F + 2 * c : -1;
              j += dj;
              c += dc;
              if (c >= P2) { c -= P2; ++j; }
            }
#pragma unroll
            for (int i = 0; i < kGB; ++i)
              if (dst[i] >= 0) *reinterpret_cast<f2v*>(s_tile + dst[i]) = v[i];
          }
        } else {
          for (int p = lane; p < 64 * F; p += 64) {
            const int j = p / F, c = p - j * F;
            const int64_t rj = c0 + s_q[e0 + (j < cnt_b ? j : 0)];
            s_tile[j * F + c] = X[rj * F + c];
          }
        }
        const int lab_old = labels[r];
        const int la = lab_old < k ? lab_old : 0;
        const float ub = ubuf[r] + s_drift[la];
        const float lbv = lbuf[r] - dmax;
        const float thr = fmaxf(lbv, s_half[la]);
        finish_rows(valid, valid, lab_old, ub, lbv, thr,
                    [&](bool v, bool ch, int lab, float u, float l) {
                      if (v) {
                        if (ch) labels[r] = (uint8_t)lab;
                        ubuf[r] = u;
                        lbuf[r] = l;
                      }
                    });
      }
      __syncthreads();
      if (t == 0) s_qn = 0;
      __syncthreads();
    }
  } else if constexpr (MODE == 0 && KIND == kList) {
    // ============================ list pass =============================
    // One stage per wave: the listed rows 64 at a time (their row state
    // loaded with the list entries, before the gather), then finish_rows on
    // the batch: the own-center distance tightens the upper bound, and the
    // rows it does not decide run the k-distance E-step in the same wave
    // (lanes of decided rows idle).  The decisions are those of every other
    // pass kind (same tests, same arithmetic): same labels, same sums.
    const int G = (int)(gridDim.x / n);
    const char* wsb = reinterpret_cast<const char*>(fit.ws);
    const size_t loff = lloyd_list_off(G, k, F);
    const int nq = reinterpret_cast<const int*>(wsb + loff)[blk];
    if (t == 0) inert = nq;  // mode 0: the record's inertia slots count the rows read
    const int* __restrict__ list =
        reinterpret_cast<const int*>(wsb + loff + lloyd_al256((size_t)G * 4)) + (size_t)blk * R;
    int* s_row = s_lab;  // the batch's 64 row indices (per wave)
    for (int e0 = wid * 64; e0 < nq; e0 += nw * 64) {
      const int cnt_b = min(64, nq - e0);
      const bool valid = lane < cnt_b;
      const int64_t r = list[e0 + (valid ? lane : 0)];
      // the row state does not depend on the gather: its loads go out first
      const int lab_old = labels[r];
      const float ub_in = ubuf[r], lb_in = lbuf[r];
      s_row[lane] = (int)r;
      __builtin_amdgcn_wave_barrier();
      gather(s_row, cnt_b);
      const int la = lab_old < k ? lab_old : 0;
      const float ub = ub_in + s_drift[la];
      const float lbv = lb_in - dmax;
      const float thr = fmaxf(lbv, s_half[la]);
      finish_rows(valid, valid, lab_old, ub, lbv, thr,
                  [&](bool v, bool ch, int lab, float u, float l) {
                    if (v) {
                      if (ch) labels[r] = (uint8_t)lab;
                      ubuf[r] = u;
                      lbuf[r] = l;
                    }
                  });
      __builtin_amdgcn_wave_barrier();  // s_row is rewritten by the next batch
    }
  } else {
    // ========================== streamed tiles ==========================
    if (MODE == 0 && t == 0) inert = nb;  // mode 0: the record's inertia slots count the rows read
    const int ntile = hi > lo ? (int)((hi - lo + 63) / 64) : 0;
    const __amdgpu_buffer_rsrc_t rx = make_rsrc(X + lo * F, (S - lo) * F * 4);
    const __amdgpu_buffer_rsrc_t rl = make_rsrc(labels + lo, nb);
    const __amdgpu_buffer_rsrc_t ru = make_rsrc(ubuf ? (void*)(ubuf + lo) : (void*)X, ubuf ? nb * 4 : 0);
    const __amdgpu_buffer_rsrc_t rw = make_rsrc(lbuf ? (void*)(lbuf + lo) : (void*)X, lbuf ? nb * 4 : 0);
    const int tile_bytes = 64 * F * 4;
    const int kk = lane >> 4, mm = lane & 15;  // MFMA operand lane map
    // kFirst: MBT blocks of 16 labels x NB blocks of 16 features in fp64
    // accumulators (the launcher picks MBT = ceil(k / 16), MBT * NB <= 4)
    constexpr int MBX = MBT * NB;
    constexpr int MB = MBT;
    constexpr bool mfma_m = MODE == 0 && KIND == kFirst;
    // kFirstSum: lane = feature, one fp64 sum per label of the q of the
    // label's rows (integers below 2^41: exact; flushed every 32 tiles)
    constexpr int KS = (MODE == 0 && KIND == kFirstSum) ? 16 : 1;
    double fsum[KS];
#pragma unroll
    for (int j = 0; j < KS; ++j) fsum[j] = 0.0;
    const int fe = lane < F ? s_e[lane] : 0;
    static_assert(KIND != kFirstAtomic || MODE == 0, "atomic first pass is mode 0");
    typedef double d4v __attribute__((ext_vector_type(4)));
    d4v acc[mfma_m ? MBX : 1];
#pragma unroll
    for (int i = 0; i < (mfma_m ? MBX : 1); ++i) acc[i] = d4v{0.0, 0.0, 0.0, 0.0};
    int since_flush = 0;
    auto flush = [&]() {
      if constexpr (MODE == 0 && KIND == kFirst) {
#pragma unroll
        for (int i = 0; i < MBX; ++i) {
          {
            const int mb = i / NB, nbk = i - mb * NB;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int lab_i = 16 * mb + kk + 4 * r, f = 16 * nbk + mm;  // f64 D map: row (l>>4)+4r, col l&15
              if (lab_i < k && f < F && acc[i][r] != 0.0)
                atomicAdd(&s_acc[lab_i * F + f], (unsigned long long)(long long)acc[i][r]);
            }
          }
          acc[i] = d4v{0.0, 0.0, 0.0, 0.0};
        }
      }
      if constexpr (MODE == 0 && KIND == kFirstSum) {
#pragma unroll
        for (int j = 0; j < KS; ++j) {
          if (j < k && lane < F && fsum[j] != 0.0)
            atomicAdd(&s_acc[j * F + lane], (unsigned long long)(long long)fsum[j]);
          fsum[j] = 0.0;
        }
      }
    };

    f4v v[NV];
    int lab_next = 0;
    float ub_next = 0.f, lb_next = 0.f;
    auto fetch = [&](int tt) {
      tt = tt < ntile ? tt : ntile - 1;
      lab_next = __builtin_amdgcn_raw_buffer_load_b8(rl, lane, tt * 64, 0);
      if (BOUNDS) {
        ub_next = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(ru, lane * 4, tt * 256, kStreamAux));
        lb_next = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rw, lane * 4, tt * 256, kStreamAux));
      }
#pragma unroll
      for (int i = 0; i < NV; ++i)  // only the vectors that hold the tile's 64 x F floats
        if (FMAX != 64 || i * 1024 < tile_bytes)
          v[i] = __builtin_bit_cast(f4v, __builtin_amdgcn_raw_buffer_load_b128(rx, lane * 16 + i * 1024,
                                                                               tt * tile_bytes, kStreamAux));
    };
    int tc = wid;
    if (tc < ntile) fetch(tc);
    for (; tc < ntile; tc += nw) {
      const int64_t r0 = lo + (int64_t)tc * 64;
      const int nrow = (int)min((int64_t)64, hi - r0);
      const bool valid = lane < nrow;
      const int lab_old = lab_next;
      const float ub_in = ub_next, lb_in = lb_next;
      {
        f4v* s4 = reinterpret_cast<f4v*>(s_tile);
#pragma unroll
        for (int i = 0; i < NV; ++i)
          if (FMAX != 64 || (lane + i * 64) * 4 < 64 * F) s4[lane + i * 64] = v[i];
      }
      wt_tail(nrow * F, r0 * F, n4, X, total, s_tile, lane);
      fetch(tc + nw);  // the next tile's loads stay in flight during this tile
      if constexpr (BOUNDS) {
        // ---- kTile: bound test, then finish the undecided rows ----
        const int la = lab_old < k ? lab_old : 0;
        const float ub = ub_in + s_drift[la];
        const float lbv = lb_in - dmax;
        const float thr = fmaxf(lbv, s_half[la]);
        const bool need = valid && (lab_old >= k || !(ub * (1.f + kEps) < thr));
        auto store = [&](bool v, bool ch, int lab, float u, float l) {
          if (v) {
            if (ch) __builtin_amdgcn_raw_buffer_store_b8((unsigned char)lab, rl, lane, tc * 64, 0);
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(int, u), ru, lane * 4, tc * 256, 0);
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(int, l), rw, lane * 4, tc * 256, 0);
          }
        };
        if (__ballot(need) != 0ull) finish_rows(valid, need, lab_old, ub, lbv, thr, store);
        else store(valid, false, lab_old, ub, lbv);
        continue;
      } else {
        f2v x2[FMAX / 2];
        load_scaled_row<FMAX>(s_tile, lane, F, s_a, s_b, x2);
        if (MODE == 2) {
          const float d = dist_one<FMAX>(x2, s_cT, lab_old < k ? lab_old : 0);
          if (valid) inert += fixq(d, iexp);
          continue;
        }
        int lab;
        float m1, m2;
        nearest_centers<FMAX, 64, true>(x2, s_cT, k, lab, m1, m2);
        recomputed += valid ? 1 : 0;
        const bool ch = valid && lab != lab_old;
        changed += ch ? 1 : 0;
        if (valid) __builtin_amdgcn_raw_buffer_store_b8((unsigned char)lab, rl, lane, tc * 64, 0);
        if (MODE == 1) {
          if (valid) inert += fixq(m1, iexp);
          continue;
        }
        // ---- MODE 0 kFirst: bounds, sizes, sums ----
        if (valid) {
          __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(int, sqrtf(m1)), ru, lane * 4, tc * 256, 0);
          __builtin_amdgcn_raw_buffer_store_b32(
              __builtin_bit_cast(int, k > 1 ? sqrtf(m2) : __builtin_inff()), rw, lane * 4, tc * 256, 0);
        }
        if constexpr (MODE == 0 && KIND == kFirstAtomic) {
          move_rows(__ballot(ch), lab, 255);
          continue;
        }
        if constexpr (MODE == 0 && KIND == kFirstSum) {
          // per label: its rows by their ballot bits (scalar bit scans), 4
          // LDS reads in flight, lane = feature
          const float* xcol = s_tile + (lane < F ? lane : 0);
#pragma unroll
          for (int j = 0; j < KS; ++j) {
            if (j >= k) break;  // wave-uniform
            unsigned long long m = __ballot(valid && lab == j);
            if (lane == 0 && m) atomicAdd(&s_cnt[j], __popcll(m));
            double sj = 0.0;
            while (m != 0ull) {  // wave-uniform
              int r[4];
#pragma unroll
              for (int u = 0; u < 4; ++u) {
                r[u] = m != 0ull ? __builtin_ctzll(m) : -1;
                m &= m - 1ull;
              }
              float xv[4];
#pragma unroll
              for (int u = 0; u < 4; ++u) xv[u] = r[u] >= 0 ? xcol[r[u] * F] : 0.f;
#pragma unroll
              for (int u = 0; u < 4; ++u) sj += fixq64(xv[u], fe);
            }
            fsum[j] += sj;
          }
          if (++since_flush == 32) {  // sums stay below 32 * 64 * 2^41 = 2^52: exact
            flush();
            since_flush = 0;
          }
        }
        if constexpr (MODE == 0 && KIND == kFirst) {
          if (valid) atomicAdd(&s_cnt[lab], 1);
          s_lab[lane] = valid ? lab : -1;
          __builtin_amdgcn_wave_barrier();
#pragma unroll
          for (int st = 0; st < 16; ++st) {  // k-steps of 4 rows
            const int row = 4 * st + kk;
            const int lr = s_lab[row];
            double bq[NB];
#pragma unroll
            for (int nbk = 0; nbk < NB; ++nbk) {
              const int f = 16 * nbk + mm;
              bq[nbk] = f < F ? fixq64(s_tile[row * F + f], s_e[f]) : 0.0;
            }
#pragma unroll
            for (int i = 0; i < MBX; ++i) {
              const int mb = i / NB, nbk = i - mb * NB;
              const double a = lr == 16 * mb + mm ? 1.0 : 0.0;
              acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, bq[nbk], acc[i], 0, 0, 0);
            }
          }
          if (++since_flush == 32) {  // sums stay below 32 * 64 * 2^41 = 2^52: exact
            flush();
            since_flush = 0;
          }
        }
      }
    }
    flush();
  }
  // ---- block record: [dQ_hi kF | dQ_lo kF | dcount k | changed | recomputed | in_hi | in_lo] ----
  const double ch = block_sum((double)changed, s_red);
  const double rc = block_sum((double)recomputed, s_red);
  const long long in = block_sum(inert, s_red64);
  __syncthreads();
  const int rlen = lloyd_rec(k, F);
  double* out = reinterpret_cast<double*>(fit.ws) + (size_t)blk * rlen;
  if (MODE == 0) {
    for (int q = t; q < k * F; q += blockDim.x) {
      double h, l;
      limbs((long long)s_acc[q], h, l);
      out[q] = h;
      out[k * F + q] = l;
    }
    for (int j = t; j < k; j += blockDim.x) out[2 * k * F + j] = (double)s_cnt[j];
  } else {
    for (int q = t; q < 2 * k * F + k; q += blockDim.x) out[q] = 0.0;
  }
  if (t == 0) {
    double h, l;
    limbs(in, h, l);
    out[2 * k * F + k] = ch;
    out[2 * k * F + k + 1] = rc;
    out[2 * k * F + k + 2] = h;
    out[2 * k * F + k + 3] = l;
  }
}

template <int FMAX, int MODE, int KIND, int MBT>
__global__ void __launch_bounds__(256) lloyd_pass_kernel(const float* __restrict__ X, int64_t S, int F,
                                                         const float* __restrict__ ga,
                                                         const float* __restrict__ gb,
                                                         const int* __restrict__ qexp,
                                                         const LloydFitsArg fits, int n, int64_t R) {
  lloyd_pass_body<FMAX, MODE, KIND, MBT>(X, S, F, ga, gb, qexp, fits, n, R);
}
// the first pass at F > 32 under a two-waves-per-SIMD register bound (the
// unbounded instance holds 256 VGPRs + 33 AGPRs: one wave per SIMD; this one
// 256 VGPRs and an 8-byte spill).  Config-5 cohort fit (2 x 40k^2 x 50
// slides, same box, profiles/r04/bench_c5x2_synth*.json): 476.3 -> 460.4 ms.
// The default; MW_LLOYD_FIRST_W2=0 takes the unbounded instance (same bits)
template <int FMAX, int KIND>
__global__ void __launch_bounds__(256, 2) lloyd_first_w2_kernel(const float* __restrict__ X, int64_t S, int F,
                                                               const float* __restrict__ ga,
                                                               const float* __restrict__ gb,
                                                               const int* __restrict__ qexp,
                                                               const LloydFitsArg fits, int n, int64_t R) {
  lloyd_pass_body<FMAX, 0, KIND, 1>(X, S, F, ga, gb, qexp, fits, n, R);
}

// the first pass at 17..32 features under a three-waves-per-SIMD bound (the
// unbounded instance holds 167 VGPRs + 16 AGPRs: two waves per SIMD; this one
// 168 VGPRs, no AGPRs, no spill): 0.88-0.92 -> 0.83 ms per config-2 pass,
// fit 7.43-7.45 -> 7.35-7.40 ms (profiles/r04/lloyd_w3_*).  The default;
// MW_LLOYD_FIRST_W3=0 takes the unbounded instance (same bits)
template <int FMAX, int KIND>
__global__ void __launch_bounds__(256, 3) lloyd_first_w3_kernel(const float* __restrict__ X, int64_t S, int F,
                                                               const float* __restrict__ ga,
                                                               const float* __restrict__ gb,
                                                               const int* __restrict__ qexp,
                                                               const LloydFitsArg fits, int n, int64_t R) {
  lloyd_pass_body<FMAX, 0, KIND, 1>(X, S, F, ga, gb, qexp, fits, n, R);
}

// kList, first launch: the bound test of every row of the block's range from
// the row state alone (4 consecutive rows per lane, 4 groups of 256 rows per
// wave in flight, no barrier until the end).  Decided rows get their drifted
// bounds written back; undecided rows go to the block's list, in any order
// (the pass's sums are integer sums and its other outputs are per row).
__global__ void __launch_bounds__(256) lloyd_mark_kernel(const LloydFitsArg fits, int n, int64_t S,
                                                         int F, int64_t R) {
  __shared__ float s_drift[64], s_half[64];
  __shared__ int s_n;
  const int g = blockIdx.x % n, blk = blockIdx.x / n, G = (int)(gridDim.x / n);
  const mw_lloyd_fit& fit = fits.f[g];
  const int k = fit.k;
  const int t = threadIdx.x, lane = t & 63, nw = blockDim.x >> 6;
  const int wid = __builtin_amdgcn_readfirstlane(t >> 6);
  for (int j = t; j < 64; j += blockDim.x) {
    s_drift[j] = j < k ? fit.drift[j] : 0.f;
    s_half[j] = j < k ? fit.half_sep[j] : 0.f;
  }
  if (t == 0) s_n = 0;
  __syncthreads();
  const float dmax = fit.drift_max;
  char* wsb = reinterpret_cast<char*>(fit.ws);
  const size_t loff = lloyd_list_off(G, k, F);
  int* __restrict__ list = reinterpret_cast<int*>(wsb + loff + lloyd_al256((size_t)G * 4)) + (size_t)blk * R;
  const uint8_t* __restrict__ labels = fit.labels;
  float* __restrict__ ubuf = fit.ub;
  float* __restrict__ lbuf = fit.lb;
  const int64_t lo = (int64_t)blk * R, hi = min(S, lo + R);
  constexpr int NI = 4;
  for (int64_t c0 = lo; c0 < hi; c0 += (int64_t)NI * nw * 256) {
    uint32_t lab4[NI];
    f4v ub4[NI], lb4[NI];
#pragma unroll
    for (int it = 0; it < NI; ++it) {
      const int64_t r0 = c0 + (int64_t)(it * nw + wid) * 256 + 4 * lane;  // a multiple of 4
      if (r0 + 3 < hi) {
        lab4[it] = *reinterpret_cast<const uint32_t*>(labels + r0);
        ub4[it] = *reinterpret_cast<const f4v*>(ubuf + r0);
        lb4[it] = *reinterpret_cast<const f4v*>(lbuf + r0);
      } else {
        lab4[it] = 0xFFFFFFFFu;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          if (r0 + i < hi) {
            lab4[it] = (lab4[it] & ~(0xFFu << (8 * i))) | ((uint32_t)labels[r0 + i] << (8 * i));
            ub4[it][i] = ubuf[r0 + i];
            lb4[it][i] = lbuf[r0 + i];
          }
        }
      }
    }
#pragma unroll
    for (int it = 0; it < NI; ++it) {
      const int64_t g0 = c0 + (int64_t)(it * nw + wid) * 256;
      if (g0 >= hi) break;  // wave-uniform
      const int64_t r0 = g0 + 4 * lane;
      bool skip[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int lab_old = (lab4[it] >> (8 * i)) & 0xFF;
        const int la = lab_old < k ? lab_old : 0;
        const float ub = ub4[it][i] + s_drift[la];
        const float lbv = lb4[it][i] - dmax;
        const float thr = fmaxf(lbv, s_half[la]);
        const bool valid = r0 + i < hi;
        const bool need = valid && (lab_old >= k || !(ub * (1.f + kEps) < thr));
        skip[i] = valid && !need;
        ub4[it][i] = ub;
        lb4[it][i] = lbv;
        const unsigned long long m = __ballot(need);
        if (m != 0ull) {
          int qb = 0;
          if (lane == 0) qb = atomicAdd(&s_n, __popcll(m));
          qb = __shfl(qb, 0, 64);
          if (need) list[qb + __popcll(m & ((1ull << lane) - 1ull))] = (int)(r0 + i);
        }
      }
      if (skip[0] && skip[1] && skip[2] && skip[3]) {
        *reinterpret_cast<f4v*>(ubuf + r0) = ub4[it];
        *reinterpret_cast<f4v*>(lbuf + r0) = lb4[it];
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (skip[i]) {
            ubuf[r0 + i] = ub4[it][i];
            lbuf[r0 + i] = lb4[it][i];
          }
      }
    }
  }
  __syncthreads();
  if (t == 0) reinterpret_cast<int*>(wsb + loff)[blk] = s_n;
}

// The kList row lists of a fold (mw_kpp_step_fold): per row block of the
// Lloyd grid, the rows that move to the new center (bit *best of moved[]),
// in the layout lloyd_mark_kernel writes; the list pass (kind 8) then
// recomputes exactly those rows against the k final centers.
__global__ void __launch_bounds__(256) lloyd_list_moved_kernel(const uint8_t* __restrict__ moved,
                                                               const int* __restrict__ best, int64_t S,
                                                               int64_t R, char* __restrict__ wsb, size_t loff,
                                                               int G) {
  __shared__ int s_n;
  const int t = threadIdx.x, lane = t & 63;
  if (t == 0) s_n = 0;
  __syncthreads();
  const int b = *best;
  const int blk = blockIdx.x;
  int* __restrict__ list = reinterpret_cast<int*>(wsb + loff + lloyd_al256((size_t)G * 4)) + (size_t)blk * R;
  const int64_t lo = (int64_t)blk * R, hi = min(S, lo + R);
  for (int64_t r0 = lo + 4 * (int64_t)t; r0 < hi; r0 += 4 * 256) {  // lo is a multiple of 256
    uint32_t m4 = 0;
    if (r0 + 3 < hi) {
      m4 = *reinterpret_cast<const uint32_t*>(moved + r0);
    } else {
      for (int i = 0; i < 4; ++i)
        if (r0 + i < hi) m4 |= (uint32_t)moved[r0 + i] << (8 * i);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const bool need = r0 + i < hi && ((m4 >> (8 * i + b)) & 1u);
      const unsigned long long m = __ballot(need);
      if (m != 0ull) {
        int qb = 0;
        if (lane == 0) qb = atomicAdd(&s_n, __popcll(m));
        qb = __shfl(qb, 0, 64);
        if (need) list[qb + __popcll(m & ((1ull << lane) - 1ull))] = (int)(r0 + i);
      }
    }
  }
  __syncthreads();
  if (t == 0) reinterpret_cast<int*>(wsb + loff)[blk] = s_n;
}

// one fit per blockIdx.y: fixed-order fold of its G block records
__global__ void __launch_bounds__(256) lloyd_reduce_fits_kernel(const LloydFitsArg fits, int G, int F) {
  const mw_lloyd_fit& fit = fits.f[blockIdx.y];
  const int rl = lloyd_rec(fit.k, F);
  if ((int)blockIdx.x * 32 >= rl) return;  // block-uniform
  rec_reduce_body(reinterpret_cast<const double*>(fit.ws), G, rl, fit.out);
}

// ---- column max |x| (fixed-point exponents of the M-step) ----
// The launcher makes the grid stride a multiple of F, so each thread walks
// one residue class of F (its column, computed once) and keeps a register
// max; one LDS atomic per thread at the end.
__global__ void __launch_bounds__(256) col_absmax_kernel(const float* __restrict__ X, int64_t S, int F,
                                                         unsigned* __restrict__ out) {
  extern __shared__ unsigned s_m[];  // F column maxima (dynamic: any F up to kColAbsMaxF)
  for (int f = threadIdx.x; f < F; f += blockDim.x) s_m[f] = 0u;
  __syncthreads();
  const int64_t total = S * (int64_t)F;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;  // a multiple of F
  const int64_t e0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int f = (int)(e0 % F);
  unsigned m = 0u;  // non-negative floats order as their bits
  int64_t e = e0;
  for (; e + 3 * stride < total; e += 4 * stride) {
    const float x0 = fabsf(X[e]), x1 = fabsf(X[e + stride]);
    const float x2 = fabsf(X[e + 2 * stride]), x3 = fabsf(X[e + 3 * stride]);
    m = max(m, max(max(__builtin_bit_cast(unsigned, x0), __builtin_bit_cast(unsigned, x1)),
                   max(__builtin_bit_cast(unsigned, x2), __builtin_bit_cast(unsigned, x3))));
  }
  for (; e < total; e += stride) m = max(m, __builtin_bit_cast(unsigned, fabsf(X[e])));
  atomicMax(&s_m[f], m);
  __syncthreads();
  for (int q = threadIdx.x; q < F; q += blockDim.x) atomicMax(&out[q], s_m[q]);
}

constexpr int kColAbsMaxF = 16384;  // columns of col_absmax_kernel (F x 4 bytes of LDS)

// grid of col_absmax_kernel: <= 2048 blocks, block count a multiple of F / gcd(256, F)
static int col_absmax_blocks(int64_t total, int F) {
  int a = 256, b = F;
  while (b) { const int r = a % b; a = b; b = r; }
  const int unit = F / a;
  int nb = (int)std::min<int64_t>((total + 255) / 256, 2048);
  nb = std::max(unit, (nb / unit) * unit);
  return nb;
}

}  // namespace mw

#include "lloyd_dense.h"
#include "lloyd_dense2.h"

using namespace mw;

extern "C" {

int mw_lloyd_rec_len(int k, int F) { return lloyd_rec(k, F); }

size_t mw_lloyd_ws_bytes(int64_t S, int k, int F) {
  const int G = lloyd_blocks(S, F);  // records, then the kList lengths and lists
  return lloyd_list_off(G, k, F) + lloyd_al256((size_t)G * 4) + (size_t)G * lloyd_rows(S, F) * 4 + 256;
}

size_t mw_lloyd_ws_bytes_kinds(int64_t S, int k, int F, int with_list) {
  if (with_list && S < ((int64_t)1 << 31)) return mw_lloyd_ws_bytes(S, k, F);
  return lloyd_list_off(lloyd_blocks(S, F), k, F) + 256;  // records only: kind 4 is never passed
}

int mw_col_absmax(const float* d_X, int64_t S, int F, float* d_out, void* stream) {
  MW_CHECK_ARG(d_X && d_out && S > 0 && F > 0 && F <= kColAbsMaxF, "mw_col_absmax: bad arguments (F <= %d)",
               kColAbsMaxF);
  hipStream_t s = as_stream(stream);
  MW_HIP(hipMemsetAsync(d_out, 0, sizeof(float) * F, s));
  const int64_t total = S * (int64_t)F;
  const int nb = col_absmax_blocks(total, F);
  hipLaunchKernelGGL(col_absmax_kernel, dim3(nb), dim3(256), (size_t)F * sizeof(unsigned), s, d_X, S, F,
                     reinterpret_cast<unsigned*>(d_out));
  MW_LAUNCH_CHECK();
  return MW_OK;
}

// max |x| per column folded into d_out (not reset first): a slide's column
// maxima band after band (the exact QC sums take their fixed point from them)
int mw_col_absmax_acc(const float* d_X, int64_t S, int F, float* d_out, void* stream) {
  MW_CHECK_ARG(d_X && d_out && S > 0 && F > 0 && F <= kColAbsMaxF, "mw_col_absmax_acc: bad arguments (F <= %d)",
               kColAbsMaxF);
  hipStream_t s = as_stream(stream);
  const int64_t total = S * (int64_t)F;
  const int nb = col_absmax_blocks(total, F);
  hipLaunchKernelGGL(col_absmax_kernel, dim3(nb), dim3(256), (size_t)F * sizeof(unsigned), s, d_X, S, F,
                     reinterpret_cast<unsigned*>(d_out));
  MW_LAUNCH_CHECK();
  return MW_OK;
}

int mw_lloyd_list_moved(const uint8_t* d_moved, const int* d_best, int64_t S, int F, int k, void* d_ws,
                        void* stream) {
  MW_CHECK_ARG(d_moved && d_best && d_ws && S > 0 && S < ((int64_t)1 << 31) && F > 0 && k >= 1,
               "mw_lloyd_list_moved: bad arguments");
  const int G = lloyd_blocks(S, F);
  hipLaunchKernelGGL(lloyd_list_moved_kernel, dim3(G), dim3(256), 0, as_stream(stream), d_moved, d_best, S,
                     lloyd_rows(S, F), static_cast<char*>(d_ws), lloyd_list_off(G, k, F), G);
  MW_LAUNCH_CHECK();
  return MW_OK;
}

int mw_lloyd_pass(const float* d_X, int64_t S, int F, const float* d_a, const float* d_b,
                  const int32_t* d_qexp, int n, const mw_lloyd_fit* h_fits, int mode, int kind,
                  void* stream) {
  MW_CHECK_ARG(d_X && d_a && d_b && d_qexp && h_fits, "mw_lloyd_pass: null pointer");
  MW_CHECK_ARG(S > 0 && F > 0 && n >= 1 && n <= kMaxFits, "mw_lloyd_pass: bad shape (1 <= n <= %d)",
               kMaxFits);
  MW_CHECK_ARG(mode >= 0 && mode <= 2, "mw_lloyd_pass: bad mode %d", mode);
  MW_CHECK_ARG(kind >= 0 && kind <= 6 || kind == kListGiven, "mw_lloyd_pass: bad kind %d", kind);
  // kind 8: a kList pass over lists written beforehand (mw_lloyd_list_moved)
  const bool lists_given = kind == kListGiven;
  if (lists_given) {
    MW_CHECK_ARG(mode == 0 && S < ((int64_t)1 << 31), "mw_lloyd_pass: kind 8 needs mode 0 and S < 2^31");
    kind = kList;
  }
  if (mode != 0) kind = kFirst;  // modes 1 and 2 stream every tile
  if (kind == kList && S >= ((int64_t)1 << 31)) kind = kQueue;  // int32 row lists
  LloydFitsArg fits{};
  int kmax = 0;
  for (int g = 0; g < n; ++g) {
    const mw_lloyd_fit& f = h_fits[g];
    MW_CHECK_ARG(f.centers && f.labels && f.ws && f.out && f.k >= 1, "mw_lloyd_pass: fit %d: bad arguments", g);
    MW_CHECK_ARG(mode != 0 || (f.ub && f.lb && f.drift && f.half_sep),
                 "mw_lloyd_pass: fit %d: mode 0 needs ub, lb, drift, half_sep", g);
    fits.f[g] = f;
    kmax = f.k > kmax ? f.k : kmax;
  }
  if (kmax > 64 || F > 64) {
    set_error("mw_lloyd_pass: k=%d F=%d unsupported (k <= 64, F <= 64)", kmax, F);
    return MW_EUNSUPPORTED;
  }
  hipStream_t s = as_stream(stream);
  const int G = lloyd_blocks(S, F);
  const int64_t R = lloyd_rows(S, F);
  if (kind == kDense || kind == kDense + 1) {
    // dense x . C^T pass over every fit of the launch (lloyd_dense.h); kind 6
    // also writes the fits' distance bounds
    DenseArg da{};
    if (!dense_groups(h_fits, n, da)) {
      set_error("mw_lloyd_pass: dense kind needs k <= %d per fit", kDenseMaxFitK);
      return MW_EUNSUPPORTED;
    }
    MW_CHECK_ARG(kind == kDense || [&] {
      for (int g = 0; g < n; ++g)
        if (!h_fits[g].ub || !h_fits[g].lb) return false;
      return true;
    }(), "mw_lloyd_pass: kind 6 needs ub / lb");
    da.bounds = kind == kDense ? 0 : (int)((1u << n) - 1u);
    static const float bscale = [] {
      const char* e = getenv("MW_DENSE_BSCALE");  // A/B of the recheck bound (never below the default)
      const float v = e ? (float)atof(e) : kDenseBScale;
      return v > kDenseBScale ? v : kDenseBScale;
    }();
    da.bscale = bscale;
    da.G = G;
    // F <= 32: every fit in one block per row block (lloyd_dense2.h);
    // MW_DENSE2=0 keeps the grouped form (A/B)
    static const bool use2 = [] {
      const char* e = getenv("MW_DENSE2");
      return !(e && e[0] == '0');
    }();
    Dense2Arg d2{};
    if (use2 && dense2_plan(h_fits, n, S, F, d2)) {
      d2.bounds = da.bounds;
      int waves = kD2Waves;  // 3 waves per SIMD, or 2 when the LDS of the launch needs it
      size_t lds2 = dense2_lds_bytes(d2.coff[n], F, d2.ntile, waves);
      if (lds2 > 160 * 1024) {
        waves = 8;
        lds2 = dense2_lds_bytes(d2.coff[n], F, d2.ntile, waves);
      }
      if (lds2 <= 160 * 1024) {
        hipLaunchKernelGGL(lloyd_dense2_kernel, dim3((unsigned)d2.G), dim3(64 * waves), lds2, s, d_X, S, F,
                           d_a, d_b, d_qexp, fits, d2);
        MW_LAUNCH_CHECK();
        const int rlmax = lloyd_rec(kmax, F);
        hipLaunchKernelGGL(lloyd_reduce_fits_kernel, dim3((rlmax + 31) / 32, n), dim3(256), 0, s, fits, d2.G, F);
        MW_LAUNCH_CHECK();
        return MW_OK;
      }
    }
    const dim3 gridd((unsigned)((G + 7) / 8 * 8) * (unsigned)da.ngroups);  // whole XCD rounds
    if (F <= 32) {
      hipLaunchKernelGGL(lloyd_dense_kernel<32>, gridd, dim3(256), dense_lds_bytes(32, F), s, d_X, S, F, d_a, d_b,
                         d_qexp, fits, da, R);
    } else {
      hipLaunchKernelGGL(lloyd_dense_kernel<64>, gridd, dim3(256), dense_lds_bytes(64, F), s, d_X, S, F, d_a, d_b,
                         d_qexp, fits, da, R);
    }
    MW_LAUNCH_CHECK();
    const int rlmax = lloyd_rec(kmax, F);
    hipLaunchKernelGGL(lloyd_reduce_fits_kernel, dim3((rlmax + 31) / 32, n), dim3(256), 0, s, fits, G, F);
    MW_LAUNCH_CHECK();
    return MW_OK;
  }
  // F in (32, 52]: 26 feature pairs instead of 32 in every distance (the 6
  // more only add exact zeros: the same bits; MW_LLOYD_FM52=0 keeps 64, A/B)
  const char* e52 = getenv("MW_LLOYD_FM52");
  const bool fm52 = !(e52 && e52[0] == '0');
  const int FM = F <= 8 ? 8 : F <= 16 ? 16 : F <= 32 ? 32 : (F <= 52 && fm52) ? 52 : 64;
  const dim3 grid((unsigned)G * (unsigned)n);
  // kFirst: fp64 accumulators for ceil(kmax / 16) label blocks x the feature
  // blocks, at most 4 (else the sums go through LDS atomics)
  const int NBF = FM <= 16 ? 1 : FM / 16, MBF = (kmax + 15) / 16;
  if (mode == 0 && kind == kFirst && MBF * NBF > 4) kind = kFirstAtomic;
  // kFirstSum at F > 32 (the config-5 fit 164.7 -> 159.4 ms per slide); at
  // F <= 32 the one-hot MFMA form measured faster (config-2 fit 7.54 vs 7.74
  // ms).  MW_LLOYD_FIRST_SUM=1 / 0 forces either.
  static const int first_sum = [] {
    const char* e = getenv("MW_LLOYD_FIRST_SUM");
    return e ? (e[0] == '1' ? 1 : 0) : -1;
  }();
  if (mode == 0 && kind == kFirst && kmax <= 16 && (first_sum == 1 || (first_sum < 0 && FM >= 52)))
    kind = kFirstSum;
  // FM = 52: the one-hot MFMA M-step takes 16-feature blocks (52 is not a multiple)
  if (mode == 0 && kind == kFirst && FM == 52) kind = kmax <= 16 ? kFirstSum : kFirstAtomic;
  const size_t lds = lloyd_lds_bytes(FM, kmax, F, mode, kind);
  if (mode == 0 && kind == kList && !lists_given) {
    hipLaunchKernelGGL(lloyd_mark_kernel, grid, dim3(256), 0, s, fits, n, S, F, R);
    MW_LAUNCH_CHECK();
  }
#define MW_LP(FMV, MO, KI, MBV)                                                                        \
  hipLaunchKernelGGL((lloyd_pass_kernel<FMV, MO, KI, MBV>), grid, dim3(256), lds, s, d_X, S, F, d_a, d_b, \
                     d_qexp, fits, n, R)
#define MW_LPF(FMV)                                                              \
  if (mode == 0) {                                                               \
    if (kind == kFirst) {                                                        \
      if (MBF == 1) MW_LP(FMV, 0, kFirst, 1);                                    \
      else if (MBF == 2) { if constexpr ((FMV <= 32)) MW_LP(FMV, 0, kFirst, 2); } \
      else { if constexpr ((FMV <= 16)) MW_LP(FMV, 0, kFirst, 4); }              \
    }                                                                            \
    else if (kind == kTile) MW_LP(FMV, 0, kTile, 1);                            \
    else if (kind == kFirstAtomic) MW_LP(FMV, 0, kFirstAtomic, 1);              \
    else if (kind == kFirstSum) MW_LP(FMV, 0, kFirstSum, 1);                    \
    else if (kind == kList) MW_LP(FMV, 0, kList, 1);                            \
    else MW_LP(FMV, 0, kQueue, 1);                                              \
  } else if (mode == 1) MW_LP(FMV, 1, kFirst, 1);                               \
  else MW_LP(FMV, 2, kFirst, 1);
  static const bool first_w2 = [] {
    const char* e = getenv("MW_LLOYD_FIRST_W2");
    return !(e && e[0] == '0');
  }();
  if (first_w2 && FM == 64 && mode == 0 && (kind == kFirst || kind == kFirstSum) && MBF == 1) {
    if (kind == kFirst)
      hipLaunchKernelGGL((lloyd_first_w2_kernel<64, kFirst>), grid, dim3(256), lds, s, d_X, S, F, d_a, d_b, d_qexp,
                         fits, n, R);
    else
      hipLaunchKernelGGL((lloyd_first_w2_kernel<64, kFirstSum>), grid, dim3(256), lds, s, d_X, S, F, d_a, d_b, d_qexp,
                         fits, n, R);
  } else if (first_w2 && FM == 52 && mode == 0 && kind == kFirstSum) {
    hipLaunchKernelGGL((lloyd_first_w2_kernel<52, kFirstSum>), grid, dim3(256), lds, s, d_X, S, F, d_a, d_b, d_qexp,
                       fits, n, R);
  } else if (FM == 32 && mode == 0 && kind == kFirst && MBF == 1 && [] {
               const char* e = getenv("MW_LLOYD_FIRST_W3");
               return !(e && e[0] == '0');
             }()) {
    hipLaunchKernelGGL((lloyd_first_w3_kernel<32, kFirst>), grid, dim3(256), lds, s, d_X, S, F, d_a, d_b, d_qexp,
                       fits, n, R);
  } else if (FM == 8) { MW_LPF(8) }
  else if (FM == 16) { MW_LPF(16) }
  else if (FM == 32) { MW_LPF(32) }
  else if (FM == 52) { MW_LPF(52) }
  else { MW_LPF(64) }
#undef MW_LPF
#undef MW_LP
  MW_LAUNCH_CHECK();
  const int rlmax = lloyd_rec(kmax, F);
  hipLaunchKernelGGL(lloyd_reduce_fits_kernel, dim3((rlmax + 31) / 32, n), dim3(256), 0, s, fits, G, F);
  MW_LAUNCH_CHECK();
  return MW_OK;
}

}  // extern "C"
