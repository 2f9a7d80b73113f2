// Shared k-means device helpers (row tiles, E-step distance stream, fixed-order
// record reduction): used by kmeans.hip (k-means++, farthest, label pass) and
// lloyd.hip (the Lloyd engine).
#pragma once

#include <stdlib.h>

#include "common.h"

namespace mw {

constexpr int kT = 256;          // rows per tile = threads per block
constexpr int kMaxG = 1024;

static inline int kmax_grid() {
  static int g = [] {
    const char* e = getenv("MW_KBLOCKS");  // tuning override (<= kMaxG)
    const int v = e ? atoi(e) : 0;
    return (v >= 1 && v <= kMaxG) ? v : kMaxG;
  }();
  return g;
}
static inline int kblocks(int64_t n) {
  int64_t tiles = (n + kT - 1) / kT;
  if (tiles < 1) tiles = 1;
  const int gm = kmax_grid();
  return (int)(tiles < gm ? tiles : gm);
}
static inline int64_t krows(int64_t n) {
  int64_t tiles = (n + kT - 1) / kT;
  int g = kblocks(n);
  return ((tiles + g - 1) / g) * kT;
}

typedef float f2v __attribute__((ext_vector_type(2)));
typedef float f4v __attribute__((ext_vector_type(4)));
__host__ __device__ constexpr int kpad4(int k) { return (k + 3) & ~3; }

// Lloyd per-block record length: [dQ_hi kF | dQ_lo kF | dcount k | changed |
// recomputed | inertia_hi | inertia_lo] (lloyd.hip)
__host__ __device__ inline int lloyd_rec(int k, int F) { return 2 * k * F + k + 4; }

// x as an exact fixed-point integer: rint(x * 2^e) (|x * 2^e| < 2^41; fp64
// holds it exactly, and sums of up to 2^12 of them).  Computed in fp32, then
// widened: x * 2^e is exact in fp32 while it is a normal number (a power-of-two
// scale of x, and |x * 2^e| < 2^41 cannot overflow); at or above 2^23 it is
// already an integer, below it rintf's result is an integer < 2^23, so both
// are exact; below 2^-126 both forms round to zero.  Same value as
// rint(ldexp((double)x, e)), with one fp64 instruction instead of three.
__device__ __forceinline__ double fixq64(float x, int e) {
  float q = rintf(ldexpf(x, e));
  asm("" : "+v"(q));  // keeps the fp32 ops (hipcc otherwise widens them back to fp64)
  return (double)q;
}
__device__ __forceinline__ long long fixq(float x, int e) { return (long long)fixq64(x, e); }

// int64 -> (hi, lo) integer-valued fp64 limbs
__device__ __forceinline__ void limbs(long long v, double& hi, double& lo) {
  const long long h = v >> 32;  // arithmetic shift: floor
  hi = (double)h;
  lo = (double)(v - h * (1LL << 32));
}

// ---- wave tiles: 64 consecutive rows of F floats (64*F floats, float4-aligned
// because tile starts are multiples of 64 rows).  Each lane fetches NV =
// FMAX/4 float4 with clamped, unconditional loads (guide §5.4c) and stores all
// of them to the wave's LDS tile of 64*FMAX floats: floats past 64*F are the
// following rows' data, read by the E-step only for padded features whose scale
// is exactly 0.  Floats past the array's last whole float4 are patched with
// scalar loads in the final tile only.  (The k-means++ and Lloyd passes at
// FMAX = 64 load and keep only the 64*F floats plus a zeroed pad instead:
// LDS, not registers, bounds their occupancy there.)
__device__ __forceinline__ void wt_tail(int nfl, int64_t e0, int64_t n4, const float* __restrict__ X,
                                        int64_t total, float* s, int lane) {
  if (e0 + nfl > n4 * 4) {  // wave-uniform
    for (int e = lane; e < nfl; e += 64) {
      const int64_t ge = e0 + e;
      if (ge >= n4 * 4 && ge < total) s[e] = X[ge];
    }
  }
}

// cache policy of the row streams' loads (buffer aux bits; 2 = nt,
// streaming): every pass reads its rows once and a pass's rows (>= 2 GB at
// config 2) do not fit the caches, so the loads need not allocate; a plain
// 2.2-GB read goes 6.3 -> 7.1 TB/s (tools/probe/hbm_probe2.hip,
// profiles/r06/hbm_probe2.txt; common.h MW_STREAM_NT for the passes' A/B)
constexpr int kStreamAux = MW_STREAM_NT ? 2 : 0;

// ---- wave-tile streaming with buffer loads: the resource covers a block's
// rows from its first row to the end of the array (32-bit block-relative
// offsets, hardware range check), the tile offset is a scalar (tile index is
// wave-uniform) and the per-lane offsets are constants, so a tile fetch costs
// no VALU.  Loads past the end return 0; stores past the range are dropped.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, int64_t nbytes) {
  const uint64_t n = nbytes < 0 ? 0 : (uint64_t)nbytes;
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0,
                                           (int)(uint32_t)(n < 0xFFFFFFFFull ? n : 0xFFFFFFFFull),
                                           0x00020000);
}
template <int NV>
__device__ __forceinline__ void tile_load(__amdgpu_buffer_rsrc_t rs, int soff, int lane, f4v (&v)[NV]) {
#pragma unroll
  for (int i = 0; i < NV; ++i)
    v[i] = __builtin_bit_cast(f4v, __builtin_amdgcn_raw_buffer_load_b128(rs, lane * 16 + i * 1024, soff, kStreamAux));
}

// ---- E-step center stream, written as inline asm so that the schedule is
// the one below (hipcc otherwise hoists every center read of the block, 128+
// VGPRs, and serialises the four distance chains).  hipcc does not count asm
// memory operations in its s_waitcnt bookkeeping, so the stream waits itself
// with counted lgkmcnt: LDS returns in order, and any LDS op the compiler
// places in between only makes a counted wait stricter.
template <int OFF>
__device__ __forceinline__ f2v ds_read8(uint32_t addr) {
  f2v r;
  asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(r) : "v"(addr), "i"(OFF));
  return r;
}
template <int N>
__device__ __forceinline__ void lgkm_wait4(f2v (&c)[4]) {
  asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(N) : "memory");
  asm volatile("" : "+v"(c[0]), "+v"(c[1]), "+v"(c[2]), "+v"(c[3]));  // uses stay below the wait
}
// acc[q] += (x - c[q])^2 for four centers, packed over a feature pair: the four
// subtractions then the four FMAs (no dependent pair back to back)
__device__ __forceinline__ void dist4(f2v x, const f2v (&c)[4], f2v (&acc)[4]) {
  f2v d0, d1, d2, d3;
  asm volatile(
      "v_pk_add_f32 %0, %8, %9 neg_lo:[0,1] neg_hi:[0,1]\n\t"
      "v_pk_add_f32 %1, %8, %10 neg_lo:[0,1] neg_hi:[0,1]\n\t"
      "v_pk_add_f32 %2, %8, %11 neg_lo:[0,1] neg_hi:[0,1]\n\t"
      "v_pk_add_f32 %3, %8, %12 neg_lo:[0,1] neg_hi:[0,1]\n\t"
      "v_pk_fma_f32 %4, %0, %0, %4\n\t"
      "v_pk_fma_f32 %5, %1, %1, %5\n\t"
      "v_pk_fma_f32 %6, %2, %2, %6\n\t"
      "v_pk_fma_f32 %7, %3, %3, %7"
      : "=&v"(d0), "=&v"(d1), "=&v"(d2), "=&v"(d3), "+v"(acc[0]), "+v"(acc[1]), "+v"(acc[2]),
        "+v"(acc[3])
      : "v"(x), "v"(c[0]), "v"(c[1]), "v"(c[2]), "v"(c[3]));
}
// dist4 with the center pairs as scalar (SGPR) operands
__device__ __forceinline__ void dist4_s(f2v x, const f2v (&c)[4], f2v (&acc)[4]) {
  f2v d0, d1, d2, d3;
  asm volatile(
      "v_pk_add_f32 %0, %8, %9 neg_lo:[0,1] neg_hi:[0,1]\n\t"
      "v_pk_add_f32 %1, %8, %10 neg_lo:[0,1] neg_hi:[0,1]\n\t"
      "v_pk_add_f32 %2, %8, %11 neg_lo:[0,1] neg_hi:[0,1]\n\t"
      "v_pk_add_f32 %3, %8, %12 neg_lo:[0,1] neg_hi:[0,1]\n\t"
      "v_pk_fma_f32 %4, %0, %0, %4\n\t"
      "v_pk_fma_f32 %5, %1, %1, %5\n\t"
      "v_pk_fma_f32 %6, %2, %2, %6\n\t"
      "v_pk_fma_f32 %7, %3, %3, %7"
      : "=&v"(d0), "=&v"(d1), "=&v"(d2), "=&v"(d3), "+v"(acc[0]), "+v"(acc[1]), "+v"(acc[2]),
        "+v"(acc[3])
      : "v"(x), "s"(c[0]), "s"(c[1]), "s"(c[2]), "s"(c[3]));
}
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)((__attribute__((address_space(3))) const char*)p);
}

// Nearest center (strict '<': the lowest index wins exact ties, as the
// reference's argmin) and, with TOP2, the second smallest distance.  Squared
// distances of the scaled row x2 to every center; the centers sit in LDS
// pair-major with a fixed center stride KS (cT[p * KS + j] = features 2p, 2p+1
// of center j; zero past k), so each read is a broadcast ds_read_b64 at an
// immediate offset.  Four centers per pass keep four independent packed-FMA
// chains; center pairs stream kAhead pairs ahead of their FMAs.  Each center's
// chain (even features in .x, odd in .y, then .x + .y) is the same fp32
// operation sequence as a one-center loop, so the result does not depend on
// the blocking.
constexpr int kAhead = 1;  // center pairs in flight ahead of their FMAs
template <int NP, int KS, int P>
__device__ __forceinline__ void nc_read(uint32_t base, f2v (&c)[4]) {
  c[0] = ds_read8<P * KS * 8>(base);
  c[1] = ds_read8<P * KS * 8 + 8>(base);
  c[2] = ds_read8<P * KS * 8 + 16>(base);
  c[3] = ds_read8<P * KS * 8 + 24>(base);
}
template <int NP, int KS, int P>
__device__ __forceinline__ void nc_pairs(uint32_t base, const f2v* x2, f2v (*c)[4], f2v (&acc)[4]) {
  if constexpr (P < NP) {
    if constexpr (P + kAhead < NP) nc_read<NP, KS, P + kAhead>(base, c[(P + kAhead) % (kAhead + 1)]);
    constexpr int after = 4 * ((P + kAhead < NP) ? kAhead : (NP - 1 - P));
    lgkm_wait4<after>(c[P % (kAhead + 1)]);
    dist4(x2[P], c[P % (kAhead + 1)], acc);
    nc_pairs<NP, KS, P + 1>(base, x2, c, acc);
  }
}
template <int NP, int KS, int P>
__device__ __forceinline__ void nc_prologue(uint32_t base, f2v (*c)[4]) {
  if constexpr (P < kAhead && P < NP) {
    nc_read<NP, KS, P>(base, c[P]);
    nc_prologue<NP, KS, P + 1>(base, c);
  }
}
template <int FMAX, int KS, bool TOP2>
__device__ __forceinline__ void nearest_centers(const f2v (&x2)[FMAX / 2], const f2v* cT, int k,
                                                int& lab, float& m1, float& m2) {
  constexpr int NP = FMAX / 2;
  const uint32_t a0 = lds_addr(cT);
  lab = 0;
  m1 = 0.f;
  m2 = __builtin_inff();
  for (int j0 = 0; j0 < k; j0 += 4) {
    const uint32_t base = a0 + (uint32_t)j0 * 8u;
    f2v c[kAhead + 1][4];  // register ring of center pairs in flight
    f2v acc[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[q] = f2v{0.f, 0.f};
    nc_prologue<NP, KS, 0>(base, c);
    nc_pairs<NP, KS, 0>(base, x2, c, acc);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int j = j0 + q;
      if (j < k) {
        const float dd = acc[q].x + acc[q].y;
        if (TOP2) {
          if (j == 0) { m1 = dd; lab = 0; }
          else if (dd < m1) { m2 = m1; m1 = dd; lab = j; }
          else if (dd < m2) { m2 = dd; }
        } else if (j == 0 || dd < m1) {
          m1 = dd;
          lab = j;
        }
      }
    }
  }
}

// nearest_centers with the pair-major image in global memory (gT, uniform
// addresses): the center pairs arrive by scalar loads (s_load_dwordx8: one
// feature pair of four centers) straight into the packed FMAs' SGPR operand,
// so the E-step puts no traffic on the LDS pipe, which the CU's four SIMDs
// share with the tile transposition (broadcast LDS reads of the centers made
// the label pass LDS-bound).  Same fp32 operation sequence per center as
// nearest_centers: bitwise the same distances.
template <int FMAX, int KS, bool TOP2>
__device__ __forceinline__ void nearest_centers_s(const f2v (&x2)[FMAX / 2],
                                                  const f2v* __restrict__ gT, int k, int& lab,
                                                  float& m1, float& m2) {
  constexpr int NP = FMAX / 2;
  lab = 0;
  m1 = 0.f;
  m2 = __builtin_inff();
  for (int j0 = 0; j0 < k; j0 += 4) {
    f2v acc[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[q] = f2v{0.f, 0.f};
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      const f2v* cp = gT + p * KS + j0;
      const f2v c[4] = {cp[0], cp[1], cp[2], cp[3]};
      dist4_s(x2[p], c, acc);  // pair order kept (asm): each pair's SGPRs die at once
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int j = j0 + q;
      if (j < k) {
        const float dd = acc[q].x + acc[q].y;
        if (TOP2) {
          if (j == 0) { m1 = dd; lab = 0; }
          else if (dd < m1) { m2 = m1; m1 = dd; lab = j; }
          else if (dd < m2) { m2 = dd; }
        } else if (j == 0 || dd < m1) {
          m1 = dd;
          lab = j;
        }
      }
    }
  }
}

// nearest_centers_s without the scaled row in registers: each pass over a
// group of four centers re-reads the row from the wave's LDS tile and scales
// it (the same fma as load_scaled_row, so the same x and bitwise the same
// distances), which frees FMAX VGPRs for more waves per SIMD (the label pass
// at C = 50 held 270 VGPRs: one wave per SIMD, latency-bound).  `xs` = this
// lane's row in LDS (F floats), `sf` the feature channels (identity: pairs
// read as 8-byte words when F is even).
template <int FMAX, int KS, bool TOP2>
__device__ __forceinline__ void nearest_centers_ls(const float* xs, int F, bool ident, const int* sf,
                                                   const f2v* sa, const f2v* sb,
                                                   const f2v* __restrict__ gT, int k, int& lab,
                                                   float& m1, float& m2) {
  constexpr int NP = FMAX / 2;
  const bool pairs = ident && (F & 1) == 0;
  const f2v* xp = reinterpret_cast<const f2v*>(xs);  // 8-byte aligned when pairs (F even)
  lab = 0;
  m1 = 0.f;
  m2 = __builtin_inff();
  for (int j0 = 0; j0 < k; j0 += 4) {
    f2v acc[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[q] = f2v{0.f, 0.f};
    if (pairs) {
#pragma unroll
      for (int p = 0; p < NP; ++p) {
        const f2v x = __builtin_elementwise_fma(xp[p], sa[p], sb[p]);
        const f2v* cp = gT + p * KS + j0;
        const f2v c[4] = {cp[0], cp[1], cp[2], cp[3]};
        dist4_s(x, c, acc);
      }
    } else {
#pragma unroll
      for (int p = 0; p < NP; ++p) {
        const f2v x = __builtin_elementwise_fma(f2v{xs[sf[2 * p]], xs[sf[2 * p + 1]]}, sa[p], sb[p]);
        const f2v* cp = gT + p * KS + j0;
        const f2v c[4] = {cp[0], cp[1], cp[2], cp[3]};
        dist4_s(x, c, acc);
      }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int j = j0 + q;
      if (j < k) {
        const float dd = acc[q].x + acc[q].y;
        if (TOP2) {
          if (j == 0) { m1 = dd; lab = 0; }
          else if (dd < m1) { m2 = m1; m1 = dd; lab = j; }
          else if (dd < m2) { m2 = dd; }
        } else if (j == 0 || dd < m1) {
          m1 = dd;
          lab = j;
        }
      }
    }
  }
}

// pair-major image (FMAX/2 x KS float pairs) of k x F row-major centers in
// global memory, for nearest_centers_s
template <int FMAX, int KS>
__global__ void __launch_bounds__(256) centers_T_kernel(const float* __restrict__ gc, int k, int F,
                                                        f2v* __restrict__ gT) {
  for (int q = threadIdx.x; q < (FMAX / 2) * KS; q += blockDim.x) {
    const int p = q / KS, j = q - p * KS;
    const int f0 = 2 * p, f1 = 2 * p + 1;
    gT[q] = f2v{(j < k && f0 < F) ? gc[j * F + f0] : 0.f, (j < k && f1 < F) ? gc[j * F + f1] : 0.f};
  }
}

// centers (k x F row-major, global) -> pair-major LDS image cT (see above)
template <int FMAX, int KS>
__device__ __forceinline__ void load_centers_T(const float* __restrict__ gc, int k, int F, f2v* cT) {
  for (int q = threadIdx.x; q < (FMAX / 2) * KS; q += blockDim.x) {
    const int p = q / KS, j = q - p * KS;
    const int f0 = 2 * p, f1 = 2 * p + 1;
    cT[q] = f2v{(j < k && f0 < F) ? gc[j * F + f0] : 0.f, (j < k && f1 < F) ? gc[j * F + f1] : 0.f};
  }
}

// the lane's row of a 64-row LDS tile (row stride F floats), scaled x*a + b;
// features past F scale to exactly 0 (a = b = 0 there)
template <int FMAX>
__device__ __forceinline__ void load_scaled_row(const float* s_tile, int lane, int F, const float* sa_,
                                                const float* sb_, f2v (&x2)[FMAX / 2]) {
  int z = 0;
  asm volatile("" : "+s"(z));  // re-read the scaler from LDS each tile (no pinned registers)
  const f2v* sa = reinterpret_cast<const f2v*>(sa_) + z;
  const f2v* sb = reinterpret_cast<const f2v*>(sb_) + z;
  const float* xs = s_tile + lane * F;
  if ((F & 1) == 0) {  // 8-byte aligned rows: ds_read_b64 pairs
    const f2v* xp = reinterpret_cast<const f2v*>(__builtin_assume_aligned(xs, 8));
#pragma unroll
    for (int p = 0; p < FMAX / 2; ++p) {
      // pairs past F read the next row (finite: times the padded scaler 0
      // they are exactly 0); the tile's last row reads past 64 * F, which
      // every caller keeps finite (full tile loads, or zeroed: lloyd kQueue)
      x2[p] = __builtin_elementwise_fma(xp[p], sa[p], sb[p]);
      // groups of 4 pairs: keeps the scaler reads from all being hoisted
      // (3 x 32 transient VGPRs)
      if ((p & 3) == 3) __builtin_amdgcn_sched_barrier(0);
    }
  } else {
#pragma unroll
    for (int p = 0; p < FMAX / 2; ++p)
      x2[p] = __builtin_elementwise_fma(f2v{xs[2 * p], xs[2 * p + 1]}, sa[p], sb[p]);
  }
}

// pair-major center image (FMAX/2 x KS float pairs)
__host__ __device__ inline size_t cent_t_bytes(int KS, int FMAX) {
  return (size_t)(FMAX / 2) * KS * 8;
}

// fixed-order sum of G per-block records: thread (q, part) sums blocks
// b = part, part+8, ... with 8 independent partial sums, then parts combine
// in order.
__device__ __forceinline__ void rec_reduce_body(const double* __restrict__ rec, int G, int rl,
                                                  double* __restrict__ out) {
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



}  // namespace mw
