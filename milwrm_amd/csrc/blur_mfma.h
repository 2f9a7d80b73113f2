// Fused log-normalise + separable Gaussian blur with the horizontal pass on
// the f32 matrix cores (img.log_normalize + img.blurring('gaussian'),
// MxIF.py:416-455 / 375-394; scipy gaussian_filter mode='nearest', truncate=4)
// — the fast path for radius 1..8 (sigma <= 2.1) and even C <= 64.
//
// A workgroup owns a band of BW = 16*BT output columns x bh output rows (BlurGrid)
// and all channels; wave (tx, ct) owns the 16-column x 16-channel output tile
// (BT x ceil(C/16) waves).  Rows stream top to bottom through three stages:
//   1. input: the halo'd row segment (BW + 2r columns x C channels, one
//      contiguous HWC byte range) arrives as 16-byte buffer loads issued a few
//      rows ahead (register ring), is log-normalised and stored as fp32 to a
//      double-buffered LDS row [column][16 * ceil(C/16) channels] (channel
//      tiles XOR-swizzled by column parity when the pitch is a multiple of 32
//      floats: conflict-free operand reads; pad channels stay 0; at the slide
//      edges the clamped halo columns are copied from the edge column);
//   2. horizontal pass = one GEMM per tile: out[16 cols][16 ch] = T[16][4K] x
//      in[4K cols][16 ch], T the banded Toeplitz matrix of the 2r+1 taps
//      (constant A operands), K/4 v_mfma_f32_16x16x4_f32 in two interleaved
//      accumulators.  The f32 MFMA is an exact fp32 FMA chain, and the zero
//      band entries add exact zeros;
//   3. vertical pass: the last 2r+1 horizontal results (4 columns x 1 channel
//      per lane: the MFMA D layout) sit in a register ring (static indices:
//      the row loop is unrolled by 2r+1) and are combined by packed FMAs into
//      an LDS staging row laid out like the output (HWC), which the whole
//      workgroup writes to HBM as 16-byte stores one step later.
// Every HBM access is 16 bytes per lane (a blur-shaped access probe on the
// MI355X, tools/probe/band_probe.hip: 4-byte lanes 4.0 TB/s, 16-byte lanes
// 5.2 TB/s); the matrix pipe takes the horizontal taps, the VALU the vertical
// ones and the log-normalise; one workgroup barrier per row.
#pragma once

#include "blur.h"

namespace mw {

constexpr int kBlurMfmaMaxR = 8;
constexpr int kBlurMfmaBH = 512;  // output rows per band (BlurGrid)

typedef float f4m __attribute__((ext_vector_type(4)));
typedef unsigned int u4m __attribute__((ext_vector_type(4)));
typedef float f2m_ __attribute__((ext_vector_type(2)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t blur_rsrc(const void* base, uint32_t nbytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)nbytes, 0x00020000);
}

// element pair i (0-based) of a 16-byte chunk as floats
template <typename T> struct Chunk16;
template <> struct Chunk16<uint8_t> {
  static constexpr int P = 8;
  static __device__ __forceinline__ bf2 pair(const u4m& v, int i) {
    const uint32_t w = v[i >> 1] >> (16 * (i & 1));
    return bf2{(float)(w & 0xffu), (float)((w >> 8) & 0xffu)};
  }
};
template <> struct Chunk16<uint16_t> {
  static constexpr int P = 4;
  static __device__ __forceinline__ bf2 pair(const u4m& v, int i) {
    return bf2{(float)(v[i] & 0xffffu), (float)(v[i] >> 16)};
  }
};
template <> struct Chunk16<float> {
  static constexpr int P = 2;
  static __device__ __forceinline__ bf2 pair(const u4m& v, int i) {
    // whole-vector bit cast (element-wise casts of vector lanes have been
    // miscompiled by ROCm 7.2's hipcc: see the staging store in blur history)
    const f4m f = __builtin_bit_cast(f4m, v);
    return i == 0 ? bf2{f.x, f.y} : bf2{f.z, f.w};
  }
};

// Workgroup barrier for LDS hand-offs only.  __syncthreads() is a
// workgroup-scope acq_rel fence + s_barrier, and hipcc lowers the fence to
// s_waitcnt vmcnt(0) whenever a global store is outstanding — which also
// drains the input loads in flight (one counter) and flattens the row
// pipeline.  Nothing here hands data between threads through global memory.
__device__ __forceinline__ uint32_t lds_addr_u32(const void* p) {
  return (uint32_t)(uintptr_t)((__attribute__((address_space(3))) const char*)p);
}
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// LDS-DMA of 16 bytes per lane: global (SGPR base + per-lane 32-bit offset)
// -> LDS at (wave-uniform lds_dst) + lane * 16, no VGPR destination.  Inline
// asm (recipe: cdna_hip_programming.md §5.4), so hipcc neither counts it nor
// drains it: the kernel waits for it with counted vmcnt before the barrier
// that precedes the read.  The offset VGPR is set once per thread and never
// rewritten, so no later instruction can race the DMA's operand read; the
// string opens with s_nop 4 (SGPR base fresh from VALU/readfirstlane).  The
// default cache policy: with nt (the row passes' kStreamAux) the launch takes
// 4.21 instead of 4.11 ms (the bands' column halos are L2 hits;
// profiles/r06/nt_ab*/).
__device__ __forceinline__ void glds16(const void* sbase, uint32_t voff, uint32_t lds_dst) {
  unsigned keep;
  asm volatile(
      "s_nop 4\n\ts_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
      "global_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(sbase), "s"(lds_dst)
      : "memory");
}
template <int N>
__device__ __forceinline__ void vm_wait_n() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// What happens to an output row once the vertical pass has staged it in LDS:
//   kEpiStore   store the blurred row (HWC fp32): img.blurring
//   kEpiSample  write the subsample rows straight from the blur: pixel p's
//               features go to X[head[p]] (head = smallest sample slot of p,
//               mw_sample_map; the other slots of p are copied afterwards)
//   kEpiAssign  StandardScaler + nearest center + confidence per pixel
//               (KMeans.predict + estimate_confidence_score_mxif) on the
//               staged row; label and confidence go to HBM, the blurred
//               image never does
// Every epilogue but kEpiStore takes its per-row side data (head slots or mask
// bytes) through the raw DMA ring: each ring slot carries one more 1-KB DMA
// piece past the raw input row, with the side data of the output row that the
// same slot serves.
template <typename T, int R, int CT, int BT, int EPI = kEpiStore, bool H16 = false>
struct BlurMfmaCfg {
  static constexpr int NR = 2 * R + 1;
  static constexpr int BW = 16 * BT;            // output columns per band
  static constexpr int NPX = BW + 2 * R;        // halo'd input columns
  static constexpr int PS = 16 * CT;            // LDS row pitch per column (floats)
  static constexpr bool SWZ = (PS % 32) == 0;   // swizzle channel tiles by column parity
  static constexpr int NK = (16 + 2 * R + 3) / 4;  // MFMA k-steps (4 input columns each)
  static constexpr int NT = 64 * BT * CT;
  static constexpr int NW = NT / 64;
  // H16 (log-normalised input): the row is held as two f16 images, hi and lo
  // (x = hi + lo to 2^-22), each [pixel slot][U units of 16 channels] with the
  // units XOR-swizzled by slot (blur_h16_unit) so that the transposed operand
  // reads are conflict-free; NPXS slots are read by the K = 32 operand of the
  // last tile (BW + 16 >= NPX), slot NPXS is the sink of pad pairs
  static constexpr int U = CT <= 2 ? 2 : 4;
  static constexpr int NPXS = BW + 16;
  static constexpr int IMGH = (NPXS + 1) * U * 16;  // halves per f16 image
  static constexpr int ROW = H16 ? IMGH : NPX * PS;  // floats per LDS row buffer (H16: hi + lo images)
  static constexpr int STG = BW * 16 * CT;      // floats per LDS output staging row (>= BW*C)
  // raw input row segment: <= NPX * C elements, C <= 16*CT, fetched as NPC
  // lane-linear 1-KB DMA pieces (piece i: wave i % NW, round i / NW); the
  // fused epilogues add one piece for their per-row side data (index NPC)
  static constexpr int SEGMAX = NPX * 16 * CT * (int)sizeof(T);
  static constexpr int NPC = (SEGMAX + 1023) / 1024;
  static constexpr int NPIECE = NPC + (EPI == kEpiStore ? 0 : 1);
  static constexpr int NG = (NPIECE + NW - 1) / NW;  // DMA rounds (pieces of the busiest wave)
  static constexpr int LASTW = NPIECE - (NG - 1) * NW;  // waves < LASTW issue NG pieces, the rest NG-1
  static constexpr int SLOT = NPIECE * 1024;    // bytes per raw ring slot
  static constexpr int NCH = (SLOT / 16 + NT - 1) / NT;  // 16-byte chunks per thread
  static constexpr int NP = NCH * Chunk16<T>::P;  // element pairs per thread
  // kEpiAssign: per output row the k distances of its BW pixels and their
  // mask bytes, double-buffered (written one step, reduced the next)
  static constexpr size_t EXTRA =
      EPI == kEpiAssign ? 2 * ((size_t)kEpiKMax * BW * 4 + BW) + (size_t)kEpiKMax * 8 * CT * 8 : 0;
  static constexpr size_t FIXED = (2 * (size_t)ROW + 2 * (size_t)STG) * sizeof(float) + 64 + EXTRA;
  static constexpr int AUXOFF = NPC * 1024;     // side-data piece
  static constexpr int AUXW = NPC % NW;
  static constexpr int NS = NT / BW;            // epilogue threads per output column (4*CT)
  // raw ring depth: as deep as two workgroups per CU allow (160 KB of LDS),
  // up to DMAX rows (the DMA of row s+2 is waited for at step s: LA-2 steps
  // of lead); one workgroup per CU only when two do not fit a 4-row ring
  static constexpr int DMAX = 8;
  static constexpr int D2 = ((80 * 1024 - (int)FIXED) / SLOT);
  static constexpr int D1 = ((160 * 1024 - (int)FIXED) / SLOT);
  static constexpr int D = D2 >= 4 ? (D2 < DMAX ? D2 : DMAX) : (D1 >= 4 ? (D1 < DMAX ? D1 : DMAX) : 4);
  static constexpr int LA = D - 1;              // rows in flight ahead of the converted one
  static constexpr size_t lds_bytes() { return FIXED + (size_t)D * SLOT; }
};

typedef _Float16 h2m __attribute__((ext_vector_type(2)));
typedef _Float16 h8m __attribute__((ext_vector_type(8)));
typedef short s4m __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s4m lds_s4m;

// H16 image: physical 16-channel unit of channel tile ct in pixel slot x.  A
// transposed read (ds_read_b64_tr_b16) of the 16x16x32 B operand takes, per
// 32-lane half, slots 8n..8n+3 and 8n+8..8n+11 (4 lanes x 8 bytes each): with
// U = 2 units per slot the slot bit 3 flips the unit, with U = 4 slot bits 1
// and 3 do, and the 32 lanes cover all 64 banks exactly once.
template <int U>
__host__ __device__ __forceinline__ int blur_h16_unit(int x, int ct) {
  return U == 2 ? ct ^ ((x >> 3) & 1) : ct ^ (((x >> 1) & 1) | (((x >> 3) & 1) << 1));
}
// log-normalised values are scaled by 2^8 before the split (the lo half stays
// clear of f16 subnormals), the horizontal taps by 2^16; the vertical taps
// take the 2^-24 back (exact: powers of two)
// cache policy of the blurred-row stores (buffer aux bits; 2 = nt: streaming)
constexpr int kBlurStoreAux = 2;
constexpr bool kBlurH16 = true;   // log-normalised input: horizontal pass on f16 hi/lo products
constexpr float kH16XS = 256.f, kH16TS = 65536.f, kH16VS = 1.f / 16777216.f;

// Band grid: nbx column bands x nby row bands of bh rows, one workgroup each,
// launched as a 1-D grid (column band fastest).  Round 2, at 10k^2 x 30
// (tools/dev/blur_ab.sh, same box, two runs each): 512-row bands 4.72 / 4.74
// ms vs 256-row 4.79 / 4.81 (the 16 halo rows are 3 % of a 512-row band, 6 %
// of a 256-row one); 384 / 768 / 1024 rows and 128-column bands slower;
// dealing adjacent bands to one XCD (xcd = 1: block b takes logical tile
// (b % 8) * (tiles / 8) + b / 8) slower.  MW_BLUR_BH and MW_BLUR_XCD override
// both for tuning.
struct BlurGrid {
  int bh, nbx, ntiles, xcd;
  int r0, r1;  // output rows [r0, r1) of the input array (the whole array but for streamed bands)
  __device__ __forceinline__ void tile(int b, int G, int& bx, int& by) const {
    const int x = b & 7, j = b >> 3, q = G >> 3, rem = G & 7;
    const int t = xcd ? x * q + (x < rem ? x : rem) + j : b;
    by = t / nbx;
    bx = t - by * nbx;
  }
};

static inline BlurGrid blur_grid(int r0, int r1, int nbx) {
  BlurGrid g;
  g.nbx = nbx;
  g.bh = kBlurMfmaBH;
  g.xcd = 0;
  g.r0 = r0;
  g.r1 = r1;
  if (const char* e = getenv("MW_BLUR_BH")) g.bh = atoi(e) >= 16 ? atoi(e) : kBlurMfmaBH;
  if (const char* e = getenv("MW_BLUR_XCD")) g.xcd = atoi(e);
  g.ntiles = nbx * ((r1 - r0 + g.bh - 1) / g.bh);
  return g;
}

template <typename T, int R, int CT, int BT, bool LOGN, int EPI>
__global__ void __launch_bounds__(64 * BT * CT, 4) blur_mfma_kernel(const T* __restrict__ in, int H, int W,
                                                                 int C, const float* __restrict__ inv_mean,
                                                                 float pseudo, BlurTaps taps,
                                                                 float* __restrict__ out, BlurEpi ep,
                                                                 BlurGrid bg) {
  constexpr bool H16 = LOGN && kBlurH16;
  using K = BlurMfmaCfg<T, R, CT, BT, EPI, H16>;
  constexpr int NS = K::NS;
  constexpr int U = K::U, IMGH = K::IMGH, NPXS = K::NPXS;
  constexpr int NR = K::NR, BW = K::BW, NPX = K::NPX, PS = K::PS, NK = K::NK, NT = K::NT;
  constexpr int ROW = K::ROW, STG = K::STG, NCH = K::NCH, NP = K::NP, CP = Chunk16<T>::P;
  constexpr int NG = K::NG, SLOT = K::SLOT, D = K::D, LA = K::LA;
  constexpr bool SWZ = K::SWZ;
  static_assert(LA >= 3, "raw ring too shallow");
  // one step issues NG (waves < LASTW) or NG-1 DMA pieces per wave + 1 output
  // store (kEpiStore; the other epilogues issue only a data-dependent number
  // of stores, which can only make a count stricter); the DMA of row s+2
  // (issued at step s+2-LA) is followed by LA-2 steps' worth of them.  Waves
  // without pieces wait for nothing.
  constexpr int kStore = EPI == kEpiStore ? 1 : 0;
  constexpr int NGB = NG - 1;  // pieces per step of waves >= LASTW
  static_assert((LA - 2) * (NG + kStore) <= 63, "vmcnt field is 6 bits");
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* s_rows = smem;                       // 2 x ROW  (fp32 input rows)
  float* s_stg = smem + 2 * ROW;              // 2 x STG  (output staging rows, HWC)
  float* s_dummy = smem + 2 * ROW + 2 * STG;  // 64 bytes: sink of pad pairs
  char* s_raw = reinterpret_cast<char*>(smem) + K::FIXED;  // D x SLOT raw input rows
  float* s_dist = s_dummy + 16;                            // kEpiAssign: [2][k][BW] distances
  uint8_t* s_mk = reinterpret_cast<uint8_t*>(s_dist + 2 * kEpiKMax * BW);  // [2][BW] mask bytes
  f2m_* s_cen = reinterpret_cast<f2m_*>(s_mk + 2 * BW);   // [k][8 CT] center pairs
  const int t = threadIdx.x;
  const int lane = t & 63;
  const int wv = __builtin_amdgcn_readfirstlane(t >> 6);
  const int tx = wv % BT, ct = wv / BT;
  int bx, by;
  bg.tile(blockIdx.x, gridDim.x, bx, by);
  const int x0 = bx * BW;
  const int y0 = bg.r0 + by * bg.bh;
  const int y1 = min(bg.r1, y0 + bg.bh);
  const int nrows = (y1 - y0) + 2 * R;
  const int bw = min(BW, W - x0);
  // clamped input column range [xa, xb) and its position in the halo'd row
  const int xa = max(0, x0 - R), xb = min(W, x0 + BW + R);
  const int col_a = xa - (x0 - R);
  const bool edge = (xa != x0 - R) || (xb != x0 + BW + R);
  const uint32_t seg_bytes = (uint32_t)(xb - xa) * (uint32_t)C * sizeof(T);

  for (int q = t; q < 2 * ROW; q += NT) s_rows[q] = 0.f;  // pad channels stay 0

  // ---- raw chunks of this thread (chunk t + c*NT of a slot): LDS fp32
  // destination of each element pair in a row buffer (-1: pad pair, written
  // to the sink)
  int p_dst[NP];
  bf2 p_inv[NP];
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const uint32_t b0 = (uint32_t)(t + c * NT) * 16u;
#pragma unroll
    for (int i = 0; i < CP; ++i) {
      const uint32_t e = (b0 / (uint32_t)sizeof(T)) + 2u * i;  // element index in the segment
      const bool ok = e * (uint32_t)sizeof(T) < seg_bytes;
      const int px = ok ? (int)(e / (uint32_t)C) : 0;
      const int ch = ok ? (int)(e - (uint32_t)px * C) : 0;
      const int col = col_a + px, ctile = ch >> 4;
      if constexpr (H16)  // byte offset in an f16 image (pad pairs: the sink slot)
        p_dst[c * CP + i] = 2 * (ok ? col * U * 16 + 16 * blur_h16_unit<U>(col, ctile) + (ch & 15) : NPXS * U * 16);
      else
        p_dst[c * CP + i] = ok ? col * PS + 16 * (SWZ ? (ctile ^ (col & 1)) : ctile) + (ch & 15) : -1;
      p_inv[c * CP + i] = (LOGN && ok) ? bf2{inv_mean[ch], inv_mean[ch + 1]} : bf2{1.f, 1.f};
    }
  }
  // DMA source offset of this lane's piece g: chunk t + g*NT, clamped into the segment
  uint32_t g_off[NG];
#pragma unroll
  for (int g = 0; g < NG; ++g) {
    const uint32_t b = (uint32_t)(t + g * NT) * 16u;
    g_off[g] = b < seg_bytes ? b : 0u;
  }
  const uint32_t raw0 = lds_addr_u32(s_raw);

  // ---- MFMA operands: A = banded Toeplitz taps (row m = output column, k =
  // input column of the tile's halo'd span), B = LDS row reads
  const int m = lane & 15, kq = lane >> 4;
  float a_op[NK];
  const float tap_scale = LOGN ? 0.30102999566398120f : 1.f;  // log2 -> log10 (log2norm2)
  if constexpr (!H16) {
#pragma unroll
    for (int st = 0; st < NK; ++st) {
      const int j = 4 * st + kq - m;
      a_op[st] = (j >= 0 && j <= 2 * R) ? taps.w[j] * tap_scale : 0.f;
    }
  }
  // H16: A[m][k = 8kq + i] = tap k - m (x 2^16, split hi + lo); B = rows of the
  // hi / lo images by two transposed reads each (slots 16tx + 8kq + 4r + q,
  // channels 16ct + 4p .. +3 from lane 4q + p of the group)
  h8m a_hi, a_lo;
  uint32_t b_addr[2] = {0u, 0u};
  if constexpr (H16) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int j = 8 * kq + i - m;
      // taps arrive x 2^-24 (the vertical pass's descale, launch_blur_mfma_one)
      const float w = (j >= 0 && j <= 2 * R) ? taps.w[j] * (tap_scale * kH16TS * 16777216.f) : 0.f;
      const _Float16 h = (_Float16)w;
      a_hi[i] = h;
      a_lo[i] = (_Float16)(w - (float)h);
    }
    const int q = (lane & 15) >> 2, p = lane & 3;
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int x = 16 * tx + 8 * kq + 4 * r + q;
      b_addr[r] = lds_addr_u32(s_rows) + 2u * (uint32_t)(x * U * 16 + 16 * blur_h16_unit<U>(x, ct) + 4 * p);
    }
  }
  // B[k][n] for k-step st: column 16*tx + 4*st + kq, channel 16*ct + n (n = m)
  const int b_ct = SWZ ? (ct ^ (kq & 1)) : ct;  // (16*tx + 4*st + kq) & 1 == kq & 1
  const int b_base = (16 * tx + kq) * PS + 16 * b_ct + m;
  // staging slot of D[r]: column 16*tx + 4*kq + r, channel 16*ct + m (HWC, pitch C)
  const bool st_ok = 16 * ct + m < C;
  const int st_base = (16 * tx + 4 * kq) * C + 16 * ct + m;
  // output: the band's row segment is bw*C floats (a multiple of 4: host
  // check); thread t stores 16-byte chunk t, past the segment the range check drops it
  const uint32_t out_bytes = (uint32_t)bw * (uint32_t)C * 4u;

  // ---- epilogue: thread (column ecol, part esub) of the staged output row
  const int ecol = t / NS, esub = t % NS;
  int fo[2][2];  // kEpiSample: channel of features 2*(esub + NS*i) + {0,1}, -1 past F
  float sc_a = 1.f, sc_b = 0.f;  // kEpiAssign: scaler of this lane's vertical-pass channel
  uint32_t aux_off = 0;
  if constexpr (EPI == kEpiSample) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int f0 = 2 * (esub + NS * i);
      fo[i][0] = f0 < ep.F ? ep.feat[f0] : -1;
      fo[i][1] = f0 + 1 < ep.F ? ep.feat[f0 + 1] : -1;
    }
    aux_off = (uint32_t)lane * 16u < (uint32_t)(BW + 2) * 8u ? (uint32_t)lane * 16u : 0u;
  }
  if constexpr (EPI == kEpiAssign) {
    for (int q = t; q < kEpiKMax * 8 * CT; q += NT) {
      const int j = q / (8 * CT), p2 = q - j * (8 * CT);
      const bool ok = j < ep.k && 2 * p2 < C;  // C even (launcher)
      s_cen[q] = ok ? f2m_{ep.centers[j * C + 2 * p2], ep.centers[j * C + 2 * p2 + 1]} : f2m_{0.f, 0.f};
    }
    if (st_ok) {
      sc_a = ep.a[16 * ct + m];
      sc_b = ep.b[16 * ct + m];
    }
    aux_off = (uint32_t)lane * 16u < (uint32_t)(BW + 16) ? (uint32_t)lane * 16u : 0u;
  }

  f4m ring[NR];
#pragma unroll
  for (int j = 0; j < NR; ++j) ring[j] = f4m{0.f, 0.f, 0.f, 0.f};

  // DMA of input row q (clamped; past the band: a harmless re-read) into slot q % D
  auto dma_row = [&](int q) {
    int yy = y0 - R + q;
    yy = yy < 0 ? 0 : (yy >= H ? H - 1 : yy);
    const char* src = reinterpret_cast<const char*>(in + ((int64_t)yy * W + xa) * C);
    const uint32_t slot = raw0 + (uint32_t)(q % D) * SLOT;
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      if (g == NG - 1 && wv >= K::LASTW) continue;  // piece past the slot
      if constexpr (EPI != kEpiStore) {
        if (g == NG - 1 && wv == K::AUXW) {
          // side data of output row y0 + q - 2 - 2R (the row stored at step q),
          // from the 16-byte aligned address at or below its first pixel
          int yq = y0 + q - 2 - 2 * R;
          yq = yq < y0 ? y0 : (yq >= y1 ? y1 - 1 : yq);
          const int64_t rp = (int64_t)(yq + ep.row_off) * W + x0;  // slide pixel
          const char* asrc = EPI == kEpiSample
                                 ? reinterpret_cast<const char*>(ep.slots) + ((rp * 8) & ~(int64_t)15)
                                 : reinterpret_cast<const char*>(ep.mask) + (rp & ~(int64_t)15);
          glds16(asrc, aux_off, slot + (uint32_t)(g * NT + 64 * wv) * 16u);
          continue;
        }
      }
      glds16(src, g_off[g], slot + (uint32_t)(g * NT + 64 * wv) * 16u);
    }
  };
  auto convert_row = [&](int q) {
    float* dst = s_rows + (q & 1) * ROW;
    const char* raw = s_raw + (q % D) * SLOT;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      // waves whose chunks are all past the segment skip the conversion (pad
      // pairs only; wave-uniform branch): with BW*C small enough that the
      // segment fits four waves, every SIMD converts one chunk per row
      if ((uint32_t)(64 * wv + c * NT) * 16u >= seg_bytes) continue;
      // chunks past the slot (SLOT is not a multiple of NT*16) are pad pairs
      const u4m v = (c + 1) * NT * 16 <= SLOT || (t + c * NT) * 16 < SLOT
                        ? *reinterpret_cast<const u4m*>(raw + (t + c * NT) * 16)
                        : u4m{0u, 0u, 0u, 0u};
#pragma unroll
      for (int i = 0; i < CP; ++i) {
        bf2 x = Chunk16<T>::pair(v, i);
        if constexpr (H16) {
          // x * 2^8 = hi + lo, both f16 (hi round-to-nearest, the residual exact in fp32)
          x = log2norm2(x, p_inv[c * CP + i], pseudo) * bf2{kH16XS, kH16XS};
          const h2m h = __builtin_convertvector(x, h2m);
          const h2m l = __builtin_convertvector(x - __builtin_convertvector(h, bf2), h2m);
          char* img = reinterpret_cast<char*>(dst) + p_dst[c * CP + i];
          *reinterpret_cast<h2m*>(img) = h;
          *reinterpret_cast<h2m*>(img + 2 * IMGH) = l;
          continue;
        }
        if (LOGN) x = log2norm2(x, p_inv[c * CP + i], pseudo);  // log10(2): in the taps
        const int d = p_dst[c * CP + i];
        *reinterpret_cast<bf2*>(d >= 0 ? dst + d : s_dummy) = x;  // pad pairs: the sink
      }
    }
    if (H16 && edge) {  // clamped halo columns: copies of the edge column, both images
      lds_barrier();
      const int nl = col_a, nr = NPX - (col_a + (xb - xa));
      uint32_t* img = reinterpret_cast<uint32_t*>(dst);
      for (int q2 = t; q2 < (nl + nr) * CT * 8 * 2; q2 += NT) {
        const int im = q2 & 1, f = (q2 >> 1) & 7, u = (q2 >> 4) % CT, h = (q2 >> 4) / CT;
        const int col = h < nl ? h : col_a + (xb - xa) + (h - nl);
        const int src = h < nl ? col_a : col_a + (xb - xa) - 1;
        const int o = im * IMGH / 2;  // in pairs
        img[o + col * U * 8 + 8 * blur_h16_unit<U>(col, u) + f] = img[o + src * U * 8 + 8 * blur_h16_unit<U>(src, u) + f];
      }
    } else if (edge) {  // clamped halo columns ('nearest'): copies of the edge column
      lds_barrier();
      const int nl = col_a, nr = NPX - (col_a + (xb - xa));
      for (int q2 = t; q2 < (nl + nr) * PS; q2 += NT) {
        const int h = q2 / PS, f = q2 - h * PS;
        const int col = h < nl ? h : col_a + (xb - xa) + (h - nl);
        const int src = h < nl ? col_a : col_a + (xb - xa) - 1;
        // (the channel-tile swizzle depends on the column parity)
        const int ctile = f >> 4;
        const int fs = SWZ ? 16 * (ctile ^ (src & 1)) + (f & 15) : f;
        const int fd = SWZ ? 16 * (ctile ^ (col & 1)) + (f & 15) : f;
        dst[col * PS + fd] = dst[src * PS + fs];
      }
    }
  };
  // one 16-byte store per thread and step; rows outside the band are dropped
  // by an empty range (every step issues exactly one store: counted waits)
  auto store_out = [&](int stg_buf, int yo, bool valid) {
    const f4m v = *reinterpret_cast<const f4m*>(s_stg + stg_buf * STG + 4 * t);
    const __amdgpu_buffer_rsrc_t ro =
        blur_rsrc(out + ((int64_t)(valid ? yo - bg.r0 : 0) * W + x0) * C, valid ? out_bytes : 0u);
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4m, v), ro, t * 16, 0, kBlurStoreAux);
  };

  // kEpiSample / kEpiAssign on the output row staged at step s-1 (buffer s & 1)
  auto epilogue = [&](int s) {
    asm volatile("" : "+s"(s));  // per-step values stay per step (no hoisting across the unroll)
    const int yo = y0 + s - 2 - 2 * R;
    const int64_t rowpix = (int64_t)(yo + ep.row_off) * W + x0;  // slide pixel (side data, outputs)
    const char* auxp = s_raw + (s % D) * SLOT + K::AUXOFF;
    const float* srow = s_stg + (s & 1) * STG + ecol * C;
    if constexpr (EPI == kEpiSample) {
      // the pixel's first two sample slots (mw_sample_map; -1: none): this
      // thread's features from the staged row, one store per slot
      const int2 sl = reinterpret_cast<const int2*>(auxp)[(int)(rowpix & 1) + ecol];
      if (ecol < bw && (uint64_t)(uint32_t)sl.x < (uint64_t)ep.S) {
        const bool dup = (uint64_t)(uint32_t)sl.y < (uint64_t)ep.S;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const int f0 = 2 * (esub + NS * i);
          if (fo[i][0] < 0) continue;
          const bool two = fo[i][1] >= 0;
          const f2m_ v = f2m_{srow[fo[i][0]], two ? srow[fo[i][1]] : 0.f};
#pragma unroll
          for (int u = 0; u < 2; ++u) {
            if (u == 1 && !dup) break;
            float* dst = ep.X + (int64_t)(u ? sl.y : sl.x) * ep.F;
            if (two && (ep.F & 1) == 0) {
              *reinterpret_cast<f2m_*>(dst + f0) = v;
            } else {
              dst[f0] = v.x;
              if (two) dst[f0 + 1] = v.y;
            }
          }
        }
      }
    } else {
      // distance phase: wave w takes centers w, w + NW, ... (wave-uniform:
      // the center comes by scalar loads), lane = pixel column of the staged
      // row; the Lloyd/assign E-step chain (even features in .x, odd in .y,
      // pair order, then .x + .y), so the distances are the assign kernel's
      // bits.  The argmin over the k tables runs next step (argmin_phase).
      const int np = C >> 1;
      const f2m_* xp = reinterpret_cast<const f2m_*>(s_stg + (s & 1) * STG + lane * C);
      float* dst = s_dist + (s & 1) * kEpiKMax * BW;
      for (int c0 = wv; c0 < ep.k; c0 += K::NW) {
        const f2m_* cj = s_cen + c0 * (8 * CT);  // wave-uniform address: broadcast reads
        f2m_ acc = f2m_{0.f, 0.f};
#pragma unroll 4
        for (int p2 = 0; p2 < np; ++p2) {
          const f2m_ d = xp[p2] - cj[p2];
          acc = __builtin_elementwise_fma(d, d, acc);
        }
        dst[c0 * BW + lane] = acc.x + acc.y;
      }
      if (wv == K::NW - 1 && lane < BW)  // the row's mask bytes travel with its distances
        s_mk[(s & 1) * BW + lane] = reinterpret_cast<const uint8_t*>(auxp)[(int)(rowpix & 15) + lane];
    }
  };
  // argmin phase for the row whose distances were written at step s - 1:
  // strict argmin in center order + second smallest (nearest_centers<TOP2>),
  // confidence (d2 - d1) / d2; one wave, lane = pixel column
  auto argmin_phase = [&](int s) {
    asm volatile("" : "+s"(s));
    if (wv != (s % K::NW) || lane >= bw) return;
    const int yo = y0 + (s - 1) - 2 - 2 * R;
    const int64_t rowpix = (int64_t)(yo + ep.row_off) * W + x0;
    const float* dd = s_dist + ((s - 1) & 1) * kEpiKMax * BW + lane;
    int lab = 0;
    float m1 = dd[0], m2 = __builtin_inff();
#pragma unroll 4
    for (int j = 1; j < ep.k; ++j) {
      const float d = dd[j * BW];
      if (d < m1) { m2 = m1; m1 = d; lab = j; }
      else if (d < m2) { m2 = d; }
    }
    const bool in_mask = s_mk[((s - 1) & 1) * BW + lane] != 0;
    ep.lab[rowpix + lane] = (int8_t)(in_mask ? lab : -1);
    ep.conf[rowpix + lane] = in_mask ? (m2 - m1) / m2 : __builtin_nanf("");  };

  lds_barrier();  // zero fill done
#pragma unroll
  for (int q = 0; q < LA; ++q) dma_row(q);
  // the wait counts of this wave (full: NG pieces per row, else NG-1)
  const bool full = wv < K::LASTW;
  if (full) vm_wait_n<(LA - 1) * NG>();  // row 0 landed (this wave's pieces)
  else if (NGB > 0) vm_wait_n<(LA - 1) * (NGB > 0 ? NGB : 1)>();
  lds_barrier();
  convert_row(0);
  if (full) vm_wait_n<(LA - 2) * NG>();  // row 1 landed
  else if (NGB > 0) vm_wait_n<(LA - 2) * (NGB > 0 ? NGB : 1)>();
  lds_barrier();
  // step s: convert input row s+1, MFMA row s, vertical pass of row s-1 into
  // staging, store the output row staged at step s-1, DMA of row s+LA; wait
  // for row s+2's DMA; one barrier
  const int nsteps = nrows + 2;
  // One row step (j = s mod NR is a compile-time constant after unrolling, so
  // the ring indices are static).  GUARD false: the steady state, where every
  // stage is live, with no branches, so hipcc can interleave the stages.
  auto step = [&](const int s, const int j, const bool guard) {
    if (!guard || s + 1 < nrows) convert_row(s + 1);
    float b_op[NK];
    h8m b_hi, b_lo;
    if (!guard || s < nrows) {
      if constexpr (H16) {
        const uint32_t bo = (uint32_t)(s & 1) * (uint32_t)(ROW * 4);
        s4m r0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4m*)(uintptr_t)(b_addr[0] + bo));
        s4m r1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4m*)(uintptr_t)(b_addr[1] + bo));
        s4m r2 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4m*)(uintptr_t)(b_addr[0] + bo + 2 * IMGH));
        s4m r3 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4m*)(uintptr_t)(b_addr[1] + bo + 2 * IMGH));
        typedef short s8m __attribute__((ext_vector_type(8)));
        b_hi = __builtin_bit_cast(h8m, __builtin_shufflevector(r0, r1, 0, 1, 2, 3, 4, 5, 6, 7));
        b_lo = __builtin_bit_cast(h8m, __builtin_shufflevector(r2, r3, 0, 1, 2, 3, 4, 5, 6, 7));
        (void)sizeof(s8m);
      } else {
        const float* rowp = s_rows + (s & 1) * ROW + b_base;
#pragma unroll
        for (int st = 0; st < NK; ++st) b_op[st] = rowp[4 * st * PS];
      }
    }
    if (!guard || (s >= 1 && s - 1 >= 2 * R && s - 1 < nrows)) {
      // vertical pass of row s-1 over ring rows s-1-2R .. s-1 (slots j .. j+2R)
      bf2 v0 = bf2{0.f, 0.f}, v1 = bf2{0.f, 0.f}, u0 = bf2{0.f, 0.f}, u1 = bf2{0.f, 0.f};
      constexpr int NRV = NR;
#pragma unroll
      for (int i = 0; i < NRV; ++i) {
        const f4m& rg = ring[(j + i) % NR];
        const bf2 w2 = bf2{taps.w[i], taps.w[i]};  // H16: x 2^-24 (launcher)
        if (i & 1) {
          v1 = __builtin_elementwise_fma(w2, bf2{rg.x, rg.y}, v1);
          u1 = __builtin_elementwise_fma(w2, bf2{rg.z, rg.w}, u1);
        } else {
          v0 = __builtin_elementwise_fma(w2, bf2{rg.x, rg.y}, v0);
          u0 = __builtin_elementwise_fma(w2, bf2{rg.z, rg.w}, u0);
        }
      }
      bf2 va = v0 + v1, vb = u0 + u1;
      if constexpr (EPI == kEpiAssign) {  // StandardScaler: x * a + b (the assign kernel's fma)
        va = __builtin_elementwise_fma(va, bf2{sc_a, sc_a}, bf2{sc_b, sc_b});
        vb = __builtin_elementwise_fma(vb, bf2{sc_a, sc_a}, bf2{sc_b, sc_b});
      }
      if (st_ok) {
        float* sg = s_stg + ((s - 1) & 1) * STG + st_base;
        sg[0] = va.x;
        sg[C] = va.y;
        sg[2 * C] = vb.x;
        sg[3 * C] = vb.y;
      }
    }
    if constexpr (EPI == kEpiStore) {
      store_out(s & 1, y0 + s - 2 - 2 * R, !guard || s >= 2 + 2 * R);
    } else if (!guard || s >= 2 + 2 * R) {
      // kept apart from the other stages: interleaved, the epilogue's
      // temporaries would lift the kernel past 128 VGPRs (one workgroup per CU)
      __builtin_amdgcn_sched_barrier(0);
      epilogue(s);
      if constexpr (EPI == kEpiAssign)
        if (!guard || s >= 3 + 2 * R) argmin_phase(s);
      __builtin_amdgcn_sched_barrier(0);
    }
    dma_row(s + LA);
    if (!guard || s < nrows) {
      if constexpr (H16) {
        // (hi + lo)(hi + lo) less lo*lo: three f16 products accumulated in fp32
        f4m d = __builtin_amdgcn_mfma_f32_16x16x32_f16(a_hi, b_hi, f4m{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
        d = __builtin_amdgcn_mfma_f32_16x16x32_f16(a_lo, b_hi, d, 0, 0, 0);
        ring[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a_hi, b_lo, d, 0, 0, 0);
      } else {
        f4m d0 = f4m{0.f, 0.f, 0.f, 0.f}, d1 = f4m{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int st = 0; st < NK; st += 2) {
          d0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a_op[st], b_op[st], d0, 0, 0, 0);
          if (st + 1 < NK) d1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a_op[st + 1], b_op[st + 1], d1, 0, 0, 0);
        }
        ring[j] = d0 + d1;
      }
    }
    if (full) {
      if (guard && s < LA - 2) vm_wait_n<(LA - 2) * NG + kStore>();  // prologue DMAs, no stores yet
      else vm_wait_n<(LA - 2) * (NG + kStore)>();
    } else if (NGB > 0) {
      if (guard && s < LA - 2) vm_wait_n<(LA - 2) * (NGB > 0 ? NGB : 1) + kStore>();
      else vm_wait_n<(LA - 2) * ((NGB > 0 ? NGB : 1) + kStore)>();
    }
    lds_barrier();
  };
  // steady groups: NR-aligned, all of s in [2R+2, nrows-2], interior bands
  // (edge bands copy halo columns behind an extra barrier: guarded path)
  const int g0 = 2 * NR;  // first multiple of NR >= 2R+2
  const int g1 = edge ? g0 : max(g0, ((nrows - 1) / NR) * NR);  // groups [g0, g1) are steady
  int base = 0;
  for (; base < g0 && base < nsteps; base += NR) {
#pragma unroll
    for (int j = 0; j < NR; ++j)
      if (base + j < nsteps) step(base + j, j, true);
  }
  for (; base < g1; base += NR) {
#pragma unroll
    for (int j = 0; j < NR; ++j) step(base + j, j, false);
  }
  for (; base < nsteps; base += NR) {
#pragma unroll
    for (int j = 0; j < NR; ++j)
      if (base + j < nsteps) step(base + j, j, true);
  }
  if constexpr (EPI == kEpiAssign)  // the last row's argmin (its distances: the last step)
    if (nsteps - 1 >= 2 + 2 * R) argmin_phase(nsteps);
  vm_wait_n<0>();  // no DMA may still target this workgroup's LDS at exit
}

template <typename T, int R, int CT, int BT, int EPI, bool LOGN>
static int launch_blur_mfma_one(const T* in, int H, int W, int C, const float* inv_mean, float p,
                                const BlurTaps& taps, float* out, const BlurEpi& ep, hipStream_t st) {
  using K = BlurMfmaCfg<T, R, CT, BT, EPI, LOGN && kBlurH16>;  // as the kernel instance
  const size_t lds = K::lds_bytes();
  if (lds > 160 * 1024 || K::D < 4) return MW_EUNSUPPORTED;
  const int nbx = (W + K::BW - 1) / K::BW;
  // the fused epilogues output the row window [ep.r0, ep.r1); img.blurring the whole array
  const BlurGrid bg = EPI == kEpiStore ? blur_grid(0, H, nbx) : blur_grid(ep.r0, ep.r1, nbx);
  if (bg.ntiles == 0) return MW_OK;
  BlurTaps tv = taps;  // H16: the vertical taps carry the 2^-24 descale (exact)
  if (LOGN && kBlurH16)
    for (int i = 0; i <= 2 * R; ++i) tv.w[i] = taps.w[i] * kH16VS;
  hipLaunchKernelGGL((blur_mfma_kernel<T, R, CT, BT, LOGN, EPI>), dim3(bg.ntiles), dim3(K::NT), lds, st, in, H,
                     W, C, inv_mean, p, tv, out, ep, bg);
  MW_LAUNCH_CHECK();
  return MW_OK;
}

template <typename T, int R, int CT, int BT, int EPI>
static int launch_blur_mfma_rc(const T* in, int H, int W, int C, const float* inv_mean, float p,
                               const BlurTaps& taps, float* out, const BlurEpi& ep, hipStream_t st) {
  if (inv_mean) return launch_blur_mfma_one<T, R, CT, BT, EPI, true>(in, H, W, C, inv_mean, p, taps, out, ep, st);
  if constexpr (EPI == kEpiStore)
    return launch_blur_mfma_one<T, R, CT, BT, EPI, false>(in, H, W, C, inv_mean, p, taps, out, ep, st);
  return MW_EUNSUPPORTED;  // the fused epilogues follow a log-normalise
}

template <typename T, int R>
static int launch_blur_mfma_r(const T* in, int H, int W, int C, const float* inv_mean, float p,
                              const BlurTaps& taps, float* out, hipStream_t st) {
  // column tiles per band: 4 (64-column bands, two 8-wave workgroups per CU
  // at C <= 32).  128-column bands (one 16-wave workgroup per CU, 12.5 % halo
  // instead of 25 %) are 3 % faster in a blur-only loop (3.91-3.93 vs
  // 4.04-4.06 ms) but 1.5-2.5 % slower inside the bench step (4.02-4.07 vs
  // 3.96-3.98 ms, same box, tools/dev/r3_bt_sweep.sh): not taken.
  const BlurEpi ep{};
  if (C <= 16) return launch_blur_mfma_rc<T, R, 1, 4, kEpiStore>(in, H, W, C, inv_mean, p, taps, out, ep, st);
  if (C <= 32) return launch_blur_mfma_rc<T, R, 2, 4, kEpiStore>(in, H, W, C, inv_mean, p, taps, out, ep, st);
  if (C <= 48) return launch_blur_mfma_rc<T, R, 3, 4, kEpiStore>(in, H, W, C, inv_mean, p, taps, out, ep, st);
  return launch_blur_mfma_rc<T, R, 4, 4, kEpiStore>(in, H, W, C, inv_mean, p, taps, out, ep, st);
}

// fused epilogue launch (BT = 4); the per-epilogue limits depend on CT
template <typename T, int R, int CT>
static int launch_blur_epi_rc(const T* in, int H, int W, int C, const float* inv_mean, float p,
                              const BlurTaps& taps, const BlurEpi& ep, int epi, hipStream_t st) {
  constexpr int NS = BlurMfmaCfg<T, R, CT, 4>::NS;
  if (epi == kEpiSample) {
    if (ep.F > 16 * CT) return MW_EUNSUPPORTED;
    return launch_blur_mfma_rc<T, R, CT, 4, kEpiSample>(in, H, W, C, inv_mean, p, taps, nullptr, ep, st);
  }
  if (ep.k < 1 || ep.k > kEpiKMax) return MW_EUNSUPPORTED;
  return launch_blur_mfma_rc<T, R, CT, 4, kEpiAssign>(in, H, W, C, inv_mean, p, taps, nullptr, ep, st);
}
template <typename T, int R>
static int launch_blur_epi_r(const T* in, int H, int W, int C, const float* inv_mean, float p,
                             const BlurTaps& taps, const BlurEpi& ep, int epi, hipStream_t st) {
  if (C <= 16) return launch_blur_epi_rc<T, R, 1>(in, H, W, C, inv_mean, p, taps, ep, epi, st);
  if (C <= 32) return launch_blur_epi_rc<T, R, 2>(in, H, W, C, inv_mean, p, taps, ep, epi, st);
  if (C <= 48) return launch_blur_epi_rc<T, R, 3>(in, H, W, C, inv_mean, p, taps, ep, epi, st);
  return launch_blur_epi_rc<T, R, 4>(in, H, W, C, inv_mean, p, taps, ep, epi, st);
}

// the shape limits of the matrix-core kernel (all epilogues)
static inline bool blur_mfma_shape_ok(int W, int C, int r, size_t elem) {
  if (C % 2 != 0 || C > 64 || r < 1 || r > kBlurMfmaMaxR) return false;
  // 16-byte output chunks: every band's row segment is a whole number of them
  if (((int64_t)W * C) % 4 != 0) return false;
  // 16-byte DMA pieces read whole dwords of the input rows
  if (((int64_t)W * C * (int64_t)elem) % 4 != 0) return false;
  return (int64_t)W * C * 4 < 0x7FFFFFF0ll;
}

// Fused blur + kEpiSample / kEpiAssign epilogue; MW_EUNSUPPORTED when the
// shape or the epilogue limits rule it out (the caller then materialises the
// blurred image and runs the standalone gather / assign kernels).
template <typename T>
int launch_blur_epi(const T* in, int H, int W, int C, const float* inv_mean, float p,
                    const BlurTaps& taps, int r, const BlurEpi& ep, int epi, hipStream_t st) {
  if (!blur_mfma_shape_ok(W, C, r, sizeof(T)) || inv_mean == nullptr) return MW_EUNSUPPORTED;
  if (epi != kEpiSample && epi != kEpiAssign) return MW_EUNSUPPORTED;
  switch (r) {
#define MW_R(N) case N: return launch_blur_epi_r<T, N>(in, H, W, C, inv_mean, p, taps, ep, epi, st);
    MW_R(1) MW_R(2) MW_R(3) MW_R(4) MW_R(5) MW_R(6) MW_R(7) MW_R(8)
#undef MW_R
    default: return MW_EUNSUPPORTED;
  }
}

// MFMA path for even C <= 64, 1 <= r <= 8, rows that fit 32-bit offsets;
// MW_EUNSUPPORTED otherwise (the caller tries the next path).
template <typename T>
int launch_blur_mfma(const T* in, int H, int W, int C, const float* inv_mean, float p,
                     const BlurTaps& taps, int r, float* out, hipStream_t st) {
  if (!blur_mfma_shape_ok(W, C, r, sizeof(T))) return MW_EUNSUPPORTED;
  if (const char* e = getenv("MW_BLUR_IMPL"))
    if (e[0] == 'v') return MW_EUNSUPPORTED;  // force the VALU kernel (A/B tests)
  switch (r) {
#define MW_R(N) case N: return launch_blur_mfma_r<T, N>(in, H, W, C, inv_mean, p, taps, out, st);
    MW_R(1) MW_R(2) MW_R(3) MW_R(4) MW_R(5) MW_R(6) MW_R(7) MW_R(8)
#undef MW_R
    default: return MW_EUNSUPPORTED;
  }
}

// Fast paths in order: matrix-core kernel, then the VALU register-ring kernel
// (blur.h); MW_EUNSUPPORTED sends the caller to the two-pass fallback.
template <typename T>
int launch_blur_fast(const T* in, int H, int W, int C, const float* inv_mean, float p,
                     const BlurTaps& taps, int r, float* out, hipStream_t st) {
  const int rc = launch_blur_mfma<T>(in, H, W, C, inv_mean, p, taps, r, out, st);
  if (rc != MW_EUNSUPPORTED) return rc;
  return launch_blur_valu<T>(in, H, W, C, inv_mean, p, taps, r, out, st);
}

}  // namespace mw
