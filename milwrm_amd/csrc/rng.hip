// Device MT19937 for img.subsample_pixels (MxIF.py:484,490):
//   np.random.seed(seed); np.random.choice(M, S)
// reproduced bit-exactly on the GPU with jump-ahead.
//
// The output stream is cut into W segments of L words (L a multiple of 624).
// Segment w starts at recurrence window V_{wL} = A^{wL} V_0 (V_0 =
// init_genrand(seed)); its words are temper(x_{624+wL+i}), i < L, i.e. the
// tempered entries of successive in-place regenerations of V_{wL}.
//   1. seed:   V_0 on device.
//   2. jumps:  parallel prefix, level j: V_{s+2^j} = h_j(A) V_s for s < 2^j,
//              h_j = t^{L 2^j} mod phi (host tables).  One workgroup per jump,
//              block Horner: acc = A^624(acc) xor P_q, P_q[j] = xor_r h_{624q+r}
//              x_{r+j} over the 1247-word extension of V_s.
//   3. gen:    every workgroup regenerates its segment 624 words at a time,
//              tempers, applies the masked rejection (v & mask <= high-1) and
//              compacts the accepted draws in order.
//   4. scan + scatter: segment counts → offsets; first `size` draws → out.
#include "common.h"

namespace mw {

constexpr int kN = 624, kM = 397, kPolyWords = 312, kDegMT = 19937;
constexpr uint32_t kUp = 0x80000000u, kLo = 0x7FFFFFFFu, kA = 0x9908B0DFu;
constexpr int kRngThreads = 640;  // >= 624, 10 waves

__device__ __forceinline__ uint32_t twist(uint32_t a, uint32_t b, uint32_t c) {
  const uint32_t y = (a & kUp) | (b & kLo);
  return c ^ (y >> 1) ^ ((y & 1u) ? kA : 0u);
}

// in-place regeneration of a 624-word LDS window (3 phases, read-then-write)
__device__ __forceinline__ void regen_lds(uint32_t* a) {
  const int i = threadIdx.x;
  uint32_t v = 0;
  if (i < 227) v = twist(a[i], a[i + 1], a[i + kM]);
  __syncthreads();
  if (i < 227) a[i] = v;
  __syncthreads();
  if (i >= 227 && i < 454) v = twist(a[i], a[i + 1], a[i + kM - kN]);
  __syncthreads();
  if (i >= 227 && i < 454) a[i] = v;
  __syncthreads();
  if (i >= 454 && i < kN) v = twist(a[i], a[(i + 1) % kN], a[i + kM - kN]);
  __syncthreads();
  if (i >= 454 && i < kN) a[i] = v;
  __syncthreads();
}

__device__ __forceinline__ uint32_t temper(uint32_t y) {
  y ^= y >> 11;
  y ^= (y << 7) & 0x9D2C5680u;
  y ^= (y << 15) & 0xEFC60000u;
  y ^= y >> 18;
  return y;
}

__global__ void mt_seed_kernel(uint32_t seed, uint32_t* __restrict__ st0) {
  if (threadIdx.x == 0) {
    uint32_t x = seed;
    st0[0] = x;
    for (int i = 1; i < kN; ++i) {
      x = 1812433253u * (x ^ (x >> 30)) + (uint32_t)i;
      st0[i] = x;
    }
  }
}

// one level of the parallel prefix: states[b + half] = h(A) states[b], b < n
__global__ void __launch_bounds__(kRngThreads) mt_jump_kernel(uint32_t* __restrict__ states, int half,
                                                              int n, const uint64_t* __restrict__ poly) {
  __shared__ uint32_t ext[2 * kN];  // x_0 .. x_1247 of the source window
  __shared__ uint32_t acc[kN];
  __shared__ uint64_t bits[kPolyWords + 2];
  const int b = blockIdx.x;
  if (b >= n) return;
  const int i = threadIdx.x;
  const uint32_t* src = states + (size_t)b * kN;
  uint32_t* dst = states + (size_t)(b + half) * kN;
  for (int q = i; q < kPolyWords; q += blockDim.x) bits[q] = poly[q];
  if (i < 2) bits[kPolyWords + i] = 0;
  if (i < kN) {
    ext[i] = src[i];
    ext[kN + i] = src[i];
    acc[i] = 0;
  }
  __syncthreads();
  regen_lds(ext + kN);  // ext[624..1247] = x_624 .. x_1247
  const int Q = (kDegMT - 1) / kN;  // 31
  __shared__ int s_list[kN];
  __shared__ int s_cnt;
  for (int q = Q; q >= 0; --q) {
    if (q < Q) regen_lds(acc);  // acc = A^624 acc
    // set-bit positions r of coefficients [624q, 624q+624) → LDS list (wave 0)
    if (i < 64) {
      int base = 0;
      const int c0 = q * kN;
      for (int r0 = 0; r0 < kN; r0 += 64) {
        const int c = c0 + r0;
        bool set = false;
        if (c + i < kDegMT && r0 + i < kN) set = (bits[(c + i) >> 6] >> ((c + i) & 63)) & 1ull;
        const unsigned long long m = __ballot(set);
        if (set) s_list[base + __popcll(m & ((1ull << i) - 1ull))] = r0 + i;
        base += __popcll(m);
      }
      if (i == 0) s_cnt = base;
    }
    __syncthreads();
    if (i < kN) {
      const int n = s_cnt;
      uint32_t p0 = 0, p1 = 0, p2 = 0, p3 = 0;
      int u = 0;
      for (; u + 8 <= n; u += 8) {  // 8 independent LDS reads in flight
        p0 ^= ext[s_list[u + 0] + i] ^ ext[s_list[u + 4] + i];
        p1 ^= ext[s_list[u + 1] + i] ^ ext[s_list[u + 5] + i];
        p2 ^= ext[s_list[u + 2] + i] ^ ext[s_list[u + 6] + i];
        p3 ^= ext[s_list[u + 3] + i] ^ ext[s_list[u + 7] + i];
      }
      for (; u < n; ++u) p0 ^= ext[s_list[u] + i];
      acc[i] ^= (p0 ^ p1) ^ (p2 ^ p3);
    }
    __syncthreads();
  }
  if (i < kN) dst[i] = acc[i];
}

// in-place regeneration of a 624-word LDS window by one wave (no workgroup
// barriers): each phase reads all its old words, then writes; a wave's LDS
// operations complete in order, and the wavefront fence keeps the compiler
// from moving a lane's store above another lane's load of the same word
__device__ __forceinline__ void wave_fence() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}
template <int LO, int HI, int OFF2>
__device__ __forceinline__ void regen_phase(uint32_t* a, int lane) {
  constexpr int R = (HI - LO + 63) / 64;
  uint32_t v[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int i = LO + r * 64 + lane;
    if (i < HI) v[r] = twist(a[i], a[i + 1 < kN ? i + 1 : 0], a[i + OFF2]);
  }
  wave_fence();
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int i = LO + r * 64 + lane;
    if (i < HI) a[i] = v[r];
  }
  wave_fence();
}
__device__ __forceinline__ void regen_wave(uint32_t* a, int lane) {
  regen_phase<0, 227, kM>(a, lane);
  regen_phase<227, 454, kM - kN>(a, lane);
  regen_phase<454, kN, kM - kN>(a, lane);
}

// per segment (one wave each): regenerate L words, temper, masked rejection,
// ordered compaction (word 64 r + lane: ballot per r, in word order).  One
// wave per segment: the former 10-wave workgroup spent 8 workgroup barriers
// per 624 words (mt_gen 0.61 ms per config-2 draw -> 0.35 ms, mt_scatter 0.22
// -> 0.18 ms with the 624 x 32-word segments).  Staging the compacted words in
// an LDS ring for aligned 256-B stores measured slower (0.50 ms), and the
// segment length does not matter between 624 x 8 and x 32 (0.34 / 0.35 ms)
__global__ void __launch_bounds__(64) mt_gen_kernel(const uint32_t* __restrict__ states,
                                                    int64_t L, uint32_t mask, uint32_t rng,
                                                    uint32_t* __restrict__ tmp,
                                                    int64_t* __restrict__ cnt) {
  __shared__ uint32_t a[kN];
  const int w = blockIdx.x, lane = threadIdx.x;
  for (int i = lane; i < kN; i += 64) a[i] = states[(size_t)w * kN + i];
  wave_fence();
  uint32_t* out = tmp + (size_t)w * L;
  int64_t count = 0;
  const int64_t nblk = L / kN;
  for (int64_t blk = 0; blk < nblk; ++blk) {
    regen_wave(a, lane);
#pragma unroll
    for (int r = 0; r < (kN + 63) / 64; ++r) {
      const int i = r * 64 + lane;
      uint32_t v = 0;
      bool ok = false;
      if (i < kN) {
        v = temper(a[i]) & mask;
        ok = v <= rng;
      }
      const unsigned long long m = __ballot(ok);
      if (ok) out[count + __popcll(m & ((1ull << lane) - 1ull))] = v;
      count += __popcll(m);
    }
    wave_fence();  // the next regeneration's stores after this pass's loads
  }
  if (lane == 0) cnt[w] = count;
}

__global__ void __launch_bounds__(1024) mt_scan_kernel(int64_t* __restrict__ cnt, int W,
                                                       int64_t* __restrict__ total) {
  __shared__ long long s[1024];
  const int t = threadIdx.x;
  const int per = (W + 1023) / 1024;
  const int lo = t * per, hi = min(W, lo + per);
  long long loc = 0;
  for (int i = lo; i < hi; ++i) loc += cnt[i];
  s[t] = loc;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {
    const long long v = t >= o ? s[t - o] : 0;
    __syncthreads();
    s[t] += v;
    __syncthreads();
  }
  long long run = s[t] - loc;
  for (int i = lo; i < hi; ++i) {
    const long long c = cnt[i];
    cnt[i] = run;  // exclusive offset
    run += c;
  }
  if (t == 1023) *total = s[1023];
}

__global__ void mt_scatter_kernel(const uint32_t* __restrict__ tmp, const int64_t* __restrict__ off,
                                  const int64_t* __restrict__ total, int W, int64_t L, int64_t size,
                                  int32_t* __restrict__ out) {
  const int w = blockIdx.y;
  const int64_t o = off[w];
  const int64_t n = (w + 1 < W ? off[w + 1] : *total) - o;
  const uint32_t* src = tmp + (size_t)w * L;
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < n; q += (int64_t)gridDim.x * blockDim.x) {
    const int64_t d = o + q;
    if (d < size) out[d] = (int32_t)src[q];
  }
}

struct RngPlan {
  int64_t W;
  uint32_t mask, rng;
};
static RngPlan rng_plan(int64_t high, int64_t size, int64_t L) {
  RngPlan p;
  const uint64_t r = (uint64_t)(high - 1);
  uint64_t m = r;
  m |= m >> 1; m |= m >> 2; m |= m >> 4; m |= m >> 8; m |= m >> 16;
  p.mask = (uint32_t)m;
  p.rng = (uint32_t)r;
  const double acc = (double)(r + 1) / (double)(m + 1);  // acceptance probability
  const double mean = (double)size / acc;
  const double D = mean * 1.001 + 16.0 * sqrt(mean / acc) + 2.0 * L;
  p.W = (int64_t)((D + L - 1) / L);
  if (p.W < 1) p.W = 1;
  return p;
}

}  // namespace mw

using namespace mw;

extern "C" {

size_t mw_legacy_randint_ws_bytes(int64_t high, int64_t size, int64_t L) {
  if (high < 2 || size <= 0 || L <= 0) return 256;
  const RngPlan p = rng_plan(high, size, L);
  return (size_t)p.W * kN * 4 + (size_t)p.W * L * 4 + (size_t)(p.W + 1) * 8 + 1024;
}

int64_t mw_legacy_randint_segments(int64_t high, int64_t size, int64_t L) {
  if (high < 2 || size <= 0 || L <= 0) return 0;
  return rng_plan(high, size, L).W;
}

size_t mw_legacy_randint_gen_ws_bytes(int64_t high, int64_t size, int64_t L) {
  if (high < 2 || size <= 0 || L <= 0) return 256;
  const RngPlan p = rng_plan(high, size, L);
  return (size_t)p.W * L * 4 + (size_t)(p.W + 1) * 8 + 1024;
}

int mw_mt_segment_states(uint32_t seed, int64_t W, const uint64_t* d_tables, int J,
                         uint32_t* d_states, void* stream) {
  MW_CHECK_ARG(d_states && d_tables, "mw_mt_segment_states: null pointer");
  MW_CHECK_ARG(W >= 1 && W <= 1024 * 1024, "mw_mt_segment_states: bad segment count %lld",
               (long long)W);
  int levels = 0;
  while ((1ll << levels) < W) ++levels;
  MW_CHECK_ARG(levels <= J, "mw_mt_segment_states: %lld segments need %d jump levels, tables have %d",
               (long long)W, levels, J);
  hipStream_t st = as_stream(stream);
  hipLaunchKernelGGL(mt_seed_kernel, dim3(1), dim3(64), 0, st, seed, d_states);
  MW_LAUNCH_CHECK();
  for (int j = 0; j < levels; ++j) {
    const int64_t half = 1ll << j;
    const int64_t n = std::min<int64_t>(half, W - half);
    if (n <= 0) break;
    hipLaunchKernelGGL(mt_jump_kernel, dim3((unsigned)n), dim3(kRngThreads), 0, st, d_states,
                       (int)half, (int)n, d_tables + (size_t)j * kPolyWords);
    MW_LAUNCH_CHECK();
  }
  return MW_OK;
}

// generation half: regenerate / temper / filter each segment from its start
// state, scan the per-segment counts, scatter the first `size` draws
static int randint_gen(const uint32_t* states, const RngPlan& p, int64_t size, int64_t L,
                       int32_t* d_out, int64_t* d_total, uint32_t* tmp, int64_t* cnt,
                       hipStream_t st) {
  hipLaunchKernelGGL(mt_gen_kernel, dim3((unsigned)p.W), dim3(64), 0, st, states, L, p.mask,
                     p.rng, tmp, cnt);
  MW_LAUNCH_CHECK();
  MW_CHECK_ARG(p.W <= 1024 * 1024, "mw_legacy_randint: too many segments");
  hipLaunchKernelGGL(mt_scan_kernel, dim3(1), dim3(1024), 0, st, cnt, (int)p.W, d_total);
  MW_LAUNCH_CHECK();
  const unsigned gx = (unsigned)std::max<int64_t>(1, std::min<int64_t>((L + 8191) / 8192, 64));
  hipLaunchKernelGGL(mt_scatter_kernel, dim3(gx, (unsigned)p.W), dim3(256), 0, st, tmp, cnt,
                     d_total, (int)p.W, L, size, d_out);
  MW_LAUNCH_CHECK();
  return MW_OK;
}

// numpy's special cases: size 0 draws nothing, high 1 returns zeros
static int randint_trivial(int64_t high, int64_t size, int32_t* d_out, int64_t* d_total,
                           hipStream_t st, bool* done) {
  *done = true;
  if (size == 0) {
    MW_HIP(hipMemsetAsync(d_total, 0, sizeof(int64_t), st));
    return MW_OK;
  }
  if (high == 1) {
    MW_HIP(hipMemsetAsync(d_out, 0, sizeof(int32_t) * (size_t)size, st));
    const int64_t s = size;
    MW_HIP(hipMemcpyAsync(d_total, &s, sizeof(int64_t), hipMemcpyHostToDevice, st));
    MW_HIP(hipStreamSynchronize(st));
    return MW_OK;
  }
  *done = false;
  return MW_OK;
}

int mw_legacy_randint_from_states(const uint32_t* d_states, int64_t W_avail, int64_t high,
                                  int64_t size, int64_t L, int32_t* d_out, int64_t* d_total,
                                  void* d_ws, void* stream) {
  MW_CHECK_ARG(d_out && d_total && d_ws, "mw_legacy_randint_from_states: null pointer");
  MW_CHECK_ARG(high >= 1 && high <= 2147483648LL && size >= 0, "mw_legacy_randint_from_states: bad range");
  MW_CHECK_ARG(L > 0 && L % kN == 0, "mw_legacy_randint_from_states: L must be a positive multiple of 624");
  hipStream_t st = as_stream(stream);
  bool done;
  const int rc = randint_trivial(high, size, d_out, d_total, st, &done);
  if (done) return rc;
  const RngPlan p = rng_plan(high, size, L);
  MW_CHECK_ARG(d_states && W_avail >= p.W,
               "mw_legacy_randint_from_states: %lld segment states needed, %lld given",
               (long long)p.W, (long long)W_avail);
  uint32_t* tmp = reinterpret_cast<uint32_t*>(d_ws);
  int64_t* cnt = reinterpret_cast<int64_t*>(tmp + (size_t)p.W * L);
  return randint_gen(d_states, p, size, L, d_out, d_total, tmp, cnt, st);
}

int mw_legacy_randint_device(uint32_t seed, int64_t high, int64_t size, const uint64_t* d_tables,
                             int J, int64_t L, int32_t* d_out, int64_t* d_total, void* d_ws,
                             void* stream) {
  MW_CHECK_ARG(d_out && d_total && d_ws, "mw_legacy_randint_device: null pointer");
  MW_CHECK_ARG(high >= 1 && high <= 2147483648LL && size >= 0, "mw_legacy_randint_device: bad range");
  MW_CHECK_ARG(L > 0 && L % kN == 0, "mw_legacy_randint_device: L must be a positive multiple of 624");
  hipStream_t st = as_stream(stream);
  bool done;
  const int rc0 = randint_trivial(high, size, d_out, d_total, st, &done);
  if (done) return rc0;
  MW_CHECK_ARG(d_tables != nullptr, "mw_legacy_randint_device: jump tables required");
  const RngPlan p = rng_plan(high, size, L);
  char* base = reinterpret_cast<char*>(d_ws);
  uint32_t* states = reinterpret_cast<uint32_t*>(base);
  uint32_t* tmp = states + (size_t)p.W * kN;
  int64_t* cnt = reinterpret_cast<int64_t*>(tmp + (size_t)p.W * L);
  const int rc = mw_mt_segment_states(seed, p.W, d_tables, J, states, stream);
  if (rc != MW_OK) return rc;
  return randint_gen(states, p, size, L, d_out, d_total, tmp, cnt, st);
}

}  // extern "C"
