// Host-side legacy NumPy MT19937 (MxIF.py:484,490):
//   np.random.seed(seed); np.random.choice(high, size)
// == RandomState(seed).randint(0, high, size) == masked rejection on the raw
// 32-bit MT19937 stream (numpy random_bounded_uint64_fill →
// buffered_bounded_masked_uint32 for 0 < high-1 < 2^32-1).
//
// Also the GF(2) machinery for the device generator's jump-ahead:
//   * the characteristic polynomial phi(t) of the MT19937 transition, found
//     by Berlekamp-Massey on 2*19937 bits of the recurrence sequence;
//   * jump polynomials h_j(t) = t^(L*2^j) mod phi(t) (squarings only);
//   * a reference host jump (Horner) used by the tests.
#include <stdint.h>
#include <string.h>

#include <vector>

#include "../../include/milwrm_amd.h"

namespace mw {
void set_error(const char* fmt, ...);

static const uint32_t kUpper = 0x80000000u, kLower = 0x7FFFFFFFu, kMatA = 0x9908B0DFu;

void mt_init_genrand(uint32_t seed, uint32_t* mt) {
  mt[0] = seed;
  for (int i = 1; i < 624; ++i) mt[i] = 1812433253u * (mt[i - 1] ^ (mt[i - 1] >> 30)) + (uint32_t)i;
}

// in-place regeneration: window x_k..x_{k+623} → x_{k+624}..x_{k+1247}
void mt_regen(uint32_t* mt) {
  int i = 0;
  for (; i < 624 - 397; ++i) {
    const uint32_t y = (mt[i] & kUpper) | (mt[i + 1] & kLower);
    mt[i] = mt[i + 397] ^ (y >> 1) ^ ((y & 1u) ? kMatA : 0u);
  }
  for (; i < 623; ++i) {
    const uint32_t y = (mt[i] & kUpper) | (mt[i + 1] & kLower);
    mt[i] = mt[i + 397 - 624] ^ (y >> 1) ^ ((y & 1u) ? kMatA : 0u);
  }
  const uint32_t y = (mt[623] & kUpper) | (mt[0] & kLower);
  mt[623] = mt[396] ^ (y >> 1) ^ ((y & 1u) ? kMatA : 0u);
}

static inline uint32_t temper(uint32_t y) {
  y ^= y >> 11;
  y ^= (y << 7) & 0x9D2C5680u;
  y ^= (y << 15) & 0xEFC60000u;
  y ^= y >> 18;
  return y;
}

// ---------------------------------------------------------------- GF(2)[t]
constexpr int kDeg = 19937;
constexpr int kWords = (kDeg + 63) / 64;  // 312

struct Poly {  // bit i = coefficient of t^i
  std::vector<uint64_t> w;
  explicit Poly(int nbits = kDeg + 1) : w((nbits + 63) / 64, 0) {}
  int bit(int i) const { return (int)((w[i >> 6] >> (i & 63)) & 1); }
  void flip(int i) { w[i >> 6] ^= 1ull << (i & 63); }
};

// XOR (src << sh) into dst (bit arrays)
static void xor_shifted(std::vector<uint64_t>& dst, const std::vector<uint64_t>& src, int sh) {
  const int ws = sh >> 6, bs = sh & 63;
  const int n = (int)src.size();
  for (int i = n - 1; i >= 0; --i) {
    const uint64_t v = src[i];
    if (!v) continue;
    const int d = i + ws;
    if (d < (int)dst.size()) dst[d] ^= v << bs;
    if (bs && d + 1 < (int)dst.size()) dst[d + 1] ^= v >> (64 - bs);
  }
}

static Poly g_phi;
static bool g_phi_ready = false;

static bool compute_phi() {
  if (g_phi_ready) return true;
  // sequence: top bit of x_k (k >= 624) from seed 5489
  const int N = 2 * kDeg + 64;
  std::vector<uint8_t> s(N);
  uint32_t mt[624];
  mt_init_genrand(5489u, mt);
  for (int k = 0; k < N;) {
    mt_regen(mt);
    for (int i = 0; i < 624 && k < N; ++i, ++k) s[k] = (uint8_t)(mt[i] >> 31);
  }
  // Berlekamp-Massey over GF(2); C(x) = 1 + c1 x + ... + cL x^L.  The
  // sequence is stored bit-reversed (bit N-1-k = s_k) so the discrepancy
  // window s_k, s_{k-1}, ..., s_{k-L} is the contiguous slice starting at bit
  // N-1-k: one AND + parity per 64 coefficients.
  const int NW = (N + 63) / 64 + 2;
  std::vector<uint64_t> SR(NW, 0);
  for (int k = 0; k < N; ++k)
    if (s[k]) SR[(N - 1 - k) >> 6] |= 1ull << ((N - 1 - k) & 63);
  std::vector<uint64_t> C(NW, 0), B(NW, 0), T;
  C[0] = 1;
  B[0] = 1;
  int L = 0, m = 1;
  for (int k = 0; k < N; ++k) {
    const int o = N - 1 - k, ow = o >> 6, ob = o & 63;
    uint64_t acc = 0;
    const int nw = (L >> 6) + 1;
    for (int w = 0; w < nw; ++w) {
      uint64_t v = SR[ow + w] >> ob;
      if (ob) v |= SR[ow + w + 1] << (64 - ob);
      acc ^= v & C[w];
    }
    // mask coefficients beyond L in the last word
    const int lb = L & 63;
    if (lb != 63) {
      uint64_t last;
      {
        uint64_t v = SR[ow + nw - 1] >> ob;
        if (ob) v |= SR[ow + nw] << (64 - ob);
        last = v & C[nw - 1];
      }
      acc ^= last & ~((2ull << lb) - 1);
    }
    int d = __builtin_popcountll(acc) & 1;
    if (!d) {
      ++m;
    } else if (2 * L <= k) {
      T = C;
      xor_shifted(C, B, m);
      L = k + 1 - L;
      B = T;
      m = 1;
    } else {
      xor_shifted(C, B, m);
      ++m;
    }
  }
  if (L != kDeg) return false;
  // phi(t) = t^L C(1/t): phi_i = c_{L-i}
  g_phi = Poly(kDeg + 1);
  for (int i = 0; i <= L; ++i)
    if ((C[(L - i) >> 6] >> ((L - i) & 63)) & 1) g_phi.flip(i);
  g_phi_ready = true;
  return true;
}

// r (up to 2*kDeg bits) mod phi → kDeg bits
static void reduce(std::vector<uint64_t>& r) {
  const int nbits = (int)r.size() * 64;
  for (int i = nbits - 1; i >= kDeg; --i)
    if ((r[i >> 6] >> (i & 63)) & 1) xor_shifted(r, g_phi.w, i - kDeg);
  r.resize(kWords);
  // clear bits >= kDeg in the last word
  r[kWords - 1] &= (kDeg % 64) ? ((1ull << (kDeg % 64)) - 1) : ~0ull;
}

static std::vector<uint64_t> sqr_mod(const std::vector<uint64_t>& a) {
  std::vector<uint64_t> r(2 * kWords + 1, 0);
  for (int i = 0; i < kWords; ++i) {
    uint64_t v = a[i];
    uint64_t lo = 0, hi = 0;
    for (int b = 0; b < 32; ++b) {
      lo |= ((v >> b) & 1ull) << (2 * b);
      hi |= ((v >> (b + 32)) & 1ull) << (2 * b);
    }
    r[2 * i] ^= lo;
    r[2 * i + 1] ^= hi;
  }
  reduce(r);
  return r;
}

static std::vector<uint64_t> mul_t_mod(const std::vector<uint64_t>& a) {
  std::vector<uint64_t> r(kWords + 1, 0);
  xor_shifted(r, a, 1);
  reduce(r);
  return r;
}

// t^e mod phi
static std::vector<uint64_t> pow_t(uint64_t e) {
  std::vector<uint64_t> r(kWords, 0);
  r[0] = 1;  // t^0
  int top = 63;
  while (top >= 0 && !((e >> top) & 1)) --top;
  for (int b = top; b >= 0; --b) {
    r = sqr_mod(r);
    if ((e >> b) & 1) r = mul_t_mod(r);
  }
  return r;
}

// host reference jump: state window (x_k..x_{k+623}) → window at k + J where
// J is encoded by poly (t^J mod phi).  Horner, one transition per coefficient.
void mt_jump_host(const uint32_t* in, const uint64_t* poly, uint32_t* out) {
  uint32_t acc[624];
  memset(acc, 0, sizeof(acc));
  int s = 0;  // acc window starts at ring index s
  uint32_t ring[624];
  memcpy(ring, acc, sizeof(acc));
  for (int i = kDeg - 1; i >= 0; --i) {
    // acc = A(acc): new word from the window, written over the oldest slot
    const uint32_t y = (ring[s] & kUpper) | (ring[(s + 1) % 624] & kLower);
    const uint32_t v = ring[(s + 397) % 624] ^ (y >> 1) ^ ((y & 1u) ? kMatA : 0u);
    ring[s] = v;
    s = (s + 1) % 624;
    if ((poly[i >> 6] >> (i & 63)) & 1)
      for (int j = 0; j < 624; ++j) ring[(s + j) % 624] ^= in[j];
  }
  for (int j = 0; j < 624; ++j) out[j] = ring[(s + j) % 624];
}

}  // namespace mw

extern "C" int mw_legacy_randint_host(uint32_t seed, int64_t high, int64_t size, int32_t* h_out) {
  if (!h_out || size < 0 || high < 1 || high > 2147483648LL) {
    mw::set_error("mw_legacy_randint_host: bad args (high=%lld size=%lld)", (long long)high,
                  (long long)size);
    return MW_EINVAL;
  }
  const uint64_t rng = (uint64_t)(high - 1);
  if (rng == 0) {
    memset(h_out, 0, sizeof(int32_t) * (size_t)size);
    return MW_OK;
  }
  uint64_t mask = rng;
  mask |= mask >> 1; mask |= mask >> 2; mask |= mask >> 4; mask |= mask >> 8; mask |= mask >> 16;
  uint32_t mt[624];
  mw::mt_init_genrand(seed, mt);
  int pos = 624;
  const uint32_t m32 = (uint32_t)mask, r32 = (uint32_t)rng;
  for (int64_t j = 0; j < size;) {
    if (pos >= 624) {
      mw::mt_regen(mt);
      pos = 0;
    }
    const uint32_t v = mw::temper(mt[pos++]) & m32;
    if (v <= r32) h_out[j++] = (int32_t)v;
  }
  return MW_OK;
}

extern "C" int mw_mt_jump_tables(int64_t L, int J, uint64_t* h_tables) {
  if (!h_tables || L <= 0 || J <= 0 || J > 48) {
    mw::set_error("mw_mt_jump_tables: bad args");
    return MW_EINVAL;
  }
  if (!mw::compute_phi()) {
    mw::set_error("mw_mt_jump_tables: Berlekamp-Massey did not find degree 19937");
    return MW_EHIP;
  }
  std::vector<uint64_t> h = mw::pow_t((uint64_t)L);
  for (int j = 0; j < J; ++j) {
    memcpy(h_tables + (size_t)j * mw::kWords, h.data(), sizeof(uint64_t) * mw::kWords);
    if (j + 1 < J) h = mw::sqr_mod(h);
  }
  return MW_OK;
}

extern "C" int mw_mt_jump_host(const uint32_t* h_state_in, const uint64_t* h_poly,
                               uint32_t* h_state_out) {
  if (!h_state_in || !h_poly || !h_state_out) {
    mw::set_error("mw_mt_jump_host: null pointer");
    return MW_EINVAL;
  }
  mw::mt_jump_host(h_state_in, h_poly, h_state_out);
  return MW_OK;
}

extern "C" int mw_mt_seed_state(uint32_t seed, uint32_t* h_state) {
  if (!h_state) return MW_EINVAL;
  mw::mt_init_genrand(seed, h_state);
  return MW_OK;
}
