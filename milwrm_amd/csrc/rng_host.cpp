// Host-side legacy NumPy MT19937 index generation (MxIF.py:484,490):
//   np.random.seed(seed); np.random.choice(high, size)
// == RandomState(seed).randint(0, high, size) == masked rejection on the raw
// 32-bit MT19937 stream (numpy random_bounded_uint64_fill →
// buffered_bounded_masked_uint32 for 0 < high-1 < 2^32-1).
#include <stdint.h>
#include <string.h>

#include "../../include/milwrm_amd.h"

namespace mw {
void set_error(const char* fmt, ...);

struct MT19937 {
  uint32_t mt[624];
  int pos;
  explicit MT19937(uint32_t seed) {  // init_genrand
    mt[0] = seed;
    for (int i = 1; i < 624; ++i) mt[i] = 1812433253u * (mt[i - 1] ^ (mt[i - 1] >> 30)) + (uint32_t)i;
    pos = 624;
  }
  void regen() {
    static const uint32_t mag[2] = {0u, 0x9908B0DFu};
    int i = 0;
    for (; i < 624 - 397; ++i) {
      const uint32_t y = (mt[i] & 0x80000000u) | (mt[i + 1] & 0x7FFFFFFFu);
      mt[i] = mt[i + 397] ^ (y >> 1) ^ mag[y & 1u];
    }
    for (; i < 623; ++i) {
      const uint32_t y = (mt[i] & 0x80000000u) | (mt[i + 1] & 0x7FFFFFFFu);
      mt[i] = mt[i + 397 - 624] ^ (y >> 1) ^ mag[y & 1u];
    }
    const uint32_t y = (mt[623] & 0x80000000u) | (mt[0] & 0x7FFFFFFFu);
    mt[623] = mt[396] ^ (y >> 1) ^ mag[y & 1u];
    pos = 0;
  }
  inline uint32_t next() {
    if (pos >= 624) regen();
    uint32_t y = mt[pos++];
    y ^= y >> 11;
    y ^= (y << 7) & 0x9D2C5680u;
    y ^= (y << 15) & 0xEFC60000u;
    y ^= y >> 18;
    return y;
  }
};
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
  mw::MT19937 g(seed);
  const uint32_t m32 = (uint32_t)mask, r32 = (uint32_t)rng;
  for (int64_t j = 0; j < size;) {
    const uint32_t v = g.next() & m32;
    if (v <= r32) h_out[j++] = (int32_t)v;
  }
  return MW_OK;
}
