// Host-side expansion of the label pass's compact outputs into the arrays the
// reference hands back (MILWRM.py:275-276: tissue_IDs[i] = labels as float64
// with NaN outside the mask; MILWRM.py:444-445: confidence_IDs[i] float64
// with NaN outside the mask).  The device keeps int8 labels (-1 = no domain)
// and fp32 confidences (NaN outside the mask); after one D2H copy of those
// (5 bytes per pixel) these loops write the 8-byte host values on several
// threads, so the output pages are also first touched in parallel.
#include <stdint.h>

#include <algorithm>
#include <cmath>
#include <thread>
#include <vector>

#include "../../include/milwrm_amd.h"

namespace mw {
void set_error(const char* fmt, ...);

template <typename F>
static void host_parallel(int64_t n, int threads, F&& body) {
  const int64_t kMinChunk = 1 << 20;
  int nt = std::max(1, std::min<int>(threads, (int)((n + kMinChunk - 1) / kMinChunk)));
  if (nt == 1) {
    body((int64_t)0, n);
    return;
  }
  std::vector<std::thread> pool;
  pool.reserve(nt);
  const int64_t step = (n + nt - 1) / nt;
  for (int i = 0; i < nt; ++i) {
    const int64_t a = std::min(n, i * step), b = std::min(n, a + step);
    pool.emplace_back([&body, a, b] { body(a, b); });
  }
  for (auto& t : pool) t.join();
}
}  // namespace mw

extern "C" int mw_host_labels_f64(const int8_t* h_lab, int64_t n, double* h_out, int threads) {
  if (n < 0 || (n > 0 && (!h_lab || !h_out))) {
    mw::set_error("mw_host_labels_f64: bad arguments");
    return MW_EINVAL;
  }
  const double nan = std::nan("");
  mw::host_parallel(n, threads, [&](int64_t a, int64_t b) {
    for (int64_t i = a; i < b; ++i) {
      const int8_t v = h_lab[i];
      h_out[i] = v < 0 ? nan : (double)v;
    }
  });
  return MW_OK;
}

extern "C" int mw_host_f32_to_f64(const float* h_in, int64_t n, double* h_out, int threads) {
  if (n < 0 || (n > 0 && (!h_in || !h_out))) {
    mw::set_error("mw_host_f32_to_f64: bad arguments");
    return MW_EINVAL;
  }
  mw::host_parallel(n, threads, [&](int64_t a, int64_t b) {
    for (int64_t i = a; i < b; ++i) h_out[i] = (double)h_in[i];
  });
  return MW_OK;
}
