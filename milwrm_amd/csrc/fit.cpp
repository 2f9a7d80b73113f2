// mw_kmeans_fit: sklearn KMeans(algorithm="lloyd").fit as one C entry
// (sklearn _kmeans.py:1427-1554; MILWRM calls it at MILWRM.py:706-737 and,
// per k, in kMeansRes MILWRM.py:29-54), for callers that bind the C ABI
// rather than the Python package.  The host control flow is the one of
// milwrm_amd/kmeans.py (KMeans.fit -> _kmeans_plusplus_device -> lloyd_fits
// with one fit), step for step and with the same fp64 expressions, so both
// front ends return bitwise the same centers, labels, inertia and n_iter:
//   * tolerance: tol * mean(var of the scaled rows)      (_kmeans.py:279-287)
//   * k-means++ from RandomState(seed): the choice draw, then n_local_trials
//     = 2 + int(ln k) uniforms per step                 (_kmeans.py:174-272)
//   * Lloyd: mw_lloyd_pass per iteration (exact fixed-point sums), strict
//     convergence on zero changed labels, else the center-shift test;
//     empty-cluster relocation and averaging   (_k_means_common.pyx:181-311)
//   * the extra E-step when not strictly converged, and the inertia.
// numpy's reductions used by the Python side (pairwise sums) are restated
// (np_sum) so the host arithmetic matches it bit for bit.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstring>
#include <limits>
#include <vector>

#include "common.h"

#pragma clang fp contract(off)

namespace mw {
void mt_init_genrand(uint32_t seed, uint32_t* mt);
void mt_regen(uint32_t* mt);

namespace {

// numpy RandomState(seed) (MT19937, init_genrand) -> random_sample()
struct LegacyRandom {
  uint32_t mt[624];
  int pos = 624;
  explicit LegacyRandom(uint32_t seed) { mt_init_genrand(seed, mt); }
  uint32_t next() {
    if (pos >= 624) { mt_regen(mt); pos = 0; }
    uint32_t y = mt[pos++];
    y ^= y >> 11;
    y ^= (y << 7) & 0x9D2C5680u;
    y ^= (y << 15) & 0xEFC60000u;
    y ^= y >> 18;
    return y;
  }
  double sample() {  // genrand_res53
    const uint32_t a = next() >> 5, b = next() >> 6;
    return (a * 67108864.0 + b) / 9007199254740992.0;
  }
};

// numpy's pairwise_sum of a contiguous double run (n <= 128: eight partial
// sums, combined as ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)), then the tail)
double np_sum(const double* a, int64_t n) {
  if (n < 8) {
    double r = 0.0;  // numpy: -0.0 start only for n == 0 paths we never take
    for (int64_t i = 0; i < n; ++i) r += a[i];
    return r;
  }
  if (n <= 128) {
    double r[8];
    for (int j = 0; j < 8; ++j) r[j] = a[j];
    int64_t i = 8;
    for (; i < n - (n % 8); i += 8)
      for (int j = 0; j < 8; ++j) r[j] += a[i + j];
    double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < n; ++i) res += a[i];
    return res;
  }
  int64_t n2 = n / 2;
  n2 -= n2 % 8;
  return np_sum(a, n2) + np_sum(a + n2, n - n2);
}

// RandomState.choice(n, p=ones(n)/n) given its uniform draw u: cdf = the
// sequential cumsum of c = 1/n, normalised by its last entry, searchsorted
// 'right'.  Inside a binade the running sum advances by a constant increment
// (after one explicit step that fixes the rounding parity), so the sum is
// evaluated run by run (rng.py _runs / _s_at, the same fp64 operations).
struct CdfRun {
  int64_t i0;
  double s0, inc;
  int64_t m;
};
static std::vector<CdfRun> cdf_runs(int64_t n) {
  std::vector<CdfRun> runs;
  const double c = 1.0 / (double)n;
  int64_t i = 0;
  double s = c;
  while (i < n) {
    runs.push_back({i, s, 0.0, 1});
    i += 1;
    if (i >= n) break;
    const double t = s + c;
    const double u = t + c;
    const double inc = u - t;
    int m_exp;
    std::frexp(t, &m_exp);
    const double top = std::ldexp(1.0, m_exp);
    int64_t m;
    if (inc > 0) {
      int64_t j = (int64_t)((top - t) / inc);
      while (j > 0 && t + (double)j * inc >= top) --j;
      while (t + (double)(j + 1) * inc < top) ++j;
      m = std::min(j + 1, n - i);
    } else {
      m = n - i;
    }
    runs.push_back({i, t, inc, m});
    i += m;
    s = (t + (double)(m - 1) * inc) + c;
  }
  return runs;
}
int64_t first_center_index(int64_t n, double u) {
  const std::vector<CdfRun> runs = cdf_runs(n);
  const CdfRun& last = runs.back();
  const double total = last.s0 + (double)(last.m - 1) * last.inc;
  for (const CdfRun& r : runs) {
    if ((r.s0 + (double)(r.m - 1) * r.inc) / total > u) {
      int64_t lo = 0, hi = r.m - 1;  // first j with s_j / total > u
      while (lo < hi) {
        const int64_t mid = (lo + hi) / 2;
        if ((r.s0 + (double)mid * r.inc) / total > u) hi = mid;
        else lo = mid + 1;
      }
      return r.i0 + lo;
    }
  }
  return n;
}

int exp_below(double bound) {  // e with bound * 2^e <= 2^40 (0 for 0)
  if (!std::isfinite(bound) || bound <= 0.0) return 0;
  int e;
  std::frexp(bound, &e);
  return 40 - e;
}

float round_f32(double x, bool up) {
  float f = (float)x;
  if (up && (double)f < x) f = std::nextafter(f, std::numeric_limits<float>::infinity());
  if (!up && (double)f > x) f = std::nextafter(f, -std::numeric_limits<float>::infinity());
  return f;
}

struct DevBuf {
  void* p = nullptr;
  ~DevBuf() { if (p) (void)hipFree(p); }
};

#define MW_TRY(call)                 \
  do {                               \
    const int rc_ = (call);          \
    if (rc_ != MW_OK) return rc_;    \
  } while (0)

template <typename T>
int dev_alloc(DevBuf& b, size_t n) {
  MW_HIP(hipMalloc(&b.p, std::max<size_t>(n * sizeof(T), 256)));
  return MW_OK;
}

// Page-locked staging for the driver's small transfers (one per thread,
// grown on demand, never freed): copies from pageable std::vectors are staged
// by the runtime synchronously, ~20 us of host time each, while the GPU waits
// for the next launch.  Regions: [0, 32K) center tables (H2D), [32K, 160K)
// pass records (D2H), [160K, 176K) gathered rows (D2H), [176K, 178K) setup
// arrays (H2D).  Every region is reused only after a stream synchronisation
// that follows its previous copy.
constexpr size_t kPinTab = 0, kPinRec = 32 << 10, kPinRows = 160 << 10, kPinSetup = 176 << 10,
                 kPinIdx = 178 << 10, kPinBytes = 180 << 10;
// A fit that returns before its last copies ran (mw_kmeans_fit_async)
// records this event after them: the next user of the staging waits for it.
static thread_local hipEvent_t pin_busy = nullptr;
static char* pinned_staging() {
  static thread_local char* p = nullptr;
  if (!p && hipHostMalloc(reinterpret_cast<void**>(&p), kPinBytes, 0) != hipSuccess) p = nullptr;
  if (pin_busy) {
    (void)hipEventSynchronize(pin_busy);
    (void)hipEventDestroy(pin_busy);
    pin_busy = nullptr;
  }
  return p;
}

// rows X[idx[i]] (idx[0] replaced by `first` when first >= 0) -> out, n x F
__global__ void rows_gather_kernel(const float* __restrict__ X, int F, const int64_t* __restrict__ idx,
                                   int64_t first, int n, float* __restrict__ out) {
  const int i = blockIdx.x, f = threadIdx.x;
  if (i < n && f < F) {
    const int64_t r = (i == 0 && first >= 0) ? first : idx[i];
    out[(size_t)i * F + f] = X[r * F + f];
  }
}

struct Fit {
  int64_t S;
  int F, k;
  hipStream_t st;
  const float* X;
  float *a32, *b32, *par;
  int32_t* qexp;
  uint8_t* labels;
  float *ub, *lb;
  void* ws;
  double* out;
  int rl;
  std::vector<double> a64, b64;
  std::vector<float> prev32;
  bool have_prev = false;
  float drift_max = 0.f, prev_dmax = 0.f;

  // centers / drift / half-separation tables of the next pass (kmeans.py
  // _bound_tables; the values only steer which rows skip the E-step)
  std::vector<float> h;  // staging of the uploaded tables (outlives the async copy)
  int upload(const std::vector<double>& c) {
    h.assign((size_t)k * F + 2 * k, 0.f);
    for (size_t i = 0; i < (size_t)k * F; ++i) h[i] = (float)c[i];
    std::vector<double> drift(k, 0.0), half(k, std::numeric_limits<double>::infinity()), tmp(F);
    for (int j = 0; j < k; ++j) {
      if (have_prev) {
        for (int f = 0; f < F; ++f) {
          const double d = (double)h[(size_t)j * F + f] - (double)prev32[(size_t)j * F + f];
          tmp[f] = d * d;
        }
        drift[j] = std::sqrt(np_sum(tmp.data(), F));
      }
      if (k > 1) {
        double m = std::numeric_limits<double>::infinity();
        for (int i = 0; i < k; ++i) {
          if (i == j) continue;
          for (int f = 0; f < F; ++f) {
            const double d = (double)h[(size_t)j * F + f] - (double)h[(size_t)i * F + f];
            tmp[f] = d * d;
          }
          m = std::min(m, np_sum(tmp.data(), F));
        }
        half[j] = 0.5 * std::sqrt(m);
      }
    }
    float dmax = 0.f;
    for (int j = 0; j < k; ++j) {
      const float d32 = round_f32(drift[j], true);
      h[(size_t)k * F + j] = d32;
      dmax = j == 0 ? d32 : std::max(dmax, d32);
      h[(size_t)k * F + k + j] = round_f32(half[j], false);
    }
    prev_dmax = have_prev ? drift_max : 0.f;
    drift_max = dmax;
    prev32.assign(h.begin(), h.begin() + (size_t)k * F);
    have_prev = true;
    char* pin = pinned_staging();
    if (pin && h.size() * sizeof(float) <= kPinRec - kPinTab) {
      std::memcpy(pin + kPinTab, h.data(), h.size() * sizeof(float));
      MW_HIP(hipMemcpyAsync(par, pin + kPinTab, h.size() * sizeof(float), hipMemcpyHostToDevice, st));
    } else {
      MW_HIP(hipMemcpyAsync(par, h.data(), h.size() * sizeof(float), hipMemcpyHostToDevice, st));
    }
    return MW_OK;
  }

  // fold_rec: the first pass of a k-means++ fold (kind 8): the record is the
  // list pass's moves plus the fold pass's base sums (out + rl), with the fold
  // record's counters (every row changed from unlabelled and was computed)
  int pass(int mode, int kind, int iexp, std::vector<double>& rec, bool fold_rec = false) {
    mw_lloyd_fit f{};
    f.centers = par;
    f.drift = par + (size_t)k * F;
    f.half_sep = par + (size_t)k * F + k;
    f.labels = labels;
    f.ub = ub;
    f.lb = lb;
    f.ws = ws;
    f.out = out;
    f.k = k;
    f.drift_max = drift_max;
    f.inertia_exp = iexp;
    MW_TRY(mw_lloyd_pass(X, S, F, a32, b32, qexp, 1, &f, mode, kind, st));
    const int nr = fold_rec ? 2 * rl : rl;
    rec.resize(nr);
    char* pin = pinned_staging();
    if (pin && (size_t)nr * sizeof(double) <= kPinRows - kPinRec) {
      MW_HIP(hipMemcpyAsync(pin + kPinRec, out, nr * sizeof(double), hipMemcpyDeviceToHost, st));
      MW_HIP(hipStreamSynchronize(st));
      std::memcpy(rec.data(), pin + kPinRec, nr * sizeof(double));
    } else {
      MW_HIP(hipMemcpyAsync(rec.data(), out, nr * sizeof(double), hipMemcpyDeviceToHost, st));
      MW_HIP(hipStreamSynchronize(st));
    }
    if (fold_rec) {  // integer-valued limbs and counts: exact fp64 sums
      const int ns = 2 * k * F + k;
      for (int i = 0; i < ns; ++i) rec[i] += rec[rl + i];
      for (int i = ns; i < rl; ++i) rec[i] = rec[rl + i];
      rec.resize(rl);
    }
    return MW_OK;
  }

  // pass() without the download's wait: the record goes to the caller's
  // page-locked h_rec when the stream gets there
  int pass_async(int mode, int kind, int iexp, double* h_rec) {
    mw_lloyd_fit f{};
    f.centers = par;
    f.drift = par + (size_t)k * F;
    f.half_sep = par + (size_t)k * F + k;
    f.labels = labels;
    f.ub = ub;
    f.lb = lb;
    f.ws = ws;
    f.out = out;
    f.k = k;
    f.drift_max = drift_max;
    f.inertia_exp = iexp;
    MW_TRY(mw_lloyd_pass(X, S, F, a32, b32, qexp, 1, &f, mode, kind, st));
    MW_HIP(hipMemcpyAsync(h_rec, out, rl * sizeof(double), hipMemcpyDeviceToHost, st));
    return MW_OK;
  }

  // the same for indices on the device (idx[0] = first when first >= 0): one
  // gather kernel into `tmp` (n x F floats of device scratch) and one copy
  int scaled_rows_dev(const int64_t* d_idx, int64_t first, int n, const double* mu, const double* inv,
                      float* tmp, std::vector<double>& outv, int64_t* h_idx = nullptr) {
    char* pin = pinned_staging();
    const size_t nb = (size_t)n * F * sizeof(float);
    if (!pin || nb > kPinSetup - kPinRows || n > 64) return -1;
    hipLaunchKernelGGL(rows_gather_kernel, dim3(n), dim3(64), 0, st, X, F, d_idx, first, n, tmp);
    MW_HIP(hipGetLastError());
    MW_HIP(hipMemcpyAsync(pin + kPinRows, tmp, nb, hipMemcpyDeviceToHost, st));
    if (h_idx) MW_HIP(hipMemcpyAsync(pin + kPinIdx, d_idx, (size_t)n * 8, hipMemcpyDeviceToHost, st));
    MW_HIP(hipStreamSynchronize(st));
    if (h_idx) {
      std::memcpy(h_idx, pin + kPinIdx, (size_t)n * 8);
      if (first >= 0) h_idx[0] = first;
    }
    const float* r = reinterpret_cast<const float*>(pin + kPinRows);
    outv.resize((size_t)n * F);
    for (int i = 0; i < n; ++i)
      for (int f = 0; f < F; ++f)
        outv[(size_t)i * F + f] = ((double)r[(size_t)i * F + f] - mu[f]) * inv[f];
    return MW_OK;
  }

  // raw rows idx[i] -> scaled fp64 (x - mu) * inv
  int scaled_rows(const int64_t* idx, int n, const double* mu, const double* inv,
                  std::vector<double>& outv) {
    std::vector<float> r((size_t)n * F);
    outv.resize((size_t)n * F);
    for (int i = 0; i < n; ++i)
      MW_HIP(hipMemcpyAsync(r.data() + (size_t)i * F, X + idx[i] * F, F * sizeof(float),
                            hipMemcpyDeviceToHost, st));
    MW_HIP(hipStreamSynchronize(st));
    for (int i = 0; i < n; ++i)
      for (int f = 0; f < F; ++f)
        outv[(size_t)i * F + f] = ((double)r[(size_t)i * F + f] - mu[f]) * inv[f];
    return MW_OK;
  }
};

// Workspace (256-aligned sections): small arrays | par | ub | lb | Lloyd
// records | out | one region shared by the column statistics (tolerance),
// the k-means++ state and the relocation scratch (never live together).
struct FitLayout {
  size_t small, par, ub, lb, lws, out, big, fold, total;
};
static inline size_t fal(size_t x) { return (x + 255) & ~(size_t)255; }
static int lloyd_queue_kind() {  // MW_LLOYD_LIST=0: one-kernel kQueue (A/B)
  static const int q = [] {
    const char* e = getenv("MW_LLOYD_LIST");
    return (e && e[0] == '0') ? 2 : 4;  // as kmeans.QUEUE_KIND
  }();
  return q;
}
static FitLayout fit_layout(int64_t S, int F, int k) {
  const int T = 2 + (int)std::log((double)(k < 1 ? 1 : k));
  FitLayout L;
  L.small = 0;
  L.par = fal(64 * 4 * 4 + 64 * 8 * 2 + 64 * 64 * 8 + 64 * 8 * 2 + 130 * 8 + 64 * 8);
  L.ub = L.par + fal(((size_t)k * F + 2 * k) * 4);
  L.lb = L.ub + fal((size_t)S * 4);
  L.lws = L.lb + fal((size_t)S * 4);
  // the records of a k-means++ fold pass (kpp grid) share the Lloyd records' region
  L.out = L.lws + fal(std::max(mw_lloyd_ws_bytes_kinds(S, k, F, lloyd_queue_kind() == 4),
                               mw_kpp_fold_rec_bytes(S, k, F)));
  L.big = L.out + fal((size_t)2 * mw_lloyd_rec_len(k, F) * 8);  // pass record | fold record
  size_t big = mw_gather_ws_bytes(S, F);
  if (T <= 8) big = std::max(big, mw_kpp_ws_bytes(S, T));
  big = std::max(big, mw_farthest_ws_bytes(S));
  L.fold = L.big + fal(big);  // fold: center image (8 KB) | moved bits (S bytes)
  L.total = L.fold + fal(8192) + fal((size_t)S);
  return L;
}

}  // namespace
}  // namespace mw

using namespace mw;

extern "C" size_t mw_kmeans_fit_ws_bytes(int64_t S, int F, int k) {
  if (S <= 0 || F < 1 || F > 64 || k < 1 || k > 64) return 0;
  return fit_layout(S, F, k).total;
}

static int kmeans_fit_impl(const float* d_X, int64_t S, int F, const double* h_mu, const double* h_inv,
                           const double* h_feature_var, const float* h_xmax, int k, const double* h_init,
                           uint32_t seed, int max_iter, double tol, uint8_t* d_labels, double* h_centers,
                           double* h_inertia, int* h_n_iter, int64_t* h_init_idx, void* d_ws, size_t ws_bytes,
                           double* h_final_rec, int* h_inertia_exp, void* stream);

// per pass of the thread's last single fit: kind, changed, recomputed, rows read
static thread_local std::vector<int64_t> fit_hist;

extern "C" int mw_kmeans_fit_history(int64_t* out, int cap) {
  const int n = (int)(fit_hist.size() / 4);
  if (out)
    for (int i = 0; i < std::min(n, cap) * 4; ++i) out[i] = fit_hist[i];
  return n;
}

extern "C" int mw_kmeans_fit(const float* d_X, int64_t S, int F, const double* h_mu,
                             const double* h_inv, const double* h_feature_var, const float* h_xmax,
                             int k, const double* h_init, uint32_t seed, int max_iter, double tol,
                             uint8_t* d_labels, double* h_centers, double* h_inertia, int* h_n_iter,
                             int64_t* h_init_idx, void* d_ws, size_t ws_bytes, void* stream) {
  return kmeans_fit_impl(d_X, S, F, h_mu, h_inv, h_feature_var, h_xmax, k, h_init, seed, max_iter, tol,
                         d_labels, h_centers, h_inertia, h_n_iter, h_init_idx, d_ws, ws_bytes, nullptr, nullptr,
                         stream);
}

extern "C" int mw_kmeans_fit_async(const float* d_X, int64_t S, int F, const double* h_mu,
                                   const double* h_inv, const double* h_feature_var, const float* h_xmax,
                                   int k, const double* h_init, uint32_t seed, int max_iter, double tol,
                                   uint8_t* d_labels, double* h_centers, int* h_n_iter, int64_t* h_init_idx,
                                   void* d_ws, size_t ws_bytes, double* h_final_rec, int* h_inertia_exp,
                                   void* stream) {
  MW_CHECK_ARG(h_final_rec && h_inertia_exp, "mw_kmeans_fit_async: null final-record pointer");
  double unused = 0.0;
  return kmeans_fit_impl(d_X, S, F, h_mu, h_inv, h_feature_var, h_xmax, k, h_init, seed, max_iter, tol,
                         d_labels, h_centers, &unused, h_n_iter, h_init_idx, d_ws, ws_bytes, h_final_rec,
                         h_inertia_exp, stream);
}

static int kmeans_fit_impl(const float* d_X, int64_t S, int F, const double* h_mu, const double* h_inv,
                           const double* h_feature_var, const float* h_xmax, int k, const double* h_init,
                           uint32_t seed, int max_iter, double tol, uint8_t* d_labels, double* h_centers,
                           double* h_inertia, int* h_n_iter, int64_t* h_init_idx, void* d_ws, size_t ws_bytes,
                           double* h_final_rec, int* h_inertia_exp, void* stream) {
  MW_CHECK_ARG(d_X && h_mu && h_inv && d_labels && h_centers && h_inertia && h_n_iter,
               "mw_kmeans_fit: null pointer");
  MW_CHECK_ARG(F >= 1 && F <= 64, "mw_kmeans_fit: F=%d outside [1, 64]", F);
  MW_CHECK_ARG(k >= 1 && k <= 64, "mw_kmeans_fit: n_clusters=%d outside [1, 64]", k);
  MW_CHECK_ARG(S >= k, "mw_kmeans_fit: n_samples=%lld should be >= n_clusters=%d", (long long)S, k);
  MW_CHECK_ARG(max_iter >= 1 && tol >= 0.0, "mw_kmeans_fit: bad max_iter / tol");
  const int T = 2 + (int)std::log((double)k);
  MW_CHECK_ARG(h_init || T <= 8, "mw_kmeans_fit: n_local_trials > 8");
  const FitLayout L = fit_layout(S, F, k);
  MW_CHECK_ARG(!d_ws || ws_bytes >= L.total, "mw_kmeans_fit: workspace %zu < %zu bytes", ws_bytes,
               L.total);
  hipStream_t st = as_stream(stream);
  DevBuf own;
  if (!d_ws) {
    MW_TRY(dev_alloc<char>(own, L.total));
    d_ws = own.p;
  }
  char* base = static_cast<char*>(d_ws);

  Fit fit;
  fit.S = S;
  fit.F = F;
  fit.k = k;
  fit.st = st;
  fit.X = d_X;
  fit.rl = mw_lloyd_rec_len(k, F);
  // small: a32[64] b32[64] qexp[64] absmax[64] | mu64[64] inv64[64] | c64[64 x 64] |
  //        topv[64] topi[64] | stats[130] | idx[64]
  char* sp = base + L.small;
  fit.a32 = reinterpret_cast<float*>(sp);
  fit.b32 = fit.a32 + 64;
  fit.qexp = reinterpret_cast<int32_t*>(fit.b32 + 64);
  float* d_absmax = reinterpret_cast<float*>(fit.qexp + 64);
  double* d_mu = reinterpret_cast<double*>(d_absmax + 64);
  double* d_inv = d_mu + 64;
  double* d_c64 = d_inv + 64;
  double* d_topv = d_c64 + 64 * 64;
  int64_t* d_topi = reinterpret_cast<int64_t*>(d_topv + 64);
  double* d_stats = reinterpret_cast<double*>(d_topi + 64);
  int64_t* d_idx = reinterpret_cast<int64_t*>(d_stats + 130);
  fit.par = reinterpret_cast<float*>(base + L.par);
  fit.ub = reinterpret_cast<float*>(base + L.ub);
  fit.lb = reinterpret_cast<float*>(base + L.lb);
  fit.ws = base + L.lws;
  fit.out = reinterpret_cast<double*>(base + L.out);
  void* big = base + L.big;
  fit.labels = d_labels;
  // MW_KPP_FOLD=1: the first Lloyd E-step folded into the last k-means++
  // pass (kpp.hip mw_kpp_step_fold) for a seeded k-means++ init
  // (mw_kpp_fold_supported: 3 <= k <= 16, T <= 4, F <= 32) with kList passes.
  // Same bits as the separate first pass (tests/test_gpu_fit_c.py); not the
  // default: the fused pass (1.15 ms at config 2) costs what the two passes
  // it replaces do (0.49 + 0.77 ms) and the moved rows' list pass comes on
  // top
  const bool fold_env = [] {  // read per fit (tests compare both forms in one process)
    const char* e = getenv("MW_KPP_FOLD");
    return e && e[0] == '1';
  }();
  const bool fold = fold_env && !h_init && mw_kpp_fold_supported(k, F, T) && S < ((int64_t)1 << 31) &&
                    lloyd_queue_kind() == 4;
  uint8_t* d_moved = reinterpret_cast<uint8_t*>(base + L.fold + 8192);

  // folded scaler: x' = x * a + b (fp32), as DeviceRows
  std::vector<float> a32(F), b32(F);
  fit.a64.resize(F);
  fit.b64.resize(F);
  for (int f = 0; f < F; ++f) {
    a32[f] = (float)h_inv[f];
    b32[f] = (float)(-h_mu[f] * h_inv[f]);
    fit.a64[f] = (double)a32[f];
    fit.b64[f] = (double)b32[f];
  }

  // tolerance: tol * mean over features of the scaled rows' variance
  double tol_abs = 0.0;
  if (tol > 0.0) {
    std::vector<double> var(F);
    if (h_feature_var) {
      for (int f = 0; f < F; ++f) var[f] = h_feature_var[f];
    } else {
      MW_TRY(mw_col_stats_rows(d_X, S, F, big, st));
      MW_TRY(mw_col_stats_finalize(big, S, F, d_stats, 0, st));
      std::vector<double> hs(1 + 2 * F);
      MW_HIP(hipMemcpyAsync(hs.data(), d_stats, hs.size() * 8, hipMemcpyDeviceToHost, st));
      MW_HIP(hipStreamSynchronize(st));
      for (int f = 0; f < F; ++f) var[f] = hs[1 + F + f] / hs[0] * h_inv[f] * h_inv[f];
    }
    tol_abs = np_sum(var.data(), F) / (double)F * tol;
  }

  // fixed-point exponents of the M-step from the column max |x|
  std::vector<float> xmax(F);
  if (h_xmax) {  // taken beside the scaler statistics by the producer of the rows
    for (int f = 0; f < F; ++f) xmax[f] = h_xmax[f];
  } else {
    MW_TRY(mw_col_absmax(d_X, S, F, d_absmax, st));
    MW_HIP(hipMemcpyAsync(xmax.data(), d_absmax, F * 4, hipMemcpyDeviceToHost, st));
    MW_HIP(hipStreamSynchronize(st));
  }
  std::vector<int32_t> qe(F);
  std::vector<double> qscale(F);
  for (int f = 0; f < F; ++f) {
    qe[f] = exp_below((double)xmax[f]);
    qscale[f] = std::ldexp(1.0, -qe[f]);
  }
  // a32[64] b32[64] qexp[64] absmax[64] | mu64[64] inv64[64]: one copy
  {
    std::vector<char> blk(64 * 4 * 4 + 64 * 8 * 2, 0);
    float* fa = reinterpret_cast<float*>(blk.data());
    int32_t* qi = reinterpret_cast<int32_t*>(fa + 128);
    double* dm = reinterpret_cast<double*>(blk.data() + 64 * 4 * 4);
    for (int f = 0; f < F; ++f) {
      fa[f] = a32[f];
      fa[64 + f] = b32[f];
      qi[f] = qe[f];
      fa[192 + f] = xmax[f];
      dm[f] = h_mu[f];
      dm[64 + f] = h_inv[f];
    }
    char* pin = pinned_staging();
    const void* src = blk.data();
    if (pin) {
      std::memcpy(pin + kPinSetup, blk.data(), blk.size());
      src = pin + kPinSetup;
    }
    MW_HIP(hipMemcpyAsync(fit.a32, src, blk.size(), hipMemcpyHostToDevice, st));
    if (!pin) MW_HIP(hipStreamSynchronize(st));  // pageable source must outlive the copy
  }

  // initial centers
  std::vector<double> centers((size_t)k * F);
  if (h_init) {
    std::memcpy(centers.data(), h_init, centers.size() * sizeof(double));
  } else {
    LegacyRandom rs(seed);
    const double u0 = rs.sample();
    const int64_t first = first_center_index(S, u0);
    MW_TRY(mw_kpp_init(d_X, S, F, d_mu, d_inv, d_X + first * F, T, big, st));
    std::vector<double> u(T);
    for (int c = 1; c < k; ++c) {
      for (int t = 0; t < T; ++t) u[t] = rs.sample();
      if (fold && c == k - 1)
        MW_TRY(mw_kpp_step_fold(d_X, S, F, d_mu, d_inv, c, u.data(), T, big, first, fit.a32, fit.b32, fit.qexp,
                                d_labels, fit.ub, fit.lb, d_moved, base + L.fold, reinterpret_cast<double*>(fit.ws),
                                fit.out + fit.rl, st));
      else
        MW_TRY(mw_kpp_step(d_X, S, F, d_mu, d_inv, c, u.data(), T, big, st));
    }
    MW_TRY(mw_kpp_indices(big, S, T, k, d_idx, st));
    std::vector<int64_t> idx(k);
    if (fit.scaled_rows_dev(d_idx, first, k, h_mu, h_inv, reinterpret_cast<float*>(d_c64), centers,
                            idx.data()) == MW_OK) {
      if (h_init_idx) std::memcpy(h_init_idx, idx.data(), k * sizeof(int64_t));
    } else {
      MW_HIP(hipMemcpyAsync(idx.data(), d_idx, k * 8, hipMemcpyDeviceToHost, st));
      MW_HIP(hipStreamSynchronize(st));
      idx[0] = first;
      MW_TRY(fit.scaled_rows(idx.data(), k, h_mu, h_inv, centers));
      if (h_init_idx) std::memcpy(h_init_idx, idx.data(), k * sizeof(int64_t));
    }
  }

  // Lloyd iterations (the fold pass labelled every row already)
  fit_hist.clear();
  if (!fold) MW_HIP(hipMemsetAsync(d_labels, 255, (size_t)S, st));
  std::vector<int64_t> q_hi((size_t)k * F, 0), q_lo((size_t)k * F, 0), count(k, 0);
  std::vector<double> rec, cnew((size_t)k * F), weight(k), tmp(std::max(F, k));
  int64_t last_recomputed = -1;
  int n_iter = 0;
  bool done = false, strict = false;
  for (int it = 0; it < max_iter && !done; ++it) {
    MW_TRY(fit.upload(centers));
    static const int first_kind = [] {  // MW_LLOYD_FIRST_ATOMIC=1: LDS-atomic first M-step (A/B)
      const char* e = getenv("MW_LLOYD_FIRST_ATOMIC");
      return (e && e[0] == '1') ? 3 : 0;
    }();
    static const double queue_below = [] {  // MW_LLOYD_QUEUE_BELOW: kTile/kQueue threshold (A/B)
      const char* e = getenv("MW_LLOYD_QUEUE_BELOW");
      return e ? atof(e) : 0.3;  // as kmeans.QUEUE_BELOW
    }();
    const int queue_kind = lloyd_queue_kind();
    int kind = first_kind;  // first pass
    if (last_recomputed >= 0) {
      double frac = (double)last_recomputed / (double)S;
      if (fit.prev_dmax > 0.f && std::isfinite(fit.drift_max))
        frac *= std::min(1.0, (double)fit.drift_max / (double)fit.prev_dmax);
      kind = frac > queue_below ? 1 : queue_kind;
    }
    if (fold && it == 0) {
      // the k-means++ fold: the winner's moved rows, listed, then recomputed
      // against the k final centers (kind 8) -- the first pass's record
      MW_TRY(mw_lloyd_list_moved(d_moved, mw_kpp_best_ptr(big, S, T), S, F, k, fit.ws, st));
      MW_TRY(fit.pass(0, 8, 0, rec, true));
    } else {
      MW_TRY(fit.pass(0, kind, 0, rec));
    }
    for (size_t i = 0; i < (size_t)k * F; ++i) {
      q_hi[i] += (int64_t)rec[i];
      q_lo[i] += (int64_t)rec[(size_t)k * F + i];
      const int64_t carry = q_lo[i] >> 32;
      q_hi[i] += carry;
      q_lo[i] -= carry << 32;
    }
    for (int j = 0; j < k; ++j) count[j] += (int64_t)rec[2 * (size_t)k * F + j];
    const double* tail = rec.data() + 2 * (size_t)k * F + k;
    const int64_t changed = (int64_t)tail[0];
    last_recomputed = (int64_t)tail[1];
    fit_hist.insert(fit_hist.end(), {(int64_t)(fold && it == 0 ? 8 : kind), changed, last_recomputed,
                                     (int64_t)(tail[2] * 4294967296.0 + tail[3])});
    for (int j = 0; j < k; ++j) {
      weight[j] = (double)count[j];
      for (int f = 0; f < F; ++f) {
        const size_t i = (size_t)j * F + f;
        const double sx = ((double)q_hi[i] * 4294967296.0 + (double)q_lo[i]) * qscale[f];
        cnew[i] = fit.a64[f] * sx + fit.b64[f] * weight[j];
      }
    }
    // empty-cluster relocation (_k_means_common.pyx:181-226)
    std::vector<int> empty;
    for (int j = 0; j < k; ++j)
      if (weight[j] == 0.0) empty.push_back(j);
    if (!empty.empty()) {
      const int ne = (int)empty.size();
      MW_HIP(hipMemcpyAsync(d_c64, centers.data(), centers.size() * 8, hipMemcpyHostToDevice, st));
      MW_TRY(mw_farthest(d_X, S, F, fit.a32, fit.b32, d_c64, k, d_labels, ne, d_topi, d_topv,
                         big, st));
      std::vector<int64_t> far_i(ne);
      std::vector<double> far_v(ne);
      MW_HIP(hipMemcpyAsync(far_i.data(), d_topi, ne * 8, hipMemcpyDeviceToHost, st));
      MW_HIP(hipMemcpyAsync(far_v.data(), d_topv, ne * 8, hipMemcpyDeviceToHost, st));
      MW_HIP(hipStreamSynchronize(st));
      double vmax = far_v[0];
      for (double v : far_v) vmax = std::max(vmax, v);
      if (vmax != 0.0) {
        std::vector<double> xs;
        MW_TRY(fit.scaled_rows(far_i.data(), ne, h_mu, h_inv, xs));
        std::vector<uint8_t> olds(ne);
        for (int e = 0; e < ne; ++e)
          MW_HIP(hipMemcpyAsync(&olds[e], d_labels + far_i[e], 1, hipMemcpyDeviceToHost, st));
        MW_HIP(hipStreamSynchronize(st));
        for (int e = 0; e < ne; ++e) {
          const uint8_t old = olds[e];
          for (int f = 0; f < F; ++f) {
            cnew[(size_t)old * F + f] -= xs[(size_t)e * F + f];
            cnew[(size_t)empty[e] * F + f] = xs[(size_t)e * F + f];
          }
          weight[empty[e]] = 1.0;
          weight[old] -= 1.0;
        }
      }
    }
    // _average_centers (_k_means_common.pyx:229-258)
    int amax = 0;
    for (int j = 1; j < k; ++j)
      if (weight[j] > weight[amax]) amax = j;
    for (int j = 0; j < k; ++j) {
      if (weight[j] > 0.0) {
        const double r = 1.0 / weight[j];
        for (int f = 0; f < F; ++f) cnew[(size_t)j * F + f] *= r;
      } else {
        for (int f = 0; f < F; ++f) cnew[(size_t)j * F + f] = cnew[(size_t)amax * F + f];
      }
    }
    std::vector<double> shift2(k);
    for (int j = 0; j < k; ++j) {
      for (int f = 0; f < F; ++f) {
        const double d = cnew[(size_t)j * F + f] - centers[(size_t)j * F + f];
        tmp[f] = d * d;
      }
      const double sh = std::sqrt(np_sum(tmp.data(), F));
      shift2[j] = sh * sh;
    }
    centers.swap(cnew);
    n_iter = it + 1;
    if (changed == 0) {
      strict = done = true;
    } else if (np_sum(shift2.data(), k) <= tol_abs) {
      done = true;
    }
  }
  if (!done) n_iter = max_iter;

  // final pass: extra E-step unless strictly converged, and inertia
  std::vector<double> xs2(F), cn(k);
  for (int f = 0; f < F; ++f) {
    const double v = std::fabs(fit.a64[f]) * (double)xmax[f] + std::fabs(fit.b64[f]);
    xs2[f] = v * v;
  }
  const double xnorm = std::sqrt(np_sum(xs2.data(), F));
  double cmax = 0.0;
  for (int j = 0; j < k; ++j) {
    for (int f = 0; f < F; ++f) tmp[f] = centers[(size_t)j * F + f] * centers[(size_t)j * F + f];
    const double v = std::sqrt(np_sum(tmp.data(), F));
    cmax = j == 0 ? v : std::max(cmax, v);
  }
  const double xc = xnorm + cmax;
  const int iexp = exp_below(xc * xc * 1.01);
  MW_TRY(fit.upload(centers));
  fit_hist.insert(fit_hist.end(), {(int64_t)(strict ? 12 : 11), -1, -1, S});  // the final pass reads every row
  *h_n_iter = n_iter;
  std::memcpy(h_centers, centers.data(), centers.size() * sizeof(double));
  if (h_final_rec && !own.p && pinned_staging()) {  // (a workspace allocated here is freed on return: synchronous end)
    // asynchronous end: the final pass and its record's copy into the caller's
    // page-locked h_final_rec are queued; the caller reads the inertia,
    // (rec[rl - 2] * 2^32 + rec[rl - 1]) * 2^-iexp, after `stream` reaches
    // here (the labels likewise: stream-ordered).  The staging the table came
    // from stays busy until then.
    MW_TRY(fit.pass_async(strict ? 2 : 1, 0, iexp, h_final_rec));
    *h_inertia_exp = iexp;
    hipEvent_t ev;
    MW_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    MW_HIP(hipEventRecord(ev, st));
    pin_busy = ev;
    *h_inertia = std::numeric_limits<double>::quiet_NaN();
    return MW_OK;
  }
  MW_TRY(fit.pass(strict ? 2 : 1, 0, iexp, rec));
  const double* tail = rec.data() + fit.rl - 4;
  *h_inertia = (tail[2] * 4294967296.0 + tail[3]) * std::ldexp(1.0, -iexp);
  if (h_final_rec) {
    std::memcpy(h_final_rec, rec.data(), (size_t)fit.rl * sizeof(double));
    *h_inertia_exp = iexp;
  }
  return MW_OK;
}

// ---------------------------------------------------------------------------
// mw_lloyd_fits: kmeans.py lloyd_fits (one process, no sharding) -- the
// batched Lloyd iterations of several independent fits over the same rows,
// host control flow step for step, so both front ends return the same bits.
// Per iteration: one table upload, the passes grouped by kind (24 fits per
// launch at most), one record download; the per-fit fp64 host arithmetic is
// the one of mw_kmeans_fit above (numpy's reductions restated by np_sum).
namespace mw {
namespace {

constexpr int kFitsMaxPerLaunch = 24;
constexpr int kKindFirst = 0, kKindTile = 1, kKindDense = 5;

struct FitsFit {
  int k = 0;
  std::vector<double> centers;
  std::vector<float> prev32;
  bool have_prev = false;
  std::vector<int64_t> q_hi, q_lo, count;
  bool done = false, strict = false, bounds_ok = true;
  int n_iter = 0;
  double drift_max = 0.0, prev_dmax = 0.0;  // float32 values (or inf), as the Python floats
  int iexp = 0;
  std::vector<int64_t> hist;  // (changed, recomputed) per pass
};

// kmeans.py _bound_tables + upload: the fp32 centers | drift | half
// separation of one fit into `h` (k*F + 2k floats)
void fits_tables(FitsFit& fs, int F, bool nobound, float* h) {
  const int k = fs.k;
  for (size_t i = 0; i < (size_t)k * F; ++i) h[i] = (float)fs.centers[i];
  const float inf = std::numeric_limits<float>::infinity();
  std::vector<float> drift32(k), half32(k);
  double dmax;
  if (nobound) {
    for (int j = 0; j < k; ++j) drift32[j] = inf, half32[j] = 0.f;
    dmax = std::numeric_limits<double>::infinity();
  } else {
    std::vector<double> tmp(F);
    for (int j = 0; j < k; ++j) {
      double drift = 0.0;
      if (fs.have_prev) {
        for (int f = 0; f < F; ++f) {
          const double d = (double)h[(size_t)j * F + f] - (double)fs.prev32[(size_t)j * F + f];
          tmp[f] = d * d;
        }
        drift = std::sqrt(np_sum(tmp.data(), F));
      }
      double half = std::numeric_limits<double>::infinity();
      if (k > 1) {
        double m = std::numeric_limits<double>::infinity();
        for (int i = 0; i < k; ++i) {
          if (i == j) continue;
          for (int f = 0; f < F; ++f) {
            const double d = (double)h[(size_t)j * F + f] - (double)h[(size_t)i * F + f];
            tmp[f] = d * d;
          }
          m = std::min(m, np_sum(tmp.data(), F));
        }
        half = 0.5 * std::sqrt(m);
      }
      drift32[j] = round_f32(drift, true);
      half32[j] = round_f32(half, false);
    }
    float m = drift32[0];
    for (int j = 1; j < k; ++j) m = std::max(m, drift32[j]);
    dmax = (double)m;
  }
  if (!fs.bounds_ok) {  // after dense passes: every row recomputed, bounds rewritten
    for (int j = 0; j < k; ++j) drift32[j] = inf;
    dmax = std::numeric_limits<double>::infinity();
  }
  fs.prev_dmax = fs.have_prev ? fs.drift_max : 0.0;
  fs.prev32.assign(h, h + (size_t)k * F);
  fs.have_prev = true;
  fs.drift_max = dmax;
  for (int j = 0; j < k; ++j) {
    h[(size_t)k * F + j] = drift32[j];
    h[(size_t)k * F + k + j] = half32[j];
  }
}

// Message layout of a sharded run in the caller's d_msg (fp64): the fits'
// records (d_out == d_msg) | the local top-64 (distance, global row) pairs of
// a relocation | their all-gather (world x 64 pairs) | the winners' (raw row,
// old label) from their owners (64 x (F + 1)).
struct MsgLayout {
  int64_t vi, gathered, owners, total;
};
MsgLayout msg_layout(int64_t rec_total, int F, int world) {
  MsgLayout L;
  L.vi = rec_total;
  L.gathered = L.vi + 2 * 64;
  L.owners = L.gathered + (int64_t)world * 2 * 64;
  L.total = L.owners + 64 * (int64_t)(F + 1);
  return L;
}

// hipEvent pairs of the per-launch timing, destroyed on every return path
struct TimedLaunches {
  struct T {
    hipEvent_t a, b;
    int slot;
    double bytes;
  };
  std::vector<T> v;
  ~TimedLaunches() {
    for (T& t : v) {
      (void)hipEventDestroy(t.a);
      (void)hipEventDestroy(t.b);
    }
  }
};

int lloyd_fits_impl(const float* d_X, int64_t S, int F, const float* d_a32, const float* d_b32,
                    const int32_t* d_qexp, const float* h_a32, const float* h_b32, const int32_t* h_qexp,
                    const float* h_xmax, const double* h_mu, const double* h_inv, int n, const int* h_k,
                    const double* h_init, uint8_t* const* d_labels, float* const* d_ub, float* const* d_lb,
                    void* const* d_ws, float* d_par, double* d_out, int max_iter, double tol, int first_kind,
                    int queue_kind, double queue_below, int dense_min, int nobound, double* h_centers,
                    double* h_inertia, int* h_n_iter, int64_t* h_hist, int hist_cap, int* h_hist_len,
                    double* h_timing, const mw_fit_comm* comm, void* stream);

}  // namespace
}  // namespace mw

extern "C" int mw_lloyd_fits(const float* d_X, int64_t S, int F, const float* d_a32, const float* d_b32,
                             const int32_t* d_qexp, const float* h_a32, const float* h_b32,
                             const int32_t* h_qexp, const float* h_xmax, const double* h_mu,
                             const double* h_inv, int n, const int* h_k, const double* h_init,
                             uint8_t* const* d_labels, float* const* d_ub, float* const* d_lb,
                             void* const* d_ws, float* d_par, double* d_out, int max_iter, double tol,
                             int first_kind, int queue_kind, double queue_below, int dense_min,
                             int nobound, double* h_centers, double* h_inertia, int* h_n_iter,
                             int64_t* h_hist, int hist_cap, int* h_hist_len, double* h_timing,
                             void* stream) {
  return lloyd_fits_impl(d_X, S, F, d_a32, d_b32, d_qexp, h_a32, h_b32, h_qexp, h_xmax, h_mu, h_inv, n, h_k,
                         h_init, d_labels, d_ub, d_lb, d_ws, d_par, d_out, max_iter, tol, first_kind, queue_kind,
                         queue_below, dense_min, nobound, h_centers, h_inertia, h_n_iter, h_hist, hist_cap,
                         h_hist_len, h_timing, nullptr, stream);
}

extern "C" int64_t mw_lloyd_fits_msg_len(int64_t rec_total, int F, int world) {
  if (rec_total < 0 || F < 1 || F > 64 || world < 1) return 0;
  return msg_layout(rec_total, F, world).total;
}

extern "C" int mw_lloyd_fits_sharded(const float* d_X, int64_t S, int F, const float* d_a32,
                                     const float* d_b32, const int32_t* d_qexp, const float* h_a32,
                                     const float* h_b32, const int32_t* h_qexp, const float* h_xmax,
                                     const double* h_mu, const double* h_inv, int n, const int* h_k,
                                     const double* h_init, uint8_t* const* d_labels, float* const* d_ub,
                                     float* const* d_lb, void* const* d_ws, float* d_par, double* d_out,
                                     int max_iter, double tol, int first_kind, int queue_kind,
                                     double queue_below, int dense_min, int nobound, double* h_centers,
                                     double* h_inertia, int* h_n_iter, int64_t* h_hist, int hist_cap,
                                     int* h_hist_len, double* h_timing, const mw_fit_comm* comm,
                                     void* stream) {
  MW_CHECK_ARG(comm && comm->d_msg && comm->all_reduce_sum && comm->all_gather,
               "mw_lloyd_fits_sharded: null comm");
  MW_CHECK_ARG(comm->world >= 1 && comm->rank >= 0 && comm->rank < comm->world && comm->row_offset >= 0 &&
                   comm->rows_total >= S + comm->row_offset,
               "mw_lloyd_fits_sharded: bad world / rank / row range");
  MW_CHECK_ARG(d_out == comm->d_msg, "mw_lloyd_fits_sharded: d_out must be comm->d_msg (records at offset 0)");
  return lloyd_fits_impl(d_X, S, F, d_a32, d_b32, d_qexp, h_a32, h_b32, h_qexp, h_xmax, h_mu, h_inv, n, h_k,
                         h_init, d_labels, d_ub, d_lb, d_ws, d_par, d_out, max_iter, tol, first_kind, queue_kind,
                         queue_below, dense_min, nobound, h_centers, h_inertia, h_n_iter, h_hist, hist_cap,
                         h_hist_len, h_timing, comm, stream);
}

namespace mw {
namespace {

int lloyd_fits_impl(const float* d_X, int64_t S, int F, const float* d_a32, const float* d_b32,
                    const int32_t* d_qexp, const float* h_a32, const float* h_b32, const int32_t* h_qexp,
                    const float* h_xmax, const double* h_mu, const double* h_inv, int n, const int* h_k,
                    const double* h_init, uint8_t* const* d_labels, float* const* d_ub, float* const* d_lb,
                    void* const* d_ws, float* d_par, double* d_out, int max_iter, double tol, int first_kind,
                    int queue_kind, double queue_below, int dense_min, int nobound, double* h_centers,
                    double* h_inertia, int* h_n_iter, int64_t* h_hist, int hist_cap, int* h_hist_len,
                    double* h_timing, const mw_fit_comm* comm, void* stream) {
  MW_CHECK_ARG(d_X && d_a32 && d_b32 && d_qexp && h_a32 && h_b32 && h_qexp && h_xmax && h_mu && h_inv &&
                   h_k && h_init && d_labels && d_ub && d_lb && d_ws && d_par && d_out && h_centers &&
                   h_inertia && h_n_iter,
               "mw_lloyd_fits: null pointer");
  MW_CHECK_ARG(n >= 1 && F >= 1 && F <= 64 && S >= 1 && max_iter >= 1 && tol >= 0.0,
               "mw_lloyd_fits: bad n / F / S / max_iter / tol");
  hipStream_t st = as_stream(stream);
  // rows over all shards (the pass-kind policy compares the global recomputed count with it)
  const int64_t S_glob = comm ? comm->rows_total : S;
  std::vector<FitsFit> fits(n);
  std::vector<int64_t> poff(n + 1, 0), roff(n + 1, 0);
  size_t coff = 0;
  for (int g = 0; g < n; ++g) {
    const int k = h_k[g];
    MW_CHECK_ARG(k >= 1 && k <= 64 && S >= k, "mw_lloyd_fits: fit %d: k=%d", g, k);
    FitsFit& fs = fits[g];
    fs.k = k;
    fs.centers.assign(h_init + coff, h_init + coff + (size_t)k * F);
    coff += (size_t)k * F;
    fs.q_hi.assign((size_t)k * F, 0);
    fs.q_lo.assign((size_t)k * F, 0);
    fs.count.assign(k, 0);
    poff[g + 1] = poff[g] + (int64_t)k * F + 2 * k;
    roff[g + 1] = roff[g] + mw_lloyd_rec_len(k, F);
  }
  std::vector<double> a64(F), b64(F), qscale(F);
  for (int f = 0; f < F; ++f) {
    a64[f] = (double)h_a32[f];
    b64[f] = (double)h_b32[f];
    qscale[f] = std::ldexp(1.0, -h_qexp[f]);
  }
  int kmax = 1;
  for (int g = 0; g < n; ++g) kmax = std::max(kmax, h_k[g]);
  const bool dense_ok = dense_min >= 0 && kmax <= 20;  // dense_min < 0: never (the caller checks F)

  // host staging: pinned when the tables / records fit its regions
  char* pin = pinned_staging();
  const size_t par_bytes = (size_t)poff[n] * 4, rec_bytes = (size_t)roff[n] * 8;
  std::vector<float> host_par_v;
  std::vector<double> rec_v;
  float* host_par;
  double* rec;
  const bool pin_par = pin && par_bytes <= kPinRec - kPinTab;
  const bool pin_rec = pin && rec_bytes <= kPinRows - kPinRec;
  if (pin_par) {
    host_par = reinterpret_cast<float*>(pin + kPinTab);
  } else {
    host_par_v.assign(poff[n], 0.f);
    host_par = host_par_v.data();
  }
  std::memset(host_par, 0, par_bytes);
  if (pin_rec) {
    rec = reinterpret_cast<double*>(pin + kPinRec);
  } else {
    rec_v.assign(roff[n], 0.0);
    rec = rec_v.data();
  }

  // per-launch timing (bench.py's profiling): slot = kind (mode 0) or 6 + mode
  TimedLaunches timed;

  auto upload = [&](const std::vector<int>& sel) -> int {
    for (int g : sel) fits_tables(fits[g], F, nobound != 0, host_par + poff[g]);
    MW_HIP(hipMemcpyAsync(d_par, host_par, par_bytes, hipMemcpyHostToDevice, st));
    if (!pin_par) MW_HIP(hipStreamSynchronize(st));
    return MW_OK;
  };
  auto launch = [&](const std::vector<int>& gs, int mode, int kind) -> int {
    for (size_t i0 = 0; i0 < gs.size(); i0 += kFitsMaxPerLaunch) {
      const size_t i1 = std::min(gs.size(), i0 + kFitsMaxPerLaunch);
      std::vector<mw_lloyd_fit> arr(i1 - i0);
      double nbytes = 0.0;
      for (size_t i = i0; i < i1; ++i) {
        const int g = gs[i];
        const FitsFit& fs = fits[g];
        mw_lloyd_fit& f = arr[i - i0];
        float* base = d_par + poff[g];
        f.centers = base;
        f.drift = base + (size_t)fs.k * F;
        f.half_sep = base + (size_t)fs.k * F + fs.k;
        f.labels = d_labels[g];
        f.ub = d_ub[g];
        f.lb = d_lb[g];
        f.ws = d_ws[g];
        f.out = d_out + roff[g];
        f.k = fs.k;
        f.drift_max = (float)fs.drift_max;
        f.inertia_exp = fs.iexp;
        if (kind == kKindDense && mode == 0)  // rows once per launch, labels per fit
          nbytes += 2.0 * S + (i == i0 ? (double)S * F * 4 : 0.0);
        else
          nbytes += 9.0 * S + ((mode || (kind != 2 && kind != 4)) ? (double)S * F * 4 : 0.0);
      }
      TimedLaunches::T t{};
      if (h_timing) {
        MW_HIP(hipEventCreate(&t.a));
        if (hipEventCreate(&t.b) != hipSuccess) {
          (void)hipEventDestroy(t.a);
          set_error("mw_lloyd_fits: hipEventCreate failed");
          return MW_EHIP;
        }
        t.slot = mode ? 6 + mode : kind;
        t.bytes = nbytes;
        timed.v.push_back(t);
        MW_HIP(hipEventRecord(t.a, st));
      }
      MW_TRY(mw_lloyd_pass(d_X, S, F, d_a32, d_b32, d_qexp, (int)arr.size(), arr.data(), mode, kind, st));
      if (h_timing) MW_HIP(hipEventRecord(t.b, st));
    }
    return MW_OK;
  };
  // the caller's collectives (sharded rows): a failing callback ends the fit
  auto comm_call = [&](int rc_cb, const char* what) -> int {
    if (rc_cb == 0) return MW_OK;
    set_error("mw_lloyd_fits_sharded: the %s callback returned %d", what, rc_cb);
    return MW_EHIP;
  };
  // one all-reduce of the exact records over the shards (the only exchange of
  // a pass), then one download
  // host time per iteration (h_timing): from a record's arrival to the next
  // pass queued, and inside the caller's collectives
  using clk = std::chrono::steady_clock;
  auto ms_since = [](clk::time_point a) {
    return std::chrono::duration<double, std::milli>(clk::now() - a).count();
  };
  double host_ms = 0.0, comm_ms = 0.0;
  int host_n = 0;
  clk::time_point t_ready{};
  bool have_ready = false;
  auto download = [&]() -> int {
    if (comm) {
      const clk::time_point t0 = clk::now();
      MW_TRY(comm_call(comm->all_reduce_sum(comm->ctx, 0, roff[n], stream), "all_reduce_sum"));
      comm_ms += ms_since(t0);
    }
    MW_HIP(hipMemcpyAsync(rec, d_out, rec_bytes, hipMemcpyDeviceToHost, st));
    MW_HIP(hipStreamSynchronize(st));
    t_ready = clk::now();
    have_ready = true;
    return MW_OK;
  };
  auto host_mark = [&]() {  // the next pass is about to be queued
    if (have_ready) {
      host_ms += ms_since(t_ready);
      ++host_n;
      have_ready = false;
    }
  };
  const MsgLayout ML = msg_layout(roff[n], F, comm ? comm->world : 1);
  if (comm) MW_CHECK_ARG(comm->msg_len >= ML.total, "mw_lloyd_fits_sharded: msg_len %lld < %lld",
                         (long long)comm->msg_len, (long long)ML.total);

  // relocation scratch (allocated on the first empty cluster)
  DevBuf far_buf;
  size_t far_ws = 0;
  double* d_c64 = nullptr;
  int64_t* d_topi = nullptr;
  double* d_topv = nullptr;
  void* d_farws = nullptr;

  int rc = MW_OK;
  std::vector<double> cnew, weight, tmp(std::max(F, kmax));
  for (int it = 0; it < max_iter && rc == MW_OK; ++it) {
    std::vector<int> active;
    for (int g = 0; g < n; ++g)
      if (!fits[g].done) active.push_back(g);
    if (active.empty()) break;
    const bool dense_now = dense_ok && it > 0 && (int)active.size() >= dense_min;
    if ((rc = upload(active)) != MW_OK) break;
    // kind_of (kmeans.py): first pass, dense, else kTile / the few-undecided kind
    std::vector<int> by_kind[8];
    for (int g : active) {
      const FitsFit& fs = fits[g];
      int kind;
      if (fs.hist.empty()) {
        kind = first_kind;
      } else if (dense_now) {
        kind = kKindDense;
      } else if (!fs.bounds_ok) {
        kind = kKindTile;
      } else {
        double frac = (double)fs.hist.back() / (double)std::max<int64_t>(S_glob, 1);
        if (fs.prev_dmax > 0 && std::isfinite(fs.drift_max)) frac *= std::min(1.0, fs.drift_max / fs.prev_dmax);
        kind = frac > queue_below ? kKindTile : queue_kind;
      }
      by_kind[kind].push_back(g);
    }
    host_mark();
    for (int kind = 0; kind < 8 && rc == MW_OK; ++kind)
      if (!by_kind[kind].empty()) rc = launch(by_kind[kind], 0, kind);
    if (rc != MW_OK || (rc = download()) != MW_OK) break;
    for (int g : active) {
      FitsFit& fs = fits[g];
      const int k = fs.k;
      if (it > 0) fs.bounds_ok = !dense_now;
      const double* r = rec + roff[g];
      for (size_t i = 0; i < (size_t)k * F; ++i) {
        fs.q_hi[i] += (int64_t)r[i];
        fs.q_lo[i] += (int64_t)r[(size_t)k * F + i];
        const int64_t carry = fs.q_lo[i] >> 32;
        fs.q_hi[i] += carry;
        fs.q_lo[i] -= carry << 32;
      }
      for (int j = 0; j < k; ++j) fs.count[j] += (int64_t)r[2 * (size_t)k * F + j];
      const double* tail = r + 2 * (size_t)k * F + k;
      const int64_t changed = (int64_t)tail[0];
      fs.hist.push_back(changed);
      fs.hist.push_back((int64_t)tail[1]);
      cnew.assign((size_t)k * F, 0.0);
      weight.assign(k, 0.0);
      for (int j = 0; j < k; ++j) {
        weight[j] = (double)fs.count[j];
        for (int f = 0; f < F; ++f) {
          const size_t i = (size_t)j * F + f;
          const double sx = ((double)fs.q_hi[i] * 4294967296.0 + (double)fs.q_lo[i]) * qscale[f];
          cnew[i] = a64[f] * sx + b64[f] * weight[j];
        }
      }
      // empty-cluster relocation (_k_means_common.pyx:181-226)
      std::vector<int> empty;
      for (int j = 0; j < k; ++j)
        if (weight[j] == 0.0) empty.push_back(j);
      if (!empty.empty()) {
        const int ne = (int)empty.size();
        if (!far_buf.p) {
          far_ws = fal(mw_farthest_ws_bytes(S));
          if ((rc = dev_alloc<char>(far_buf, far_ws + fal(64 * 64 * 8) + 64 * 16)) != MW_OK) break;
          d_farws = far_buf.p;
          d_c64 = reinterpret_cast<double*>(static_cast<char*>(far_buf.p) + far_ws);
          d_topi = reinterpret_cast<int64_t*>(static_cast<char*>(far_buf.p) + far_ws + fal(64 * 64 * 8));
          d_topv = reinterpret_cast<double*>(d_topi + 64);
        }
        MW_HIP(hipMemcpyAsync(d_c64, fs.centers.data(), fs.centers.size() * 8, hipMemcpyHostToDevice, st));
        const int m = (int)std::min<int64_t>(ne, S);  // this shard's candidates (S >= 1)
        if ((rc = mw_farthest(d_X, S, F, d_a32, d_b32, d_c64, k, d_labels[g], m, d_topi, d_topv, d_farws,
                              st)) != MW_OK)
          break;
        std::vector<int64_t> far_i(m);
        std::vector<double> far_v(m);
        MW_HIP(hipMemcpyAsync(far_i.data(), d_topi, m * 8, hipMemcpyDeviceToHost, st));
        MW_HIP(hipMemcpyAsync(far_v.data(), d_topv, m * 8, hipMemcpyDeviceToHost, st));
        MW_HIP(hipStreamSynchronize(st));
        std::vector<float> xr((size_t)ne * F);
        std::vector<uint8_t> olds(ne);
        if (comm) {
          // dist.DistComm.farthest: every shard's local top n as (distance,
          // global row) pairs, all-gathered and ordered by (distance desc, row
          // asc); the winners' raw rows and old labels all-reduced from their
          // owners (zeros elsewhere; fp32 values and labels are exact in fp64)
          std::vector<double> vi(2 * (size_t)ne, -1.0);
          for (int e = 0; e < m; ++e) {
            vi[2 * e] = far_v[e];
            vi[2 * e + 1] = (double)(far_i[e] + comm->row_offset);
          }
          MW_HIP(hipMemcpyAsync(comm->d_msg + ML.vi, vi.data(), vi.size() * 8, hipMemcpyHostToDevice, st));
          MW_HIP(hipStreamSynchronize(st));
          if ((rc = comm_call(comm->all_gather(comm->ctx, ML.vi, 2 * ne, ML.gathered, stream), "all_gather")) !=
              MW_OK)
            break;
          std::vector<double> gv((size_t)comm->world * 2 * ne);
          MW_HIP(hipMemcpyAsync(gv.data(), comm->d_msg + ML.gathered, gv.size() * 8, hipMemcpyDeviceToHost, st));
          MW_HIP(hipStreamSynchronize(st));
          std::vector<std::pair<double, int64_t>> cand;  // (distance, global row) of every shard
          for (size_t i = 0; i < gv.size() / 2; ++i)
            if (gv[2 * i + 1] >= 0) cand.push_back({gv[2 * i], (int64_t)gv[2 * i + 1]});
          std::sort(cand.begin(), cand.end(), [](const std::pair<double, int64_t>& a,
                                                 const std::pair<double, int64_t>& b) {
            return a.first != b.first ? a.first > b.first : a.second < b.second;
          });
          cand.resize(std::min<size_t>(cand.size(), (size_t)ne));
          far_i.assign(ne, 0);
          far_v.assign(ne, 0.0);
          for (size_t e = 0; e < cand.size(); ++e) far_v[e] = cand[e].first, far_i[e] = cand[e].second;
          double vmax = far_v[0];
          for (double v : far_v) vmax = std::max(vmax, v);
          std::vector<double> own((size_t)ne * (F + 1), 0.0);
          for (int e = 0; e < ne; ++e) {
            const int64_t loc = far_i[e] - comm->row_offset;
            if (loc < 0 || loc >= S) continue;
            MW_HIP(hipMemcpyAsync(xr.data() + (size_t)e * F, d_X + loc * F, F * sizeof(float),
                                  hipMemcpyDeviceToHost, st));
            MW_HIP(hipMemcpyAsync(&olds[e], d_labels[g] + loc, 1, hipMemcpyDeviceToHost, st));
          }
          MW_HIP(hipStreamSynchronize(st));
          for (int e = 0; e < ne; ++e) {
            const int64_t loc = far_i[e] - comm->row_offset;
            if (loc < 0 || loc >= S) continue;
            for (int f = 0; f < F; ++f) own[(size_t)e * (F + 1) + f] = (double)xr[(size_t)e * F + f];
            own[(size_t)e * (F + 1) + F] = (double)olds[e];
          }
          MW_HIP(hipMemcpyAsync(comm->d_msg + ML.owners, own.data(), own.size() * 8, hipMemcpyHostToDevice, st));
          MW_HIP(hipStreamSynchronize(st));
          if ((rc = comm_call(comm->all_reduce_sum(comm->ctx, ML.owners, (int64_t)own.size(), stream),
                              "all_reduce_sum")) != MW_OK)
            break;
          MW_HIP(hipMemcpyAsync(own.data(), comm->d_msg + ML.owners, own.size() * 8, hipMemcpyDeviceToHost, st));
          MW_HIP(hipStreamSynchronize(st));
          if (vmax == 0.0) far_v.clear();  // nothing to move (as _relocate_empty: far_val.max() == 0)
          for (int e = 0; e < ne; ++e) {
            for (int f = 0; f < F; ++f) xr[(size_t)e * F + f] = (float)own[(size_t)e * (F + 1) + f];
            olds[e] = (uint8_t)own[(size_t)e * (F + 1) + F];
          }
        } else {
          double vmax = far_v[0];
          for (double v : far_v) vmax = std::max(vmax, v);
          if (vmax == 0.0) {
            far_v.clear();
          } else {
            for (int e = 0; e < ne; ++e) {
              MW_HIP(hipMemcpyAsync(xr.data() + (size_t)e * F, d_X + far_i[e] * F, F * sizeof(float),
                                    hipMemcpyDeviceToHost, st));
              MW_HIP(hipMemcpyAsync(&olds[e], d_labels[g] + far_i[e], 1, hipMemcpyDeviceToHost, st));
            }
            MW_HIP(hipStreamSynchronize(st));
          }
        }
        if (!far_v.empty()) {
          for (int e = 0; e < ne; ++e) {
            const uint8_t old = olds[e];
            for (int f = 0; f < F; ++f) {
              const double x = ((double)xr[(size_t)e * F + f] - h_mu[f]) * h_inv[f];
              cnew[(size_t)old * F + f] -= x;
              cnew[(size_t)empty[e] * F + f] = x;
            }
            weight[empty[e]] = 1.0;
            weight[old] -= 1.0;
          }
        }
      }
      // _average_centers (_k_means_common.pyx:229-258)
      int amax = 0;
      for (int j = 1; j < k; ++j)
        if (weight[j] > weight[amax]) amax = j;
      for (int j = 0; j < k; ++j) {
        if (weight[j] > 0.0) {
          const double rr = 1.0 / weight[j];
          for (int f = 0; f < F; ++f) cnew[(size_t)j * F + f] *= rr;
        } else {
          for (int f = 0; f < F; ++f) cnew[(size_t)j * F + f] = cnew[(size_t)amax * F + f];
        }
      }
      std::vector<double> shift2(k);
      for (int j = 0; j < k; ++j) {
        for (int f = 0; f < F; ++f) {
          const double d = cnew[(size_t)j * F + f] - fs.centers[(size_t)j * F + f];
          tmp[f] = d * d;
        }
        const double sh = std::sqrt(np_sum(tmp.data(), F));
        shift2[j] = sh * sh;
      }
      fs.centers.swap(cnew);
      fs.n_iter = it + 1;
      if (changed == 0) {
        fs.strict = fs.done = true;
      } else if (np_sum(shift2.data(), k) <= tol) {
        fs.done = true;
      }
      if (fs.done) MW_HIP(hipMemsetAsync(d_out + roff[g], 0, (size_t)(roff[g + 1] - roff[g]) * 8, st));
    }
  }
  if (rc != MW_OK) return rc;
  for (FitsFit& fs : fits)
    if (!fs.done) fs.n_iter = max_iter;

  // final pass: the extra E-step when not strictly converged, and inertia
  std::vector<double> xs2(F);
  for (int f = 0; f < F; ++f) {
    const double v = std::fabs(a64[f]) * (double)h_xmax[f] + std::fabs(b64[f]);
    xs2[f] = v * v;
  }
  const double xnorm = std::sqrt(np_sum(xs2.data(), F));
  std::vector<int> all(n);
  for (int g = 0; g < n; ++g) {
    all[g] = g;
    FitsFit& fs = fits[g];
    double cmax = 0.0;
    for (int j = 0; j < fs.k; ++j) {
      for (int f = 0; f < F; ++f) tmp[f] = fs.centers[(size_t)j * F + f] * fs.centers[(size_t)j * F + f];
      const double v = std::sqrt(np_sum(tmp.data(), F));
      cmax = j == 0 ? v : std::max(cmax, v);
    }
    const double xc = xnorm + cmax;
    fs.iexp = exp_below(xc * xc * 1.01);
  }
  if ((rc = upload(all)) == MW_OK) {
    host_mark();
    for (int mode = 1; mode <= 2 && rc == MW_OK; ++mode) {
      std::vector<int> sel;
      for (int g = 0; g < n; ++g)
        if ((fits[g].strict ? 2 : 1) == mode) sel.push_back(g);
      if (!sel.empty()) rc = launch(sel, mode, kKindFirst);
    }
  }
  if (rc == MW_OK) rc = download();
  if (rc != MW_OK) return rc;
  size_t c = 0;
  for (int g = 0; g < n; ++g) {
    const FitsFit& fs = fits[g];
    const double* tail = rec + roff[g + 1] - 4;
    h_inertia[g] = (tail[2] * 4294967296.0 + tail[3]) * std::ldexp(1.0, -fs.iexp);
    h_n_iter[g] = fs.n_iter;
    std::memcpy(h_centers + c, fs.centers.data(), fs.centers.size() * sizeof(double));
    c += fs.centers.size();
    if (h_hist && h_hist_len) {
      const int m = (int)std::min<size_t>(fs.hist.size() / 2, (size_t)hist_cap);
      std::memcpy(h_hist + (size_t)g * hist_cap * 2, fs.hist.data(), (size_t)m * 2 * sizeof(int64_t));
      h_hist_len[g] = m;
    }
  }
  if (h_timing) {  // [slot][count, ms, bytes], slots 0..8; then host intervals, host ms, comm ms
    for (int i = 0; i < 27; ++i) h_timing[i] = 0.0;
    h_timing[27] = host_n;
    h_timing[28] = host_ms;
    h_timing[29] = comm_ms;
    for (TimedLaunches::T& t : timed.v) {
      float ms = 0.f;
      (void)hipEventElapsedTime(&ms, t.a, t.b);
      h_timing[3 * t.slot] += 1.0;
      h_timing[3 * t.slot + 1] += ms;
      h_timing[3 * t.slot + 2] += t.bytes;
    }
  }
  return MW_OK;  // (the events are destroyed with `timed`)
}

}  // namespace
}  // namespace mw
