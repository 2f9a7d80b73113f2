/*
 * milwrm_amd — C ABI of the MI355X-native MILWRM pixel-clustering hot path.
 *
 * Plain pointers and sizes only (no torch types).  Every pointer named d_* is
 * device memory (HBM) owned by the caller; h_* is host memory.  `stream` is a
 * hipStream_t passed as void*.  All launches are asynchronous on `stream`
 * unless a function says it synchronises.  Workspace buffers (d_ws) are
 * caller-allocated; their sizes come from the matching *_ws_bytes() query.
 * The library never frees caller memory and never allocates inside a launch
 * function.  Status: 0 = ok, < 0 = error; mw_last_error() gives the text.
 *
 * Reference interfaces replaced (file:line in codyheiser/MILWRM unless noted;
 * sklearn/scipy paths are the pinned third-party engines the reference calls):
 *   mw_nz_stats        img.calculate_non_zero_mean        MxIF.py:519-541
 *   mw_lognorm         img.log_normalize                  MxIF.py:416-455
 *   mw_blur            img.blurring('gaussian') → skimage.filters.gaussian →
 *                      scipy.ndimage.gaussian_filter       MxIF.py:375-394
 *   mw_block_mean      img.downsample → skimage block_reduce MxIF.py:494-517
 *   mw_mask_rank,
 *   mw_gather_rows     img.subsample_pixels (mask gather + fancy index)
 *                                                          MxIF.py:457-492
 *   mw_legacy_randint_* np.random.seed(16); np.random.choice(M, S)
 *                                                          MxIF.py:484,490
 *   mw_col_stats_finalize StandardScaler.fit               MILWRM.py:1742-1745
 *   mw_kpp_*           sklearn _kmeans_plusplus            _kmeans.py:174-272
 *   mw_lloyd_pass      sklearn lloyd_iter_chunked_dense    _k_means_lloyd.pyx:23-218
 *                      (+ _inertia_dense                   _k_means_common.pyx:94-124)
 *   mw_farthest        sklearn _relocate_empty_clusters_dense _k_means_common.pyx:181-226
 *   mw_assign_conf     KMeans.predict + estimate_confidence_score_mxif
 *                                                          MILWRM.py:237-277, 389-450
 */
#ifndef MILWRM_AMD_H
#define MILWRM_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* status codes */
#define MW_OK 0
#define MW_EINVAL (-1)      /* bad argument (ValueError on the Python side) */
#define MW_EHIP (-2)        /* HIP runtime error */
#define MW_EUNSUPPORTED (-3) /* shape/parameter outside what the kernels take */

/* element types of image planes */
#define MW_U8 0
#define MW_U16 1
#define MW_F32 2

int mw_version(void);
const char* mw_last_error(void);
/* Number of streaming workgroups the reductions use for `n` rows; partial
 * buffers are sized from it.  Fixed per n (not per device) so results are
 * identical across runs and shard layouts. */
int mw_stream_blocks(int64_t n);

/* ---- img.calculate_non_zero_mean (MxIF.py:519-541) --------------------------
 * HWC image of n_pix pixels x C channels.  Outputs per channel: sum of the
 * non-zero values (fp64) and their count (int64).  Deterministic. */
size_t mw_nz_stats_ws_bytes(int64_t n_pix, int C);
int mw_nz_stats(const void* d_img, int dtype, int64_t n_pix, int C,
                double* d_sum, int64_t* d_cnt, void* d_ws, void* stream);

/* ---- img.log_normalize (MxIF.py:416-455) ------------------------------------
 * out = log10(x * inv_mean[c] + pseudoval), HWC, fp32 out. */
int mw_lognorm(const void* d_img, int dtype, int64_t n_pix, int C,
               const float* d_inv_mean, float pseudoval, float* d_out, void* stream);

/* ---- img.blurring('gaussian', sigma) (MxIF.py:375-394) ----------------------
 * Separable Gaussian, per channel, edge-replicate ('nearest'), radius r =
 * int(4*sigma+0.5) <= 32, taps h_w[0..2r] (scipy _gaussian_kernel1d).
 * Optional fused log-normalise prologue when d_inv_mean != NULL.  HWC in,
 * HWC fp32 out (out must not alias in).  Even C and r <= 12: single
 * streaming pass (register ring); otherwise two passes through d_ws
 * (mw_blur_ws_bytes). */
size_t mw_blur_ws_bytes(int H, int W, int C, int radius);
int mw_blur(const void* d_img, int dtype, int H, int W, int C,
            const float* d_inv_mean, float pseudoval,
            const float* h_w, int radius, float* d_out, void* d_ws, void* stream);

/* ---- img.downsample(fact, np.mean) (MxIF.py:494-517) ------------------------
 * block mean over fact x fact, zero padded to a multiple of fact, pad zeros
 * included.  HWC in, fp32 HWC out of ceil(H/f) x ceil(W/f) x C. */
int mw_block_mean(const void* d_img, int dtype, int H, int W, int C, int fact,
                  float* d_out, void* stream);

/* ---- mask row-major rank → pixel (MxIF.py:486-488) --------------------------
 * d_rank2pix[r] = flat index of the r-th pixel with mask != 0.  d_count gets
 * the number of such pixels (int64 on device). */
size_t mw_mask_rank_ws_bytes(int64_t n_pix);
int mw_mask_rank(const uint8_t* d_mask, int64_t n_pix, uint32_t* d_rank2pix,
                 int64_t* d_count, void* d_ws, void* stream);

/* The same rank as a compact index (img.subsample_pixels' mask gather,
 * MxIF.py:486-488, without a rank -> pixel table): per 64-pixel word its mask
 * bits and the tissue pixels before it, per 64 ranks the word holding the
 * first: mw_rank_index_bytes(n_pix) bytes (~n_pix / 6), d_count = M.  The *_ri
 * forms below look a rank up in it (+ pix_off: the index of a slide band
 * inside a larger array) -- the random lookups of a subsample then stay in
 * the on-die caches instead of reading an HBM line per draw. */
size_t mw_rank_index_bytes(int64_t n_pix);
int mw_mask_rank_index(const uint8_t* d_mask, int64_t n_pix, void* d_index, int64_t* d_count, void* d_ws,
                       void* stream);

/* ---- subsample gather (MxIF.py:490-491) -------------------------------------
 * X[j, f] = img[rank2pix[idx[j]], feat[f]] as fp32 rows (S x F), plus per
 * block column statistics (count, mean, M2 in fp64) for StandardScaler.
 * d_img is fp32 HWC with C channels. */
size_t mw_gather_ws_bytes(int64_t S, int F);
int mw_gather_rows(const float* d_img, int C, const int32_t* d_feat, int F,
                   const int32_t* d_idx, const uint32_t* d_rank2pix, int64_t S,
                   float* d_X, void* d_ws, void* stream);
int mw_gather_rows_ri(const float* d_img, int C, const int32_t* d_feat, int F, const int32_t* d_idx,
                      const void* d_index, int64_t n_pix, int64_t pix_off, int64_t S, float* d_X, void* d_ws,
                      void* stream);
/* The draws as pixels: d_idx[j] = pixel of rank d_idx[j] (+ pix_off) through
 * the rank index, in place -- a pass over the draws that keeps the random
 * lookups in the on-die caches (it runs beside the blur); then
 * mw_gather_rows_px reads X[j, f] = img[d_pix[j], feat[f]] with no lookup.
 * Same rows and records as mw_gather_rows over the same draws. */
int mw_rank_to_pixel_ri(int32_t* d_idx, int64_t S, const void* d_index, int64_t n_pix, int64_t pix_off,
                        void* stream);
int mw_gather_rows_px(const float* d_img, int C, const int32_t* d_feat, int F, const int32_t* d_pix, int64_t S,
                      float* d_X, void* d_ws, void* stream);
/* Column statistics of rows already in X (same per-block records as
 * mw_gather_rows, same order: identical numbers for identical rows); then
 * mw_col_stats_finalize. */
int mw_col_stats_rows(const float* d_X, int64_t S, int F, void* d_ws, void* stream);

/* ---- fused blur + subsample (MxIF.py:375-394 + 457-492, MILWRM.py:1716-1733)
 * The subsample rows are written by the blur itself, so the blurred slide is
 * never stored:
 *   mw_sample_map:      slots[2p], slots[2p+1] = the first two sample slots j
 *                       of pixel p (rank2pix[idx[j]] == p; -1 where absent;
 *                       d_slots holds mw_sample_slot_elems(n_pix) int32), the
 *                       later slots of p on the overflow list d_ovf (S + 1
 *                       int32: [0] = count, then the slots);
 *   mw_blur_sample:     lognorm + blur of the slide; X[j, f] = blurred[p,
 *                       feat[f]] for both table slots j of every sampled p;
 *   mw_sample_overflow: X[j] = X[slots[2p]] for the overflow slots;
 * then mw_col_stats_rows.  X ends up equal to mw_blur + mw_gather_rows.
 * mw_blur_sample returns MW_EUNSUPPORTED (nothing launched) for shapes the
 * fused kernel does not take (odd C, C > 64, radius 0 or > 8, F > C rounded
 * up to 16, no log-normalise); the caller then materialises the blur. */
size_t mw_sample_slot_elems(int64_t n_pix);
int mw_sample_map(const int32_t* d_idx, const uint32_t* d_rank2pix, int64_t S, int64_t n_pix,
                  int32_t* d_slots, int32_t* d_ovf, void* stream);
int mw_blur_sample(const void* d_img, int dtype, int H, int W, int C, const float* d_inv_mean,
                   float pseudoval, const float* h_weights, int radius, const int32_t* d_slots,
                   int64_t S, const int32_t* d_feat, int F, float* d_X, void* stream);
int mw_sample_overflow(const int32_t* d_idx, const uint32_t* d_rank2pix, const int32_t* d_slots,
                       const int32_t* d_ovf, int64_t S, int F, float* d_X, void* stream);
int mw_sample_map_ri(const int32_t* d_idx, const void* d_index, int64_t n_index, int64_t pix_off, int64_t S,
                     int64_t n_pix, int32_t* d_slots, int32_t* d_ovf, void* stream);
int mw_sample_overflow_ri(const int32_t* d_idx, const void* d_index, int64_t n_index, int64_t pix_off,
                          const int32_t* d_slots, const int32_t* d_ovf, int64_t S, int F, float* d_X,
                          void* stream);
/* Row-window form for a slide streamed in row bands (img.subsample_pixels over a
 * slide that is not resident in HBM, MxIF.py:457-492): d_img holds the H rows
 * [row_off, row_off + H) of the slide (a band and its +-radius halo rows);
 * only its rows [r0, r1) are blurred into samples, d_slots is the whole
 * slide's table (indexed by slide pixel).  Calling it for bands that tile the
 * slide writes exactly the rows of one mw_blur_sample over the whole slide. */
int mw_blur_sample_rows(const void* d_img, int dtype, int H, int W, int C, int64_t row_off, int r0, int r1,
                        const float* d_inv_mean, float pseudoval, const float* h_weights, int radius,
                        const int32_t* d_slots, int64_t S, const int32_t* d_feat, int F, float* d_X,
                        void* stream);
/* The same rows from a band already blurred into fp32 (any shape the fused
 * kernel does not take): d_band = n_pix HWC fp32 pixels, slide pixels
 * [pix_off, pix_off + n_pix); X[j] = band[p - pix_off, feat] for both table
 * slots j of every sampled pixel p of the band. */
int mw_slot_gather(const float* d_band, int C, int64_t n_pix, int64_t pix_off, const int32_t* d_slots,
                   int64_t S, const int32_t* d_feat, int F, float* d_X, void* stream);

/* Chan-merge the per-block stats of the last gather(s) into d_stats =
 * [n, mean[F], M2[F]] (fp64).  `n_parts` gathers may be accumulated: pass
 * the workspace of each; merged in call order. */
int mw_col_stats_finalize(const void* d_ws, int64_t S, int F, double* d_stats,
                          int accumulate, void* stream);
/* Column max |x| of the same rows (fp32 d_out[F]; maxed into d_out when
 * accumulating): the fixed-point exponents of mw_lloyd_pass come from it
 * (replaces a separate mw_col_absmax pass over the rows). */
int mw_col_stats_absmax(const void* d_ws, int64_t S, int F, float* d_out, int accumulate,
                        void* stream);

/* ---- legacy MT19937 subsample indices (MxIF.py:484,490) ---------------------
 * Bit-exact np.random.RandomState(seed).randint(0, high, size) (== choice),
 * masked rejection on MT19937.  Host implementation (single thread). */
int mw_legacy_randint_host(uint32_t seed, int64_t high, int64_t size, int32_t* h_out);

/* ---- device MT19937 with jump-ahead (bit-exact legacy randint) -------------
 * One-time host tables: h_j(t) = t^(L*2^j) mod phi(t), j < J (312 uint64 per
 * polynomial; phi = characteristic polynomial of the MT19937 transition,
 * found by Berlekamp-Massey).  The device builds the start state of every
 * L-word segment by a parallel prefix of jumps (block Horner), then every
 * workgroup regenerates, tempers and filters its segment; accepted draws are
 * compacted in stream order.  Output identical to mw_legacy_randint_host. */
int mw_mt_jump_tables(int64_t L, int J, uint64_t* h_tables);
int mw_mt_jump_host(const uint32_t* h_state_in, const uint64_t* h_poly, uint32_t* h_state_out);
int mw_mt_seed_state(uint32_t seed, uint32_t* h_state);
size_t mw_legacy_randint_ws_bytes(int64_t high, int64_t size, int64_t L);
int mw_legacy_randint_device(uint32_t seed, int64_t high, int64_t size, const uint64_t* d_tables,
                             int J, int64_t L, int32_t* d_out, int64_t* d_total, void* d_ws,
                             void* stream);
/* The same in two halves.  The segment start states depend only on (seed, L):
 * every image of a batch reseeds with 16 (MxIF.py:484), so a caller may build
 * them once (mw_mt_segment_states, W x 624 uint32 in d_states) and draw any
 * (high, size) needing at most W segments from them
 * (mw_legacy_randint_from_states; workspace mw_legacy_randint_gen_ws_bytes). */
int64_t mw_legacy_randint_segments(int64_t high, int64_t size, int64_t L);
int mw_mt_segment_states(uint32_t seed, int64_t W, const uint64_t* d_tables, int J,
                         uint32_t* d_states, void* stream);
size_t mw_legacy_randint_gen_ws_bytes(int64_t high, int64_t size, int64_t L);
int mw_legacy_randint_from_states(const uint32_t* d_states, int64_t W_avail, int64_t high,
                                  int64_t size, int64_t L, int32_t* d_out, int64_t* d_total,
                                  void* d_ws, void* stream);

/* ---- k-means++ (sklearn _kmeans.py:174-272) ---------------------------------
 * Rows are scaled on the fly: x' = (x - mu) * inv_sigma  (fp64 affine).
 * The workspace keeps the closest distance of every row (fp64) and per-block
 * / per-64-row-tile sums of the step's T trial arrays (the arrays themselves
 * are recomputed where the search needs them, never stored).
 * Single device: mw_kpp_init + (k-1) x mw_kpp_step + mw_kpp_indices keep all
 * state on the device (no host synchronisation between steps).
 * Row-sharded (one shard per rank): mw_kpp_init, then per step c
 * mw_kpp_pots → (host all-gather, global argmin, targets) → mw_kpp_search
 * with explicit local targets → (host all-reduce of candidate rows) →
 * mw_kpp_trial. */
size_t mw_kpp_ws_bytes(int64_t S, int T);
/* distances to one center row (raw fp32 features, device) */
int mw_kpp_init(const float* d_X, int64_t S, int F, const double* d_mu,
                const double* d_inv, const float* d_center_row, int T, void* d_ws,
                void* stream);
/* single-device step for center c (1..k-1); h_u = the T uniform draws */
int mw_kpp_step(const float* d_X, int64_t S, int F, const double* d_mu,
                const double* d_inv, int c, const double* h_u, int T,
                void* d_ws, void* stream);
/* single-device: chosen indices (int64 [k]) into d_idx_out */
int mw_kpp_indices(const void* d_ws, int64_t S, int T, int k, int64_t* d_idx_out,
                   void* stream);
/* single-device last step (c = k-1 >= 2, mw_kpp_fold_supported) with the
 * first Lloyd E-step folded into its pass (the fit driver's default; no
 * reference counterpart: it replaces the pass over the rows that sklearn's
 * first lloyd_iter_chunked_dense makes after _kmeans_plusplus, _kmeans.py:
 * 624-752): besides the step's trial sums, every row gets its label among the
 * k-1 centers so far (labels), distance bounds valid whichever candidate wins
 * (ub, lb), the bits "moves to the new center if candidate t wins" (moved,
 * S bytes) and the base cluster sums as Lloyd block records (d_rec,
 * mw_kpp_fold_rec_bytes) folded into d_rec_out (mw_lloyd_rec_len(k, F) fp64).
 * first = the first center's row; d_a32 / d_b32 / d_qexp as mw_lloyd_pass;
 * d_centers_img = 8 KB of device scratch.  After mw_kpp_indices, the winner's
 * moved rows are listed (mw_lloyd_list_moved) and a mode-0 mw_lloyd_pass of
 * kind 8 over the k final centers moves them: its record plus d_rec_out's
 * sums and counts are those of a kind-0 first pass, bit for bit. */
int mw_kpp_step_fold(const float* d_X, int64_t S, int F, const double* d_mu, const double* d_inv, int c,
                     const double* h_u, int T, void* d_ws, int64_t first, const float* d_a32,
                     const float* d_b32, const int32_t* d_qexp, uint8_t* d_labels, float* d_ub, float* d_lb,
                     uint8_t* d_moved, void* d_centers_img, double* d_rec, double* d_rec_out, void* stream);
size_t mw_kpp_fold_rec_bytes(int64_t S, int k, int F);
/* 1 when mw_kpp_step_fold takes (k, F, T): 3 <= k <= 16, T <= 4, F <= 32 and
 * its LDS fits four blocks per CU */
int mw_kpp_fold_supported(int k, int F, int T);
/* device address of the k-means++ workspace's selected-array index (int) */
const int* mw_kpp_best_ptr(const void* d_ws, int64_t S, int T);
/* sharded: local potentials (fp64) of the arrays finished before step c
 * (1 array after init, T after a trial) */
int mw_kpp_pots(const void* d_ws, int64_t S, int T, int c, double* d_pots, void* stream);
/* sharded: search array `best` of step c-1 (recomputed from the rows where
 * needed) for local targets d_rv[T] (fp64, < 0 = not on this shard); local
 * row indices (int64, -1 if skipped) */
int mw_kpp_search(const float* d_X, int64_t S, int F, void* d_ws, int T, int c, int best,
                  const double* d_rv, int64_t* d_local_idx, void* stream);
/* sharded: pass of step c against candidate rows d_rows (T x F raw fp32),
 * after folding in array `best` of step c-1 */
int mw_kpp_trial(const float* d_X, int64_t S, int F, const double* d_mu,
                 const double* d_inv, int c, int best, const float* d_rows, int T,
                 void* d_ws, void* stream);

/* ---- Lloyd iteration (sklearn lloyd_iter_chunked_dense, _k_means_lloyd.pyx:23-218;
 *      _inertia_dense, _k_means_common.pyx:94-124) -----------------------------
 * One pass over S rows for n independent fits (n = 1 for KMeans.fit, all k of
 * the find_optimal_k sweep, MILWRM.py:29-90, batched).  Rows x' = x*a[f] +
 * b[f] (fp32, the folded StandardScaler); labels = argmin of the direct
 * squared distance, lowest index on ties.  Per fit the caller owns:
 *   centers   k x F fp32 (scaled space)
 *   labels    S uint8 (255 = none yet; k <= 64)
 *   ub, lb    S fp32 distance bounds (mode 0; contents ignored where label = 255)
 *   drift     k fp32 |c_j - c_j(previous pass)|, rounded up (0 on the first pass)
 *   half_sep  k fp32 0.5 * min_{i != j} |c_i - c_j|, rounded down (+inf for k = 1)
 *   drift_max max_j drift[j]
 *   ws        mw_lloyd_ws_bytes(S, k, F) bytes of per-block records and row lists
 *             (mw_lloyd_ws_bytes_kinds(S, k, F, 0): records only, no kind 4)
 *   out       mw_lloyd_rec_len(k, F) fp64, the fixed-order fold of the records:
 *             [dQ_hi k*F | dQ_lo k*F | dcount k | changed | recomputed | in_hi | in_lo]
 *             (mode 0: in_hi * 2^32 + in_lo = the rows whose features the pass
 *             read -- all of them for kinds 0 / 1, the queued or listed ones
 *             for kinds 2 / 4; 0 for the dense kinds)
 * mode 0: E-step (rows whose bounds prove the label skip the distances) and
 *         the M-step change of the per-cluster sums: every raw value rounds
 *         once to q = rint(x * 2^qexp[f]) (|q| < 2^41) and a relabelled row
 *         moves its q from the old cluster to the new one; dQ = dQ_hi * 2^32 +
 *         dQ_lo (exact integers), dcount the change of the cluster sizes.
 * mode 1: full E-step (labels updated) and inertia = (in_hi * 2^32 + in_lo) *
 *         2^-inertia_exp of the new labels (each distance rounded once to that
 *         fixed point);  mode 2: inertia of the given labels.
 * Every sum is an integer sum: identical for any row order or sharding.
 * `kind` (mode 0): 0 = first pass (every label 255: sums of all rows on the
 * fp64 matrix cores), 1 = stream every row, the bounds skip the E-step per
 * row (most rows undecided), 2 = stream the row state only and read just the
 * undecided rows (few undecided), chunk by chunk in one kernel, 4 = the same
 * as two kernels: the bound test over the whole row state lists the undecided
 * rows, then a second launch reads only those (falls back to 2 when S >= 2^31;
 * ws then also holds the lists).  Same results for any kind.
 * k <= 64, F <= 64, n <= 24.  h_fits is a host array. */
typedef struct mw_lloyd_fit {
  const float* centers;
  const float* drift;
  const float* half_sep;
  uint8_t* labels;
  float* ub;
  float* lb;
  void* ws;
  double* out;
  int k;
  float drift_max;
  int inertia_exp;  /* modes 1 / 2: inertia fixed point 2^-inertia_exp */
} mw_lloyd_fit;
int mw_lloyd_rec_len(int k, int F);
size_t mw_lloyd_ws_bytes(int64_t S, int k, int F);
/* The workspace without the kList row lists (4 bytes per row) when with_list
 * is 0 or S >= 2^31 (kind 4 falls back to kind 2 there): a fit whose passes
 * never take kind 4 (MW_LLOYD_LIST=0) needs only its per-block records. */
size_t mw_lloyd_ws_bytes_kinds(int64_t S, int k, int F, int with_list);
/* kind 8 = kind 4 over row lists written beforehand into ws: the rows of
 * d_moved (mw_kpp_step_fold) whose bit *d_best is set (S < 2^31) */
int mw_lloyd_list_moved(const uint8_t* d_moved, const int* d_best, int64_t S, int F, int k, void* d_ws,
                        void* stream);
int mw_lloyd_pass(const float* d_X, int64_t S, int F, const float* d_a, const float* d_b,
                  const int32_t* d_qexp, int n, const mw_lloyd_fit* h_fits, int mode, int kind,
                  void* stream);
/* per-column max |x| of S x F fp32 rows (F <= 16384), fp32 out */
int mw_col_absmax(const float* d_X, int64_t S, int F, float* d_out, void* stream);
/* The same maxima folded into d_out (fp32 [F], >= 0) without resetting it:
 * the column maxima of a slide processed band after band. */
int mw_col_absmax_acc(const float* d_X, int64_t S, int F, float* d_out, void* stream);

/* Per pass of the calling thread's last mw_kmeans_fit / mw_kmeans_fit_async
 * (k-means++ passes excluded): 4 int64 each -- kind (0..8; 10 + mode for the
 * final pass), rows relabelled, rows recomputed, rows whose features the pass
 * read -- up to cap passes into out; returns the number of passes.  For the
 * measurement of the bytes a pruned fit really reads (bench.py). */
int mw_kmeans_fit_history(int64_t* out, int cap);

/* ---- whole fit: sklearn KMeans(algorithm="lloyd").fit (_kmeans.py:1427-1554)
 * Replaces the reference's `KMeans(n_clusters=k, random_state=seed).fit(X)`
 * (MILWRM.py:706-737 find_tissue_regions; MILWRM.py:29-54 kMeansRes) for a
 * caller of the C ABI; KMeans.fit of the Python package runs through it too
 * (single process, one k-means++ init from an int seed or an explicit init).
 * Rows: S x F raw fp32 on the device, scaled on the fly x' = (x - mu) * inv
 * (fp64 host arrays; mu = 0, inv = 1 for rows that are already standardised).
 * k-means++ seeded from RandomState(seed) (or the k x F scaled centers
 * h_init, then no seeding), Lloyd with sklearn's strict and tolerance
 * convergence (tol relative: tol * mean of the scaled rows' per-feature
 * variance, from h_feature_var[F] when given, else computed on the device),
 * empty-cluster relocation, the extra E-step and inertia.  h_xmax[F]: the
 * rows' column max |x| when the producer already has it (else one pass).
 * Outputs: d_labels (S uint8, device), h_centers (k x F fp64, scaled space),
 * *h_inertia, *h_n_iter, h_init_idx (k int64, may be NULL; untouched with
 * h_init).  d_ws: mw_kmeans_fit_ws_bytes(S, F, k) bytes of device workspace
 * (NULL: allocated and freed inside).  Caps: 1 <= k <= 64 (uint8 labels,
 * centers in LDS / scalar registers), 1 <= F <= 64 (one feature per lane of
 * a wave); S >= k.  Synchronises `stream` before returning. */
size_t mw_kmeans_fit_ws_bytes(int64_t S, int F, int k);
int mw_kmeans_fit(const float* d_X, int64_t S, int F, const double* h_mu,
                  const double* h_inv, const double* h_feature_var, const float* h_xmax,
                  int k, const double* h_init, uint32_t seed, int max_iter, double tol,
                  uint8_t* d_labels, double* h_centers, double* h_inertia, int* h_n_iter,
                  int64_t* h_init_idx, void* d_ws, size_t ws_bytes, void* stream);
/* The same fit with an asynchronous end: returns once the final E-step
 * (labels, inertia) is queued on `stream`, so the caller can queue the label
 * pass behind it without a host round trip (the centers, n_iter and k-means++
 * indices are final at return; d_labels is stream-ordered).  The final pass's
 * record (mw_lloyd_rec_len(k, F) fp64) is copied to the caller's PAGE-LOCKED
 * h_final_rec when the stream gets there; after synchronising the stream the
 * inertia is (rec[rl - 2] * 2^32 + rec[rl - 1]) * 2^-(*h_inertia_exp).  A
 * d_ws of NULL (workspace allocated inside) makes the end synchronous, with
 * the same outputs. */
int mw_kmeans_fit_async(const float* d_X, int64_t S, int F, const double* h_mu,
                        const double* h_inv, const double* h_feature_var, const float* h_xmax,
                        int k, const double* h_init, uint32_t seed, int max_iter, double tol,
                        uint8_t* d_labels, double* h_centers, int* h_n_iter, int64_t* h_init_idx,
                        void* d_ws, size_t ws_bytes, double* h_final_rec, int* h_inertia_exp,
                        void* stream);

/* ---- batched fits: the find_optimal_k sweep's Lloyd iterations ----------------
 * Replaces kMeansRes' per-k `KMeans(n_clusters=k, random_state=seed).fit(X)`
 * (MILWRM.py:29-54, called per k by find_optimal_k MILWRM.py:659-704) for n
 * fits over the same rows, from given k x F scaled initial centers (h_init,
 * the fits' blocks concatenated; the caller seeds them with mw_kpp_*): one
 * iteration = one mw_lloyd_pass per pass kind for every fit still running,
 * one record download; each fit returns exactly what mw_kmeans_fit returns
 * for it alone (strict / tolerance convergence, tol absolute here,
 * relocation, the extra E-step, inertia).  Rows as mw_lloyd_pass (d_a32,
 * d_b32, d_qexp on the device; h_a32, h_b32, h_qexp, the column max |x|
 * h_xmax[F] and the scaler h_mu / h_inv on the host).  Per fit g the caller
 * owns d_labels[g] (S uint8, filled with 255), d_ub[g], d_lb[g] (S fp32) and
 * d_ws[g] (mw_lloyd_ws_bytes); d_par: sum of (k F + 2k) fp32, d_out: sum of
 * mw_lloyd_rec_len(k, F) fp64.  Pass-kind policy: first_kind (0 or 3),
 * queue_kind (2 or 4) below queue_below of the rows recomputed, the dense pass
 * while >= dense_min fits run (< 0: never), nobound != 0: no bound ever holds.
 * Outputs: h_centers (the fits' k x F fp64 blocks), h_inertia[n],
 * h_n_iter[n]; h_hist (may be NULL): per fit hist_cap x (changed, recomputed)
 * int64, h_hist_len[n] entries; h_timing (may be NULL, 30 doubles): 9 x
 * (launches, ms, algorithmic bytes) of the passes by mode-0 kind 0..6, mode 1,
 * mode 2, then (host intervals, their host ms: from a pass's records arriving
 * to the next pass queued, ms inside the caller's collectives).
 * Synchronises `stream`. */
int mw_lloyd_fits(const float* d_X, int64_t S, int F, const float* d_a32, const float* d_b32,
                  const int32_t* d_qexp, const float* h_a32, const float* h_b32,
                  const int32_t* h_qexp, const float* h_xmax, const double* h_mu,
                  const double* h_inv, int n, const int* h_k, const double* h_init,
                  uint8_t* const* d_labels, float* const* d_ub, float* const* d_lb,
                  void* const* d_ws, float* d_par, double* d_out, int max_iter, double tol,
                  int first_kind, int queue_kind, double queue_below, int dense_min,
                  int nobound, double* h_centers, double* h_inertia, int* h_n_iter,
                  int64_t* h_hist, int hist_cap, int* h_hist_len, double* h_timing,
                  void* stream);

/* ---- the same fits over row shards (one process per GPU) ----------
 * Replaces the per-iteration loop of the row-sharded fit (MILWRM.py:706-737
 * find_tissue_regions, MILWRM.py:29-90 the k sweep, with the pixels of a
 * cohort split over the GPUs of a node): mw_lloyd_fits where each rank holds
 * its S rows (ranks hold consecutive row ranges, `row_offset` its first global
 * row, `rows_total` all of them) and the caller supplies the collectives.  Per
 * pass ONE in-place sum over the ranks of the fits' records (exact
 * fixed-point limbs, so the centers, labels, n_iter and inertia are bitwise
 * those of one process over all rows); a rare empty-cluster relocation adds
 * one all-gather of 2n values and one all-sum of n (F + 1) values.  Every
 * rank calls with the same n, k, init, tolerances and policy, and S >= 1.
 * The messages live in the caller's device buffer d_msg (fp64, msg_len >=
 * mw_lloyd_fits_msg_len(sum of mw_lloyd_rec_len, F, world) elements), with
 * d_out == d_msg (the records at offset 0); the callbacks address it by
 * element offsets, return 0 on success, and must order the collective after
 * the work queued on `stream` and the later work on `stream` after it (the
 * Python package binds them to torch.distributed: RCCL on the current
 * stream, or gloo through host copies; a C caller to ncclAllReduce /
 * ncclAllGather on `stream`).  A failing callback ends the call with MW_EHIP. */
typedef struct mw_fit_comm {
  void* ctx;
  int world;
  int rank;
  int64_t rows_total;
  int64_t row_offset;
  double* d_msg;
  int64_t msg_len;
  /* d_msg[off, off + n) <- its sum over the ranks */
  int (*all_reduce_sum)(void* ctx, int64_t off, int64_t n, void* stream);
  /* d_msg[out_off + r n, out_off + (r + 1) n) <- rank r's d_msg[in_off, in_off + n) */
  int (*all_gather)(void* ctx, int64_t in_off, int64_t n, int64_t out_off, void* stream);
} mw_fit_comm;
int64_t mw_lloyd_fits_msg_len(int64_t rec_total, int F, int world);
int mw_lloyd_fits_sharded(const float* d_X, int64_t S, int F, const float* d_a32, const float* d_b32,
                          const int32_t* d_qexp, const float* h_a32, const float* h_b32,
                          const int32_t* h_qexp, const float* h_xmax, const double* h_mu,
                          const double* h_inv, int n, const int* h_k, const double* h_init,
                          uint8_t* const* d_labels, float* const* d_ub, float* const* d_lb,
                          void* const* d_ws, float* d_par, double* d_out, int max_iter, double tol,
                          int first_kind, int queue_kind, double queue_below, int dense_min,
                          int nobound, double* h_centers, double* h_inertia, int* h_n_iter,
                          int64_t* h_hist, int hist_cap, int* h_hist_len, double* h_timing,
                          const mw_fit_comm* comm, void* stream);

/* ---- empty-cluster relocation support (_k_means_common.pyx:181-226) ---------
 * fp64 distance of every row to centers[labels]; returns the n largest
 * (value desc, index asc) into d_top_idx / d_top_val (n <= 64). */
size_t mw_farthest_ws_bytes(int64_t S);
int mw_farthest(const float* d_X, int64_t S, int F, const float* d_a,
                const float* d_b, const double* d_centers, int k,
                const uint8_t* d_labels, int n, int64_t* d_top_idx,
                double* d_top_val, void* d_ws, void* stream);

/* ---- label + confidence pass (MILWRM.py:237-277, 389-450) -------------------
 * Over n_pix HWC fp32 pixels (C channels, features d_feat[F]):
 * label = argmin_j ||x' - c_j||^2 (x' = x*a + b), conf = (d2 - d1)/d2;
 * mask == 0 → label -1, conf NaN.  Per-block records per label go to d_ws,
 * mw_assign_reduce folds them into d_dom (fp64 [3k]) = [conf hi k | conf lo k
 * | count k]: the per-domain sum of the confidences in exact fixed point,
 * sum of rint(conf * 2^32) = hi * 2^32 + lo, 0 <= lo < 2^32 (value = that * 2^-32; NaN limbs
 * when a confidence of the domain is NaN), and the pixel counts.  Every entry
 * is an integer-valued fp64 below 2^53, so records of several launches (row
 * bands, ranks) add exactly: the domain sums do not depend on how the pixels
 * were split (reference: MILWRM.py:447-449, np.mean per domain). */
size_t mw_assign_ws_bytes(int64_t n_pix, int k);
int mw_assign_conf(const float* d_img, int C, const int32_t* d_feat, int F,
                   const float* d_a, const float* d_b, const float* d_centers,
                   int k, const uint8_t* d_mask, int64_t n_pix,
                   int8_t* d_label, float* d_conf, void* d_ws, void* stream);
/* Fused blur + label/confidence (features = all C channels in order): the
 * same labels and confidences as mw_blur then mw_assign_conf, without the
 * blurred slide in HBM; k <= 16 (k <= 8 for C <= 16).  d_mask must be
 * readable 128 bytes past n_pix.  MW_EUNSUPPORTED (nothing launched) as for
 * mw_blur_sample.  mw_domain_records then writes mw_assign_conf's per-block
 * records from the label/confidence maps (same partition and order), for
 * mw_assign_reduce. */
int mw_blur_assign_conf(const void* d_img, int dtype, int H, int W, int C, const float* d_inv_mean,
                        float pseudoval, const float* h_weights, int radius, const float* d_a,
                        const float* d_b, const float* d_centers, int k, const uint8_t* d_mask,
                        int8_t* d_label, float* d_conf, void* stream);
/* Row-window form (a streamed slide band, as mw_blur_sample_rows): d_img
 * holds slide rows [row_off, row_off + H); rows [r0, r1) are labelled;
 * d_mask, d_label and d_conf are indexed by slide pixel. */
int mw_blur_assign_rows(const void* d_img, int dtype, int H, int W, int C, int64_t row_off, int r0, int r1,
                        const float* d_inv_mean, float pseudoval, const float* h_weights, int radius,
                        const float* d_a, const float* d_b, const float* d_centers, int k,
                        const uint8_t* d_mask, int8_t* d_label, float* d_conf, void* stream);
int mw_domain_records(const int8_t* d_label, const float* d_conf, int64_t n_pix, int C, int k,
                      void* d_ws, void* stream);
int mw_assign_reduce(const void* d_ws, int64_t n_pix, int k, double* d_dom,
                     void* stream);

/* ---- clustering QC statistics ------------------------------------------------
 * Replaces the per-domain loops of estimate_percentage_variance_mxif
 * (MILWRM.py:280-333, dc/dm sums), estimate_mse_mxif (MILWRM.py:453-515) and
 * their ST twins estimate_percentage_variance_st / estimate_mse_st
 * (MILWRM.py:518-554, 601-644; rows as a 1-pixel-wide image).
 * Over n_pix HWC fp32 pixels, x' = x[feat[f]]*a[f] + b[f], y = x' - pivot[f] (fp64).
 * Exact: every term is rounded to the two-level fixed point of its feature,
 * q = rint(v * 2^e) and r = rint((v * 2^e - q) * 2^38) (d_qexp, int32 [3F]: e
 * for (x' - c)^2 | for y | for y^2, chosen by the caller so that |q| <= 2^38),
 * and both levels are summed as integers, so the results do not depend on how
 * the pixels are split over launches (a slide blurred band by band gives the
 * materialised slide's bits) and keep ~2^-76 of the bound.
 * d_out (fp64, M = mw_domain_sse_out_len(k, F) = 4(kF + 2F) + k) =
 * [Q hi limbs | Q lo limbs | R hi limbs | R lo limbs of the NQ = kF + 2F
 * quantities: sum over label == d0+d of (x'_f - c_df)^2 (k x F), sum y_f (F),
 * sum y_f^2 (F, over every pixel)] | pixel count per label (k); with
 * Q = Qhi * 2^32 + Qlo and R likewise, value = (Q + R * 2^-38) * 2^-e.
 * accumulate != 0 adds to d_out (band after
 * band) instead of overwriting it.  Labels outside [d0, d0+k) (other
 * domains; masked / NaN tissue_ID → -1) add to the sums only.  1 <= k <= 20
 * domains per call (more: several calls with d0 = 0, 20, 40, ...), 1 <= F <=
 * 256, at most 2^24 pixels per internal block (n_pix <= ~3.4e10). */
int mw_domain_sse_out_len(int k, int F);
size_t mw_domain_sse_ws_bytes(int64_t n_pix, int k, int F);
int mw_domain_sse(const float* d_img, int C, const int32_t* d_feat, int F, const double* d_a,
                  const double* d_b, const double* d_pivot, const double* d_centers,
                  const int32_t* d_qexp, int k, int d0, const int8_t* d_label, int64_t n_pix,
                  double* d_out, int accumulate, void* d_ws, void* stream);
/* The same over fp64 rows (n_pix x C, row-major): the ST estimators'
 * cluster_data (estimate_percentage_variance_st / estimate_mse_st,
 * MILWRM.py:518-554, 601-644), which the reference holds in float64. */
int mw_domain_sse_f64(const double* d_rows, int C, const int32_t* d_feat, int F, const double* d_a,
                      const double* d_b, const double* d_pivot, const double* d_centers,
                      const int32_t* d_qexp, int k, int d0, const int8_t* d_label, int64_t n_pix,
                      double* d_out, int accumulate, void* d_ws, void* stream);

/* ---- ST feature blur (blur_features_st, ST.py:25-77) --------------------------
 * out[i, f] = mean of X[j, f] over j in (nonzero columns of row i of the CSR
 * spatial graph, in column order) + [i] (a self-loop therefore counts twice,
 * as in the reference), NaN entries skipped (pandas mean); NaN if none.
 * CSR: d_indptr (n+1, int64), d_indices (int32); X, out: n x F fp64 row-major. */
int mw_neighbor_mean(const int64_t* d_indptr, const int32_t* d_indices, int64_t n, const double* d_X,
                     int F, double* d_out, void* stream);

/* ---- synthetic slide generator (benchmark input; SURVEY §8d shape) ----------
 * uint16 HWC + uint8 mask: Voronoi domains (seeds given), per-domain channel
 * profiles, gamma-like multiplicative noise from a counter-based hash. */
int mw_synth_slide(int H, int W, int C, const float* d_seed_yx, int n_seeds,
                   const float* d_profiles, int n_domains, int shape_k,
                   int bg_rows, uint64_t seed, uint16_t* d_img, uint8_t* d_mask,
                   void* stream);
/* Rows [y0, y1) of the same H x W slide into d_img ((y1-y0) x W x C) and, when
 * d_mask != NULL, d_mask ((y1-y0) x W): bit for bit those rows of
 * mw_synth_slide (every value is a hash of its slide pixel index).  The
 * stand-in for reading a slide band from storage in the streamed benchmark. */
int mw_synth_rows(int H, int W, int C, int y0, int y1, const float* d_seed_yx, int n_seeds,
                  const float* d_profiles, int n_domains, int shape_k, int bg_rows, uint64_t seed,
                  uint16_t* d_img, uint8_t* d_mask, void* stream);

/* ---- reference-format label-pass outputs (host) ----------------------------
 * tissue_IDs[i] / confidence_IDs[i] as the reference holds them: float64 H x W
 * with NaN outside the mask (MILWRM.py:275-276, 444-445), from the compact
 * device outputs copied to host memory (int8 labels, -1 = no domain; fp32
 * confidences).  Host loops on `threads` threads (<= 1: the calling thread). */
int mw_host_labels_f64(const int8_t* h_lab, int64_t n, double* h_out, int threads);
int mw_host_f32_to_f64(const float* h_in, int64_t n, double* h_out, int threads);

#ifdef __cplusplus
}
#endif
#endif /* MILWRM_AMD_H */
