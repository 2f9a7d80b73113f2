"""CPU-only tests: the C-ABI library loads and exports every declared symbol,
the host-side RNG plumbing is bit-exact with NumPy, and the host API checks
behave like the reference's (no compute calls — no GPU here)."""
import ctypes
import os
import re

import numpy as np
import pandas as pd
import pytest

from tests.conftest import ROOT


def _declared_symbols():
    txt = open(os.path.join(ROOT, "include", "milwrm_amd.h")).read()
    return sorted(set(re.findall(r"\b(mw_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_all_header_symbols():
    from milwrm_amd import _native as N

    lib = N.load()
    syms = _declared_symbols()
    assert len(syms) >= 25
    for s in syms:
        assert hasattr(lib, s), f"missing export {s}"
    assert set(syms) == set(N.EXPORTED), "ctypes prototypes out of sync with include/milwrm_amd.h"
    assert lib.mw_version() >= 10000


def test_legacy_randint_host_bit_exact():
    from milwrm_amd.rng import subsample_indices

    for M, fr in [(6540, 0.2), (1, 0.9), (2, 0.5), (1000, 0.5), (2**20, 0.01), (2**20 + 1, 0.01),
                  (123457, 0.3), (2**31 - 1, 1e-6), (85_000_000, 0.001)]:
        np.random.seed(16)
        ref = np.random.choice(M, int(M * fr))
        got = subsample_indices(M, fr, 16)
        np.testing.assert_array_equal(got, ref, err_msg=f"M={M}")


def test_first_center_index_matches_numpy_choice():
    from milwrm_amd.rng import first_center_index, kpp_draws

    for n in (1, 2, 3, 5, 17, 6297, 65537, 100003, 999999, 2**20 + 7):
        for seed in (18, 0, 12345):
            ref = np.random.RandomState(seed).choice(n, p=np.ones(n) / n)
            u0, _ = kpp_draws(seed, 2, 2)
            assert first_center_index(n, u0) == ref, (n, seed)


def test_kpp_draws_consume_like_sklearn():
    from milwrm_amd.rng import kpp_draws

    rs = np.random.RandomState(18)
    u0 = rs.random_sample()
    steps = [rs.uniform(size=4) for _ in range(7)]
    a0, a = kpp_draws(18, 8, 4)
    assert a0 == u0
    for x, y in zip(a, steps):
        np.testing.assert_array_equal(x, y)


def test_gaussian_taps_match_scipy():
    import scipy.ndimage as ndi

    from milwrm_amd.device import gaussian_taps

    for s in (0.5, 1.0, 2.0, 3.7):
        w = gaussian_taps(s)
        imp = np.zeros(101)
        imp[50] = 1.0
        ref = ndi.gaussian_filter1d(imp, s, mode="nearest", truncate=4.0)
        r = (len(w) - 1) // 2
        np.testing.assert_allclose(w[::-1], ref[50 - r:50 + r + 1], rtol=1e-6)


def test_img_and_labeler_validation_like_reference():
    import milwrm_amd as M

    with pytest.raises(AssertionError, match="enough dimensions"):
        M.img(np.zeros(5))
    with pytest.raises(Exception, match="Channels must be given in a list"):
        M.img(np.zeros((4, 4, 2)), channels=("a", "b"))
    with pytest.raises(AssertionError, match="Shape of mask"):
        M.img(np.zeros((4, 4, 2)), mask=np.ones((3, 4)))
    im = M.img(np.zeros((4, 4, 2)))
    assert im.ch == ["ch_0", "ch_1"] and im.n_ch == 2
    with pytest.raises(Exception, match="Image_df must be given"):
        M.mxif_labeler(pd.DataFrame({"Img": [im], "batch": ["a"], "mean": [[1]], "pixels": [1]}))
    df = pd.DataFrame({"Img": [im, "p"], "batch_names": ["a", "a"], "mean estimators": [[1], [1]],
                       "pixels": [1, 1]})
    with pytest.raises(Exception, match="Img column"):
        M.mxif_labeler(df)
    lab = M.mxif_labeler(df.iloc[:1])
    with pytest.raises(Exception, match="No cluster data found"):
        lab.find_optimal_k()
    with pytest.raises(Exception, match="No cluster data found"):
        lab.find_tissue_regions(k=3)
    with pytest.raises(Exception, match="filter name should be"):
        im.blurring("nope")
    with pytest.raises(TypeError):
        im.blurring("median", sigma=2)  # the reference's median branch raises (MxIF.py:403)


def test_scaler_constant_feature_rule():
    from milwrm_amd.kmeans import StandardScaler

    X = np.column_stack([np.arange(10.0), np.full(10, 3.0)])
    s = StandardScaler().fit(X)
    assert s.scale_[1] == 1.0
    st = np.concatenate([[10.0], X.mean(0), X.var(0) * 10])
    s2 = StandardScaler.from_stats(st)
    np.testing.assert_allclose(s2.scale_, s.scale_)


def test_mt_jump_tables_and_host_jump_match_sequential_stream():
    """phi from Berlekamp-Massey + t^(L 2^j) mod phi: jumping the seeded
    window by L*2^j equals advancing the generator sequentially."""
    from milwrm_amd import _native as N
    from oracle.milwrm_oracle import mt19937_init

    L, J = 624 * 3, 3
    tab = np.zeros((J, 312), dtype=np.uint64)
    N.call("mw_mt_jump_tables", L, J, tab.ctypes.data)
    st0 = np.zeros(624, dtype=np.uint32)
    N.call("mw_mt_seed_state", 16, st0.ctypes.data)
    np.testing.assert_array_equal(st0, mt19937_init(16))

    def regen(mt):
        mt = mt.astype(np.uint64).copy()
        for i in range(624):
            y = (int(mt[i]) & 0x80000000) | (int(mt[(i + 1) % 624]) & 0x7FFFFFFF)
            mt[i] = int(mt[(i + 397) % 624]) ^ (y >> 1) ^ (0x9908B0DF if y & 1 else 0)
        return mt.astype(np.uint32)

    wins = [st0]
    for _ in range(12):
        wins.append(regen(wins[-1]))
    for j in range(J):
        out = np.zeros(624, dtype=np.uint32)
        N.call("mw_mt_jump_host", st0.ctypes.data, tab[j].ctypes.data, out.ctypes.data)
        ref = wins[(L << j) // 624]
        np.testing.assert_array_equal(out[1:], ref[1:])
        assert (out[0] >> 31) == (ref[0] >> 31)


def test_lloyd_workspace_holds_records_and_row_lists():
    """mw_lloyd_ws_bytes covers the per-block records plus the kList pass's
    per-block lengths and row lists (at least 4 bytes per row): callers that
    size the workspace from the query get the list pass without changes."""
    from milwrm_amd import _native as N

    for S, k, F in [(1, 1, 1), (1000, 8, 30), (17_000_000, 20, 30), (270_000_000, 8, 50)]:
        ws = N.query("mw_lloyd_ws_bytes", S, k, F)
        rec = N.query("mw_lloyd_rec_len", k, F) * 8
        assert ws >= rec + 4 * S, (S, k, F, ws)
        # without kList: the records only (MW_LLOYD_LIST=0, or S >= 2^31)
        ws0 = N.query("mw_lloyd_ws_bytes_kinds", S, k, F, 0)
        assert rec <= ws0 and ws - ws0 >= 4 * S, (S, k, F, ws0)
        assert N.query("mw_lloyd_ws_bytes_kinds", S, k, F, 1) == ws
    assert N.query("mw_lloyd_ws_bytes_kinds", 1 << 31, 8, 30, 1) == N.query("mw_lloyd_ws_bytes_kinds", 1 << 31, 8, 30, 0)


def test_stream_band_plan_covers_rows():
    """stream.bands over a resident source (views, no GPU needed): output rows
    tile [r0, r1) once, each band's raw rows are its output rows plus the
    halo clipped to the slide."""
    import torch

    from milwrm_amd import stream

    H = 53
    t = torch.arange(H * 3 * 2, dtype=torch.int16).reshape(H, 3, 2)
    src = stream.DeviceSource(t)
    for band, halo, r0, r1 in [(7, 3, 0, H), (53, 8, 0, H), (1, 0, 0, H), (10, 8, 5, 41), (100, 2, 0, H)]:
        seen = []
        for y0, y1, a, raw in stream.bands(src, band, halo, r0, r1):
            assert a == max(0, y0 - halo)
            assert raw.shape[0] == min(H, y1 + halo) - a
            assert torch.equal(raw, t[a:a + raw.shape[0]])
            seen.extend(range(y0, y1))
        assert seen == list(range(r0, r1))


def test_stream_parse_bytes_and_host_dtypes():
    import torch

    from milwrm_amd import stream

    assert stream._parse_bytes("64G") == 64 << 30
    assert stream._parse_bytes("1.5M") == int(1.5 * (1 << 20))
    assert stream._parse_bytes("12345") == 12345
    assert stream.device_dtype_of(np.zeros((2, 2, 2), np.uint8)) == torch.uint8
    assert stream.device_dtype_of(np.zeros((2, 2, 2), np.uint16)) == torch.int16
    assert stream.device_dtype_of(np.full((2, 2, 2), 70000, np.int32)) == torch.float32
    assert stream.device_dtype_of(np.full((2, 2, 2), 700, np.int64)) == torch.int16
    assert stream.device_dtype_of(np.zeros((2, 2, 2), np.float64)) == torch.float32
    hs = stream.HostSource(np.arange(5 * 4 * 3, dtype=np.uint16).reshape(5, 4, 3) + 60000)
    rows = hs._host_rows(1, 3)
    assert rows.dtype == torch.int16 and tuple(rows.shape) == (2, 4, 3)
    assert int(rows.view(torch.int16).to(torch.int32)[0, 0, 0]) & 0xFFFF == 60000 + 12


def test_blur_bound_bounds_lognorm_blur():
    """img._blur_bound (the QC fixed point's pixel bound, known before the
    blur): |blur(lognorm(raw))| <= bound on every channel of the oracle's fp64
    pipeline, for uint16 / uint8 slides, with and without a log_normalize;
    None for float slides and once the pixels are no longer raw."""
    import milwrm_amd as M
    from oracle import milwrm_oracle as O

    raw, _ = O.synth_slide(40, 48, 5, seed=11, mode="hard")
    raw[3, 4, 1] = 65535  # the dtype max itself
    mean = raw.reshape(-1, 5).mean(0)
    for a, mx in ((raw, 65535.0), (np.minimum(raw, 255).astype(np.uint8), 255.0)):
        im = M.img(a.copy())
        assert im._raw_int_max() == mx
        assert np.all(im._blur_bound() >= np.abs(O.gaussian_blur(a.astype(np.float64))).max((0, 1)))
        for p in (1.0, 0.25):
            inv = (1.0 / mean).astype(np.float32)
            im._pending, im._lognorm_host = ("device", p), (inv, p)  # as log_normalize leaves them
            ref = O.gaussian_blur(O.log_normalize(a, mean, pseudoval=p))
            assert np.all(im._blur_bound() >= np.abs(ref).max((0, 1)))
            im._lognorm_host = None  # a pending transform of pixels that were not raw
            assert im._blur_bound() is None
    assert M.img(raw.astype(np.float32))._blur_bound() is None
