"""Lloyd pass kinds are exact: with every bounded pass forced to kTile, or to
kQueue, or to kList (twice), or the default mix, the fits equal the plain Lloyd E-step every pass
(MW_LLOYD_NOBOUND) bit for bit — labels, centers, n_iter — for k = 8..20 in
one batched launch, and repeated runs agree; so does the dense pass (the
f16-split x . C^T of every fit on the matrix cores, exact recheck of near
ties), every iteration or until fewer than 9 fits run (then bounded passes
from recomputed bounds); at F = 30 (FMAX = 32) and at
F = 50 / 45 (FMAX = 52 instances: 26 feature pairs, 52-float tile rows with a
zeroed pad; odd F takes the scalar gather).  test_fm52_instances_equal_fm64
checks those against the FMAX = 64 instances (F-sized LDS tiles, masked tile
stores, the kList gather into the smaller tile) bit for bit.
The k-means++ passes at F > 32 (F-sized tiles, pipelined table loads) pick
the oracle's indices on the same fp32 rows.  Regression: the queue pass
gathers only the F floats of each row into LDS, and the scaled-row read
took the padded pair of the tile's last row from LDS no pass had written
(NaN * 0 = NaN): a few labels per pass changed from run to run."""
import contextlib
import os
import sys

import numpy as np
import pandas as pd
import pytest

pytestmark = pytest.mark.gpu


def _rows(C=30, size=1536):
    import milwrm_amd as M
    from milwrm_amd import device as D

    raw, mask = D.synth_slide(size, size, C, seed=20251015, mode="hard")
    im = M.img.from_device(raw, mask)
    with contextlib.redirect_stdout(sys.stderr):
        est, pix = im.calculate_non_zero_mean()
        df = pd.DataFrame({"Img": [im], "batch_names": ["b"], "mean estimators": [est],
                           "pixels": [pix]})
        lab = M.mxif_labeler(df)
        lab.prep_cluster_data(features=list(range(C)), sigma=2, fract=0.2)
    return lab._rows


@pytest.mark.timeout(300)
@pytest.mark.parametrize("C,size", [(30, 1536), (50, 1024), (45, 1024)])
def test_pass_kinds_equal_full_estep(gpu, monkeypatch, C, size):
    from milwrm_amd import kmeans as KM

    rows = _rows(C, size)
    ks = list(range(8, 21))
    out = {}
    # (name, queue threshold, few-undecided kind, no bounds, dense pass from how many fits)
    for name, qb, qk, nobound, dmin in [("full", -1.0, KM.KIND_QUEUE, True, None),
                                        ("tile", -1.0, KM.KIND_QUEUE, False, None),
                                        ("queue", 2.0, KM.KIND_QUEUE, False, None),
                                        ("queue_again", 2.0, KM.KIND_QUEUE, False, None),
                                        ("list", 2.0, KM.KIND_LIST, False, None),
                                        ("list_again", 2.0, KM.KIND_LIST, False, None),
                                        ("dense", 2.0, KM.KIND_LIST, False, 1),
                                        ("dense_again", 2.0, KM.KIND_LIST, False, 1),
                                        ("dense_then_bounds", KM.QUEUE_BELOW, KM.QUEUE_KIND, False, 9),
                                        ("default", KM.QUEUE_BELOW, KM.QUEUE_KIND, False, KM.DENSE_MIN_FITS)]:
        monkeypatch.setattr(KM, "QUEUE_BELOW", qb)
        monkeypatch.setattr(KM, "QUEUE_KIND", qk)
        monkeypatch.setattr(KM, "USE_DENSE", dmin is not None)
        monkeypatch.setattr(KM, "DENSE_MODE", "1")  # F = 50 / 45: the grouped dense form too
        monkeypatch.setattr(KM, "DENSE_MIN_FITS", dmin or 1)
        if nobound:
            monkeypatch.setenv("MW_LLOYD_NOBOUND", "1")
        else:
            monkeypatch.delenv("MW_LLOYD_NOBOUND", raising=False)
        with contextlib.redirect_stdout(sys.stderr):
            fits = KM.fit_many(rows, ks, random_state=18)
        out[name] = [(np.asarray(m.labels_).copy(), m.cluster_centers_.copy(), m.n_iter_) for m in fits]
    for name in ("tile", "queue", "queue_again", "list", "list_again", "dense", "dense_again",
                 "dense_then_bounds", "default"):
        for i, k in enumerate(ks):
            a, b = out["full"][i], out[name][i]
            assert a[2] == b[2], f"k={k} {name}: n_iter {b[2]} vs {a[2]}"
            np.testing.assert_array_equal(b[0], a[0], err_msg=f"k={k} {name} labels")
            np.testing.assert_array_equal(b[1], a[1], err_msg=f"k={k} {name} centers")


@pytest.mark.timeout(300)
@pytest.mark.parametrize("dense", [True, False])
def test_fits_driver_equals_python_loop(gpu, monkeypatch, dense):
    """mw_lloyd_fits (the batched iterations in C++) against lloyd_fits'
    Python loop: labels, centers, inertia, n_iter and every pass's (changed,
    recomputed) bit for bit, with the dense pass and with the bounded kinds
    only; an empty cluster is forced (duplicated initial centers) so the
    relocation runs in both."""
    from milwrm_amd import kmeans as KM

    rows = _rows(30, 768)
    rng = np.random.default_rng(3)
    inits = []
    for k in (2, 5, 9, 14, 20):
        c = rows.scaled_rows(rng.choice(rows.S, size=k, replace=False))
        if k >= 5:
            c[1] = c[0]  # two identical centers: one of them ends empty
        inits.append(c)
    monkeypatch.setattr(KM, "USE_DENSE", dense)
    out = {}
    for name, use_c in [("py", False), ("c", True)]:
        monkeypatch.setattr(KM, "USE_C_FITS", use_c)
        res = KM.lloyd_fits(rows, [c.copy() for c in inits], 300, 1e-6)
        out[name] = ([(r[0].cpu().numpy().copy(), r[1], r[2].copy(), r[3]) for r in res],
                     [list(h) for h in KM.LAST_STATS["history"]])
    for i, (a, b) in enumerate(zip(out["py"][0], out["c"][0])):
        np.testing.assert_array_equal(b[0], a[0], err_msg=f"fit {i} labels")
        np.testing.assert_array_equal(b[2], a[2], err_msg=f"fit {i} centers")
        assert b[1] == a[1] and b[3] == a[3], f"fit {i}: inertia / n_iter {b[1], b[3]} vs {a[1], a[3]}"
    assert out["c"][1] == out["py"][1]


@pytest.mark.timeout(300)
@pytest.mark.parametrize("outlier", [300.0, 3000.0])
def test_dense_keys_far_rows_equal_full_estep(gpu, monkeypatch, outlier):
    """The dense pass's folded norms and keyed top two (lloyd_dense2.h) at
    its edges: an odd number of fits with k = 1 and fits spanning two MFMA
    tiles, rows whose |x|^2 passes kD2NormMax (their fits go to the exact
    chain) and, at the larger outliers, centers past it too (the whole launch
    on the exact chain).  Labels, centers and n_iter equal the plain E-step."""
    import torch

    from milwrm_amd import kmeans as KM

    rng = np.random.default_rng(7)
    S, F = 120_000, 30
    cent = rng.normal(0.0, 6.0, size=(12, F))
    X = cent[rng.integers(0, 12, size=S)] + rng.normal(0.0, 1.0, size=(S, F))
    far = rng.choice(S, size=S // 100, replace=False)
    X[far, :4] += rng.uniform(0.5, 1.0, size=(far.size, 4)) * outlier
    rows = KM.DeviceRows.from_host(X.astype(np.float32))
    ks = [1, 2, 3, 5, 9, 17, 20]
    out = {}
    for name, nobound, dense in [("full", True, False), ("dense", False, True)]:
        monkeypatch.setattr(KM, "USE_DENSE", dense)
        monkeypatch.setattr(KM, "DENSE_MIN_FITS", 1)
        if nobound:
            monkeypatch.setenv("MW_LLOYD_NOBOUND", "1")
        else:
            monkeypatch.delenv("MW_LLOYD_NOBOUND", raising=False)
        with contextlib.redirect_stdout(sys.stderr):
            fits = KM.fit_many(rows, ks, random_state=11)
        out[name] = [(np.asarray(m.labels_).copy(), m.cluster_centers_.copy(), m.n_iter_) for m in fits]
    torch.cuda.synchronize()
    for i, k in enumerate(ks):
        a, b = out["full"][i], out["dense"][i]
        assert a[2] == b[2], f"k={k}: n_iter {b[2]} vs {a[2]}"
        np.testing.assert_array_equal(b[0], a[0], err_msg=f"k={k} labels")
        np.testing.assert_array_equal(b[1], a[1], err_msg=f"k={k} centers")


@pytest.mark.timeout(300)
@pytest.mark.parametrize("C", [50, 45])
def test_kpp_indices_wide_rows(gpu, C):
    """k-means++ at F > 32 (FMAX = 64 instances) against the oracle's
    _kmeans_plusplus restatement on the same fp32 rows (scaled, centered as
    KMeans.fit does), k = 8 and 20."""
    import torch

    from milwrm_amd.kmeans import KMeans
    from oracle import milwrm_oracle as O

    rows = _rows(C, 768)
    Xs = ((rows.X.double() - torch.from_numpy(rows.mu).cuda()) * torch.from_numpy(rows.inv).cuda()).cpu().numpy()
    Xs -= Xs.mean(axis=0)
    for k in (8, 20):
        with contextlib.redirect_stdout(sys.stderr):
            km = KMeans(n_clusters=k, random_state=18).fit(rows)
        _, idx = O.kmeans_plusplus(Xs, k, np.random.RandomState(18))
        np.testing.assert_array_equal(km.init_indices_, idx, err_msg=f"F={C} k={k}")


@pytest.mark.timeout(300)
def test_sweep_in_slide_order_equals_draw_order(gpu, monkeypatch):
    """fit_many runs the Lloyd passes over the rows in slide order
    (DeviceRows.spatial_order) and puts the labels back in draw order: every
    fit bitwise equal to the passes over the draw order (labels, centers,
    n_iter, inertia), k = 2..20."""
    from milwrm_amd import kmeans as KM

    rows = _rows(30, 1024)
    assert rows.spatial_order() is not None
    out = {}
    for flag in (False, True):
        monkeypatch.setattr(KM, "SWEEP_SORT", flag)
        with contextlib.redirect_stdout(sys.stderr):
            fits = KM.fit_many(rows, list(range(2, 21)), random_state=18)
        out[flag] = [(np.asarray(m.labels_).copy(), m.cluster_centers_.copy(), m.n_iter_, m.inertia_) for m in fits]
    for k, a, b in zip(range(2, 21), out[False], out[True]):
        assert a[2] == b[2], f"k={k} n_iter"
        assert a[3] == b[3], f"k={k} inertia"
        np.testing.assert_array_equal(b[0], a[0], err_msg=f"k={k} labels")
        np.testing.assert_array_equal(b[1], a[1], err_msg=f"k={k} centers")


@pytest.mark.timeout(300)
@pytest.mark.parametrize("C", [50, 45, 33])
def test_fm52_instances_equal_fm64(gpu, monkeypatch, C):
    """At 33 <= F <= 52 the Lloyd passes run the FMAX = 52 instances (26
    feature pairs per distance; the first pass's M-step by label-sorted sums
    or LDS atomics, never the 16-feature MFMA blocks): every fit bitwise the
    FMAX = 64 instances' (MW_LLOYD_FM52=0) -- labels, centers, n_iter,
    inertia -- for k = 8..20 batched and k = 8 alone through KMeans."""
    from milwrm_amd import kmeans as KM

    rows = _rows(C, 768)
    ks = [8, 12, 17, 20]
    out = {}
    for fm in ("0", "1"):
        monkeypatch.setenv("MW_LLOYD_FM52", fm)
        with contextlib.redirect_stdout(sys.stderr):
            fits = KM.fit_many(rows, ks, random_state=18)
            one = KM.KMeans(n_clusters=8, random_state=18).fit(rows)
        out[fm] = ([(np.asarray(m.labels_).copy(), m.cluster_centers_.copy(), m.n_iter_, m.inertia_)
                    for m in fits], (np.asarray(one.labels_).copy(), one.cluster_centers_.copy(),
                                     one.n_iter_, one.inertia_))
    for (a, b), k in zip(zip(out["0"][0], out["1"][0]), ks):
        assert a[2] == b[2], f"F={C} k={k}: n_iter {b[2]} vs {a[2]}"
        np.testing.assert_array_equal(a[0], b[0], err_msg=f"F={C} k={k} labels")
        np.testing.assert_array_equal(a[1], b[1], err_msg=f"F={C} k={k} centers")
        assert a[3] == b[3]
    a, b = out["0"][1], out["1"][1]
    assert a[2] == b[2] and a[3] == b[3]
    np.testing.assert_array_equal(a[0], b[0])
    np.testing.assert_array_equal(a[1], b[1])


@pytest.mark.timeout(300)
def test_first_pass_three_waves_equals_unbounded(gpu, monkeypatch):
    """The first pass at F <= 32 under the three-waves-per-SIMD register bound
    (lloyd_first_w3_kernel, the default) gives the unbounded instance's
    fits (MW_LLOYD_FIRST_W3=0) bit for bit: labels, centers, n_iter,
    inertia."""
    from milwrm_amd import kmeans as KM

    rows = _rows(30, 1024)
    out = {}
    for w3 in ("0", "1"):
        monkeypatch.setenv("MW_LLOYD_FIRST_W3", w3)
        with contextlib.redirect_stdout(sys.stderr):
            one = KM.KMeans(n_clusters=8, random_state=18).fit(rows)
            fits = KM.fit_many(rows, [5, 8, 13], random_state=18)
        out[w3] = [(np.asarray(m.labels_).copy(), m.cluster_centers_.copy(), m.n_iter_, m.inertia_)
                   for m in [one] + list(fits)]
    for a, b in zip(out["0"], out["1"]):
        assert a[2] == b[2] and a[3] == b[3]
        np.testing.assert_array_equal(a[0], b[0])
        np.testing.assert_array_equal(a[1], b[1])
