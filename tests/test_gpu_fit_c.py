"""The whole-fit C entry ``mw_kmeans_fit`` (include/milwrm_amd.h), called
directly through ctypes as a non-Python caller would bind it, against the
reference's golden fit (tests/golden/mxif_small.npz: sklearn KMeans(k,
random_state=18) on the reference's own cluster_data) and bitwise against
the Python ``KMeans.fit`` on the same device rows."""
import ctypes as C

import numpy as np
import pytest

from oracle import milwrm_oracle as O

pytestmark = pytest.mark.gpu


def _c_fit(X_dev, mu, inv, k, seed=18, var=None, init=None, max_iter=300, tol=1e-4):
    import torch

    from milwrm_amd import _native as N
    from milwrm_amd import device as D

    S, F = X_dev.shape
    mu = np.ascontiguousarray(mu, dtype=np.float64)
    inv = np.ascontiguousarray(inv, dtype=np.float64)
    var = None if var is None else np.ascontiguousarray(var, dtype=np.float64)
    init = None if init is None else np.ascontiguousarray(init, dtype=np.float64)
    labels = torch.empty(S, dtype=torch.uint8, device=X_dev.device)
    centers = np.zeros((k, F))
    inertia = C.c_double()
    n_iter = C.c_int()
    idx = np.full(k, -1, dtype=np.int64)
    N.call("mw_kmeans_fit", D.P(X_dev), S, F, mu.ctypes.data, inv.ctypes.data,
           None if var is None else var.ctypes.data, None, k,
           None if init is None else init.ctypes.data, seed, max_iter, tol, D.P(labels),
           centers.ctypes.data, C.addressof(inertia), C.addressof(n_iter), idx.ctypes.data,
           None, 0, D.stream())
    return dict(labels=labels.cpu().numpy().astype(np.int32), centers=centers,
                inertia=inertia.value, n_iter=n_iter.value, idx=idx)


def _py_fit(rows, k, seed=18, init="k-means++"):
    """The Python host loop (KMeans.fit with the C driver switched off)."""
    from milwrm_amd import kmeans as K

    K.USE_C_FIT = False
    try:
        km = K.KMeans(n_clusters=k, random_state=seed, init=init).fit(rows)
    finally:
        K.USE_C_FIT = True
    return dict(labels=km.labels_, centers=km.cluster_centers_, inertia=km.inertia_,
                n_iter=km.n_iter_, idx=km.init_indices_)


def _same(a, b):
    np.testing.assert_array_equal(a["labels"], b["labels"])
    np.testing.assert_array_equal(a["centers"], b["centers"])
    assert a["inertia"] == b["inertia"]
    assert a["n_iter"] == b["n_iter"]


def test_c_fit_vs_reference_golden(gpu, golden):
    """k = the golden's k on the reference's cluster_data: k-means++ indices,
    n_iter and labels exact, centers and inertia to 1e-6 (fp32 rows)."""
    from milwrm_amd.kmeans import DeviceRows

    g = golden("mxif_small")
    X = g["cluster_data"]
    k = int(g["k"])
    rows = DeviceRows.from_host(X)
    F = X.shape[1]
    got = _c_fit(rows.X, np.zeros(F), np.ones(F), k, var=np.var(X, axis=0))
    np.testing.assert_array_equal(got["idx"], g["kpp_indices"][k, :k])
    assert got["n_iter"] == int(g["n_iter"])
    np.testing.assert_array_equal(got["labels"], g["labels"])
    np.testing.assert_allclose(got["centers"], g["centers"], rtol=1e-6, atol=1e-6)
    assert abs(got["inertia"] - float(g["inertia"])) / float(g["inertia"]) < 1e-6
    ref = _py_fit(rows, k)
    _same(got, ref)
    np.testing.assert_array_equal(got["idx"], ref["idx"])


@pytest.mark.parametrize("k", [2, 7, 20])
def test_c_fit_folded_scaler_matches_python(gpu, k):
    """Raw rows with the scaler folded in (mu, inv), the tolerance's variance
    computed on the device (h_feature_var NULL) vs given: bitwise the Python
    fit on the same DeviceRows; and the oracle fit on the scaled rows."""
    import torch

    from milwrm_amd import device as D
    from milwrm_amd.kmeans import DeviceRows

    rng = np.random.default_rng(k)
    cents = rng.normal(0, 2.0, size=(9, 12))
    raw = (cents[rng.integers(0, 9, 20000)] + rng.normal(0, 1.0, size=(20000, 12))) * 3.0 + 7.0
    raw32 = raw.astype(np.float32)
    mu = raw32.astype(np.float64).mean(0)
    sd = raw32.astype(np.float64).std(0)
    inv = 1.0 / sd
    Xs = (raw32.astype(np.float64) - mu) * inv
    fv = Xs.var(0)
    rows = DeviceRows(torch.from_numpy(raw32).to(D.device()), mu, inv, feature_var=fv)
    got = _c_fit(rows.X, mu, inv, k, var=fv)
    ref = _py_fit(rows, k)
    _same(got, ref)
    np.testing.assert_array_equal(got["idx"], ref["idx"])
    dev_var = _c_fit(rows.X, mu, inv, k)  # variance from device column statistics
    assert dev_var["n_iter"] in (got["n_iter"], got["n_iter"] - 1, got["n_iter"] + 1)
    np.testing.assert_allclose(dev_var["centers"], got["centers"], rtol=1e-3, atol=1e-3)
    orc = O.kmeans_fit(Xs, k, random_state=18)
    np.testing.assert_array_equal(got["idx"], orc["init_indices"])
    assert got["n_iter"] == orc["n_iter_"]
    np.testing.assert_allclose(got["centers"], orc["cluster_centers_"], rtol=1e-4, atol=1e-5)


def test_c_fit_given_init_and_errors(gpu, golden):
    """An explicit init (no seeding, indices untouched) equals the Python fit
    from the same array; out-of-range k / F are rejected with the error text."""
    from milwrm_amd.kmeans import DeviceRows

    g = golden("mxif_small")
    X = g["cluster_data"]
    rows = DeviceRows.from_host(X)
    F = X.shape[1]
    init = g["lloyd1_centers_in"]
    got = _c_fit(rows.X, np.zeros(F), np.ones(F), init.shape[0], var=np.var(X, axis=0), init=init)
    assert np.all(got["idx"] == -1)
    _same(got, _py_fit(rows, init.shape[0], init=init))
    with pytest.raises(ValueError, match="n_clusters=65"):
        _c_fit(rows.X, np.zeros(F), np.ones(F), 65)
    with pytest.raises(ValueError, match="n_samples=10 should be >= n_clusters=20"):
        _c_fit(rows.X[:10], np.zeros(F), np.ones(F), 20)
    with pytest.raises(ValueError, match="max_iter"):
        _c_fit(rows.X, np.zeros(F), np.ones(F), 4, max_iter=0)


@pytest.mark.parametrize("k,F", [(3, 30), (8, 30), (12, 17), (16, 32), (8, 8)])
def test_kpp_fold_equals_separate_first_pass(gpu, monkeypatch, k, F):
    """MW_KPP_FOLD=1 (the first Lloyd E-step folded into the last k-means++
    pass, then the winner's moved rows through a kind-8 list pass) against
    the separate kind-0 first pass: k-means++ indices, labels, centers,
    inertia and n_iter bitwise, on overlapping clusters (many moved rows,
    near ties)."""
    import torch

    from milwrm_amd import _native as N

    assert N.load().mw_kpp_fold_supported(k, F, 2 + int(np.log(k))) == 1
    rng = np.random.default_rng(100 + k)
    S = 150_000 + 37 * k
    cen = rng.normal(0, 1.5, size=(k + 3, F))
    X = (cen[rng.integers(0, k + 3, S)] + rng.normal(0, 1.0, size=(S, F))).astype(np.float32)
    X[:50] = X[50:100]  # exact duplicate rows: exact distance ties
    Xd = torch.from_numpy(X).cuda()
    mu, inv = X.mean(0).astype(np.float64), 1.0 / (X.std(0).astype(np.float64) + 0.5)
    var = (np.var(X.astype(np.float64), axis=0) * inv * inv)
    monkeypatch.setenv("MW_KPP_FOLD", "0")
    a = _c_fit(Xd, mu, inv, k, var=var)
    monkeypatch.setenv("MW_KPP_FOLD", "1")
    b = _c_fit(Xd, mu, inv, k, var=var)
    _same(a, b)
    np.testing.assert_array_equal(a["idx"], b["idx"])
