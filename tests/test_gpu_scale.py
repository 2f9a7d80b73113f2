"""GPU parity at larger sizes and at the 50-channel shape of BASELINE config 5
(the FMAX = 64 instances of every k-means kernel and the 4-channel-tile blur),
end to end against the CPU oracle (oracle/milwrm_oracle.py, pinned to the
reference's golden vectors by tests/test_oracle_golden.py).

Tolerances (north_star): labels bit-exact except near-ties (oracle cID <
1e-5), centers / inertia / confidence within 1e-4 relative."""
import numpy as np
import pandas as pd
import pytest

from oracle import milwrm_oracle as O

pytestmark = pytest.mark.gpu
TAU = 1e-5
RTOL = 1e-4


def _rel(a, b):
    a, b = np.asarray(a, dtype=np.float64), np.asarray(b, dtype=np.float64)
    return np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-30)


def _labels_match(got, ref, cid_ref):
    got = np.nan_to_num(np.asarray(got, dtype=np.float64), nan=-1)
    ref = np.nan_to_num(np.asarray(ref, dtype=np.float64), nan=-1)
    near = np.nan_to_num(cid_ref, nan=1.0) < TAU
    bad = (got != ref) & ~near
    assert not bad.any(), f"{int(bad.sum())} non-tie label mismatches"


def _run_labeler(slides, masks, C, k):
    import milwrm_amd as M

    imgs = [M.img(s.copy(), mask=m.copy()) for s, m in zip(slides, masks)]
    ests, pix = zip(*[im.calculate_non_zero_mean() for im in imgs])
    df = pd.DataFrame({"Img": imgs, "batch_names": ["b"] * len(imgs),
                       "mean estimators": list(ests), "pixels": list(pix)})
    lab = M.mxif_labeler(df)
    lab.prep_cluster_data(features=list(range(C)), sigma=2, fract=0.2)
    lab.label_tissue_regions(k=k, plot_out=False, random_state=18)
    lab.confidence_score_images()
    return lab


def _check_against_oracle(lab, ref, k):
    km = ref["kmeans"]
    np.testing.assert_allclose(lab.scaler.mean_, ref["scaler_mean"], rtol=1e-5)
    np.testing.assert_allclose(lab.scaler.scale_, ref["scaler_scale"], rtol=1e-5)
    np.testing.assert_array_equal(lab.kmeans.init_indices_, km["init_indices"])
    assert lab.kmeans.n_iter_ == km["n_iter_"], (lab.kmeans.n_iter_, km["n_iter_"])
    assert _rel(lab.kmeans.cluster_centers_, km["cluster_centers_"]) < RTOL
    assert abs(lab.kmeans.inertia_ - km["inertia_"]) / km["inertia_"] < RTOL
    for i in range(len(ref["tissue_IDs"])):
        cid = ref["confidence_IDs"][i]
        _labels_match(lab.tissue_IDs[i], ref["tissue_IDs"][i], cid)
        ok = ~np.isnan(cid)
        np.testing.assert_array_equal(np.isnan(lab.confidence_IDs[i]), np.isnan(cid))
        np.testing.assert_allclose(lab.confidence_IDs[i][ok], cid[ok], rtol=RTOL, atol=RTOL)
    ref_df = np.array([[m[j] for j in range(k)] for m in ref["confidence_means"]])
    np.testing.assert_allclose(lab.confidence_score_df.values, ref_df, rtol=RTOL, atol=1e-6)


def test_e2e_2048_hard_vs_oracle(gpu):
    """One 2048^2 x 30 hard slide (713k clustering rows), k = 8: k-means++
    indices, n_iter, centers, inertia, every pixel's label (except near-ties)
    and confidence, and the confidence frame, against the oracle pipeline."""
    raw, mask = O.synth_slide(2048, 2048, 30, seed=20251015, mode="hard")
    ref = O.mxif_pipeline([raw], [mask], ["b"], list(range(30)), k=8)
    lab = _run_labeler([raw], [mask], 30, 8)
    _check_against_oracle(lab, ref, 8)


@pytest.mark.parametrize("k,fused", [(8, "0"), (8, "1"), (8, "band"), (20, "0"), (20, "1")])
def test_e2e_50_channels_vs_oracle(gpu, monkeypatch, k, fused):
    """BASELINE config 5's 50 channels on two 320 x 384 slides: blur with four
    16-channel tiles, the FMAX = 64 k-means++ / Lloyd / label kernels, the
    fused sample and (k = 8) assign epilogues, end to end against the oracle."""
    from milwrm_amd import device as D

    monkeypatch.setenv("MW_FUSED_BLUR", "0" if fused == "0" else "1")
    monkeypatch.setenv("MW_DEFERRED_ASSIGN", "band" if fused == "band" else "fused")
    monkeypatch.setenv("MW_ASSIGN_BAND_ROWS", "72")
    before = dict(D.FUSED_USED)
    slides, masks = zip(*[O.synth_slide(320, 384, 50, seed=77 + s, mode="hard") for s in range(2)])
    ref = O.mxif_pipeline(list(slides), list(masks), ["b", "b"], list(range(50)), k=k)
    lab = _run_labeler(slides, masks, 50, k)
    _check_against_oracle(lab, ref, k)
    if fused != "0":
        assert D.FUSED_USED["sample"] > before["sample"]
        if fused == "band":
            assert D.FUSED_USED["assign_banded"] > before["assign_banded"]
        elif k <= 16:
            assert D.FUSED_USED["assign"] > before["assign"]


def test_sweep_50_features_equals_separate_fits(gpu):
    """The batched k sweep at F = 50 (FMAX = 64; k = 17..20 need two label
    blocks): every fit bitwise equal to a separate KMeans fit."""
    from milwrm_amd.kmeans import DeviceRows, KMeans, fit_many

    rng = np.random.default_rng(50)
    cents = rng.normal(0, 2.0, size=(12, 50))
    X = cents[rng.integers(0, 12, 30000)] + rng.normal(0, 1.0, size=(30000, 50))
    rows = DeviceRows.from_host((X - X.mean(0)) / X.std(0))
    ks = [2, 3, 8, 16, 17, 20]
    many = fit_many(rows, ks, random_state=18)
    for k, b in zip(ks, many):
        a = KMeans(n_clusters=k, random_state=18).fit(rows)
        np.testing.assert_array_equal(a.init_indices_, b.init_indices_)
        assert a.n_iter_ == b.n_iter_, (k, a.n_iter_, b.n_iter_)
        assert a.inertia_ == b.inertia_
        np.testing.assert_array_equal(a.cluster_centers_, b.cluster_centers_)
        np.testing.assert_array_equal(a.labels_, b.labels_)
    ref = O.kmeans_fit(rows.to_host_scaled(), 20, random_state=18)
    assert many[-1].n_iter_ == ref["n_iter_"]
    assert _rel(many[-1].cluster_centers_, ref["cluster_centers_"]) < RTOL


def test_rows_beyond_hbm_raise_clearly(gpu, monkeypatch):
    """Config 5 at 1-2 GPUs: sampled rows beyond the free HBM raise a
    MemoryError naming the remedy before any allocation (free HBM faked)."""
    import torch

    from milwrm_amd.MILWRM import _check_rows_fit

    _check_rows_fit(1000, 50, torch.device("cuda", 0))  # small: fine
    monkeypatch.setattr(torch.cuda, "mem_get_info", lambda *a: (1 << 30, 288 << 30))
    with pytest.raises(MemoryError, match="shard the images over more GPUs"):
        _check_rows_fit(4_350_000_000, 50, torch.device("cuda", 0))
