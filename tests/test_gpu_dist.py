"""Sharded execution on the GPU: 2 ranks (spawned processes, gloo for the
small messages, both on cuda:0) each preprocess their own slides, then the
k = 6 fit, the labels / confidences and the k = 2..20 sweep run sharded.
Everything must be BITWISE the single-process run over all slides: the
scaler (per-image statistics merged in global image order), the k-means++
indices (global argmin / owner search), n_iter, centers and inertia (exact
fixed-point Lloyd records, all-reduced), every pixel's label, and the sweep
curve.  Host-side logic of the same collectives: tests/test_dist_gloo.py."""
import os
import socket

import numpy as np
import pandas as pd
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
SHARDS = {0: [0, 1], 1: [2]}  # rank -> slides (uneven on purpose)
BATCHES = ["b1", "b1", "b2"]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _slides():
    from oracle.milwrm_oracle import synth_slide

    return [synth_slide(160, 192 + 32 * i, 8, seed=300 + i, mode="hard") for i in range(3)]


def _run(slides, batches, comm):
    import milwrm_amd as M
    from milwrm_amd import kmeans as KM

    used = dict(KM.FITS_C_USED)
    imgs = [M.img(r.copy(), mask=m.copy()) for r, m in slides]
    ests, pix = zip(*[im.calculate_non_zero_mean() for im in imgs])
    df = pd.DataFrame({"Img": imgs, "batch_names": batches, "mean estimators": list(ests),
                       "pixels": list(pix)})
    lab = M.mxif_labeler(df)
    lab.prep_cluster_data(features=list(range(8)), sigma=2, fract=0.2, comm=comm)
    lab.label_tissue_regions(k=6, plot_out=False, random_state=18, comm=comm)
    lab.confidence_score_images()
    out = dict(mean=lab.scaler.mean_, scale=lab.scaler.scale_, idx=lab.kmeans.init_indices_,
               n_iter=lab.kmeans.n_iter_, centers=lab.kmeans.cluster_centers_,
               inertia=lab.kmeans.inertia_, rows_labels=lab.kmeans.labels_,
               tid=[np.nan_to_num(t, nan=-1) for t in lab.tissue_IDs],
               cid=[np.nan_to_num(c, nan=-1) for c in lab.confidence_IDs])
    out["kpp_host_ms"] = list(getattr(comm, "kpp_host_ms", []))
    lab.find_optimal_k(random_state=18, alpha=0.05)
    out["best_k"] = int(lab.k)
    out["curve"] = lab.inertia_curve_["Scaled Inertia"].values
    out["fits_c"] = {key: KM.FITS_C_USED[key] - used[key] for key in used}
    return out


def _worker(rank, world, port, q):
    import torch
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        from milwrm_amd.dist import DistComm

        from milwrm_amd import kmeans as KM

        slides = _slides()
        mine = SHARDS[rank]
        res = _run([slides[i] for i in mine], [BATCHES[i] for i in mine],
                   DistComm(device=torch.device("cpu")))
        # the same run with the sharded fits in the Python loop (MW_LLOYD_FITS_C=0)
        KM.USE_C_FITS = False
        try:
            res["pyloop"] = _run([slides[i] for i in mine], [BATCHES[i] for i in mine],
                                 DistComm(device=torch.device("cpu")))
        finally:
            KM.USE_C_FITS = True
        torch.cuda.synchronize()
        q.put((rank, res))
    except Exception as e:  # surface the failure in the parent
        q.put((rank, repr(e)))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(600)
def test_two_shards_bitwise_equal_single_process(gpu):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    got = dict(q.get(timeout=540) for _ in ps)
    for p in ps:
        p.join(60)
    for r in (0, 1):
        assert not isinstance(got[r], str), got[r]
        assert ps[r].exitcode == 0
    ref = _run(_slides(), BATCHES, None)
    for r in (0, 1):
        g = got[r]
        for key in ("mean", "scale", "idx", "centers", "curve"):
            np.testing.assert_array_equal(g[key], ref[key], err_msg=key)
        assert g["n_iter"] == ref["n_iter"]
        # host time per sharded k-means++ step (sync -> next trial pass queued:
        # targets, owner search, the candidate all-reduce over gloo)
        ms = g["kpp_host_ms"]
        assert len(ms) == 5 and max(ms) < 50.0, ms
        print(f"rank {r}: sharded k-means++ host time per step {np.mean(ms):.2f} ms (max {max(ms):.2f})")
        assert g["inertia"] == ref["inertia"]
        assert g["best_k"] == ref["best_k"]
        for j, i in enumerate(SHARDS[r]):
            np.testing.assert_array_equal(g["tid"][j], ref["tid"][i])
            np.testing.assert_array_equal(g["cid"][j], ref["cid"][i])
    # clustering rows: rank order = image order
    np.testing.assert_array_equal(np.concatenate([got[0]["rows_labels"], got[1]["rows_labels"]]),
                                  ref["rows_labels"])
    for r in (0, 1):
        # the sharded fit (k = 6) and the sweep ran in the C driver
        # (mw_lloyd_fits_sharded), the single process in mw_kmeans_fit /
        # mw_lloyd_fits; the Python loop over the same shards gives the same bits
        g = got[r]
        assert g["fits_c"]["sharded"] >= 2 and g["fits_c"]["local"] == 0, g["fits_c"]
        py = g["pyloop"]
        assert py["fits_c"]["sharded"] == 0, py["fits_c"]
        for key in ("idx", "centers", "curve", "rows_labels"):
            np.testing.assert_array_equal(py[key], g[key], err_msg=f"python loop vs C: {key}")
        assert py["n_iter"] == g["n_iter"] and py["inertia"] == g["inertia"] and py["best_k"] == g["best_k"]
        for j in range(len(SHARDS[r])):
            np.testing.assert_array_equal(py["tid"][j], g["tid"][j])
            np.testing.assert_array_equal(py["cid"][j], g["cid"][j])


def _band_worker(rank, world, port, q):
    """One slide in row bands (milwrm_amd.bands): rank b preprocesses rows
    [y0, y1) (+ 8 halo rows), the sampled rows move by one all-to-all to
    the rank owning their draw positions, the fit runs row-sharded."""
    import torch
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        import milwrm_amd as M
        from milwrm_amd import bands
        from milwrm_amd.dist import DistComm

        comm = DistComm(device=torch.device("cpu"))
        raw, mask = _band_slide()
        im = bands.band_image(raw, mask, rank, world, halo=8)
        est, pix = im.calculate_non_zero_mean(comm)
        df = pd.DataFrame({"Img": [im], "batch_names": ["b1"], "mean estimators": [est],
                           "pixels": [pix]})
        lab = M.mxif_labeler(df)
        lab.prep_cluster_data(features=list(range(8)), sigma=2, fract=0.2, comm=comm)
        lab.label_tissue_regions(k=6, plot_out=False, random_state=18, comm=comm)
        lab.confidence_score_images()
        out = dict(est=np.asarray(est), pix=pix, mean=lab.scaler.mean_, scale=lab.scaler.scale_,
                   idx=lab.kmeans.init_indices_, n_iter=lab.kmeans.n_iter_,
                   centers=lab.kmeans.cluster_centers_, inertia=lab.kmeans.inertia_,
                   rows_labels=lab.kmeans.labels_, tid=np.nan_to_num(lab.tissue_IDs[0], nan=-1),
                   cid=np.nan_to_num(lab.confidence_IDs[0], nan=-1),
                   conf_df=lab.confidence_score_df.values, rows=(im._band.y0, im._band.y1))
        torch.cuda.synchronize()
        q.put((rank, out))
    except Exception as e:
        q.put((rank, repr(e)))
        raise
    finally:
        dist.destroy_process_group()


def _band_slide():
    from oracle.milwrm_oracle import synth_slide

    return synth_slide(208, 176, 8, seed=411, mode="hard")


@pytest.mark.timeout(600)
def test_row_bands_equal_single_process(gpu):
    """a single slide split into 2 row bands over 2 ranks gives
    the single-process result: the same estimators, k-means++ indices,
    n_iter, every pixel's label; centers / inertia / confidences to fp64
    rounding (the scaler statistics of the two row ranges are Chan-merged)."""
    import milwrm_amd as M

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_band_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    got = dict(q.get(timeout=540) for _ in ps)
    for p in ps:
        p.join(60)
    for r in (0, 1):
        assert not isinstance(got[r], str), got[r]
        assert ps[r].exitcode == 0
    raw, mask = _band_slide()
    im = M.img(raw.copy(), mask=mask.copy())
    est, pix = im.calculate_non_zero_mean()
    df = pd.DataFrame({"Img": [im], "batch_names": ["b1"], "mean estimators": [est],
                       "pixels": [pix]})
    lab = M.mxif_labeler(df)
    lab.prep_cluster_data(features=list(range(8)), sigma=2, fract=0.2)
    lab.label_tissue_regions(k=6, plot_out=False, random_state=18)
    lab.confidence_score_images()
    tid = np.nan_to_num(lab.tissue_IDs[0], nan=-1)
    cid = np.nan_to_num(lab.confidence_IDs[0], nan=-1)
    for r in (0, 1):
        g = got[r]
        np.testing.assert_array_equal(g["est"], np.asarray(est))
        assert g["pix"] == pix
        np.testing.assert_allclose(g["mean"], lab.scaler.mean_, rtol=1e-13)
        np.testing.assert_allclose(g["scale"], lab.scaler.scale_, rtol=1e-13)
        np.testing.assert_array_equal(g["idx"], lab.kmeans.init_indices_)
        assert g["n_iter"] == lab.kmeans.n_iter_
        np.testing.assert_allclose(g["centers"], lab.kmeans.cluster_centers_, rtol=1e-10, atol=1e-12)
        assert abs(g["inertia"] - lab.kmeans.inertia_) <= 1e-10 * abs(lab.kmeans.inertia_)
        y0, y1 = g["rows"]
        np.testing.assert_array_equal(g["tid"], tid[y0:y1])
        np.testing.assert_allclose(g["cid"], cid[y0:y1], rtol=1e-6, atol=1e-7)
        np.testing.assert_allclose(g["conf_df"], lab.confidence_score_df.values, rtol=1e-10)
    np.testing.assert_array_equal(np.concatenate([got[0]["rows_labels"], got[1]["rows_labels"]]),
                                  lab.kmeans.labels_)
