"""The RCCL message path on one GPU: a one-rank "nccl" process group with
``DistComm(force=True)`` runs every collective of the sharded path (device
message tensors, all_gather_into_tensor, all_reduce, all_to_all_single,
all_gather_object) through RCCL.  Whole slides per rank, one slide in a
single row band, and that band with its blur deferred into the fused
epilogues (MW_FUSED_BLUR=1) must all be BITWISE the LocalComm run: scaler,
k-means++ indices, n_iter, centers, inertia, every row's and pixel's label
and confidence, the confidence frame, and the k = 2..20 sweep curve.
(Two ranks cannot share one GPU under RCCL; the multi-rank logic of the same
collectives runs with gloo in tests/test_gpu_dist.py and test_dist_gloo.py.)"""
import os
import socket

import numpy as np
import pandas as pd
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
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


def _band_slide():
    from oracle.milwrm_oracle import synth_slide

    return synth_slide(208, 176, 8, seed=411, mode="hard")


def _result(lab, with_sweep):
    out = dict(mean=lab.scaler.mean_, scale=lab.scaler.scale_, idx=lab.kmeans.init_indices_,
               n_iter=lab.kmeans.n_iter_, centers=lab.kmeans.cluster_centers_,
               inertia=lab.kmeans.inertia_, rows_labels=lab.kmeans.labels_,
               tid=[np.nan_to_num(t, nan=-1) for t in lab.tissue_IDs],
               cid=[np.nan_to_num(c, nan=-1) for c in lab.confidence_IDs],
               conf_df=lab.confidence_score_df.values)
    if with_sweep:
        lab.find_optimal_k(random_state=18, alpha=0.05)
        out["best_k"] = int(lab.k)
        out["curve"] = lab.inertia_curve_["Scaled Inertia"].values
    return out


def _run_slides(comm):
    import milwrm_amd as M

    imgs = [M.img(r.copy(), mask=m.copy()) for r, m in _slides()]
    ests, pix = zip(*[im.calculate_non_zero_mean() for im in imgs])
    df = pd.DataFrame({"Img": imgs, "batch_names": BATCHES, "mean estimators": list(ests),
                       "pixels": list(pix)})
    lab = M.mxif_labeler(df)
    lab.prep_cluster_data(features=list(range(8)), sigma=2, fract=0.2, comm=comm)
    lab.label_tissue_regions(k=6, plot_out=False, random_state=18, comm=comm)
    lab.confidence_score_images()
    return _result(lab, True)


def _run_band(comm):
    """The band slide as one image (comm None) or as band 0 of 1 over comm."""
    import milwrm_amd as M
    from milwrm_amd import bands

    raw, mask = _band_slide()
    if comm is None:
        im = M.img(raw.copy(), mask=mask.copy())
        est, pix = im.calculate_non_zero_mean()
    else:
        im = bands.band_image(raw, mask, 0, 1, halo=8)
        est, pix = im.calculate_non_zero_mean(comm)
    df = pd.DataFrame({"Img": [im], "batch_names": ["b1"], "mean estimators": [est],
                       "pixels": [pix]})
    lab = M.mxif_labeler(df)
    lab.prep_cluster_data(features=list(range(8)), sigma=2, fract=0.2, comm=comm)
    lab.label_tissue_regions(k=6, plot_out=False, random_state=18, comm=comm)
    lab.confidence_score_images()
    out = _result(lab, False)
    out["est"], out["pix"] = np.asarray(est), pix
    return out


def _worker(port, q):
    import torch
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    os.environ.pop("MW_FUSED_BLUR", None)
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        from milwrm_amd import device as D
        from milwrm_amd.dist import LOCAL_COMM, DistComm

        from milwrm_amd import kmeans as KM

        comm = DistComm(force=True)
        assert comm.device.type == "cuda" and comm.sharded()
        res = {"local": _run_slides(LOCAL_COMM)}
        used = dict(KM.FITS_C_USED)
        res["nccl"] = _run_slides(comm)  # the fits in mw_lloyd_fits_sharded, records all-reduced by RCCL
        res["fits_c"] = {key: KM.FITS_C_USED[key] - used[key] for key in used}
        res.update(band_local=_run_band(None), band_nccl=_run_band(comm))
        before = dict(D.FUSED_USED)
        os.environ["MW_FUSED_BLUR"] = "1"
        res["band_fused"] = _run_band(comm)
        res["fused_used"] = {k: D.FUSED_USED[k] - before[k] for k in before}
        torch.cuda.synchronize()
        q.put(res)
    except Exception as e:  # surface the failure in the parent
        q.put(repr(e))
        raise
    finally:
        dist.destroy_process_group()


def _equal(a, b, what):
    for key in a:
        x, y = a[key], b[key]
        if isinstance(x, list):
            for i, (u, v) in enumerate(zip(x, y)):
                np.testing.assert_array_equal(u, v, err_msg=f"{what}: {key}[{i}]")
        else:
            np.testing.assert_array_equal(x, y, err_msg=f"{what}: {key}")


@pytest.mark.timeout(600)
def test_rccl_message_path_bitwise_equal_local(gpu):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(_free_port(), q))
    p.start()
    res = q.get(timeout=540)
    p.join(60)
    assert not isinstance(res, str), res
    assert p.exitcode == 0
    _equal(res["local"], res["nccl"], "whole slides, nccl vs local")
    assert res["fits_c"]["sharded"] >= 2 and res["fits_c"]["local"] == 0, res["fits_c"]
    _equal(res["band_local"], res["band_nccl"], "one band, nccl vs local")
    _equal(res["band_local"], res["band_fused"], "one band with deferred blur vs local")
    # the deferred band really took the fused sample epilogue and the banded label pass
    assert res["fused_used"]["sample"] >= 1 and res["fused_used"]["assign_banded"] >= 1
