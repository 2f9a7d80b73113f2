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
    lab.find_optimal_k(random_state=18, alpha=0.05)
    out["best_k"] = int(lab.k)
    out["curve"] = lab.inertia_curve_["Scaled Inertia"].values
    return out


def _worker(rank, world, port, q):
    import torch
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        from milwrm_amd.dist import DistComm

        slides = _slides()
        mine = SHARDS[rank]
        res = _run([slides[i] for i in mine], [BATCHES[i] for i in mine],
                   DistComm(device=torch.device("cpu")))
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
        assert g["inertia"] == ref["inertia"]
        assert g["best_k"] == ref["best_k"]
        for j, i in enumerate(SHARDS[r]):
            np.testing.assert_array_equal(g["tid"][j], ref["tid"][i])
            np.testing.assert_array_equal(g["cid"][j], ref["cid"][i])
    # clustering rows: rank order = image order
    np.testing.assert_array_equal(np.concatenate([got[0]["rows_labels"], got[1]["rows_labels"]]),
                                  ref["rows_labels"])
