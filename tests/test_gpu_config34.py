"""BASELINE configs 3 and 4 at their full per-rank size: two 20k x 20k x 30
slides (the per-GPU share of config 3's 8-slide set) as 2 ranks on one GPU
(spawned processes, gloo for the messages), against the single-process run
over both slides:

* config 3 (prep + k = 8 fit + labels + confidences, row-sharded fit with one
  all-reduce of exact fixed-point records per Lloyd pass): BITWISE equal --
  scaler, k-means++ indices, n_iter, centers, inertia, every row label, and
  every pixel's label and confidence (compared by digest: 4e8 pixels each);
* config 4 (the k = 2..20 find_optimal_k sweep over the 1.36e8 rows, all
  fits batched per Lloyd pass): the curve and best_k bitwise equal to the
  single-process sweep, and every k's inertia within 1e-6 of an fp64
  recompute from its labels and centers.
"""
import hashlib
import os
import socket

import numpy as np
import pandas as pd
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
SIZE, C, K = 20_000, 30, 8
SEEDS = [20251015, 20251016]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _digest(t: torch.Tensor) -> str:
    return hashlib.sha256(t.contiguous().cpu().numpy().tobytes()).hexdigest()


def _run(seeds, comm):
    import milwrm_amd as M
    from milwrm_amd import device as D

    imgs = [M.img.from_device(*D.synth_slide(SIZE, SIZE, C, seed=s)) for s in seeds]
    ests, pix = zip(*[im.calculate_non_zero_mean() for im in imgs])
    df = pd.DataFrame({"Img": imgs, "batch_names": ["b"] * len(imgs), "mean estimators": list(ests),
                       "pixels": list(pix)})
    lab = M.mxif_labeler(df)
    lab.prep_cluster_data(features=list(range(C)), sigma=2, fract=0.2, comm=comm)
    lab.label_tissue_regions(k=K, plot_out=False, random_state=18, comm=comm)
    lab.confidence_score_images()
    out = dict(mean=lab.scaler.mean_, scale=lab.scaler.scale_, idx=lab.kmeans.init_indices_,
               n_iter=lab.kmeans.n_iter_, centers=lab.kmeans.cluster_centers_,
               inertia=lab.kmeans.inertia_, rows_digest=_digest(lab.kmeans._labels_dev),
               S=lab._rows.S, conf_df=lab.confidence_score_df.values,
               tid=[_digest(t) for t in lab._labels_dev], cid=[_digest(c) for c in lab._conf_dev])
    del imgs, df
    lab.find_optimal_k(random_state=18, alpha=0.05)
    out["best_k"] = int(lab.k)
    out["curve"] = lab.inertia_curve_["Scaled Inertia"].values
    return out, lab


def _worker(rank, world, port, q):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        from milwrm_amd.dist import DistComm

        res, _ = _run([SEEDS[rank]], DistComm(device=torch.device("cpu")))
        torch.cuda.synchronize()
        q.put((rank, res))
    except Exception as e:  # surface the failure in the parent
        q.put((rank, repr(e)))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(1200)
def test_config3_config4_two_ranks_full_size(gpu):
    from milwrm_amd import device as D
    from milwrm_amd.kmeans import fit_many

    D.WS.clear()
    torch.cuda.empty_cache()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    got = dict(q.get(timeout=1000) for _ in ps)
    for p in ps:
        p.join(120)
    for r in (0, 1):
        assert not isinstance(got[r], str), got[r]
        assert ps[r].exitcode == 0
    ref, lab = _run(SEEDS, None)
    assert ref["S"] == got[0]["S"] + got[1]["S"] > 1.3e8
    for r in (0, 1):
        g = got[r]
        for key in ("mean", "scale", "idx", "centers", "curve"):
            np.testing.assert_array_equal(g[key], ref[key], err_msg=key)
        np.testing.assert_array_equal(g["conf_df"], ref["conf_df"][r:r + 1])  # this rank's slide
        assert g["n_iter"] == ref["n_iter"]
        assert g["inertia"] == ref["inertia"]
        assert g["best_k"] == ref["best_k"]
        assert g["tid"][0] == ref["tid"][r] and g["cid"][0] == ref["cid"][r]
    # the clustering rows: rank order = image order
    lab_rows = lab.kmeans._labels_dev
    S0 = got[0]["S"]
    assert _digest(lab_rows[:S0]) == got[0]["rows_digest"]
    assert _digest(lab_rows[S0:]) == got[1]["rows_digest"]
    # config 4: every k's inertia against an fp64 recompute from its labels and centers
    rows = lab._device_rows()
    fits = fit_many(rows, list(range(2, 21)), random_state=18)
    smu = torch.from_numpy(rows.mu).cuda()
    sinv = torch.from_numpy(rows.inv).cuda()
    inertia_o = rows.S * float(np.sum(rows.feature_var()))
    curve = [km.inertia_ / inertia_o + 0.05 * k for km, k in zip(fits, range(2, 21))]
    np.testing.assert_array_equal(np.asarray(curve), ref["curve"])
    step = 4_000_000
    for km in fits:
        Cn = torch.from_numpy(km.cluster_centers_).cuda()
        labels = km._labels_dev.long()
        tot = 0.0
        for a in range(0, rows.S, step):
            b = min(rows.S, a + step)
            xs = (rows.X[a:b].double() - smu) * sinv
            tot += float(((xs - Cn[labels[a:b]]) ** 2).sum())
        assert abs(km.inertia_ - tot) <= 1e-6 * tot, (km.n_clusters, km.inertia_, tot)
