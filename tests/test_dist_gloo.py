"""world_size-2 gloo tests (CPU) of the sharded path's host-side collectives:
batch means, Chan-merged scaler statistics, per-batch sums."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from milwrm_amd.dist import DistComm

        comm = DistComm(device=__import__("torch").device("cpu"))
        rng = np.random.default_rng(rank)
        X = rng.normal(rank, 1 + rank, size=(100 + 37 * rank, 5))
        st = np.concatenate([[X.shape[0]], X.mean(0), X.var(0) * X.shape[0]])
        merged = comm.merge_stats(st, 5)
        est = [10.0 * (rank + 1), 20.0]
        e, p = comm.batch_stats(est, 7 + rank)
        per = {"a": (np.array([1.0 + rank, 2.0]), 3 + rank)}
        if rank == 1:
            per["b"] = (np.array([5.0, 6.0]), 9)
        sb = comm.sum_batches(per)
        q.put((rank, merged, e, p, {k: (v[0].tolist(), float(v[1])) for k, v in sb.items()}))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_gloo_world2_collectives():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict((r[0], r[1:]) for r in [q.get(timeout=90) for _ in ps])
    for p in ps:
        p.join(30)
        assert p.exitcode == 0
    rng0, rng1 = np.random.default_rng(0), np.random.default_rng(1)
    X = np.vstack([rng0.normal(0, 1, size=(100, 5)), rng1.normal(1, 2, size=(137, 5))])
    for r in (0, 1):
        merged, e, p, sb = res[r]
        assert merged[0] == 237
        np.testing.assert_allclose(merged[1:6], X.mean(0), rtol=1e-12)
        np.testing.assert_allclose(merged[6:] / 237, X.var(0), rtol=1e-12)
        assert e == [30.0, 40.0] and p == 15
        assert sb["a"] == ([3.0, 4.0], 7.0) and sb["b"] == ([5.0, 6.0], 9.0)
