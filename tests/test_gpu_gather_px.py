"""The draws-as-pixels gather (MW_GATHER_PX=1: mw_rank_to_pixel_ri through
the compact rank index, then the lookup-free mw_gather_rows_px) gives the
rank-table gather's rows and column-statistics records bit for bit, on a
ragged mask (rows of no tissue, isolated pixels) and a band offset."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("pix_off", [0, 777])
def test_pixel_gather_equals_table_gather(gpu, pix_off):
    from milwrm_amd import device as D

    H, W, C, F = 300, 420, 12, 7
    rng = np.random.default_rng(5)
    img = torch.from_numpy(rng.normal(size=(H, W, C)).astype(np.float32)).to(gpu)
    mask = (rng.random((H, W)) < 0.55).astype(np.uint8)
    mask[40:70] = 0
    mask[100, ::37] = 1
    m = torch.from_numpy(mask).to(gpu).reshape(-1)
    n = H * W
    M = int(mask.sum())
    table = torch.empty(n, dtype=torch.int32, device=gpu)
    cnt = torch.empty(1, dtype=torch.int64, device=gpu)
    ws = torch.empty(D.N.query("mw_mask_rank_ws_bytes", n), dtype=torch.uint8, device=gpu)
    D.N.call("mw_mask_rank", D.P(m), n, D.P(table), D.P(cnt), D.P(ws), D.stream())
    buf = torch.empty(D.N.query("mw_rank_index_bytes", n), dtype=torch.uint8, device=gpu)
    D.N.call("mw_mask_rank_index", D.P(m), n, D.P(buf), D.P(cnt), D.P(ws), D.stream())
    assert int(cnt.item()) == M
    feat = torch.tensor([0, 3, 4, 5, 8, 10, 11], dtype=torch.int32, device=gpu)
    S = 9000
    idx = torch.from_numpy(rng.integers(0, M, size=S).astype(np.int32)).to(gpu)
    # the table form over an image whose first pix_off pixels are a pad
    big = torch.cat([torch.zeros((pix_off, C), device=gpu), img.reshape(-1, C)]).reshape(1, -1, C)
    X_t = torch.empty((S, F), dtype=torch.float32, device=gpu)
    st_t = torch.zeros(1 + 2 * F, dtype=torch.float64, device=gpu)
    shifted = (table[:M] + pix_off).contiguous()
    D.gather_rows(big, feat, idx, shifted, X_t, st_t, False)
    pix = idx.clone()
    D.rank_to_pixel(pix, D.RankIndex(buf, n, pix_off))
    assert torch.equal(pix, shifted[idx.long()])
    X_p = torch.empty_like(X_t)
    st_p = torch.zeros_like(st_t)
    D.gather_rows(big, feat, pix, None, X_p, st_p, False)
    assert torch.equal(X_p, X_t)
    assert torch.equal(st_p, st_t)
