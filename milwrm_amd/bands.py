"""One slide split into row bands over the ranks of a process group (SURVEY
§8(e): "a single slide ... is split into row bands with ±r halo rows read from
the input"; config 2 on more than one GPU).

Rank b holds rows [y0, y1) of the slide plus up to ``halo`` rows above and
below (read from the input, no exchange), so its blur of the band rows is the
whole-slide blur of those rows, operation for operation.  What couples the
bands, and how:

* ``calculate_non_zero_mean`` (MxIF.py:519-541): exact integer-valued channel
  sums and counts of the band rows, all-reduced — every band reports the
  slide's estimators; the batch means count the slide once (band 0).
* ``subsample_pixels`` (MxIF.py:457-492): the draws index the slide's masked
  pixels in row-major order, i.e. band 0's, then band 1's...  Band b's mask
  rank is offset by the masked pixels above it (all-gather of the counts);
  every rank generates the same S draws on its device (legacy MT19937).  The
  clustering rows must stay in draw order with each rank owning a contiguous
  range of it (the sharded k-means++ and relocation rely on that), so rank b
  gathers the rows of the draws that fall in its band and ONE all-to-all moves
  every row to the rank that owns its draw position ``j`` — the path's only
  bulk exchange (S x F x 4 bytes in total).
* StandardScaler: column statistics of each rank's rows, Chan-merged in rank
  order (= draw order).
* the fit: the existing row-sharded KMeans (one all-reduce per Lloyd pass).
* labels / confidence: each band labels its own rows; the per-domain sums of
  the confidence frame are all-reduced.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import torch

from . import device as D


@dataclass(frozen=True)
class BandInfo:
    H: int        # slide rows
    y0: int       # band rows [y0, y1) of the slide
    y1: int
    lo: int       # local array rows = slide rows [lo, hi) (band + halo)
    hi: int
    band: int
    n_bands: int
    halo: int

    @property
    def rows(self) -> slice:
        """The band rows inside the local (halo'd) array."""
        return slice(self.y0 - self.lo, self.y1 - self.lo)


def band_rows(H: int, n_bands: int, band: int, halo: int = 8):
    """(y0, y1, lo, hi) of band ``band`` of ``n_bands`` near-equal row bands of
    an H-row slide, with up to ``halo`` input rows on each side."""
    if not (0 <= band < n_bands <= H):
        raise ValueError(f"band {band} of {n_bands} for a slide of {H} rows")
    y0, y1 = H * band // n_bands, H * (band + 1) // n_bands
    return y0, y1, max(0, y0 - halo), min(H, y1 + halo)


def band_image(slide, mask, band: int, n_bands: int, halo: int = 8, channels=None):
    """The ``img`` of band ``band`` cut from a whole slide (host array or HWC
    device tensor; only rows [lo, hi) are kept).  A loader that reads rows
    itself passes the halo'd rows with ``band_image_rows``."""
    H = int(slide.shape[0])
    y0, y1, lo, hi = band_rows(H, n_bands, band, halo)
    m = None if mask is None else mask[lo:hi]
    return band_image_rows(slide[lo:hi], m, H, band, n_bands, halo, channels)


def band_image_rows(rows, mask, H: int, band: int, n_bands: int, halo: int = 8, channels=None):
    """``img`` from the halo'd rows [lo, hi) of band ``band`` (see band_rows)."""
    from .MxIF import img

    y0, y1, lo, hi = band_rows(H, n_bands, band, halo)
    if int(rows.shape[0]) != hi - lo:
        raise ValueError(f"band {band}: {rows.shape[0]} rows given, rows [{lo}, {hi}) expected")
    if isinstance(rows, torch.Tensor):
        im = img.from_device(rows.contiguous(), mask=None if mask is None else mask.contiguous(),
                             channels=channels)
    else:
        im = img(np.ascontiguousarray(rows), channels=channels,
                 mask=None if mask is None else np.ascontiguousarray(mask))
    im._band = BandInfo(H, y0, y1, lo, hi, band, n_bands, halo)
    return im


def check_group(images, comm):
    """Banded prep needs exactly one band image per rank, band index = rank,
    as many bands as ranks."""
    if len(images) != 1:
        raise NotImplementedError("a rank holding a slide band holds no other image")
    b = images[0]._band
    world = comm.world if comm.sharded() else 1
    rank = comm.rank if comm.sharded() else 0
    if b.n_bands != world or b.band != rank:
        raise ValueError(f"band {b.band} of {b.n_bands} on rank {rank} of {world}: "
                         "band index must equal the rank and the bands span the group")
    return b


def owner_bounds(S: int, world: int) -> np.ndarray:
    """Draw positions [bnd[r], bnd[r+1]) owned by rank r (contiguous, rank order)."""
    return np.array([S * r // world for r in range(world + 1)], dtype=np.int64)


def exchange_rows(rows: torch.Tensor, send_counts, comm) -> tuple[torch.Tensor, list]:
    """All-to-all of row blocks: ``rows`` holds the rows for rank 0, then rank
    1, ... (``send_counts`` of them); returns the rows received, source 0
    first, and the per-source counts.  Message tensors live on comm.device
    (RCCL: the rows stay in HBM; gloo: staged through host memory)."""
    F = int(rows.shape[1])
    send_counts = [int(c) for c in send_counts]
    recv_counts = [int(c) for c in comm.all_to_all_counts(send_counts)]
    dev = comm.device
    src = rows.reshape(-1).to(dev) if rows.device != dev else rows.reshape(-1)
    out = torch.empty(sum(recv_counts) * F, dtype=rows.dtype, device=dev)
    comm.all_to_all_single(out, src.contiguous(), [c * F for c in recv_counts],
                           [c * F for c in send_counts])
    return out.reshape(-1, F).to(rows.device), recv_counts


def placement(src_of: torch.Tensor) -> torch.Tensor:
    """Row positions (in draw order) of the received blocks: the rows from
    source s arrive in increasing draw order, so position order = a stable
    sort of the owned draws by their source band."""
    return torch.sort(src_of, stable=True).indices


def route_draws(idx64: torch.Tensor, off, band: int, bnd):
    """The draws (global mask ranks ``idx64``, draw order) that fall in band
    ``band`` (ranks [off[band], off[band+1])): their draw positions j, their
    ranks inside the band (int32, for the gather) and how many go to each
    rank (rank d owns positions [bnd[d], bnd[d+1]); positions ascend, so the
    rows are already grouped by destination)."""
    lo, hi = int(off[band]), int(off[band + 1])
    pos = torch.nonzero((idx64 >= lo) & (idx64 < hi)).reshape(-1)
    local_idx = (idx64[pos] - lo).to(torch.int32).contiguous()
    bnd_t = torch.as_tensor(np.asarray(bnd, dtype=np.int64), device=idx64.device)
    dest = torch.searchsorted(bnd_t, pos, right=True) - 1
    send = torch.bincount(dest, minlength=len(bnd) - 1).cpu().tolist()
    return pos, local_idx, send


def assemble_rows(recv: torch.Tensor, idx64: torch.Tensor, off, bnd, rank: int) -> torch.Tensor:
    """This rank's rows in draw order from the blocks received (source band
    0 first, each in increasing draw position)."""
    lo_j, hi_j = int(bnd[rank]), int(bnd[rank + 1])
    off_t = torch.as_tensor(np.asarray(off, dtype=np.int64), device=idx64.device)
    src_of = torch.searchsorted(off_t, idx64[lo_j:hi_j], right=True) - 1
    X = torch.empty((hi_j - lo_j, recv.shape[1]), dtype=recv.dtype, device=recv.device)
    if hi_j > lo_j:
        X[placement(src_of).to(recv.device)] = recv
    return X


def prep_banded(image, batch, means, features, filter_name, sigma, fract, comm):
    """mxif_labeler.prep_cluster_data for one band per rank (module docstring).
    Returns (X rows of this rank in draw order, per-rank column stats, xmax).
    A band whose blur is deferred (D.defer_blur: its fp32 blurred copy would
    not fit beside the raw rows) gathers its sampled rows straight from the
    fused blur epilogue over the halo'd rows, like the whole-slide path."""
    b = check_group([image], comm)
    dev = D.device()
    r = int(4.0 * float(sigma) + 0.5)
    if filter_name == "gaussian" and r > b.halo and b.n_bands > 1:
        raise ValueError(f"blur radius {r} exceeds the band halo of {b.halo} rows")
    image.log_normalize(mean=means[batch])
    image.blurring(filter_name=filter_name, sigma=sigma)
    W = int(image.shape[1])
    # mask rank of the band rows, global offsets from the bands above
    mb = D.padded_mask(image._mask_device()[b.rows].contiguous())
    r2p, Mb = D.mask_rank(mb.reshape(-1))
    Ms = comm.all_gather_np(np.array([Mb], dtype=np.int64))[:, 0] if comm.sharded() else np.array([Mb])
    off = np.concatenate([[0], np.cumsum(Ms)]).astype(np.int64)
    M = int(off[-1])
    F = len(image._features(features))
    np.random.seed(16)
    from .rng import check_total, set_global_state_after_draws, subsample_indices_device

    idx, total = subsample_indices_device(M, fract, 16, dev)
    S = int(idx.shape[0])
    world = b.n_bands
    from .MILWRM import _check_rows_fit, _gather_deferred

    _check_rows_fit(S // world + 1, F, dev)
    bnd = owner_bounds(S, world)
    idx64 = idx.to(torch.int64)
    pos, local_idx, send_counts = route_draws(idx64, off, b.band, bnd)
    rows = torch.empty((int(pos.numel()), F), dtype=torch.float32, device=dev)
    if rows.shape[0]:
        feat = D.h2d(np.asarray(image._features(features), dtype=np.int32), dev)
        # pixel index of each band-row rank inside the local (halo'd) array
        k = (b.y0 - b.lo) * W
        r2p_local = (r2p.offset(k) if isinstance(r2p, D.RankIndex) else r2p + k) if k else r2p
        if not _gather_deferred(image, feat, local_idx, r2p_local, rows):
            src = D.as_float32(image._materialize())  # band + halo rows, blurred
            scratch = torch.zeros(1 + 2 * F, dtype=torch.float64, device=dev)
            D.gather_rows(src[b.rows], feat, local_idx, r2p, rows, scratch, accumulate=False)
    # rows move to the rank owning their draw position
    recv = exchange_rows(rows, send_counts, comm)[0] if world > 1 else rows
    X = assemble_rows(recv, idx64, off, bnd, b.band)
    check_total(total, S)
    set_global_state_after_draws()
    stats = torch.zeros((1, 1 + 2 * F), dtype=torch.float64, device=dev)
    xmax = torch.zeros(F, dtype=torch.float32, device=dev)
    D.col_stats_rows(X, stats[0], accumulate=False, absmax=xmax)
    return X, stats, xmax
