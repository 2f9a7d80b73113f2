"""ST-side plumbing of MILWRM (ST.py).  Only ``blur_features_st`` is on the
st_labeler path: the neighbour mean over the spatial graph runs on the device
(``mw_neighbor_mean``, a CSR sparse product).  The Visium image utilities are
out of scope."""
from __future__ import annotations

import numpy as np
import scipy.sparse as sp
import torch


def blur_features_st(adata, tmp, spatial_graph_key=None, n_rings=1):
    """ST.py:25-77: each spot's features averaged (NaN skipped, as pandas'
    mean) with its non-zero spatial neighbours; a self-loop in the graph
    counts twice, as in the reference."""
    if spatial_graph_key is not None:
        assert spatial_graph_key in adata.obsp.keys(), \
            "Spatial connectivities key '{}' not found.".format(spatial_graph_key)
    else:
        try:
            import squidpy as sq
        except ImportError as e:
            raise ImportError("computing a spatial graph needs squidpy; pass spatial_graph_key "
                              "for a precomputed graph") from e
        print("Computing spatial graph with {} hexagonal rings".format(n_rings))
        sq.gr.spatial_neighbors(adata, coord_type="grid", n_rings=n_rings)
        spatial_graph_key = "spatial_connectivities"
    from . import _native as N
    from . import device as D

    A = sp.csr_matrix(adata.obsp[spatial_graph_key])
    A.sum_duplicates()
    A.eliminate_zeros()  # np.argwhere of the row: stored zeros are no neighbours
    A.sort_indices()
    n = A.shape[0]
    cols = tmp.columns
    vals = np.ascontiguousarray(tmp.loc[:, cols].values, dtype=np.float64)
    F = vals.shape[1]
    dev = D.device()
    ip = torch.from_numpy(A.indptr.astype(np.int64)).to(dev)
    ix = torch.from_numpy(A.indices.astype(np.int32)).to(dev)
    xv = torch.from_numpy(vals).to(dev)
    out = torch.empty_like(xv)
    N.call("mw_neighbor_mean", D.P(ip), D.P(ix), n, D.P(xv), F, D.P(out), D.stream())
    blurred = D.d2h(out)
    tmp2 = tmp.copy()
    tmp2.loc[:, cols] = blurred
    adata.obs[[x for x in cols]] = tmp.loc[:, cols].values
    adata.obs[["blur_" + x for x in cols]] = tmp2.loc[:, cols].values
    return tmp2.loc[:, cols]


def _out_of_scope(name):
    def f(*a, **k):
        raise NotImplementedError(f"{name} (Visium image plumbing / plotting) is outside the "
                                  "MI355X hot path")
    f.__name__ = name
    return f


map_pixels = _out_of_scope("map_pixels")
trim_image = _out_of_scope("trim_image")
assemble_pita = _out_of_scope("assemble_pita")
show_pita = _out_of_scope("show_pita")
