"""ST-side plumbing of MILWRM (ST.py).  Only ``blur_features_st`` is on the
st_labeler path; it is a tiny sparse neighbour mean over ~10^3-10^4 spots,
kept on the host (scipy.sparse), outside the GPU hot path.
The Visium image utilities are out of scope."""
from __future__ import annotations

import numpy as np
import scipy.sparse as sp


def blur_features_st(adata, tmp, spatial_graph_key=None, n_rings=1):
    """ST.py:25-77: each spot's features averaged with its non-zero spatial
    neighbours (a self-loop in the graph counts twice, as in the reference)."""
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
    A = sp.csr_matrix(adata.obsp[spatial_graph_key])
    A.eliminate_zeros()
    A.data = np.ones_like(A.data, dtype=np.float64)
    n = A.shape[0]
    M = A + sp.identity(n, format="csr")
    deg = np.asarray(A.getnnz(axis=1) + 1, dtype=np.float64)
    cols = tmp.columns
    vals = tmp.loc[:, cols].values.astype(np.float64)
    blurred = (M @ vals) / deg[:, None]
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
