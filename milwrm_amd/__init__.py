"""milwrm_amd — MI355X-native MILWRM pixel-clustering hot path.

Public API mirrors ``MILWRM/__init__.py:7-29`` (img, mxif_labeler,
st_labeler, blur_features_st, map_pixels, trim_image, assemble_pita,
show_pita) plus the sklearn-shaped ``KMeans`` / ``StandardScaler`` that run
on the HIP kernels."""
from .MILWRM import (
    chooseBestKforKMeansParallel,
    kMeansRes,
    mxif_labeler,
    st_labeler,
    tissue_labeler,
)
from .MxIF import img
from .ST import assemble_pita, blur_features_st, map_pixels, show_pita, trim_image
from .kmeans import DeviceRows, KMeans, StandardScaler

__all__ = [
    "img",
    "blur_features_st",
    "map_pixels",
    "trim_image",
    "assemble_pita",
    "show_pita",
    "mxif_labeler",
    "st_labeler",
    "tissue_labeler",
    "KMeans",
    "StandardScaler",
    "DeviceRows",
    "kMeansRes",
    "chooseBestKforKMeansParallel",
]

__version__ = "0.1.0"
