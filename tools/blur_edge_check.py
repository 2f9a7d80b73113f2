"""Blur edge cases (tests/golden/preproc_edges.npz): MFMA and VALU kernels vs the golden outputs."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from milwrm_amd import device as D  # noqa: E402

torch.cuda.set_device(0)
g = np.load(os.path.join(os.path.dirname(__file__), "..", "tests", "golden", "preproc_edges.npz"))
for i in range(5):
    a = g[f"gauss{i}_in"]
    sig = float(g[f"gauss{i}_sigma"])
    x = torch.from_numpy(a.astype(np.float32)).cuda()
    for impl in ["mfma", "valu"]:
        if impl == "valu":
            os.environ["MW_BLUR_IMPL"] = "valu"
        out = D.blur(x, sig).cpu().numpy()
        os.environ.pop("MW_BLUR_IMPL", None)
        err = np.abs(out - g[f"gauss{i}_out"])
        print(f"case {i} shape {a.shape} sigma {sig}: {impl} max abs err {err.max():.3e}", flush=True)
        if err.max() > 1e-4:
            ys, xs, cs = np.nonzero(err > 1e-4)
            print("   bad cols", np.unique(xs)[:20], "rows", np.unique(ys)[:10], "ch", np.unique(cs))
