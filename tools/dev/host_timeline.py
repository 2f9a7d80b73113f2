"""Host timeline of the config-2 bench step: wall-clock entry/exit marks of
the main host calls (monkeypatched wrappers), printed per step relative to
the step start, to see what the device may idle behind.

  python tools/dev/host_timeline.py [--steps 3]
"""
import functools
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import pandas as pd  # noqa: E402
import torch  # noqa: E402

MARKS = []


def wrap(owner, name, label=None):
    f = getattr(owner, name)
    label = label or name

    @functools.wraps(f)
    def g(*a, **k):
        MARKS.append((time.perf_counter(), ">" + label))
        try:
            return f(*a, **k)
        finally:
            MARKS.append((time.perf_counter(), "<" + label))
    setattr(owner, name, g)


def main():
    steps = int(sys.argv[sys.argv.index("--steps") + 1]) if "--steps" in sys.argv else 3
    import bench
    import milwrm_amd as M
    from milwrm_amd import MILWRM as MW
    from milwrm_amd import device as D
    from milwrm_amd import kmeans as KM
    from milwrm_amd import MxIF as MX
    from milwrm_amd.dist import make_comm

    torch.cuda.set_device(0)
    slides = bench.Slides(10000, 10000, 30, [20251015], "device", "hard")
    step = bench.make_step(slides, 30, 8, make_comm())
    wrap(MX.img, "calculate_non_zero_mean", "nzmean")
    wrap(pd, "DataFrame")
    wrap(MW.mxif_labeler, "__init__", "labeler_init")
    wrap(MW.mxif_labeler, "prep_cluster_data", "prep")
    wrap(MW.mxif_labeler, "_batch_means")
    wrap(MX.img, "log_normalize")
    wrap(MX.img, "blurring")
    wrap(D, "blur")
    wrap(D, "d2h")
    wrap(D, "mask_rank")
    wrap(MW, "_draws_beside")
    wrap(D, "gather_rows")
    wrap(MW, "set_global_state_after_draws")
    wrap(KM.KMeans, "fit", "kmeans_fit")
    wrap(MW.mxif_labeler, "label_tissue_regions", "label")
    wrap(MW, "_assign_img")
    wrap(MW.mxif_labeler, "confidence_score_images", "conf")
    for _ in range(2):
        step()
    torch.cuda.synchronize()
    for s in range(steps):
        MARKS.clear()
        t0 = time.perf_counter()
        step()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"--- step {s}: host {1e3 * (t1 - t0):.3f} ms, +sync {1e3 * (t2 - t0):.3f} ms")
        for t, lab in MARKS:
            print(f"{1e3 * (t - t0):9.3f}  {lab}")
    print("[host_timeline] done")


if __name__ == "__main__":
    main()
