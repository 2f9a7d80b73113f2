"""MFMA blur vs VALU blur on small slides: where do they differ?"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from milwrm_amd import device as D  # noqa: E402

torch.cuda.set_device(0)
for (H, W, C) in [(40, 70, 30), (300, 300, 30), (256 + 40, 64 * 3 + 5, 16)]:
    raw, mask = D.synth_slide(H, W, C, seed=3, mode="hard")
    inv = torch.rand(C, device="cuda", dtype=torch.float32) * 1e-2 + 1e-3
    a = D.blur(raw, 2.0, inv_mean=inv)
    os.environ["MW_BLUR_IMPL"] = "valu"
    b = D.blur(raw, 2.0, inv_mean=inv)
    del os.environ["MW_BLUR_IMPL"]
    torch.cuda.synchronize()
    d = (a - b).abs().cpu().numpy()
    bad = d > 1e-5 * np.abs(b.cpu().numpy()).max()
    print(f"{H}x{W}x{C}: max abs {d.max():.3e}, bad {bad.sum()} of {bad.size}", flush=True)
    if bad.any():
        ys, xs, cs = np.nonzero(bad)
        print("  rows", np.unique(ys)[:20], "n", len(np.unique(ys)))
        print("  cols", np.unique(xs)[:40], "n", len(np.unique(xs)))
        print("  chans", np.unique(cs))
        i = 0
        print("  sample", ys[i], xs[i], cs[i], a[ys[i], xs[i], cs[i]].item(), b[ys[i], xs[i], cs[i]].item())
