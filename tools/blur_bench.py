"""Blur-only timing on one synthetic 30-channel uint16 slide: kernel time per
launch (HIP events on the launch stream) for several band geometries
(env overrides, e.g. MW_BLUR_BH=256 MW_BLUR_BT=3), plus a bitwise cross-check
between the variants."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from milwrm_amd import device as D  # noqa: E402

size = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
C = int(sys.argv[2]) if len(sys.argv) > 2 else 30
torch.cuda.set_device(0)
raw, mask = D.synth_slide(size, size, C, seed=7, mode="hard")
inv = ((torch.arange(C, device="cuda", dtype=torch.float32) * 37) % 11 + 1) * 1e-4  # deterministic
ref = None
variants = sys.argv[3].split(",") if len(sys.argv) > 3 else ["", "MW_BLUR_BH=256"]
for bw in variants:
    for kv in ("MW_BLUR_BH", "MW_BLUR_XCD", "MW_BLUR_BT", "MW_BLUR_BT8"):
        os.environ.pop(kv, None)
    for kv in filter(None, bw.split(";")):
        k, v = kv.split("=")
        os.environ[k] = v
    out = D.blur(raw, 2.0, inv_mean=inv)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = 10
    e0.record()
    for _ in range(n):
        out = D.blur(raw, 2.0, inv_mean=inv)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / n
    gb = size * size * C * (raw.element_size() + 4) / 1e9
    same = None if ref is None else bool(torch.equal(out, ref))
    if ref is None:
        ref = out.clone()
        if os.environ.get("BLUR_SAVE"):  # strided sample of the first variant, for cross-library checks
            import numpy as np
            np.save(os.environ["BLUR_SAVE"], out.view(size, size, C)[::37, ::41].cpu().numpy())
    print(f"BW={bw or 'default'}: {ms:.3f} ms/launch, {gb / ms * 1e3:.0f} GB/s algorithmic, same={same}",
          flush=True)
