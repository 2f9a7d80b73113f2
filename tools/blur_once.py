"""One warm + a few timed launches of the fused blur on a 10000^2 x 30 u16 slide
(profiling target)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from milwrm_amd import device as D  # noqa: E402

size = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
torch.cuda.set_device(0)
raw, mask = D.synth_slide(size, size, 30, seed=7, mode="hard")
inv = torch.rand(30, device="cuda", dtype=torch.float32) * 1e-3 + 1e-4
for _ in range(3):
    out = D.blur(raw, 2.0, inv_mean=inv)
torch.cuda.synchronize()
print("ok", float(out[0, 0, 0]))
