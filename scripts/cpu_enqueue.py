"""CPU cost of enqueueing one configs[2] training step (eager launches) against
the GPU time of the same steps: is the eager step bound by the host's launch
rate?  Prints per-step CPU enqueue time (no sync inside the timed loop, so the
host runs ahead unless it is the slower side) and per-step wall time."""
import time

import numpy as np
import torch

from posecnn_amd import _lib, synth
from posecnn_amd.pipeline import PoseStep

_lib.load()
dev = torch.device("cuda", 0)
B, H, W, C = 8, 480, 640, 22
fr = synth.make_frames(B, H, W, num_classes=C, objects_per_image=6, seed=3)
g = torch.Generator(device=dev)
g.manual_seed(1234)
to = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
inputs = dict(label=to(fr["label"]), vertex=to(fr["vertex"]), extents=to(fr["extents"]), meta=to(fr["meta"]),
              gt=to(fr["gt"]), conv4=torch.randn((B, H // 8, W // 8, 512), generator=g, device=dev),
              conv5=torch.randn((B, H // 16, W // 16, 512), generator=g, device=dev))
pts, sym = synth.rescaled_points(C)
inputs["points"], inputs["symmetry"] = to(pts), to(sym)
step = PoseStep(B, H, W, C, dev, is_train=1, skip_pixels=10)
for _ in range(5):
    step.step(inputs)
torch.cuda.synchronize()
N = 50
t0 = time.perf_counter()
cpu = []
for _ in range(N):
    a = time.perf_counter()
    step.step(inputs)
    cpu.append(time.perf_counter() - a)
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print(f"enqueue per step: median {np.median(cpu) * 1e3:.3f} ms, min {np.min(cpu) * 1e3:.3f} ms")
print(f"host loop {1e3 * (t1 - t0) / N:.3f} ms/step; wall incl. drain {1e3 * (t2 - t0) / N:.3f} ms/step")
