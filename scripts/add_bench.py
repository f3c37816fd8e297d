"""Time the ADD loss forward on the bench's own rows (configs[2]: B=8 train-mode
Hough targets/weights, 22 classes, random normalised predictions) with HIP
events.    python scripts/add_bench.py [--iters 20]"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from posecnn_amd import synth  # noqa: E402
from posecnn_amd.hough_voting_gpu_layer import hough_voting_gpu_op as hv  # noqa: E402
from posecnn_amd.average_distance_loss import average_distance_loss_op as adl  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--iters", type=int, default=20)
a = p.parse_args()
D = torch.device("cuda")
B, H, W, C = 8, 480, 640, 22
fr = synth.make_frames(B, H, W, num_classes=C, objects_per_image=6, seed=3)
to = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(D)
o = hv.hough_voting_gpu_capacity(to(fr["label"]), to(fr["vertex"]), to(fr["extents"]), to(fr["meta"]), to(fr["gt"]),
                                 1, -1.0, 0.02, 10)
nr = o["num_rois"][1:2]
pts, sym = synth.rescaled_points(C)
pts, sym = to(pts), to(sym)
g = torch.Generator(device=D).manual_seed(7)
pred = torch.nn.functional.normalize(torch.randn(o["target"].shape, generator=g, device=D), dim=1)
loss = torch.zeros((1,), device=D)
diff = torch.zeros_like(pred)
fn = lambda: adl.average_distance_loss(pred, o["target"], o["weight"], pts, sym, 0.01, num_rois=nr, out=(loss, diff))
for _ in range(3):
    fn()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(a.iters):
    fn()
e1.record()
torch.cuda.synchronize()
import hashlib  # noqa: E402
dig = hashlib.sha256(diff.cpu().numpy().tobytes()).hexdigest()[:16]
print(f"rows {int(nr.item())} add_fwd {e0.elapsed_time(e1) / a.iters * 1e3:9.1f} us loss {float(loss.item()).hex()} "
      f"diff sha {dig}", flush=True)
