"""Time hough_voting_gpu (capacity form) on the bench's frames (configs[2]: B=8
train mode, or --test for configs[1]-style test mode) with HIP events.
    python scripts/hough_bench.py [--iters 20] [--batch 8] [--test]"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from posecnn_amd import synth  # noqa: E402
from posecnn_amd.hough_voting_gpu_layer import hough_voting_gpu_op as hv  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--iters", type=int, default=20)
p.add_argument("--batch", type=int, default=8)
p.add_argument("--test", action="store_true")
a = p.parse_args()
D = torch.device("cuda")
B, H, W, C = a.batch, 480, 640, 22
fr = synth.make_frames(B, H, W, num_classes=C, objects_per_image=6, seed=3)
to = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(D)
inp = [to(fr[k]) for k in ("label", "vertex", "extents", "meta", "gt")]
out = {}
train = 0 if a.test else 1
fn = lambda: out.__setitem__("o", hv.hough_voting_gpu_capacity(*inp, train, -1.0, 0.02, 10, out=out.get("o")))
for _ in range(3):
    fn()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(a.iters):
    fn()
e1.record()
torch.cuda.synchronize()
us = e0.elapsed_time(e1) / a.iters * 1e3
print(f"B={B} {'test' if a.test else 'train'} rows {int(out['o']['num_rois'][0].item())} hough {us:9.1f} us "
      f"({us / B:.1f} us/frame)", flush=True)
