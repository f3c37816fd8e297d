"""PCIe-inclusive rate of the Hough vote op: the same B=8
train-mode frames as bench.py, but with label + vertex maps starting in pinned
host memory, copied H2D on the launch stream and voted on.  The C-ABI takes
device pointers (as the reference's TF op takes GPU tensors), so this is a
note beside `value`, never `value` itself.
    python scripts/pcie_rate.py [--iters 20]"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from posecnn_amd import synth  # noqa: E402
from posecnn_amd.hough_voting_gpu_layer import hough_voting_gpu_op as hv  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--iters", type=int, default=20)
a = p.parse_args()
D = torch.device("cuda")
B, H, W, C = 8, 480, 640, 22
fr = synth.make_frames(B, H, W, num_classes=C, objects_per_image=6, seed=3)
to = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(D)
pin = lambda x: torch.from_numpy(np.ascontiguousarray(x)).pin_memory()
h_lab, h_vtx = pin(fr["label"]), pin(fr["vertex"])
d_lab, d_vtx = torch.empty_like(h_lab, device=D), torch.empty_like(h_vtx, device=D)
d_lab.copy_(h_lab)
d_vtx.copy_(h_vtx)
rest = (to(fr["extents"]), to(fr["meta"]), to(fr["gt"]), 1, -1.0, 0.02, 10)
o = hv.hough_voting_gpu_capacity(d_lab, d_vtx, *rest)


def timeit(fn):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / a.iters * 1e3


def h2d():
    d_lab.copy_(h_lab, non_blocking=True)
    d_vtx.copy_(h_vtx, non_blocking=True)


def vote():
    hv.hough_voting_gpu_capacity(d_lab, d_vtx, *rest, out=o)


def both():
    h2d()
    vote()


nbytes = h_lab.numel() * 4 + h_vtx.numel() * 4
t_copy, t_vote, t_both = timeit(h2d), timeit(vote), timeit(both)
print(json.dumps({
    "frames": B, "h2d_bytes": nbytes, "h2d_us": round(t_copy, 1), "h2d_GBps": round(nbytes / t_copy / 1e3, 1),
    "vote_us": round(t_vote, 1), "h2d_plus_vote_us": round(t_both, 1),
    "frames_per_s_resident": round(B / t_vote * 1e6, 1), "frames_per_s_pcie_inclusive": round(B / t_both * 1e6, 1),
}))
