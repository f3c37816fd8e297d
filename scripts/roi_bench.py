"""Time RoI pooling forward / backward on the bench's own RoIs (configs[2]:
B=8 train-mode Hough rows, conv4_3 60x80 and conv5_3 30x40, 512 channels),
one op at a time with HIP events.
    python scripts/roi_bench.py [--iters 20]"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from posecnn_amd import synth  # noqa: E402
from posecnn_amd.hough_voting_gpu_layer import hough_voting_gpu_op as hv  # noqa: E402
from posecnn_amd.roi_pooling_layer import roi_pooling_op as rp  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--iters", type=int, default=20)
p.add_argument("--px", action="store_true", help="the fused step's form: uint16 pixel argmax (pair forward, px backward)")
p.add_argument("--only", default="")
a = p.parse_args()
D = torch.device("cuda")
B, H, W, C = 8, 480, 640, 22
fr = synth.make_frames(B, H, W, num_classes=C, objects_per_image=6, seed=3)
to = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(D)
o = hv.hough_voting_gpu_capacity(to(fr["label"]), to(fr["vertex"]), to(fr["extents"]), to(fr["meta"]), to(fr["gt"]),
                                 1, -1.0, 0.02, 10)
nr = o["num_rois"][1:2]
R = int(nr.item())
box = o["box"]
g = torch.Generator(device=D).manual_seed(5)
c4 = torch.randn((B, 60, 80, 512), generator=g, device=D)
c5 = torch.randn((B, 30, 40, 512), generator=g, device=D)
CAP = box.shape[0]
top = torch.zeros((CAP, 7, 7, 512), device=D)
a5 = torch.zeros((CAP, 7, 7, 512), dtype=torch.int32, device=D)
a4 = torch.zeros_like(a5)
gd = torch.randn((CAP, 7, 7, 512), generator=g, device=D)
d4, d5 = torch.empty_like(c4), torch.empty_like(c5)
a5p = torch.zeros((CAP, 7, 7, 512), dtype=torch.int16, device=D)
a4p = torch.zeros_like(a5p)
if a.px:
    rp.roi_pool_pair(c5, 1 / 16, c4, 1 / 8, box, 7, 7, num_rois=nr, out=(top, a5p, a4p), pixel_argmax=True)
cases = [
    ("fwd_conv5", lambda: rp.roi_pool(c5, box, 7, 7, 1 / 16, 0, num_rois=nr, out=(top, a5))),
    ("fwd_conv4_acc", lambda: rp.roi_pool(c4, box, 7, 7, 1 / 8, 0, num_rois=nr, out=(top, a4), accumulate=True)),
    ("fwd_pair", lambda: rp.roi_pool_pair(c5, 1 / 16, c4, 1 / 8, box, 7, 7, num_rois=nr, out=(top, a5, a4))),
    ("bwd_conv5", lambda: rp.roi_pool_grad(c5, box, a5, gd, 7, 7, 1 / 16, 0, num_rois=nr, out=d5)),
    ("bwd_conv4", lambda: rp.roi_pool_grad(c4, box, a4, gd, 7, 7, 1 / 8, 0, num_rois=nr, out=d4)),
]
if a.px:
    cases = [
        ("fwd_pair_px", lambda: rp.roi_pool_pair(c5, 1 / 16, c4, 1 / 8, box, 7, 7, num_rois=nr, out=(top, a5p, a4p),
                                                 pixel_argmax=True)),
        ("bwd_conv5_px", lambda: rp.roi_pool_grad(c5, box, a5p, gd, 7, 7, 1 / 16, 0, num_rois=nr, out=d5)),
        ("bwd_conv4_px", lambda: rp.roi_pool_grad(c4, box, a4p, gd, 7, 7, 1 / 8, 0, num_rois=nr, out=d4)),
    ]
if a.only:
    cases = [c for c in cases if c[0] in a.only.split(",")]
print(f"rows {R}", flush=True)
for name, fn in cases:
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    print(f"{name:14s} {e0.elapsed_time(e1) / a.iters * 1e3:9.1f} us", flush=True)
import hashlib  # noqa: E402
sha = lambda t: hashlib.sha256(t.cpu().numpy().tobytes()).hexdigest()[:16]
print(f"sha d4 {sha(d4)} d5 {sha(d5)}", flush=True)
print(f"checksum d4 {float(d4.double().sum()):.6e} d5 {float(d5.double().sum()):.6e}", flush=True)
