"""Backprojection microbench at the configs[4] bench size (B = 8, 640x480,
G = 64, Ch = 64, NC = 16, kernel size 1, threshold 0.02): forward and
backward op time by HIP events, the algorithmic bytes of each (forward:
top_data + top_flag + top_label written, label_3d read where a voxel has no
hit; backward: bottom_diff written + the top_diff rows of in-grid pixels
read), the forward's hit fraction and the backward's in-grid fraction --
on a scene with depth at every pixel (objects over a floor plane: surfaces
cross the grid, hit voxels gather their feature windows) and on objects-only
depth (almost no hits: a store stream).  POSECNN_HIP_LIB selects a variant
library."""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from posecnn_amd import synth
from posecnn_amd.backprojecting_layer import backprojecting_op as bpo

ap = argparse.ArgumentParser()
ap.add_argument("--iters", type=int, default=50)
ap.add_argument("--batch", type=int, default=8)
ap.add_argument("--scene", choices=["scene", "objects", "both"], default="both",
                help="one scene only (the rocprofv3 --pmc passes of scripts/bp_pmc.py take one scene per run)")
a = ap.parse_args()
B, H, W, C, G, CH = a.batch, 480, 640, 16, 64, 64
dev = torch.device("cuda")
voxel = ([1.2 / G, 0.9 / G, 1.2 / G], [-0.6, -0.45, 0.9])  # as bench.py --workload linemod: the frustum at 0.9-2.1 m
# "scene": depth at every pixel (objects over a tilted floor plane, bench.py's
# configs[4] workload), so object and floor surfaces cross the grid and the
# feature-averaging gather runs; "objects": depth only on the objects (holes
# elsewhere) -- nearly every voxel misses, the forward is a store stream
SCENES = {"scene": (1.0, 2.0), "objects": None}
if a.scene != "both":
    SCENES = {a.scene: SCENES[a.scene]}
frames = {k: synth.make_frames(B, H, W, num_classes=C, objects_per_image=4, seed=5,
                               extents=synth.models()["linemod_extents"], with_depth=True, voxel=voxel,
                               depth_background=v) for k, v in SCENES.items()}
g = torch.Generator(device=dev)
g.manual_seed(7)
to = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(dev)
data = torch.randn((B, H, W, CH), generator=g, device=dev)
label = torch.rand((B, H, W, C), generator=g, device=dev)
label3d = torch.rand((B, G, G, G, C), generator=g, device=dev)
grad = torch.randn((B, G, G, G, CH), generator=g, device=dev)


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
    return e0.elapsed_time(e1) * 1e3 / a.iters


res = {}
for name, fr in frames.items():
    depth, meta = to(fr["depth"]), to(fr["meta"])
    out = bpo.backproject(data, label, depth, meta, label3d, G, 1, 0.02)
    top_flag = out[2]
    hit = float((top_flag[..., 0] > 0).float().mean())
    fwd = timeit(lambda: bpo.backproject(data, label, depth, meta, label3d, G, 1, 0.02))
    gd = bpo.backproject_grad(data, depth, meta, grad, G, 1, 0.02)
    ingrid = float((gd[..., 0] != 0).float().mean())  # pixels whose top_diff row is read
    bwd = timeit(lambda: bpo.backproject_grad(data, depth, meta, grad, G, 1, 0.02))
    nvox = B * G ** 3
    # forward: outputs written + label_3d read for misses + the (2k+1)^2-pixel
    # feature / label rows a hit voxel averages (upper bound: every pixel of
    # the window passes the depth test)
    gather = hit * nvox * 9 * (CH + C + 1) * 4
    fwd_bytes = nvox * (2 * CH + C) * 4 + (1 - hit) * nvox * C * 4 + gather
    # backward: bottom_diff written (B H W Ch 4, the HBM floor) + one top_diff
    # row per in-grid pixel.  Pixels that map to one voxel re-read its row,
    # mostly from L2, so the row term over-counts HBM reads: this is an
    # algorithmic-bytes rate, not an HBM rate (scripts/bp_pmc.py adds the
    # rocprofv3 counter bytes and their rate beside it).
    bwd_write = B * H * W * CH * 4
    bwd_bytes = bwd_write * (1 + ingrid)
    res[name] = {"fwd_us": round(fwd, 1), "fwd_algorithmic_bytes": round(fwd_bytes),
                 "fwd_algorithmic_TBps": round(fwd_bytes / fwd / 1e6, 3),
                 "fwd_gather_bytes_upper": round(gather), "bwd_us": round(bwd, 1),
                 "bwd_algorithmic_bytes": round(bwd_bytes),
                 "bwd_algorithmic_TBps": round(bwd_bytes / bwd / 1e6, 3),
                 "bwd_write_TBps": round(bwd_write / bwd / 1e6, 3), "hit_fraction": round(hit, 4),
                 "hit_voxels": int(round(hit * nvox)), "bwd_ingrid_fraction": round(ingrid, 4),
                 "depth": "objects over a floor plane 1.0 -> 2.0 m" if SCENES[name] else "objects only (holes)"}
print(json.dumps({"B": B, "G": G, "Ch": CH, "NC": C, **res}))
