"""Time the RGB-only pose estimator (estimatePose2D, SURVEY §8(f) row 4;
csrc/pose2d.hip via posecnn_amd.synthesize.pose2d) on a 640x480 ray-cast box
scene (tests/pose2d_scene.py) with device-resident label / vertex maps, and
the oracle's single-thread restatement (oracle/orc_pose2d.cpp) on the same
frame beside it as the CPU baseline.  Prints one JSON line.
    python scripts/pose2d_bench.py [--objects 5] [--classes 22] [--iters 20]"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from pose2d_scene import make_scene  # noqa: E402
from posecnn_amd.synthesize import pose2d  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--objects", type=int, default=5)
p.add_argument("--classes", type=int, default=22)
p.add_argument("--iters", type=int, default=20)
p.add_argument("--noise", type=float, default=0.003)
p.add_argument("--no-cpu", action="store_true")
a = p.parse_args()

sc = make_scene(seed=11, n_obj=a.objects, C=a.classes, coord_noise=a.noise)
D = torch.device("cuda")
C = sc["C"]
lab = torch.from_numpy(sc["label"]).to(D)
vm = torch.from_numpy(sc["vertmap"]).to(D)
ext = torch.from_numpy(sc["extents"]).to(D)
poses = torch.zeros((3, 4, C), device=D)
cam = sc["camera"]


def run():
    pose2d.estimate_poses_2d(lab, vm, ext, poses, C, *cam)


for _ in range(3):
    run()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(a.iters):
    run()
torch.cuda.synchronize()
gpu_ms = (time.perf_counter() - t0) / a.iters * 1e3

found = int((poses[2, 3, :] > 0).sum())
fx, fy, px, py = cam
err = []
for c, gt in sc["poses"].items():
    t = poses[:, 3, c].cpu().numpy()
    if t[2] > 0:
        err.append(float(np.abs(np.array([fx * t[0] / t[2] + px, fy * t[1] / t[2] + py]) -
                                np.array([fx * gt["t"][0] / gt["t"][2] + px, fy * gt["t"][1] / gt["t"][2] + py])).max()))

out = {"metric": "estimatePose2D frames/s (256 hypotheses, 8 preemptive rounds, 640x480)",
       "value": round(1e3 / gpu_ms, 2), "unit": "frames/s", "ms_per_frame": round(gpu_ms, 3),
       "objects": a.objects, "classes": C, "objects_found": found,
       "max_centre_error_px": round(max(err), 3) if err else None,
       "timing": "wall clock per call (all launches on the device, one sync)",
       "data": f"synthetic (ray-cast boxes, tests/pose2d_scene.py, coordinate noise {a.noise})"}
if not a.no_cpu:
    from oracle import oracle  # CPU baseline leg only
    nb = 10
    t0 = time.perf_counter()
    for _ in range(nb):
        oracle.pose2d(sc["label"], sc["vertmap"], sc["extents"], *cam)
    cpu_ms = (time.perf_counter() - t0) / nb * 1e3
    out["cpu_baseline"] = {"value": round(1e3 / cpu_ms, 2), "unit": "frames/s", "cores": 1, "kind": "port",
                           "sample": f"{nb} calls of the oracle's estimatePose2D restatement on the same frame"}
print(json.dumps(out), flush=True)
