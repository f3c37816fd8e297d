"""Time the RANSAC pose estimators: estimatePose2D
(--mode 2d, posecnn_amd.synthesize.pose2d) or estimatePose3D (--mode 3d,
posecnn_amd.synthesize.pose3d; depth with 10 % holes and 1 mm noise), both in
csrc/pose2d.hip, on a 640x480 ray-cast box scene (tests/pose2d_scene.py) with
device-resident inputs, and the oracle's single-thread restatement
(oracle/orc_pose2d.cpp) on the same frame beside it as the CPU baseline (the
reason this lives under tests/: only tests/, smoke() and bench.py's CPU leg
run the oracle).  Prints one JSON line.
    python tests/perf_pose.py [--mode 2d|3d] [--objects 5] [--classes 22] [--iters 20]"""
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
from posecnn_amd.synthesize import pose2d, pose3d  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--objects", type=int, default=5)
p.add_argument("--classes", type=int, default=22)
p.add_argument("--iters", type=int, default=20)
p.add_argument("--noise", type=float, default=0.003)
p.add_argument("--no-cpu", action="store_true")
p.add_argument("--mode", choices=["2d", "3d"], default="2d")
a = p.parse_args()

sc = make_scene(seed=11, n_obj=a.objects, C=a.classes, coord_noise=a.noise, hole_frac=0.1, depth_noise=0.001)
D = torch.device("cuda")
C = sc["C"]
lab = torch.from_numpy(sc["label"]).to(D)
vm = torch.from_numpy(sc["vertmap"]).to(D)
ext = torch.from_numpy(sc["extents"]).to(D)
poses = torch.zeros((3, 4, C), device=D)
cam = sc["camera"]
dep = torch.from_numpy(sc["depth"].view(np.int16)).to(D)


def run():
    if a.mode == "2d":
        pose2d.estimate_poses_2d(lab, vm, ext, poses, C, *cam)
    else:
        pose3d.estimate_poses_3d(lab, dep, vm, ext, poses, C, *cam, sc["depth_factor"])


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
err, terr = [], []
for c, gt in sc["poses"].items():
    t = poses[:, 3, c].cpu().numpy()
    if t[2] > 0:
        err.append(float(np.abs(np.array([fx * t[0] / t[2] + px, fy * t[1] / t[2] + py]) -
                                np.array([fx * gt["t"][0] / gt["t"][2] + px, fy * gt["t"][1] / gt["t"][2] + py])).max()))
        terr.append(float(np.abs(t - gt["t"]).max()))

name = "estimatePose2D" if a.mode == "2d" else "estimatePose3D"
out = {"metric": f"{name} frames/s (256 hypotheses, 8 preemptive rounds, 640x480)",
       "value": round(1e3 / gpu_ms, 2), "unit": "frames/s", "ms_per_frame": round(gpu_ms, 3),
       "objects": a.objects, "classes": C, "objects_found": found,
       "max_centre_error_px": round(max(err), 3) if err else None,
       "max_translation_error_m": round(max(terr), 5) if terr else None,
       "timing": "wall clock per call (all launches on the device, one sync)",
       "data": f"synthetic (ray-cast boxes, tests/pose2d_scene.py, coordinate noise {a.noise}"
               + (", depth holes 10 %, depth noise 1 mm)" if a.mode == "3d" else ")")}
if not a.no_cpu:
    from oracle import oracle  # CPU baseline leg only
    nb = 10
    t0 = time.perf_counter()
    for _ in range(nb):
        if a.mode == "2d":
            oracle.pose2d(sc["label"], sc["vertmap"], sc["extents"], *cam)
        else:
            oracle.pose3d(sc["label"], sc["depth"], sc["vertmap"], sc["extents"], *cam, sc["depth_factor"])
    cpu_ms = (time.perf_counter() - t0) / nb * 1e3
    out["cpu_baseline"] = {"value": round(1e3 / cpu_ms, 2), "unit": "frames/s", "cores": 1, "kind": "port",
                           "sample": f"{nb} calls of the oracle's {name} restatement on the same frame"}
print(json.dumps(out), flush=True)
