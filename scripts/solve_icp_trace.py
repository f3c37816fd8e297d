"""Run solve_icp (graph-replayed box renderer, --rois RoIs, --nm Nelder-Mead
evaluations) --reps times on the synthetic scene, for a rocprofv3 kernel trace
of the call (what runs on the device, and the idle gaps the host leaves).
    python scripts/solve_icp_trace.py [--rois 1] [--nm 50] [--reps 10]"""
import argparse
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from posecnn_amd.synthesize import icp as R  # noqa: E402
from refine_scene import CAMERA, GraphBoxRenderer, scene  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--rois", type=int, default=1)
p.add_argument("--nm", type=int, default=50)
p.add_argument("--reps", type=int, default=10)
a = p.parse_args()
D = torch.device("cuda")
t = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(D)  # noqa: E731
sc = scene(0)
depth = t(sc["live"]["depth"].astype(np.int32)).to(torch.uint16)
lab = t(sc["live"]["label"])
params = list(CAMERA) + [0.25, 6.0, 10000.0]
rnd = GraphBoxRenderer(lambda o: sc["half"])
rois = np.tile(np.array([[0, sc["cls"], 0, 0, 1, 1]], np.float32), (a.rois, 1))
poses = np.tile(sc["init"].astype(np.float32)[None], (a.rois, 1))
run = lambda: R.solve_icp(lab, depth, params, rois, poses, rnd, max_error=0.02, nm_evals=a.nm)  # noqa: E731
for _ in range(3):
    run()
torch.cuda.synchronize()
ts = []
for _ in range(a.reps):
    t0 = time.perf_counter()
    run()
    torch.cuda.synchronize()
    ts.append((time.perf_counter() - t0) * 1e3)
print(f"solve_icp rois {a.rois} nm {a.nm}: median {np.median(ts):.2f} ms, min {min(ts):.2f} ms", flush=True)
