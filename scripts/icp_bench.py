"""Time the pose-refinement ops on the synthetic box scene (tests/refine_scene.py):
live vertices, icp for N problems (solveICP's 8 hypotheses) x iterations, centre.
    python scripts/icp_bench.py [--n 8] [--iters 8] [--reps 20]"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from posecnn_amd.synthesize import icp as R  # noqa: E402
from refine_scene import CAMERA, scene  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--n", type=int, default=8)
p.add_argument("--iters", type=int, default=8)
p.add_argument("--reps", type=int, default=20)
a = p.parse_args()
D = torch.device("cuda")
t = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(D)
sc = scene(0)
depth = t(sc["live"]["depth"].astype(np.int32)).to(torch.uint16)
lab = t(sc["live"]["label"])
obj = torch.tensor([sc["cls"]], dtype=torch.int32)
pv = t(np.repeat(sc["pred"]["pred_v"][None], a.n, 0))
pn = t(np.repeat(sc["pred"]["pred_n"][None], a.n, 0))
li = torch.zeros(a.n, dtype=torch.int32, device=D)
lv = R.live_vertices(depth, lab, obj, 10000.0, CAMERA)


def timed(fn):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / a.reps * 1e3


res = {"n_problems": a.n, "iterations": a.iters, "pixels_in_range": int((sc["pred"]["pred_v"][..., 2] > 0.25).sum()),
       "live_vertices_us": timed(lambda: R.live_vertices(depth, lab, obj, 10000.0, CAMERA)),
       "icp_us": timed(lambda: R.icp(lv, pv, pn, CAMERA, max_error=0.05, iterations=a.iters, live_index=li)),
       "icp_1iter_us": timed(lambda: R.icp(lv, pv, pn, CAMERA, max_error=0.05, iterations=1, live_index=li))}
print(json.dumps(res), flush=True)
