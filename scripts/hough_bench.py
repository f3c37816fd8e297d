"""Time the Hough op (B frames, train mode) with HIP events; the library may
be swapped with POSECNN_HIP_LIB for ablation builds.
    python scripts/hough_bench.py [--batch 8] [--iters 20]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from posecnn_amd import synth  # noqa: E402
from posecnn_amd.hough_voting_gpu_layer import hough_voting_gpu_op as hv  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--batch", type=int, default=8)
p.add_argument("--iters", type=int, default=20)
p.add_argument("--skip", type=int, default=10)
a = p.parse_args()
D = torch.device("cuda")
fr = synth.make_frames(a.batch, seed=3)
t = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(D)
args = [t(fr[k]) for k in ("label", "vertex", "extents", "meta", "gt")]
out = None
for _ in range(3):
    out = hv.hough_voting_gpu_capacity(*args, 1, -1.0, 0.02, a.skip, out=out)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(a.iters):
    out = hv.hough_voting_gpu_capacity(*args, 1, -1.0, 0.02, a.skip, out=out)
e1.record()
torch.cuda.synchronize()
print(f"{os.environ.get('POSECNN_HIP_LIB', 'default')}: hough op {e0.elapsed_time(e1) / a.iters * 1e3:.1f} us "
      f"rows {int(out['num_rois'][0])}", flush=True)
