"""Label producer microbench at the bench size (B=8,
640x480, C=22, train mode): argmax_2d alone, the Hough op on label_2d, the
Hough op with the argmax fused (prob input), and Hardlabel; HIP events on the
launch stream.    python scripts/label_bench.py [--iters 50]"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from posecnn_amd import synth  # noqa: E402
from posecnn_amd.label_2d import argmax_2d  # noqa: E402
from posecnn_amd.hard_label_layer import hard_label_op as hl  # noqa: E402
from posecnn_amd.hough_voting_gpu_layer import hough_voting_gpu_op as hv  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--iters", type=int, default=50)
a = p.parse_args()
D = torch.device("cuda")
B, H, W, C = 8, 480, 640, 22
fr = synth.make_frames(B, H, W, num_classes=C, objects_per_image=6, seed=3)
to = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(D)
g = torch.Generator(device=D).manual_seed(1)
lab = to(fr["label"])
score = torch.rand((B, H, W, C), generator=g, device=D)
score.scatter_(3, lab.long().unsqueeze(3), 2.0)
prob = torch.softmax(score, dim=3).contiguous()
gt_label = lab.clone()
args = (to(fr["vertex"]), to(fr["extents"]), to(fr["meta"]), to(fr["gt"]), 1, -1.0, 0.02, 10)
lab_out = torch.empty_like(lab)
o1 = hv.hough_voting_gpu_capacity(lab, *args)
o2 = hv.hough_voting_gpu_capacity(None, *args, prob=prob)
top = torch.empty((B, H, W, C), device=D)


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


res = {
    "argmax_2d_us": timeit(lambda: argmax_2d(prob, out=lab_out)),
    "hough_label_us": timeit(lambda: hv.hough_voting_gpu_capacity(lab, *args, out=o1)),
    "hough_prob_fused_us": timeit(lambda: hv.hough_voting_gpu_capacity(None, *args, out=o2, prob=prob)),
    "hard_label_us": timeit(lambda: hl.hard_label(prob, gt_label, 0.9)),
}
# class-compact vertex map: producer + vote on it vs the vote on the full map
from posecnn_amd.vertex_pred import vertex_pred_compact  # noqa: E402
K = 128
feat = torch.randn((B, H, W, K), generator=g, device=D)
vw = torch.randn((K, 3 * C), generator=g, device=D) * 0.05
vb = torch.randn((3 * C,), generator=g, device=D)
v3 = torch.empty((B, H, W, 3), device=D)
res["vertex_pred_compact_us"] = timeit(lambda: vertex_pred_compact(feat, vw, vb, lab, out=v3))
# the vote on the compact form of the frames' own vertex map (same field as hough_label_us)
vfull = args[0]
idx = (3 * lab.long()).unsqueeze(3) + torch.arange(3, device=D)
v3f = torch.gather(vfull, 3, idx).contiguous()
oc = hv.hough_voting_gpu_capacity(lab, v3f, *args[1:], vertex_compact=True)
res["hough_compact_us"] = timeit(lambda: hv.hough_voting_gpu_capacity(lab, v3f, *args[1:], out=oc, vertex_compact=True))
nr = int(o1["num_rois"][1].item())
assert torch.equal(oc["num_rois"], o1["num_rois"])
for k in ("box", "pose", "target", "weight", "domain"):
    assert torch.equal(oc[k][:nr], o1[k][:nr]), k
res["vertex_pred_compact_GBps"] = (B * H * W * (K * 4 + 4 + 12)) / (res["vertex_pred_compact_us"] * 1e-6) / 1e9
res["argmax_then_hough_us"] = res["argmax_2d_us"] + res["hough_label_us"]
prob_bytes = B * H * W * C * 4
res["argmax_2d_GBps"] = (prob_bytes + B * H * W * 4) / (res["argmax_2d_us"] * 1e-6) / 1e9
res["hard_label_GBps"] = (prob_bytes + B * H * W * 4 + B * H * W * C * 4) / (res["hard_label_us"] * 1e-6) / 1e9
assert torch.equal(o2["label"], argmax_2d(prob))
print(json.dumps({k: round(v, 2) for k, v in res.items()}), flush=True)
