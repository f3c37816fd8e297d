"""Time the ADD loss forward on the bench's own rows (configs[2]: B=8 train-mode
Hough targets/weights, 22 classes, random predictions normalised as the
step's l2_normalize does: a unit quaternion on the row's class) with HIP
events, for the pruned ADD-S search (PCNN_ADD_SEARCH=pruned) and the full scan,
and check that both give the same bits.
    python scripts/add_bench.py [--iters 20] [--near]"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from posecnn_amd import synth  # noqa: E402
from posecnn_amd.hough_voting_gpu_layer import hough_voting_gpu_op as hv  # noqa: E402
from posecnn_amd.average_distance_loss import average_distance_loss_op as adl  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--iters", type=int, default=20)
p.add_argument("--near", action="store_true", help="predictions within a few degrees of the targets")
p.add_argument("--no-check", action="store_true", help="timing ablation builds: skip the pruned == full check")
p.add_argument("--modes", default="pruned,full,pruned")
a = p.parse_args()
D = torch.device("cuda")
B, H, W, C = 8, 480, 640, 22
fr = synth.make_frames(B, H, W, num_classes=C, objects_per_image=6, seed=3)
to = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(D)
o = hv.hough_voting_gpu_capacity(to(fr["label"]), to(fr["vertex"]), to(fr["extents"]), to(fr["meta"]), to(fr["gt"]),
                                 1, -1.0, 0.02, 10)
nr = o["num_rois"][1:2]
pts, sym = synth.rescaled_points(C)
pts, sym = to(pts), to(sym)
g = torch.Generator(device=D).manual_seed(7)
raw = torch.randn(o["target"].shape, generator=g, device=D)
if a.near:
    raw = o["target"] + 0.03 * raw
pred = torch.nn.functional.normalize(raw * o["weight"], dim=1)  # unit quaternion on the class, as the step's
loss = torch.zeros((1,), device=D)
diff = torch.zeros_like(pred)
R = pred.shape[0]
ws = torch.empty(adl.workspace_bytes(R, C, pts.shape[1]), dtype=torch.uint8, device=D)
fn = lambda: adl.average_distance_loss(pred, o["target"], o["weight"], pts, sym, 0.01, num_rois=nr, out=(loss, diff),
                                       workspace=ws)
import hashlib  # noqa: E402
res = {}
for mode in a.modes.split(","):
    os.environ["PCNN_ADD_SEARCH"] = mode
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    os.environ.pop("PCNN_ADD_SEARCH", None)
    dig = hashlib.sha256(diff.cpu().numpy().tobytes()).hexdigest()[:16]
    res.setdefault(mode, []).append((loss.item(), dig))
    diag = adl.search_diagnostics(ws, R, C, pts.shape[1])
    frac = ""
    if diag is not None and mode == "pruned":
        sc, held = (int(v) for v in diag[1].cpu().numpy())
        frac = f" blocks scanned {sc}/{held} = {sc / max(held, 1):.3f}"
    print(f"{mode:6s} rows {int(nr.item())} add_fwd {e0.elapsed_time(e1) / a.iters * 1e3:9.1f} us "
          f"loss {float(loss.item()).hex()} diff sha {dig}{frac}", flush=True)
assert a.no_check or len({r for v in res.values() for r in v}) == 1, "pruned and full search differ"
