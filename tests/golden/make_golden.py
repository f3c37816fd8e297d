"""Regenerate tests/golden/golden.npz: fixed inputs and the oracle's outputs
for every §8 op at small sizes.

The reference itself cannot be built or imported here, so
these vectors are the oracle's, pinned in turn by tests/test_oracle_kat.py;
they freeze the semantics so that (a) the CPU suite catches any drift of the
oracle or of the synthetic generator and (b) the GPU suite checks the HIP
path against stored vectors, not only against a live oracle.  Large inputs
(label/vertex maps) are regenerated from posecnn_amd.synth seeds and guarded
by a SHA-256 of their bytes; small inputs are stored verbatim.

    python tests/golden/make_golden.py
"""
import hashlib
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from posecnn_amd import synth  # noqa: E402

HOUGH_CASES = [  # (name, B, H, W, C, objects, seed, is_train, vote_thr, skip)
    ("hough_test", 2, 120, 160, 8, 3, 41, 0, -1.0, 3),
    ("hough_train", 2, 120, 160, 8, 3, 42, 1, -1.0, 2),
    ("hough_nms", 1, 240, 320, 8, 4, 43, 0, 5.0, 2),
]


def sha(*arrays):
    h = hashlib.sha256()
    for a in arrays:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


def hough_frames(B, H, W, C, objects, seed):
    return synth.make_frames(B, H=H, W=W, num_classes=C, objects_per_image=objects, seed=seed)


def roi_inputs():
    rng = np.random.default_rng(51)
    B, H, W, Ch = 2, 15, 20, 16
    data = rng.normal(size=(B, H, W, Ch)).astype(np.float32)
    data[1, 3:6, 3:6, :] = 2.5  # ties: first max in scan order wins
    R = 12
    x1 = rng.uniform(-30, 300, R)
    y1 = rng.uniform(-30, 220, R)
    rois = np.stack([np.sort(rng.integers(0, B, R)), rng.integers(0, Ch, R), x1, y1,
                     x1 + rng.uniform(1, 160, R), y1 + rng.uniform(1, 160, R), np.zeros(R)], 1).astype(np.float32)
    top_diff = rng.normal(size=(R, 7, 7, Ch)).astype(np.float32)
    return data, rois, top_diff


def add_inputs():
    rng = np.random.default_rng(52)
    R, C, P = 6, 4, 64
    pred = rng.normal(size=(R, 4 * C)).astype(np.float32)
    target = rng.normal(size=(R, 4 * C)).astype(np.float32)
    weight = np.zeros((R, 4 * C), np.float32)
    for r in range(R - 1):  # last row: no weighted class (zero loss row)
        c = 1 + r % (C - 1)
        weight[r, 4 * c:4 * c + 4] = 1
    points = rng.normal(size=(C, P, 3)).astype(np.float32)
    symmetry = np.array([0, 0, 1, 0], np.float32)
    return pred, target, weight, points, symmetry


def bp_inputs():
    rng = np.random.default_rng(53)
    B, H, W, Ch, NC, G = 1, 12, 16, 4, 3, 8
    data = rng.normal(size=(B, H, W, Ch)).astype(np.float32)
    label = rng.uniform(size=(B, H, W, NC)).astype(np.float32)
    depth = rng.uniform(0.8, 1.2, size=(B, H, W, 1)).astype(np.float32)
    K = np.array([[20.0, 0, 8], [0, 20.0, 6], [0, 0, 1]])
    meta = synth.make_meta(K, B, voxel=((0.05, 0.05, 0.05), (-0.2, -0.2, 0.8)))
    label3d = rng.uniform(size=(B, G, G, G, NC)).astype(np.float32)
    top_diff = rng.normal(size=(B, G, G, G, Ch)).astype(np.float32)
    return data, label, depth, meta, label3d, top_diff, G


def compute(orc):
    out = {}
    for name, B, H, W, C, obj, seed, train, vthr, skip in HOUGH_CASES:
        fr = hough_frames(B, H, W, C, obj, seed)
        box, pose, tgt, wgt, dom, n = orc.hough_voting(fr["label"], fr["vertex"], fr["extents"], fr["meta"],
                                                       fr["gt"], train, vthr, 0.02, skip)
        out[f"{name}/sha"] = np.array(sha(fr["label"], fr["vertex"], fr["meta"], fr["gt"]))
        out[f"{name}/n"] = np.array(n, np.int32)
        for k, v in (("box", box), ("pose", pose), ("target", tgt), ("weight", wgt), ("domain", dom)):
            out[f"{name}/{k}"] = v
    data, rois, top_diff = roi_inputs()
    for pc in (0, 1):
        top, arg = orc.roi_pool_fwd(data, rois, 7, 7, 1.0 / 16, pc)
        td = top_diff if not pc else top_diff[..., :1].copy()
        out[f"roi{pc}/top"], out[f"roi{pc}/argmax"] = top, arg
        out[f"roi{pc}/bottom_diff"] = orc.roi_pool_bwd(td, arg, data.shape, rois, 7, 7, 1.0 / 16, pc)
    out["roi/data"], out["roi/rois"], out["roi/top_diff"] = data, rois, top_diff
    pred, target, weight, points, symmetry = add_inputs()
    loss, diff, rows = orc.average_distance_loss(pred, target, weight, points, symmetry, 0.01)
    out.update({"add/pred": pred, "add/target": target, "add/weight": weight, "add/points": points,
                "add/symmetry": symmetry, "add/loss": loss, "add/diff": diff, "add/rows": rows})
    data, label, depth, meta, label3d, top_diff, G = bp_inputs()
    td, tl, tf = orc.backproject_fwd(data, label, depth, meta, label3d, G, 1, 0.05)
    gb = orc.backproject_bwd(top_diff, depth, meta, data.shape[1], data.shape[2], G)
    out.update({"bp/top_data": td, "bp/top_label": tl, "bp/top_flag": tf, "bp/bottom_diff": gb})
    return out


def main():
    from oracle import oracle as orc
    orc.build()
    out = compute(orc)
    path = os.path.join(HERE, "golden.npz")
    np.savez_compressed(path, **out)
    print(f"wrote {path}: {len(out)} arrays, {os.path.getsize(path)} bytes")


if __name__ == "__main__":
    main()
