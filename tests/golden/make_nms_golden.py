"""Regenerate tests/golden/nms_golden.npz: inputs and the outputs of the
REFERENCE's own class-aware NMS (lib/utils/nms.py, pure numpy), imported from
/root/reference at generation time only — the fixture (data) is what the tests
read; nothing under tests/ or the package reads /root/reference at run time.

Cases are tie-free in score (numpy's argsort()[::-1] leaves the order of equal
scores unspecified, so only tie-free inputs pin one answer); ties are covered
by the GPU-vs-oracle test with the canonical lower-row-first order.

    python tests/golden/make_nms_golden.py
"""
import importlib.util
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference/lib/utils/nms.py"


def ref_nms():
    spec = importlib.util.spec_from_file_location("ref_nms", REF)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod.nms


def hough_like(rng, n_max, jitter=True):
    """rows as the train-mode Hough op emits them: per maximum a box and its
    8 jittered copies (+-5% of w / h, hough_voting_gpu_op.cu.cc:468-554)."""
    rows = []
    for _ in range(n_max):
        cls = float(rng.integers(1, 6))
        cx, cy = rng.uniform(0, 640), rng.uniform(0, 480)
        w, h = rng.uniform(20, 250), rng.uniform(20, 250)
        x1, y1, x2, y2 = cx - w / 2, cy - h / 2, cx + w / 2, cy + h / 2
        shifts = [(0, 0)] + ([(dx, dy) for dx in (-1, 0, 1) for dy in (-1, 0, 1) if dx or dy] if jitter else [])
        for dx, dy in shifts:
            rows.append([0.0, cls, x1 + dx * 0.05 * w, y1 + dy * 0.05 * h, x2 + dx * 0.05 * w, y2 + dy * 0.05 * h,
                         0.0])
    d = np.array(rows, np.float32)
    d[:, 6] = rng.permutation(len(d)).astype(np.float32) * 3.0 + 17.0  # distinct scores
    return d


def main():
    nms = ref_nms()
    rng = np.random.default_rng(2024)
    cases = {}
    cases["single"] = hough_like(rng, 1)
    cases["train_rows"] = hough_like(rng, 40)
    cases["test_rows"] = hough_like(rng, 30, jitter=False)
    dense = hough_like(rng, 128)  # 1152 rows: the op's capacity
    cases["capacity"] = dense
    degen = hough_like(rng, 10)
    degen[::7, 4] = degen[::7, 2] - 3.0  # x2 < x1 (negative bb, cu.cc:751-764 lets these through)
    cases["degenerate"] = degen
    out = {}
    for name, d in cases.items():
        for thr in (0.5, 0.3):
            keep = np.array(nms(d.copy(), thr), np.int64)
            out[f"{name}_{thr}_dets"] = d
            out[f"{name}_{thr}_keep"] = keep
    np.savez_compressed(os.path.join(HERE, "nms_golden.npz"), **out)
    print("wrote", {k: v.shape for k, v in out.items() if k.endswith("_keep")})


if __name__ == "__main__":
    main()
