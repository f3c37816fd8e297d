"""Centre error of the oracle's estimatePose2D over several ray-cast scenes:
the 3 px bar of tests/test_gpu_pose2d.py is a property of its scenes, not a guarantee."""
import sys, numpy as np
sys.path.insert(0, 'tests'); sys.path.insert(0, '.')
from oracle import oracle
from pose2d_scene import make_scene
for noise, seed in [(0.0, 1), (0.01, 2), (0.003, 5), (0.01, 6), (0.01, 7), (0.01, 8), (0.01, 9), (0.01, 10)]:
    sc = make_scene(seed=seed, coord_noise=noise)
    r = oracle.pose2d(sc["label"], sc["vertmap"], sc["extents"], *sc["camera"])
    fx, fy, px, py = sc["camera"]
    errs = []
    for c, p in sc["poses"].items():
        t = r["poses"][:, 3, c]
        got = np.array([fx * t[0] / t[2] + px, fy * t[1] / t[2] + py])
        want = np.array([fx * p["t"][0] / p["t"][2] + px, fy * p["t"][1] / p["t"][2] + py])
        errs.append(np.abs(got - want).max())
    print(noise, seed, np.round(errs, 2))
