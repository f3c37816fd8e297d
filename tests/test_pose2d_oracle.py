"""The estimatePose2D restatement (oracle/orc_pose2d.cpp; synthesize.cpp:1571)
pinned by known answers on ray-cast box scenes (tests/pose2d_scene.py), CPU
only: with exact object coordinates every surviving hypothesis is the true pose
(P3P recovers it from 4 exact correspondences); with coordinate noise the pose
still lands on the object (centre within 3 px); the preemptive schedule keeps
one hypothesis per object after 8 rounds, with inlier counts over the growing
subsets; a frame without a > 400-pixel object returns nothing."""
import numpy as np

from oracle import oracle
from pose2d_scene import make_scene


def _centre_px(R, t, cam):
    fx, fy, px, py = cam
    return np.array([fx * t[0] / t[2] + px, fy * t[1] / t[2] + py])


def test_exact_coordinates_recover_the_pose():
    sc = make_scene(seed=1)
    r = oracle.pose2d(sc["label"], sc["vertmap"], sc["extents"], *sc["camera"])
    assert r["n_obj"] == len(sc["poses"])
    for c, p in sc["poses"].items():
        h, inl, nh = r["final"][c]
        assert h >= 0 and nh > 0 and inl > 0
        np.testing.assert_allclose(r["poses"][:, :3, c], p["R"], atol=2e-5)
        np.testing.assert_allclose(r["poses"][:, 3, c], p["t"], atol=2e-5)
        # the survivor was counted in every round, over growing subsets
        rounds = r["inliers"][h]
        assert (rounds > 0).all() and (np.diff(rounds) >= 0).all()
        # sampled pixels belong to the object
        assert (sc["label"].reshape(-1)[r["hyp_px"][h]] == c).all()
    # each hypothesis names a present object, each object keeps exactly one
    objs = r["hyps"][:, 0]
    assert set(objs[objs >= 0].astype(int)) <= set(sc["poses"])
    assert (objs >= 0).sum() == 256


def test_noisy_coordinates_land_on_the_object():
    sc = make_scene(seed=2, coord_noise=0.01)
    r = oracle.pose2d(sc["label"], sc["vertmap"], sc["extents"], *sc["camera"])
    for c, p in sc["poses"].items():
        assert r["final"][c][0] >= 0
        got = _centre_px(r["poses"][:, :3, c], r["poses"][:, 3, c], sc["camera"])
        want = _centre_px(p["R"], p["t"], sc["camera"])
        assert np.abs(got - want).max() < 3.0, (c, got, want)


def test_preemptive_schedule():
    sc = make_scene(seed=3, n_obj=2)
    r = oracle.pose2d(sc["label"], sc["vertmap"], sc["extents"], *sc["camera"], n_hyp=64)
    for c in sc["poses"]:
        nh = int(r["final"][c][2])
        hs = np.where(r["hyps"][:, 0] == c)[0]
        assert len(hs) == nh
        # round k counts the survivors of round k - 1: n, n/2, n/4, ... (at least 1)
        alive = nh
        for k in range(8):
            assert (r["inliers"][hs, k] >= 0).sum() == alive
            alive = max(alive // 2, 1) if alive > 1 else 1


def test_no_object():
    sc = make_scene(seed=4)
    lab = np.zeros_like(sc["label"])
    lab[:10, :30] = 1  # 300 pixels: below minArea = 400
    r = oracle.pose2d(lab, sc["vertmap"], sc["extents"], *sc["camera"])
    assert r["n_obj"] == 0 and not r["poses"].any() and (r["final"] == -1).all()
