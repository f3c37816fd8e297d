"""The estimatePose3D restatement (oracle/orc_pose2d.cpp orc_pose3d;
synthesize.cpp:1769-1965) pinned by known answers on ray-cast box scenes with
depth (tests/pose2d_scene.py), CPU only: with exact object coordinates and
depth (0.1 mm quantisation) every survivor is the true pose after the refit and
the Nelder-Mead refinement; with depth holes, depth noise and coordinate noise
the pose stays within millimetres; the preemptive schedule keeps one
hypothesis per object; the camera coordinates are pxToEye's; a frame without a
> 400-pixel object, or an object without depth, returns nothing for it."""
import numpy as np

from oracle import oracle
from pose2d_scene import make_scene


def _run(sc, **kw):
    return oracle.pose3d(sc["label"], sc["depth"], sc["vertmap"], sc["extents"], *sc["camera"], sc["depth_factor"],
                         **kw)


def test_exact_coordinates_recover_the_pose():
    sc = make_scene(seed=1)
    r = _run(sc)
    assert r["n_obj"] == len(sc["poses"])
    for c, p in sc["poses"].items():
        h, inl, nh = r["final"][c]
        assert h >= 0 and nh > 0 and inl > 10
        np.testing.assert_allclose(r["poses"][:, :3, c], p["R"], atol=1e-4)
        np.testing.assert_allclose(r["poses"][:, 3, c], p["t"], atol=1e-4)
        assert 0 < r["energy"][c] < 1e-4  # mean residual of the refined pose (m)
        rounds = r["inliers"][h]
        assert (rounds > 0).all() and (np.diff(rounds) >= 0).all()
        assert (sc["label"].reshape(-1)[r["hyp_px"][h]] == c).all()
    objs = r["hyps"][:, 0]
    assert (objs >= 0).sum() == 256 and set(objs.astype(int)) <= set(sc["poses"])


def test_holes_and_noise_stay_close():
    sc = make_scene(seed=2, hole_frac=0.2, depth_noise=0.002, coord_noise=0.01)
    r = _run(sc)
    for c, p in sc["poses"].items():
        assert r["final"][c][0] >= 0
        np.testing.assert_allclose(r["poses"][:, 3, c], p["t"], atol=5e-3)
        np.testing.assert_allclose(r["poses"][:, :3, c], p["R"], atol=0.03)
        # sampled pixels have depth
        assert (sc["depth"].reshape(-1)[r["hyp_px"][r["final"][c][0]]] > 0).all()


def test_eye_is_pxtoeye():
    sc = make_scene(seed=3, n_obj=1, hole_frac=0.1)
    r = _run(sc)
    fx, fy, px, py = [np.float32(v) for v in sc["camera"]]
    d = sc["depth"].astype(np.float32)
    f = np.float32(sc["depth_factor"])
    H, W = d.shape
    x = np.arange(W, dtype=np.float32)[None, :]
    y = np.arange(H, dtype=np.float32)[:, None]
    want = np.stack([(x - px) * d / fx / f, (y - py) * d / fy / f, d / f], -1).astype(np.float32)
    want[d == 0] = 0
    np.testing.assert_array_equal(r["eye"], want)


def test_objects_without_depth_or_area():
    sc = make_scene(seed=4, n_obj=2)
    c0 = sorted(sc["poses"])[0]
    dep = sc["depth"].copy()
    dep[sc["label"] == c0] = 0  # every pixel of one object is a hole
    sc2 = dict(sc, depth=dep)
    r = _run(sc2, max_iter=300)
    assert (r["final"][c0] == -1).all() and not r["poses"][:, :, c0].any()
    for c in sc["poses"]:
        if c != c0:
            assert r["final"][c][0] >= 0
    lab = np.zeros_like(sc["label"])
    lab[:10, :30] = 1
    r = _run(dict(sc, label=lab))
    assert r["n_obj"] == 0 and not r["poses"].any() and (r["final"] == -1).all()
